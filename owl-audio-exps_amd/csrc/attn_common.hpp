// Frame-mask geometry shared by the attention kernels.
//
// Reference mask (attn.py:24-62, mask_mod):  allowed(q, kv) <=>
//     frame_kv <= frame_q                         (causal)
//   & |frame_q - frame_kv| < window               (window_len; None = all frames)
//   & doc_id[b, frame_q] == doc_id[b, frame_kv]   (packed documents)
// with frame(i) = i // tokens_per_frame and q shifted by q_offset (KV-cache decode).
// Nothing is materialised: tiles are classified EMPTY / FULL / PARTIAL from frame ranges and
// per-frame helper arrays built once per forward by the host:
//   kv_lo[b, f]     first kv frame any query of frame f may see (window + first doc occurrence)
//   q_hi[b, f]      last query frame that may see kv frame f
//   run_start[b, f] first frame of the contiguous same-doc run holding f
//   doc[b, f]       doc id (int32)
#pragma once
#include "common.hpp"

struct MaskP {
  long tpf;            // tokens per frame
  unsigned magic;      // floor(2^32 / tpf) + 1 (exact frame division for idx < 2^32 / tpf); 0 if tpf == 1
  int window;          // frames; <= 0 means unlimited
  int causal;
  long q_offset;       // tokens (KV cache)
  int n_frames;        // kv frames (Lkv / tpf, rounded up)
  const int* kv_lo;    // [B, n_frames] or null
  const int* q_hi;     // [B, n_frames] or null
  const int* run_start;
  const int* doc;
  long fstride;        // batch stride of the frame arrays
};

DEV int frame_of(const MaskP& m, long idx) {
  return m.magic ? (int)__umulhi((unsigned)idx, m.magic) : (int)idx;
}

// Packed documents (every doc one contiguous run of frames, causal): the caller passes kv_lo / q_hi
// without doc / run_start.  Then allowed(q, k) <=> kv_lo[fq] <= fk <= fq (kv_lo = max(run start,
// fq - W + 1), non-decreasing in fq) -- an index range per row, like the doc-free mask.
DEV bool runs_mode(const MaskP& m) { return !m.doc && m.kv_lo && m.causal; }

enum TileKind { TILE_EMPTY = 0, TILE_FULL = 1, TILE_PARTIAL = 2 };

// classify query frames [fq0, fq1] x kv frames [fk0, fk1] for batch b
DEV int classify(const MaskP& m, long b, int fq0, int fq1, int fk0, int fk1) {
  if (m.causal && fk0 > fq1) return TILE_EMPTY;
  if (m.window > 0) {
    if (fq0 - fk1 >= m.window) return TILE_EMPTY;
    if (!m.causal && fk0 - fq1 >= m.window) return TILE_EMPTY;
  }
  bool pure_doc = true;
  if (runs_mode(m)) {
    const int* kl = m.kv_lo + b * m.fstride;
    if (fk1 < kl[fq0]) return TILE_EMPTY;
    pure_doc = fk0 >= kl[fq1];
  }
  if (m.doc) {
    const int* rs = m.run_start + b * m.fstride;
    const int* dc = m.doc + b * m.fstride;
    const int lo = fq0 < fk0 ? fq0 : fk0, hi = fq1 > fk1 ? fq1 : fk1;
    pure_doc = rs[hi] <= lo;
    if (!pure_doc && rs[fq1] <= fq0 && rs[fk1] <= fk0 && dc[fq0] != dc[fk0]) return TILE_EMPTY;
  }
  bool full = pure_doc;
  if (m.causal) full = full && fk1 <= fq0;
  if (m.window > 0) {
    full = full && (fq1 - fk0 < m.window);
    if (!m.causal) full = full && (fk1 - fq0 < m.window);
  }
  return full ? TILE_FULL : TILE_PARTIAL;
}

// Tiles a wave sweeps form a contiguous index range that classify() would call FULL.  Without a
// document mask that range is analytic, so the tile loop only classifies tiles outside it (the
// per-tile classify is ~120 scalar instructions ahead of the first MFMA).  Half-open [lo, hi);
// empty (lo >= hi) for non-contiguous documents; packed (contiguous-run) documents narrow it by
// kv_lo / q_hi.
struct TileRange {
  int lo, hi;
};
DEV long floordiv_(long a, long b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }
// self = query frames [fq0, fq1]; swept tiles = kv rows [base + t KT, base + t KT + KT)
DEV TileRange full_range_kv(const MaskP& m, long b, int fq0, int fq1, long base, long Lkv, int KT) {
  TileRange r{1, 0};
  if (m.doc) return r;
  long cmin = base, cmax = Lkv - KT;
  if (runs_mode(m)) cmin = max(cmin, (long)m.kv_lo[b * m.fstride + fq1] * m.tpf);
  if (m.causal) cmax = min(cmax, (long)(fq0 + 1) * m.tpf - KT);
  if (m.window > 0) {
    cmin = max(cmin, (long)(fq1 - m.window + 1) * m.tpf);
    if (!m.causal) cmax = min(cmax, (long)(fq0 + m.window) * m.tpf - KT);
  }
  if (cmax < cmin) return r;
  r.lo = (int)floordiv_(cmin - base + KT - 1, KT);
  r.hi = (int)floordiv_(cmax - base, KT) + 1;
  return r;
}
// self = key frames [fk0, fk1]; swept tiles = query rows [base + t TL, base + t TL + TL)
DEV TileRange full_range_q(const MaskP& m, long b, int fk0, int fk1, long base, long Lq, int TL) {
  TileRange r{1, 0};
  if (m.doc) return r;
  long cmin = base, cmax = Lq - TL;
  if (runs_mode(m)) cmax = min(cmax, ((long)m.q_hi[b * m.fstride + fk0] + 1) * m.tpf - TL);
  if (m.causal) cmin = max(cmin, (long)fk1 * m.tpf);
  if (m.window > 0) {
    cmax = min(cmax, (long)(fk0 + m.window) * m.tpf - TL);
    if (!m.causal) cmin = max(cmin, (long)(fk1 - m.window + 1) * m.tpf);
  }
  if (cmax < cmin) return r;
  r.lo = (int)floordiv_(cmin - base + TL - 1, TL);
  r.hi = (int)floordiv_(cmax - base, TL) + 1;
  return r;
}

DEV bool allowed(const MaskP& m, long b, int fq, int fk) {
  if (m.causal && fk > fq) return false;
  if (m.window > 0) {
    const int dd = fq > fk ? fq - fk : fk - fq;
    if (dd >= m.window) return false;
  }
  if (m.doc) {
    const int* dc = m.doc + b * m.fstride;
    if (dc[fq] != dc[fk]) return false;
  }
  return true;
}

// 64-bit allowed-mask of one lane against a 64-row tile of the other side: bit i set iff
// (self, other0 + i) is allowed.  self_is_query selects which side `self` indexes.  Only built
// for PARTIAL tiles, so the FULL-tile hot path carries no mask arithmetic at all.
DEV unsigned long long range_bits(long lo, long hi) {  // bits [lo, hi) of 0..63 (clamped)
  lo = lo < 0 ? 0 : lo;
  hi = hi > 64 ? 64 : hi;
  if (hi <= lo) return 0ull;
  const unsigned long long upto = hi >= 64 ? ~0ull : ((1ull << hi) - 1ull);
  return upto & ~((1ull << lo) - 1ull);
}

DEV unsigned long long tile_bits(const MaskP& m, long b, long self, bool self_ok, long other0, long other_len,
                                 bool self_is_query) {
  unsigned long long bits = 0ull;
  if (!self_ok) return 0ull;
  const int fs = frame_of(m, self + (self_is_query ? m.q_offset : 0));
  if (!m.doc) {
    // without documents the allowed other-side rows are one contiguous index range: causal and
    // window bounds are monotone in the other side's frame (a 64-step per-element loop cost more
    // than the tile's MFMAs)
    const long tpf = m.tpf, W = m.window;
    long lo = 0, hi = other_len;
    if (runs_mode(m)) {  // packed documents: the run bounds arrive through kv_lo / q_hi
      if (self_is_query)
        lo = max(lo, (long)m.kv_lo[b * m.fstride + fs] * tpf);
      else
        hi = min(hi, ((long)m.q_hi[b * m.fstride + fs] + 1) * tpf - m.q_offset);
    }
    if (self_is_query) {  // other = keys, frame(k) in [fs - W + 1, fs] (causal) / (fs - W, fs + W)
      if (m.causal) hi = min(hi, ((long)fs + 1) * tpf);
      if (W > 0) {
        lo = max(lo, ((long)fs - W + 1) * tpf);
        if (!m.causal) hi = min(hi, ((long)fs + W) * tpf);
      }
    } else {  // other = queries (frame of o + q_offset), self = key frame fs
      if (m.causal) lo = max(lo, (long)fs * tpf - m.q_offset);
      if (W > 0) {
        hi = min(hi, ((long)fs + W) * tpf - m.q_offset);
        if (!m.causal) lo = max(lo, ((long)fs - W + 1) * tpf - m.q_offset);
      }
    }
    return range_bits(lo - other0, hi - other0);
  }
  for (int i = 0; i < 64; ++i) {
    const long o = other0 + i;
    if (o >= other_len) break;
    const int fo = frame_of(m, o + (self_is_query ? 0 : m.q_offset));
    const bool ok = self_is_query ? allowed(m, b, fs, fo) : allowed(m, b, fo, fs);
    bits |= (unsigned long long)ok << i;
  }
  return bits;
}

// Replace the elements of a 32x32 accumulator block whose bit is clear by `fill`.  `bh` is the
// tile mask shifted right by 4*h (h = lane >> 5), so element r of block BASE (0 or 32) is bit
// BASE + (r & 3) + 8 * (r >> 2) -- a compile-time index.  Callers branch on a wave-uniform
// "tile is PARTIAL" flag around this, so FULL tiles never execute it.
template <int BASE>
DEV void apply_bits(f32x16& a, unsigned long long bh, float fill) {
  __asm__ volatile("");  // keeps the caller's uniform branch a branch (no if-conversion to selects)
  const unsigned w = BASE ? (unsigned)(bh >> 32) : (unsigned)bh;
#pragma unroll
  for (int r = 0; r < 16; ++r) a[r] = (w >> ((r & 3) + 8 * (r >> 2))) & 1u ? a[r] : fill;
}

// 128-B-row (64 x bf16) tile swizzles: K is read row-wise (ds_read_b128), V through
// ds_read_b64_tr_b16; each gets its own conflict-free XOR of the 16-B chunk index.
DEV int swz_row(int r) { return (r >> 1) & 7; }
DEV int swz_tr(int r) { return ((r >> 1) & 1) << 2; }
// one image serving both row reads (32x32x16 A operand) and transposed reads: distinct chunk
// XORs among same-parity rows of every ds_read_b128 lane group, bit 2 flipping between row
// pairs (r, r+2) for the tr_b16 half-waves.
DEV int swz_dual(int r) { return ((r >> 1) & 7) ^ (((r >> 1) & 1) << 2); }

enum Swz { SW_ROW = 0, SW_TR = 1, SW_DUAL = 2 };
template <int S>
DEV int swz(int r) {
  return S == SW_ROW ? swz_row(r) : (S == SW_TR ? swz_tr(r) : swz_dual(r));
}

// 64 rows x 64 bf16 (128-B rows) tile: global -> 2 x 16 B per thread (256 threads) -> LDS
DEV void tile_load(bf16x8 (&r)[2], const bf16* base, long ld, long r0, long R) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = threadIdx.x + 256 * i;
    const long row = r0 + (c >> 3);
    r[i] = (row >= 0 && row < R) ? *(const bf16x8*)(base + row * ld + (c & 7) * 8) : bf16x8{};
  }
}

template <int S>
DEV void tile_store(char* lds, const bf16x8 (&r)[2]) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = threadIdx.x + 256 * i;
    const int row = c >> 3, ch = c & 7;
    *(bf16x8*)(lds + row * 128 + ((ch ^ swz<S>(row)) << 4)) = r[i];
  }
}

// A/B fragment of v_mfma_f32_32x32x16_bf16 read row-wise: rows row0 + (lane & 31), k = 16 s + 8 h
template <int S>
DEV bf16x8 frag_row(const char* lds, int row0, int s, int lane) {
  const int r = row0 + (lane & 31);
  return *(const bf16x8*)(lds + r * 128 + (((2 * s + (lane >> 5)) ^ swz<S>(r)) << 4));
}

// A fragment X^T-ordered for a product that consumes an accumulator tile as its B operand:
// lane (col = 32 cb + (lane & 31), half h) element j <- tile[row0 + 16 s + 8 (j >> 2) + 4 h + (j & 3)][col]
template <int S>
DEV bf16x8 frag_tr(const char* lds, int row0, int s, int cb, int lane) {
  const int g = lane >> 4, h = lane >> 5;
  const int qq = (lane & 15) >> 2, pp = lane & 3;
  const int ra = row0 + 16 * s + 4 * h + qq, rb_ = ra + 8;
  const int ch = 4 * cb + 2 * (g & 1) + (pp >> 1);
  const s16x4 lo = ds_read_tr16(lds + ra * 128 + ((ch ^ swz<S>(ra)) << 4) + 8 * (pp & 1));
  const s16x4 hi = ds_read_tr16(lds + rb_ * 128 + ((ch ^ swz<S>(rb_)) << 4) + 8 * (pp & 1));
  return join_tr(lo, hi);
}

// ---- v_mfma_f32_16x16x32_bf16 forms (lane column c = lane & 15, k-group / row group g = lane >> 4;
// C/D element r of lane (c, g) is row 4 g + r, column c).  An accumulator tile feeds the next
// product as its B operand with the k order permuted: slot j of group g is row 4 g + j (j < 4) of
// the first 16-row tile and 4 g + (j - 4) of the second; the other operand is read in that order.
template <int BASE>
DEV void apply_bits4(f32x4& a, unsigned long long bh, float fill) {
  __asm__ volatile("");  // keeps the caller's uniform branch a branch
  const unsigned w = (unsigned)(bh >> BASE);
#pragma unroll
  for (int r = 0; r < 4; ++r) a[r] = (w >> r) & 1u ? a[r] : fill;
}

// 16x16x32 A fragment read row-wise: row = row0 + (lane & 15), k = 32 ks + 8 (lane >> 4) .. + 7
template <int S = SW_DUAL>
DEV bf16x8 frag_row16(const char* lds, int row0, int ks, int lane) {
  const int r = row0 + (lane & 15);
  return *(const bf16x8*)(lds + r * 128 + (((4 * ks + (lane >> 4)) ^ swz<S>(r)) << 4));
}

// 16x16x32 A fragment of X^T in the permuted k order: element j of lane (c = lane & 15,
// g = lane >> 4) = tile[row0 + 4 g + (j & 3) + 16 (j >> 2)][16 ds + c], by two ds_read_b64_tr_b16
// (rows 4 g .. 4 g + 3 and 16 + 4 g .. + 3, columns 16 ds + 4 (c & 3) .. + 3 addressed by lane c)
template <int S = SW_DUAL>
DEV bf16x8 frag_tr16(const char* lds, int row0, int ds, int lane) {
  const int c = lane & 15, g = lane >> 4;
  const int ra = row0 + 4 * g + (c >> 2), rb_ = ra + 16;
  const int ch = 2 * ds + ((c & 3) >> 1);
  const s16x4 lo = ds_read_tr16(lds + ra * 128 + ((ch ^ swz<S>(ra)) << 4) + 8 * (c & 1));
  const s16x4 hi = ds_read_tr16(lds + rb_ * 128 + ((ch ^ swz<S>(rb_)) << 4) + 8 * (c & 1));
  return join_tr(lo, hi);
}

// two 16x16 accumulator tiles stacked along k (rows 4 g + r of tile 0, then of tile 1) -> the
// bf16 B fragment in the permuted k order frag_tr16 reads its A operand in
DEV bf16x8 pack_perm(const f32x4& a0, const f32x4& a1) {
  bf16x8 f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    f[j] = (bf16)a0[j];
    f[4 + j] = (bf16)a1[j];
  }
  return f;
}

// accumulator registers 8 s .. 8 s + 7 of a 32x32 tile -> bf16 B fragment for k-step s
DEV bf16x8 acc_frag(const f32x16& a, int s) {
  bf16x8 f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (bf16)a[8 * s + j];
  return f;
}

// row (register) index -> row of a 32x32 accumulator tile for lane half h
DEV int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// LDS-DMA (global_load_lds_dwordx4) of a 64 x 128-B tile by 4 waves: wave w moves rows
// [16w, 16w + 16) in two 1-KiB wave-instructions.  The LDS image is lane-linear, so the chunk
// swizzle is applied to the per-lane SOURCE chunk (an XOR is its own inverse).  Rows past R are
// clamped to R - 1 (valid memory; the consumer masks them).
template <int S>
DEV void tile_glds(char* lds, const bf16* base, long ld, long r0, long R, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 16 * wave + 8 * i + (lane >> 3);
    const int ch = (lane & 7) ^ swz<S>(row);
    long gr = r0 + row;
    gr = gr < R ? gr : R - 1;
    __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)(base + gr * ld + ch * 8),
                                     (void __attribute__((address_space(3)))*)(lds + (16 * wave + 8 * i) * 128), 16,
                                     0, 0);
  }
}

// Same transfer with per-lane byte offsets precomputed once (they do not depend on the tile) and
// a wave-uniform tile base, so each tile costs no VALU address arithmetic (saddr + voffset form).
// Only for tiles fully inside the tensor (the caller keeps tile_glds for the ragged last tile).
struct GldsOff {
  unsigned o[2];
};
template <int S>
DEV GldsOff glds_offsets(long ld, int wave, int lane) {
  GldsOff g;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 16 * wave + 8 * i + (lane >> 3);
    const int ch = (lane & 7) ^ swz<S>(row);
    g.o[i] = (unsigned)((row * ld + ch * 8) * 2);
  }
  return g;
}
DEV void tile_glds_fast(char* lds, const bf16* tile_base, const GldsOff& g, int wave) {
#pragma unroll
  for (int i = 0; i < 2; ++i)
    __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)((const char*)tile_base + g.o[i]),
                                     (void __attribute__((address_space(3)))*)(lds + (16 * wave + 8 * i) * 128), 16,
                                     0, 0);
}

// one 64-float row by one wave-instruction (4 B per lane, lane-linear in LDS)
DEV void glds_f32(char* lds_row, const float* src) {
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                   (void __attribute__((address_space(3)))*)lds_row, 4, 0, 0);
}

// XCD-aware workgroup order (cdna_hip_programming.md T1): consecutive workgroups are dealt to
// the 8 XCDs round-robin, so remap the linear id so that XCD x runs a CONTIGUOUS range of
// (block, head, batch) triples.  Co-resident workgroups on one XCD then hold neighbouring blocks
// of the same head and sweep the same Q/dO or K/V tiles a few tiles apart -- L2 (4 MiB/XCD) hits
// instead of re-fetches.  Bijective (the tail beyond a multiple of 8 keeps its id).
struct BlockIds {
  int x, y, z;
};
DEV BlockIds xcd_block_ids() {
  const unsigned nx = gridDim.x, ny = gridDim.y, n = nx * ny * gridDim.z;
  unsigned lin = blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z);
  const unsigned per = n / 8;
  if (lin < per * 8) lin = (lin % 8) * per + lin / 8;
  BlockIds r;
  r.x = (int)(lin % nx);
  lin /= nx;
  r.y = (int)(lin % ny);
  r.z = (int)(lin / ny);
  return r;
}

#define OWLK_VMCNT(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")
#define OWLK_BARRIER() asm volatile("s_barrier" ::: "memory")

MaskP owlk_make_mask(long tpf, int window, int causal, long q_offset, long Lkv, const int* kv_lo, const int* q_hi,
                     const int* run_start, const int* doc, long fstride);
