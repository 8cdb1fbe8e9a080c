// Attention forward with ONE wave per SIMD (head_dim 64, bounded softmax; gfx950).  Reference: the
// compiled flex_attention forward behind attn.py:13-16 with the frame mask of attn.py:24-62; the
// arithmetic is attn_fwd.hip attn_fwd16_k's (q' = bf16(c q), P = exp2(c s) without a running max,
// P in bf16 in the permuted key order, O^T += V^T P and ones^T P as MFMAs, one 16x16x32 chain per
// output tile with the key parts in sweep order).
//
// A workgroup of 4 waves takes 512 queries, each wave 128 (8 query tiles of 16): every K fragment
// read from LDS feeds 8 S MFMAs and every V^T fragment 8 O MFMAs (twice attn_fwd16_k's), and the
// wave holds q', O^T and the row sums in AGPRs (224 registers hipcc never touches: this translation
// unit is built with -amdgpu-mfma-vgpr-form -amdgpu-spill-vgpr-to-agpr=0, csrc/Makefile).  The
// 64-key tiles stream through a 3-slot LDS ring (tiles t, t + 1 resident, t + 2 landing; one barrier
// per tile).  A run of FULL tiles is ONE hand-placed statement (tools/gen_fwd4_asm.py ->
// attn_fwd4_step.inc) software-pipelined across the 32-key parts: the exponentials of one part run
// under the S and O MFMAs of its neighbours.  Masked (diagonal / window-edge / ragged) tiles take a
// one-tile statement with the per-query key range applied after the exponentials; tiles a wave does
// not see only keep the ring and the barrier.
#include "attn_fwd4.hpp"

#include <utility>

namespace owlk_fwd4 {
namespace {

#include "attn_fwd4_step.inc"

constexpr int QW = 128, KT4 = 64, SLOT4 = 16384, NSLOT4 = 3;

template <class F, int... I>
DEV void static_for4_(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
DEV void static_for4(F&& f) {
  static_for4_(f, std::make_integer_sequence<int, N>{});
}

DEV unsigned lds_u32(const void* p) { return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)p; }

__global__ __launch_bounds__(256, 1) void attn_fwd4_k(Fwd4P p) {
  // ring (48 KiB) | the epilogue's O staging reuses it and the 16 KiB after it
  __shared__ __attribute__((aligned(16))) char smem[4 * SLOT4];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = lane & 15, g = lane >> 4;
  const BlockIds bid = xcd_block_ids();
  const long b = bid.z;
  const int head = bid.y;
  const int ntq = (int)((p.Lq + FWD4_QTW - 1) / FWD4_QTW);
  const long q0 = (long)(ntq - 1 - bid.x) * FWD4_QTW;  // heaviest (latest) query blocks first
  const long r0 = q0 + QW * w;
  const MaskP& m = p.m;
  const bf16* Q = p.q + b * p.sqb + head * 64;
  const bf16* K = p.k + b * p.skb + head * 64;
  const bf16* V = p.v + b * p.svb + head * 64;

  // the workgroup's key range (attn_fwd16_k): frames of its queries, causal / window
  const long qlast = (q0 + FWD4_QTW < p.Lq ? q0 + FWD4_QTW : p.Lq) - 1;
  const int fq_lo = frame_of(m, q0), fq_hi = frame_of(m, qlast);
  const int lo_f = m.window > 0 ? max(0, fq_lo - m.window + 1) : 0;
  const int hi_f = m.causal ? fq_hi : (m.window > 0 ? min(m.n_frames - 1, fq_hi + m.window - 1) : m.n_frames - 1);
  long kv_begin = (long)lo_f * m.tpf;
  long kv_end = ((long)hi_f + 1) * m.tpf;
  if (kv_end > p.Lkv) kv_end = p.Lkv;
  kv_begin = (kv_begin / KT4) * KT4;
  const int ntiles = kv_end > kv_begin ? (int)((kv_end - kv_begin + KT4 - 1) / KT4) : 0;
  // tiles wholly inside the tensor (the ragged last one is DMA'd with clamped rows, by this code)
  const int nwhole = (int)((p.Lkv - kv_begin) / KT4) < ntiles ? (int)((p.Lkv - kv_begin) / KT4) : ntiles;

#ifndef FWD4_FORM
#define FWD4_FORM 16
#endif
  // query tiles per wave: 8 of 16 (16x16x32 form) or 4 of 32 (32x32x16 form)
  constexpr int QTN = FWD4_FORM == 32 ? 4 : 8, QTS = FWD4_FORM == 32 ? 32 : 16;
  const int qlane = FWD4_FORM == 32 ? (lane & 31) : c;  // this lane's query within a query tile
  const int kh = FWD4_FORM == 32 ? (lane >> 5) : g;     // its key-row group (4 kh + r / acc_row)
  // q' = bf16(c q) fragments, the B operand of S^T (16x16x32: d 32 kd + 8 g of query 16 t4 + c;
  // 32x32x16: d 16 ks + 8 h of query 32 qt + (lane & 31)); O^T = 0
  {
    constexpr int NK = FWD4_FORM == 32 ? 4 : 2, KW = FWD4_FORM == 32 ? 16 : 32;
    unsigned qv[QTN][NK][4];
#pragma unroll
    for (int t4 = 0; t4 < QTN; ++t4) {
      const long q = r0 + QTS * t4 + qlane;
#pragma unroll
      for (int kd = 0; kd < NK; ++kd) {
        bf16x8 x = q < p.Lq ? *(const bf16x8*)(Q + q * p.ldq + KW * kd + 8 * kh) : bf16x8{};
        float f[8];
        unpack8(x, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] *= p.scale_log2;
        const u32x4 u = __builtin_bit_cast(u32x4, pack8(f));
#pragma unroll
        for (int e = 0; e < 4; ++e) qv[t4][kd][e] = u[e];
      }
    }
#if FWD4_FORM == 32
    // the row-sum selector (A of the 16x16x32 row-sum MFMA): row (lane & 15) < 8 takes k-groups 0 and 2
    // (lanes of query n), rows >= 8 k-groups 1 and 3 (query n + 16)
    fwd4_agpr_init(qv, (((lane & 15) < 8) == (((lane >> 4) & 1) == 0)) ? 0x3F803F80u : 0u);
#else
    fwd4_agpr_init(qv, 0x3F803F80u);  // ones: bf16 1.0 pairs
#endif
  }
  // each query's allowed keys [klo, khi) (causal, window; ragged rows and queries past Lq: none)
  int klo[QTN], khi[QTN];
#pragma unroll
  for (int t4 = 0; t4 < QTN; ++t4) {
    const long q = r0 + QTS * t4 + qlane;
    const int fq = frame_of(m, q);
    const int tpf = (int)m.tpf;
    int lo = 0, hi = (int)p.Lkv;
    if (m.causal) hi = min(hi, (fq + 1) * tpf);
    if (m.window > 0) {
      lo = max(lo, (fq - m.window + 1) * tpf);
      if (!m.causal) hi = min(hi, (fq + m.window) * tpf);
    }
    if (q >= p.Lq) lo = hi = 0;
    klo[t4] = lo;
    khi[t4] = hi;
  }
  const long wlast = r0 + QW - 1 < p.Lq ? r0 + QW - 1 : p.Lq - 1;
  const bool wave_live = r0 < p.Lq;
  const int wfq0 = frame_of(m, r0), wfq1 = frame_of(m, wlast);
  TileRange full = full_range_kv(m, b, wfq0, wfq1, kv_begin, p.Lkv, KT4);
  if (!wave_live) full = TileRange{1, 0};
  if (full.lo < 0) full.lo = 0;
  if (full.hi > ntiles) full.hi = ntiles;
  full.lo = __builtin_amdgcn_readfirstlane(full.lo);
  full.hi = __builtin_amdgcn_readfirstlane(full.hi);

  // per-lane operands
  const unsigned L0 = lds_u32(smem);
  W4Lane f;
#if FWD4_FORM == 32
  // K rows (lane & 31), d chunk 2 ks + h (frag_row<SW_ROW>); V^T frag_tr<SW_TR> of d tile cb
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const int r = lane & 31;
    f.kr[ks] = L0 + (unsigned)(r * 128 + (((2 * ks + (lane >> 5)) ^ swz_row(r)) << 4));
  }
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
    const int h = lane >> 5, qq = (lane & 15) >> 2, pp = lane & 3, ra = 4 * h + qq;
    const int ch = 4 * cb + 2 * (g & 1) + (pp >> 1);
    f.vt[cb] = L0 + (unsigned)(ra * 128 + ((ch ^ swz_tr(ra)) << 4) + 8 * (pp & 1));
  }
  constexpr int SWV = SW_TR;
#else
  f.kr[0] = L0 + (unsigned)(c * 128 + (((0 + g) ^ swz_row(c)) << 4));
  f.kr[1] = L0 + (unsigned)(c * 128 + (((4 + g) ^ swz_row(c)) << 4));
#pragma unroll
  for (int ds = 0; ds < 4; ++ds) {
    const int x = 4 * g + (c >> 2), ch = 2 * ds + ((c & 3) >> 1);
    f.vt[ds] = L0 + (unsigned)(x * 128 + ((ch ^ swz_dual(x)) << 4) + 8 * (c & 1));
  }
  constexpr int SWV = SW_DUAL;
#endif
  const GldsOff gk = glds_offsets<SW_ROW>(p.ldk, w, lane), gv = glds_offsets<SWV>(p.ldv, w, lane);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    f.ko[h] = gk.o[h];
    f.vo[h] = gv.o[h];
  }
  W4Scalar sc;
  sc.m0k = __builtin_amdgcn_readfirstlane(L0 + (unsigned)(w * 2048));
  const unsigned kstep = (unsigned)(KT4 * p.ldk * 2), vstep = (unsigned)(KT4 * p.ldv * 2);

  // the ring: tile i in slot i % 3; whole tiles by the per-lane offsets, the ragged one clamped
  auto issue = [&](int i) {
    char* buf = smem + (i % NSLOT4) * SLOT4;
    const long c0 = kv_begin + (long)i * KT4;
    if (i < nwhole) {
      tile_glds_fast(buf, K + c0 * p.ldk, gk, w);
      tile_glds_fast(buf + 8192, V + c0 * p.ldv, gv, w);
    } else {
      tile_glds<SW_ROW>(buf, K, p.ldk, c0, p.Lkv, w, lane);
      tile_glds<SWV>(buf + 8192, V, p.ldv, c0, p.Lkv, w, lane);
    }
  };
  if (ntiles > 0) issue(0);
  if (ntiles > 1) issue(1);
  OWLK_VMCNT(0);
  __syncthreads();

  // the run: FULL tiles [full.lo, full.hi) as one statement when >= 2; its in-statement DMA covers the
  // whole tiles t + 2 < nwhole, so with a ragged tile R the run stops at R - 3 (R - 2 issues R here)
  int run_lo = full.lo, run_hi = full.hi - 1;
  if (nwhole < ntiles && run_hi > ntiles - 4) run_hi = ntiles - 4;
  if (run_hi - run_lo + 1 < 2) run_lo = run_hi = -1;
  run_lo = __builtin_amdgcn_readfirstlane(run_lo);
  run_hi = __builtin_amdgcn_readfirstlane(run_hi);

  for (int t = 0; t < ntiles;) {
    const long c0 = kv_begin + (long)t * KT4;
    if (t == run_lo) {
      const int n = run_hi - run_lo + 1;
      int dl = nwhole - 2 - t;  // iterations whose tile t + 2 is whole (and exists)
      dl = dl < 0 ? 0 : (dl > n ? n : dl);
      sc.kb = K + (c0 + 2 * KT4) * p.ldk;
      sc.vb = V + (c0 + 2 * KT4) * p.ldv;
      fwd4_run(t % NSLOT4, n, dl, f, sc, 0, kstep, vstep);
      t += n;
      continue;
    }
    int kind = TILE_FULL;
    if (t < full.lo || t >= full.hi) {
      const long clast = c0 + KT4 - 1 < p.Lkv ? c0 + KT4 - 1 : p.Lkv - 1;
      kind = wave_live ? classify(m, b, wfq0, wfq1, frame_of(m, c0), frame_of(m, clast)) : TILE_EMPTY;
      if (kind == TILE_FULL && c0 + KT4 > p.Lkv) kind = TILE_PARTIAL;
    }
    kind = __builtin_amdgcn_readfirstlane(kind);
    int fl = 0;
    if (t + 2 < ntiles) {
      if (t + 2 < nwhole && kind != TILE_EMPTY) {
        fl = 1;
        sc.kb = K + (c0 + 2 * KT4) * p.ldk;
        sc.vb = V + (c0 + 2 * KT4) * p.ldv;
      } else {
        issue(t + 2);
      }
    }
    if (kind == TILE_FULL) {
      fwd4_tile<false>(t % NSLOT4, f, sc, fl);
    } else if (kind == TILE_PARTIAL) {
#pragma unroll
      for (int t4 = 0; t4 < QTN; ++t4) {
        f.mlo[t4] = klo[t4] - (int)c0 - 4 * kh;
        f.mhi[t4] = khi[t4] - (int)c0 - 4 * kh;
      }
      fwd4_tile<true>(t % NSLOT4, f, sc, fl);
    }
    OWLK_VMCNT(0);
    __syncthreads();
    ++t;
  }

  // ---- epilogue: O = O^T / rowsum through this wave's 16 KiB of LDS (whole 128-B rows, chunk x of row
  // r at x ^ (r & 7)), lse = log2(rowsum)
  char* stg = smem + w * 16384;
#if FWD4_FORM == 32
  static_for4<4>([&](auto tc) {
    constexpr int qt = decltype(tc)::value;
    float o[36];
    fwd4_acc_read<qt>(o);
    // the row-sum tile: lane (n, g) holds query n (g < 2) or n + 16 (g >= 2)
    const int q31 = lane & 31, h = lane >> 5;
    const float l = __shfl(o[32], q31 < 16 ? q31 : q31 + 16, 64);
    const float inv = l > 0.f ? 1.f / l : 0.f;
    const int r = 32 * qt + q31;
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        bf16x4 v4;
#pragma unroll
        for (int e = 0; e < 4; ++e) v4[e] = (bf16)(o[16 * cb + 4 * jj + e] * inv);
        *(bf16x4*)(stg + r * 128 + (((4 * cb + jj) ^ (r & 7)) << 4) + 8 * h) = v4;
      }
    const long q = r0 + r;
    if (q < p.Lq && h == 0) p.lse[(b * p.H + head) * p.Lq + q] = l > 0.f ? __log2f(l) : -INFINITY;
  });
#else
  static_for4<8>([&](auto tc) {
    constexpr int t4 = decltype(tc)::value;
    float o[17];
    fwd4_acc_read<t4>(o);
    const float l = o[16];
    const float inv = l > 0.f ? 1.f / l : 0.f;
    const int r = 16 * t4 + c;
#pragma unroll
    for (int ds = 0; ds < 4; ++ds) {
      bf16x4 v4;
#pragma unroll
      for (int e = 0; e < 4; ++e) v4[e] = (bf16)(o[4 * ds + e] * inv);
      *(bf16x4*)(stg + r * 128 + (((2 * ds + (g >> 1)) ^ (r & 7)) << 4) + 8 * (g & 1)) = v4;
    }
    const long q = r0 + r;
    if (q < p.Lq && g == 0) p.lse[(b * p.H + head) * p.Lq + q] = l > 0.f ? __log2f(l) : -INFINITY;
  });
#endif
  wave_lds_handoff();
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int r = 8 * it + (lane >> 3), x = lane & 7;
    const long q = r0 + r;
    const bf16x8 v = *(const bf16x8*)(stg + r * 128 + ((x ^ (r & 7)) << 4));
    if (q < p.Lq) *(bf16x8*)(p.o + b * p.sob + q * p.ldo + head * 64 + 8 * x) = v;
  }
}

}  // namespace
}  // namespace owlk_fwd4

int owlk_fwd4_launch(const Fwd4P& p, hipStream_t s) {
  const MaskP& m = p.m;
  if (m.doc || m.kv_lo || m.q_offset != 0 || p.Lq != p.Lkv) return -1;
  // 32-bit per-lane DMA offsets within a tile and int key indices
  if (p.Lkv >= (1L << 31) / 2 || 64L * (p.ldk > p.ldv ? p.ldk : p.ldv) * 2 >= (1L << 31)) return -1;
  const dim3 grid((unsigned)((p.Lq + FWD4_QTW - 1) / FWD4_QTW), (unsigned)p.H, (unsigned)p.B);
  hipLaunchKernelGGL(owlk_fwd4::attn_fwd4_k, grid, dim3(256), 0, s, p);
  return 0;
}
