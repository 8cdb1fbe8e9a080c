// bf16 MFMA GEMM with fused epilogues for the owl_wms DiT training step (gfx950).
//
//   C[m, n] = epi( sum_k A(m, k) * B(n, k) )
//
//   A(m, k) = A[m*lda + k]   (a_trans = 0, k-contiguous)   or  A[k*lda + m]  (a_trans = 1)
//   B(n, k) = B[n*ldb + k]   (b_trans = 0, k-contiguous)   or  B[k*ldb + n]  (b_trans = 1)
//
// Replaces every cuBLAS nn.Linear GEMM of the reference hot path (SURVEY.md §2.2 row
// "cuBLAS nn.Linear"): forward y = x W^T (+b) uses (0,0); dX = dY W uses (0,1); dW = dY^T X
// uses (1,1).  Tiles: BM x BN x 64, 4 waves (2x2), v_mfma_f32_16x16x32_bf16, operands staged
// global -> VGPR -> LDS (double buffered, one barrier per K-step).  k-contiguous tiles are
// XOR-swizzled for conflict-free ds_read_b128; m/n-contiguous tiles are read with the
// ds_read_b64_tr_b16 hardware transpose through a 32-B block swizzle.  The epilogue goes
// through LDS so every global access is a 16-B row chunk.
#include "common.hpp"

#include <algorithm>
#include <cstdlib>

namespace {

enum Epi : int {
  EPI_STORE = 0,       // C = alpha*acc (+ bf16(bias)) (+ beta*C_old)
  EPI_SILU = 1,        // aux = bf16(acc + bias); C = bf16(silu(aux))            (MLP fc1)
  EPI_GATE_RESID = 2,  // aux = y = bf16(acc + bias); C = bf16(resid + bf16(gate[m/tpf]*y))
  EPI_DSILU = 3,       // C = bf16(bf16(acc) * silu'(aux)) (+ resid := bf16(silu(aux)))  (MLP fc1 bwd)
  EPI_AXPBY = 4,       // C = bf16(bf16(alpha*bf16(acc)) + bf16(beta*aux))        (Newton-Schulz)
  EPI_SCALE2 = 5,      // C = bf16(acc); aux = bf16(alpha*bf16(acc))   (NS: A = X X^T and c*A, muon.py:32-33)
  // C = dO = bf16(alpha*acc) (the attention output's gradient, attn.py:113 backward) and the softmax
  // backward's delta[b, h, t] = sum_c dO[r, 64 h + c] * O[r, 64 h + c] (r = b L + t, aux = O) from the
  // stored bf16 values, attn_delta_k's products in its order: internal, owlk_gemm_attn_delta only
  EPI_DELTA = 6,
  // C = qkv = bf16(acc + bias) (attn.py:82) and, for the q | k columns, the QK-RMSNorm + RoPE rows
  // (attn.py:83-89, rope.py:43-51) into aux = qkr [M, 2 H 64] with rstd [M, 2 H]: qk_rope_fwd_k's
  // operations in its order on the stored bf16 values: internal, owlk_gemm_qk_rope only
  EPI_QKROPE = 7,
};

constexpr int BK = 64;
constexpr int NT = 256;

struct GemmP {
  long M, N, K;
  const bf16* A; long lda, sA;
  const bf16* B; long ldb, sB;
  void* C; long ldc, sC;
  float alpha, beta;
  const float* bias;
  bf16* aux; long ldaux, sAux;
  const bf16* gate; long ldgate, sGate, tpf;
  unsigned tpf_mul; int tpf_shift;  // row / tpf = tpf_mul ? umulhi(row, tpf_mul) >> tpf_shift : row >> tpf_shift
  const bf16* resid; long ldres, sRes;
  int tiles_m, tiles_n;
  long kchunk;  // split-K: K range per blockIdx.y (multiple of BK)
  float* ws;    // split-K partials [split][M][N] (256^2 kernel); null: fp32 atomics combine the splits
  float* colsum_req;  // caller wants colsum[n] += sum_m C[m, n] (stored bf16 values)
  float* colsum;      // ... and the launched kernel fuses it (set by the dispatch, else a separate pass)
  float* cs_part;     // fused column sums as per-(tile row, wave row) partials [tiles_m * 2][N] (deterministic)
  int group_m;        // gemm_pp_kernel tile order: groups of group_m tile rows (<= 1: row-major)
  // frame-strided rows (gemm_pp_kernel only): row r of the operand lives at (r / 64) * fs + (r % 64) * ld
  // -- the video rows of the MMDiT joint sequence (64 video + 1 audio token per frame, mmattn.py:54-60)
  // read / written in place; 0 = plain rows r * ld
  long a_fs, b_fs, c_fs;
  float* delta;  // EPI_DELTA: [M / dl][N / 64][dl] fp32
  long dl;
  // EPI_QKROPE: rope tables [n_tab, 32] fp32 (row stride ld_tab) at row tab_off + (tpos_div ? r % tpos_div : r),
  // rstd [M][qk_cols / 64]; the q | k columns are [0, qk_cols)
  const float* rcos;
  const float* rsin;
  long ld_tab, tab_off, tpos_div;
  float* rstd;
  long qk_cols;
};
constexpr float QK_RMS_EPS = 1.1920928955078125e-07f;  // finfo(float32).eps, F.rms_norm default (elementwise.hip)

constexpr int FRAME_ROWS = 64;  // rows per frame of a frame-strided operand (OWLK_FRAME_ROWS)
#ifndef OWLK_GEMM_EPI2  // 1: gemm_pp_kernel's epilogue in paired-rounding form (epi_apply2); 0: epi_apply
#define OWLK_GEMM_EPI2 1
#endif

// element offset of row r: plain (F = false) or frame-strided
template <bool F>
DEV long row_off(long r, long ld, long fs) {
  return F ? (r >> 6) * fs + (r & 63) * ld : r * ld;
}

// 32-B block swizzle of an m/n-contiguous tile so the 8 k-rows one ds_read_b64_tr_b16 half-wave
// touches land on distinct bank slots (256-B rows for ROWS >= 128, 128-B rows for ROWS == 64)
template <int ROWS>
DEV int swz_t(int k) {
  if (ROWS >= 128) return (k & 3) | (((k >> 3) & 1) << 2);
  return ((k >> 1) & 1) | (((k >> 3) & 1) << 1);
}

// ---- staging: global -> registers for one operand tile (ROWS x 64 along k) ---------------
template <int ROWS, bool TRANS>
struct Stager {
  static constexpr int CHUNKS = ROWS * BK / 8;  // 16-byte chunks in the tile
  static constexpr int PER = CHUNKS / NT;
  bf16x8 r[PER];

  DEV void load(const bf16* base, long ld, long r0, long k0, long R, long K) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + i * NT;
      long row, col;
      bool ok;
      if (!TRANS) {  // [ROWS][64]: 8 chunks per row
        row = r0 + (c >> 3);
        col = k0 + (c & 7) * 8;
        ok = row < R && col < K;
        r[i] = ok ? *(const bf16x8*)(base + row * ld + col) : bf16x8{};
      } else {  // [64][ROWS]: ROWS/8 chunks per k-row
        constexpr int CPR = ROWS / 8;
        row = k0 + c / CPR;
        col = r0 + (c % CPR) * 8;
        ok = row < K && col < R;
        r[i] = ok ? *(const bf16x8*)(base + row * ld + col) : bf16x8{};
      }
    }
  }

  DEV void store(char* lds) const {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + i * NT;
      int off;
      if (!TRANS) {
        const int row = c >> 3, kc = c & 7;
        off = row * 128 + ((kc ^ ((row >> 1) & 7)) << 4);
      } else {
        constexpr int CPR = ROWS / 8;
        const int k = c / CPR, mc = c % CPR;
        off = k * (ROWS * 2) + (((mc >> 1) ^ swz_t<ROWS>(k)) << 5) + ((mc & 1) << 4);
      }
      *(bf16x8*)(lds + off) = r[i];
    }
  }
};

// fragment (8 bf16 along k) for rows [row0, row0+16) of an LDS operand tile, k-substep kk
template <int ROWS, bool TRANS>
DEV bf16x8 read_frag(const char* lds, int row0, int kk, int lane) {
  if (!TRANS) {
    const int r = row0 + (lane & 15);
    const int kc = 4 * kk + (lane >> 4);
    return *(const bf16x8*)(lds + r * 128 + ((kc ^ ((r >> 1) & 7)) << 4));
  } else {
    const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
    const int blk = row0 >> 4;
    const int k0 = 32 * kk + 8 * g + q;
    const int k1 = k0 + 4;
    s16x4 lo = ds_read_tr16(lds + k0 * (ROWS * 2) + ((blk ^ swz_t<ROWS>(k0)) << 5) + pp * 8);
    s16x4 hi = ds_read_tr16(lds + k1 * (ROWS * 2) + ((blk ^ swz_t<ROWS>(k1)) << 5) + pp * 8);
    return join_tr(lo, hi);
  }
}

// read_frag with the transposed reads issued through inline asm (ds_read_tr16_async): the caller
// retires them with its own s_waitcnt lgkmcnt(0) before the MFMAs (ping-pong kernel)
template <int ROWS, bool TRANS>
DEV bf16x8 read_frag_async(const char* lds, int row0, int kk, int lane) {
  if (!TRANS) return read_frag<ROWS, false>(lds, row0, kk, lane);
  const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int blk = row0 >> 4;
  const int k0 = 32 * kk + 8 * g + q;
  const int k1 = k0 + 4;
  s16x4 lo = ds_read_tr16_async(lds + k0 * (ROWS * 2) + ((blk ^ swz_t<ROWS>(k0)) << 5) + pp * 8);
  s16x4 hi = ds_read_tr16_async(lds + k1 * (ROWS * 2) + ((blk ^ swz_t<ROWS>(k1)) << 5) + pp * 8);
  return join_tr(lo, hi);
}

// epilogue for 8 consecutive outputs C[gm, gn .. gn + 8) of batch item z (v = raw accumulators)
// row -> frame (gate row) without an integer division: tpf_mul = ceil(2^(32+s) / tpf), s = floor(log2 tpf),
// exact for rows < 2^31 (the error m*tpf - 2^(32+s) < tpf <= 2^(s+1) times the row stays under 2^(32+s))
DEV unsigned frame_of(const GemmP& p, unsigned row) {
  return p.tpf_mul ? __umulhi(row, p.tpf_mul) >> p.tpf_shift : row >> p.tpf_shift;
}

template <int EPI, bool OF32>
DEV void epi_chunk(const GemmP& p, long z, long gm, long gn, float (&v)[8]) {
  float bb[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bb[e] = 0.f;
  if (p.bias) {  // two 16-B loads (gn % 8 == 0), not eight dependent scalar ones
    const f32x4 lo = *(const f32x4*)(p.bias + gn), hi = *(const f32x4*)(p.bias + gn + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      bb[e] = rb(lo[e]);
      bb[e + 4] = rb(hi[e]);
    }
  }
  if (EPI == EPI_STORE) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = p.alpha * v[e] + bb[e];
    if (OF32) {
      float* C = (float*)p.C + z * p.sC + gm * p.ldc + gn;
      if (p.beta != 0.f) {
        const f32x4 o0 = *(const f32x4*)C, o1 = *(const f32x4*)(C + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] += p.beta * o0[e];
          v[e + 4] += p.beta * o1[e];
        }
      }
      *(f32x4*)C = f32x4{v[0], v[1], v[2], v[3]};
      *(f32x4*)(C + 4) = f32x4{v[4], v[5], v[6], v[7]};
    } else {
      bf16* C = (bf16*)p.C + z * p.sC + gm * p.ldc + gn;
      if (p.beta != 0.f) {
        float o[8];
        unpack8(*(const bf16x8*)C, o);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += p.beta * o[e];
      }
      *(bf16x8*)C = pack8(v);
    }
  } else if (EPI == EPI_SILU) {
    float y[8], s[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      y[e] = rb(v[e] + bb[e]);
      s[e] = silu_f(y[e]);
    }
    *(bf16x8*)(p.aux + z * p.sAux + gm * p.ldaux + gn) = pack8(y);
    *(bf16x8*)((bf16*)p.C + z * p.sC + gm * p.ldc + gn) = pack8(s);
  } else if (EPI == EPI_GATE_RESID) {
    float y[8], g[8], r[8], o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) y[e] = rb(v[e] + bb[e]);
    unpack8(*(const bf16x8*)(p.gate + z * p.sGate + (long)frame_of(p, (unsigned)gm) * p.ldgate + gn), g);
    unpack8(*(const bf16x8*)(p.resid + z * p.sRes + gm * p.ldres + gn), r);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = r[e] + rb(g[e] * y[e]);
    if (p.aux) *(bf16x8*)(p.aux + z * p.sAux + gm * p.ldaux + gn) = pack8(y);
    *(bf16x8*)((bf16*)p.C + z * p.sC + gm * p.ldc + gn) = pack8(o);
  } else if (EPI == EPI_DSILU) {
    float x[8], o[8];
    unpack8(*(const bf16x8*)(p.aux + z * p.sAux + gm * p.ldaux + gn), x);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float sg = sigmoid_f(x[e]);
      o[e] = rb(v[e]) * sg * (1.f + x[e] * (1.f - sg));
    }
    *(bf16x8*)((bf16*)p.C + z * p.sC + gm * p.ldc + gn) = pack8(o);
    if (p.resid) {  // optional second output: the activation silu(aux) itself
      float a[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) a[e] = silu_f(x[e]);
      *(bf16x8*)((bf16*)p.resid + z * p.sRes + gm * p.ldres + gn) = pack8(a);
    }
  } else if (EPI == EPI_AXPBY) {
    float x[8], o[8];
    unpack8(*(const bf16x8*)(p.aux + z * p.sAux + gm * p.ldaux + gn), x);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = rb(rb(p.alpha * rb(v[e])) + rb(p.beta * x[e]));
    *(bf16x8*)((bf16*)p.C + z * p.sC + gm * p.ldc + gn) = pack8(o);
  } else if (EPI == EPI_SCALE2) {
    float y[8], o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      y[e] = rb(v[e]);
      o[e] = rb(p.alpha * y[e]);
    }
    *(bf16x8*)((bf16*)p.C + z * p.sC + gm * p.ldc + gn) = pack8(y);
    *(bf16x8*)(p.aux + z * p.sAux + gm * p.ldaux + gn) = pack8(o);
  }
}

// streaming output chunk: non-temporal 16-B store (epilogue outputs are not re-read by this kernel)
DEV void st_nt(bf16x8* dst, bf16x8 v) { __builtin_nontemporal_store(v, dst); }

// epi_chunk with the bias (already bf16-rounded, bb) and the aux / resid (x) and gate (g) inputs
// supplied by the caller (loaded ahead of time)
template <int EPI, bool OF32, bool CF = false>
DEV void epi_apply(const GemmP& p, long z, long gm, long gn, float (&v)[8], const float (&bb)[8], const bf16x8& x,
                   const bf16x8& g, float (&cs)[8]) {
  if (EPI == EPI_STORE) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = p.alpha * v[e] + bb[e];
    if (OF32) {
      float* C = (float*)p.C + z * p.sC + gm * p.ldc + gn;
      if (p.beta != 0.f) {
        const f32x4 o0 = *(const f32x4*)C, o1 = *(const f32x4*)(C + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] += p.beta * o0[e];
          v[e + 4] += p.beta * o1[e];
        }
      }
      *(f32x4*)C = f32x4{v[0], v[1], v[2], v[3]};
      *(f32x4*)(C + 4) = f32x4{v[4], v[5], v[6], v[7]};
    } else {
      bf16* C = (bf16*)p.C + z * p.sC + row_off<CF>(gm, p.ldc, p.c_fs) + gn;
      if (p.beta != 0.f) {
        float o[8];
        unpack8(*(const bf16x8*)C, o);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += p.beta * o[e];
      }
      st_nt((bf16x8*)C, pack8(v));
    }
  } else if (EPI == EPI_SILU) {
    float y[8], s[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      y[e] = rb(v[e] + bb[e]);
      s[e] = silu_f(y[e]);
    }
    st_nt((bf16x8*)(p.aux + z * p.sAux + gm * p.ldaux + gn), pack8(y));
    st_nt((bf16x8*)((bf16*)p.C + z * p.sC + gm * p.ldc + gn), pack8(s));
  } else if (EPI == EPI_GATE_RESID) {
    float y[8], gg[8], r[8], o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) y[e] = rb(v[e] + bb[e]);
    unpack8(g, gg);
    unpack8(x, r);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = r[e] + rb(gg[e] * y[e]);
    if (p.aux) st_nt((bf16x8*)(p.aux + z * p.sAux + gm * p.ldaux + gn), pack8(y));
    st_nt((bf16x8*)((bf16*)p.C + z * p.sC + gm * p.ldc + gn), pack8(o));
  } else if (EPI == EPI_DSILU) {
    float xx[8], o[8];
    unpack8(x, xx);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float sg = sigmoid_f(xx[e]);
      o[e] = rb(v[e]) * sg * (1.f + xx[e] * (1.f - sg));
    }
    st_nt((bf16x8*)((bf16*)p.C + z * p.sC + gm * p.ldc + gn), pack8(o));
    if (p.resid) {  // optional second output: the activation silu(aux) itself
      float a[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) a[e] = silu_f(xx[e]);
      st_nt((bf16x8*)((bf16*)p.resid + z * p.sRes + gm * p.ldres + gn), pack8(a));
    }
    if (p.colsum) {
#pragma unroll
      for (int e = 0; e < 8; ++e) cs[e] += rb(o[e]);
    }
  } else if (EPI == EPI_AXPBY) {
    float xx[8], o[8];
    unpack8(x, xx);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = rb(rb(p.alpha * rb(v[e])) + rb(p.beta * xx[e]));
    st_nt((bf16x8*)((bf16*)p.C + z * p.sC + gm * p.ldc + gn), pack8(o));
  } else if (EPI == EPI_SCALE2) {
    float y[8], o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      y[e] = rb(v[e]);
      o[e] = rb(p.alpha * y[e]);
    }
    st_nt((bf16x8*)((bf16*)p.C + z * p.sC + gm * p.ldc + gn), pack8(y));
    st_nt((bf16x8*)(p.aux + z * p.sAux + gm * p.ldaux + gn), pack8(o));
  }
}

// epi_apply in paired form (OWLK_GEMM_EPI2): every bf16 rounding of two neighbouring values is one
// v_cvt_pk_bf16_f32 whose packed word is also what gets stored (the integer rb() costs 4 VALU per value;
// the SiLU / dSiLU / gate epilogues ran 2,000-3,200 instructions per wave and tile, now 1,600-2,900:
// -2..4 % per GEMM, profiles/r5i_gemm_epi_ab.txt).  Same operations in the same order as epi_apply,
// bit-identical outputs (tools/gemm_epi_bench.py --compare).  The
// caller passes element offsets of this row chunk in C (c), aux (ao) and resid (ro), formed from per-lane
// bases plus wave-uniform row steps; x / g are the aux-or-resid and gate inputs it loaded.
template <int EPI, bool OF32>
DEV void epi_apply2(const GemmP& p, long c, long ao, long ro, float (&v)[8], const float (&bb)[8],
                    const bf16x8& x, const bf16x8& g, float (&cs)[8]) {
  const u32x4 xw = __builtin_bit_cast(u32x4, x), gw = __builtin_bit_cast(u32x4, g);
  u32x4 o, y;
  if (EPI == EPI_STORE) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = p.alpha * v[e] + bb[e];
    if (OF32) {
      float* C = (float*)p.C + c;
      if (p.beta != 0.f) {
        const f32x4 o0 = *(const f32x4*)C, o1 = *(const f32x4*)(C + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] += p.beta * o0[e];
          v[e + 4] += p.beta * o1[e];
        }
      }
      *(f32x4*)C = f32x4{v[0], v[1], v[2], v[3]};
      *(f32x4*)(C + 4) = f32x4{v[4], v[5], v[6], v[7]};
    } else {
      bf16* C = (bf16*)p.C + c;
      if (p.beta != 0.f) {
        float ob[8];
        unpack8(*(const bf16x8*)C, ob);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += p.beta * ob[e];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = cvt2(v[2 * k], v[2 * k + 1]);
      st_nt((bf16x8*)C, __builtin_bit_cast(bf16x8, o));
    }
  } else if (EPI == EPI_SILU) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      y[k] = cvt2(v[2 * k] + bb[2 * k], v[2 * k + 1] + bb[2 * k + 1]);
      o[k] = cvt2(silu_f(bf_lo(y[k])), silu_f(bf_hi(y[k])));
    }
    st_nt((bf16x8*)(p.aux + ao), __builtin_bit_cast(bf16x8, y));
    st_nt((bf16x8*)((bf16*)p.C + c), __builtin_bit_cast(bf16x8, o));
  } else if (EPI == EPI_GATE_RESID) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      y[k] = cvt2(v[2 * k] + bb[2 * k], v[2 * k + 1] + bb[2 * k + 1]);
      const unsigned t = cvt2(bf_lo(gw[k]) * bf_lo(y[k]), bf_hi(gw[k]) * bf_hi(y[k]));
      o[k] = cvt2(bf_lo(xw[k]) + bf_lo(t), bf_hi(xw[k]) + bf_hi(t));
    }
    if (p.aux) st_nt((bf16x8*)(p.aux + ao), __builtin_bit_cast(bf16x8, y));
    st_nt((bf16x8*)((bf16*)p.C + c), __builtin_bit_cast(bf16x8, o));
  } else if (EPI == EPI_DSILU) {
    u32x4 a;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const unsigned rv = cvt2(v[2 * k], v[2 * k + 1]);
      float ov[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float xx = h ? bf_hi(xw[k]) : bf_lo(xw[k]);
        const float sg = sigmoid_f(xx);
        ov[h] = (h ? bf_hi(rv) : bf_lo(rv)) * sg * (1.f + xx * (1.f - sg));
      }
      o[k] = cvt2(ov[0], ov[1]);
      a[k] = cvt2(silu_f(bf_lo(xw[k])), silu_f(bf_hi(xw[k])));  // stored only with p.resid (no branch per word)
      cs[2 * k] += bf_lo(o[k]);  // unconditional (a select per value otherwise); used only with p.colsum
      cs[2 * k + 1] += bf_hi(o[k]);
    }
    st_nt((bf16x8*)((bf16*)p.C + c), __builtin_bit_cast(bf16x8, o));
    if (p.resid) st_nt((bf16x8*)((bf16*)p.resid + ro), __builtin_bit_cast(bf16x8, a));
  } else if (EPI == EPI_AXPBY) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const unsigned r = cvt2(v[2 * k], v[2 * k + 1]);
      const unsigned s1 = cvt2(p.alpha * bf_lo(r), p.alpha * bf_hi(r));
      const unsigned s2 = cvt2(p.beta * bf_lo(xw[k]), p.beta * bf_hi(xw[k]));
      o[k] = cvt2(bf_lo(s1) + bf_lo(s2), bf_hi(s1) + bf_hi(s2));
    }
    st_nt((bf16x8*)((bf16*)p.C + c), __builtin_bit_cast(bf16x8, o));
  } else if (EPI == EPI_SCALE2) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      y[k] = cvt2(v[2 * k], v[2 * k + 1]);
      o[k] = cvt2(p.alpha * bf_lo(y[k]), p.alpha * bf_hi(y[k]));
    }
    st_nt((bf16x8*)((bf16*)p.C + c), __builtin_bit_cast(bf16x8, y));
    st_nt((bf16x8*)(p.aux + ao), __builtin_bit_cast(bf16x8, o));
  } else if (EPI == EPI_QKROPE) {  // STORE (alpha 1, bias); the stored values go back to the caller in cs
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = p.alpha * v[e] + bb[e];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      o[k] = cvt2(v[2 * k], v[2 * k + 1]);
      cs[2 * k] = bf_lo(o[k]);
      cs[2 * k + 1] = bf_hi(o[k]);
    }
    st_nt((bf16x8*)((bf16*)p.C + c), __builtin_bit_cast(bf16x8, o));
  } else if (EPI == EPI_DELTA) {
    float sd = 0.f;  // this lane's 8 products O * dO, in attn_delta_k's order (the caller joins 8 lanes)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      o[k] = cvt2(p.alpha * v[2 * k], p.alpha * v[2 * k + 1]);
      sd += bf_lo(xw[k]) * bf_lo(o[k]);
      sd += bf_hi(xw[k]) * bf_hi(o[k]);
    }
    st_nt((bf16x8*)((bf16*)p.C + c), __builtin_bit_cast(bf16x8, o));
    cs[0] = sd;
  }
}

template <int BM, int BN, bool AT, bool BT, int EPI, bool OF32>
__global__ __launch_bounds__(NT) void gemm_kernel(GemmP p) {
  constexpr int WTM = BM / 2, WTN = BN / 2;  // wave tile
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE_BYTES = 2 * (A_BYTES + B_BYTES);
  constexpr int EPI_LD = BN + 4;
  constexpr int EPI_BYTES = BM * EPI_LD * 4;
  constexpr int LDS_BYTES = STAGE_BYTES > EPI_BYTES ? STAGE_BYTES : EPI_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // XCD-aware bijective remap of the linear tile id (MI355X_MICROARCH: blocks b, b+8 share an XCD)
  const int nwg = p.tiles_m * p.tiles_n;
  int bid = blockIdx.x;
  {
    const int q = nwg / 8, r = nwg % 8, x = bid % 8;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
  }
  const int tm = bid / p.tiles_n, tn = bid % p.tiles_n;
  const long m0 = (long)tm * BM, n0 = (long)tn * BN;
  const long z = blockIdx.z;
  const bf16* A = p.A + z * p.sA;
  const bf16* B = p.B + z * p.sB;

  Stager<BM, AT> sa;
  Stager<BN, BT> sb;
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const long kbeg = (long)blockIdx.y * p.kchunk;
  const long kend = kbeg + p.kchunk < p.K ? kbeg + p.kchunk : p.K;
  const int nk = (int)((kend - kbeg + BK - 1) / BK);
  sa.load(A, p.lda, m0, kbeg, p.M, p.K);
  sb.load(B, p.ldb, n0, kbeg, p.N, p.K);
  sa.store(smem);
  sb.store(smem + A_BYTES);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      sa.load(A, p.lda, m0, kbeg + (long)(kt + 1) * BK, p.M, p.K);
      sb.load(B, p.ldb, n0, kbeg + (long)(kt + 1) * BK, p.N, p.K);
    }
    const char* la = smem + cur * (A_BYTES + B_BYTES);
    const char* lb = la + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = read_frag<BM, AT>(la, wm * WTM + 16 * i, kk, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = read_frag<BN, BT>(lb, wn * WTN + 16 * j, kk, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      char* nb = smem + (cur ^ 1) * (A_BYTES + B_BYTES);
      sa.store(nb);
      sb.store(nb + A_BYTES);
    }
    __syncthreads();
  }

  // ---- epilogue: accumulators -> LDS fp32 tile -> 16-B row chunks -------------------------
  float* ct = (float*)smem;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = wn * WTN + 16 * j + (lane & 15);
      const int row = wm * WTM + 16 * i + (lane >> 4) * 4;
#pragma unroll
      for (int r = 0; r < 4; ++r) ct[(row + r) * EPI_LD + col] = acc[i][j][r];
    }
  __syncthreads();

  if (p.ws) {
    // skinny split-K: raw fp32 partial tile to ws[split][M][N]; splitk_epi_k sums the splits in
    // order and applies the epilogue
    float* W = p.ws + (long)blockIdx.y * p.M * p.N;
    for (int c = threadIdx.x; c < BM * BN / 4; c += NT) {
      const int row = c / (BN / 4), col = (c % (BN / 4)) * 4;
      const long gm = m0 + row, gn = n0 + col;
      if (gm < p.M && gn < p.N)
        __builtin_nontemporal_store(*(const f32x4*)(ct + row * EPI_LD + col), (f32x4*)(W + gm * p.N + gn));
    }
    return;
  }
  if (OF32 && EPI == EPI_STORE && gridDim.y > 1) {
    // split-K partial: each wave-instruction adds 64 consecutive floats (256 B, full atomic rate)
    float* C = (float*)p.C + z * p.sC;
    for (int row = wave; row < BM; row += NT / 64) {
      const long gm = m0 + row;
      if (gm >= p.M) break;
#pragma unroll
      for (int cc = 0; cc < BN; cc += 64) {
        const long gn = n0 + cc + lane;
        if (gn < p.N) atomicAdd(C + gm * p.ldc + gn, p.alpha * ct[row * EPI_LD + cc + lane]);
      }
    }
    return;
  }

  constexpr int CH = BM * BN / 8;
  for (int c = threadIdx.x; c < CH; c += NT) {
    const int row = c / (BN / 8), col = (c % (BN / 8)) * 8;
    const long gm = m0 + row, gn = n0 + col;
    if (gm >= p.M || gn >= p.N) continue;  // N % 8 == 0 is required by the host
    float v[8];
    {
      const f32x4 lo = *(const f32x4*)(ct + row * EPI_LD + col);
      const f32x4 hi = *(const f32x4*)(ct + row * EPI_LD + col + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = lo[e];
        v[e + 4] = hi[e];
      }
    }
    epi_chunk<EPI, OF32>(p, z, gm, gn, v);
  }
}


// ======================================================================== 256 x 256 tiles
// 8 waves (2 x 4, each 128 x 64), BK 64, operands moved by LDS-DMA (global_load_lds_dwordx4)
// into a 2-stage ring: the next K-step's tiles stream in while the current one feeds 64 MFMAs
// per wave.  Operand bytes per FLOP are half the 128x128 kernel's, which at peak needs more
// L2 -> CU bandwidth (~64 B/clk/CU) than an XCD's L2 delivers.  The LDS-DMA image is lane-linear,
// so the operand swizzles are applied to the per-lane source chunk (XOR: its own inverse).
// Requirements (checked on the host): K % 64 == 0, tiled dims multiples of 256 for transposed
// operands, rows of k-contiguous operands may have a ragged last tile (rows clamped).
constexpr int NT8 = 512;

template <int ROWS, bool TRANS, bool F = false>
DEV void glds_tile(char* lds, const bf16* base, long ld, long r0, long k0, long R, int wave, int lane, long fs = 0) {
  if (!TRANS) {  // [ROWS][64] k-contiguous: 8 rows x 128 B per wave-instruction
#pragma unroll
    for (int i = 0; i < ROWS / 64; ++i) {
      const int rbase = (wave * (ROWS / 64) + i) * 8;
      const int row = rbase + (lane >> 3);
      const int ch = (lane & 7) ^ ((row >> 1) & 7);
      long gr = r0 + row;
      gr = gr < R ? gr : R - 1;
      __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)(base + row_off<F>(gr, ld, fs) +
                                                                                         k0 + ch * 8),
                                       (void __attribute__((address_space(3)))*)(lds + rbase * 128), 16, 0, 0);
    }
  } else {  // [64][ROWS] m/n-contiguous: 1 KiB = 1024 / (2 ROWS) k-rows per wave-instruction
    constexpr int KPI = 512 / ROWS;  // k-rows per instruction
    constexpr int CPR = ROWS / 8;    // 16-B chunks per k-row
#pragma unroll
    for (int i = 0; i < 64 / KPI / 8; ++i) {
      const int kb = (wave * (64 / KPI / 8) + i) * KPI;
      const int k = kb + lane / CPR;
      const int pch = lane % CPR;
      const int lch = ((((pch >> 1) ^ swz_t<ROWS>(k))) << 1) | (pch & 1);
      __builtin_amdgcn_global_load_lds(
          (const void __attribute__((address_space(1)))*)(base + row_off<F>(k0 + k, ld, fs) + r0 + lch * 8),
          (void __attribute__((address_space(3)))*)(lds + kb * ROWS * 2), 16, 0, 0);
    }
  }
}

// BN 256: waves 2 (M) x 4 (N) of 128 x 64, 2-stage ring (128 KiB), the next K-tile's DMA drained
//         at every K-step (one tile in flight, inside the step).
// BN 128: waves 4 x 2 of 64 x 64, 3-stage ring (3 x 48 KiB): two K-tiles in flight across the
//         raw barrier behind a counted vmcnt (cdna_hip_programming.md "Pipelining across
//         barriers"): the wait at the end of step k retires tile k+1 only.
template <int BN, bool AT, bool BT, int EPI, bool OF32>
__global__ __launch_bounds__(NT8, 1) void gemm256_kernel(GemmP p) {
  constexpr int BM = 256, WARPS_N = BN / 64, WTM = BM / (8 / WARPS_N), WTN = 64, TM = WTM / 16, TN = 4;
  constexpr int NBUF = BN == 256 ? 2 : 3;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int OPS = (BM + BN) * BK * 2 / (NT8 * 16);  // LDS-DMA instructions per wave per stage
  __shared__ __attribute__((aligned(16))) char smem[NBUF * STAGE];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / WARPS_N, wn = wave % WARPS_N;

  const int nwg = p.tiles_m * p.tiles_n;
  int bid = blockIdx.x;
  {
    const int q = nwg / 8, r = nwg % 8, x = bid % 8;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
  }
  const int tm = bid / p.tiles_n, tn = bid % p.tiles_n;
  const long m0 = (long)tm * BM, n0 = (long)tn * BN;
  const long z = blockIdx.z;
  const bf16* A = p.A + z * p.sA;
  const bf16* B = p.B + z * p.sB;
  const long kbeg = (long)blockIdx.y * p.kchunk;
  const long kend = kbeg + p.kchunk < p.K ? kbeg + p.kchunk : p.K;
  const int nk = (int)((kend - kbeg) / BK);

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto issue = [&](int kt) {
    char* buf = smem + (kt % NBUF) * STAGE;
    glds_tile<BM, AT>(buf, A, p.lda, m0, kbeg + (long)kt * BK, p.M, wave, lane);
    glds_tile<BN, BT>(buf + A_BYTES, B, p.ldb, n0, kbeg + (long)kt * BK, p.N, wave, lane);
  };
  auto wait_next = [&](bool younger_in_flight) {
    if (NBUF > 2 && younger_in_flight)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(OPS) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
#pragma unroll
  for (int i = 0; i < NBUF - 1; ++i)
    if (i < nk) issue(i);
  wait_next(nk > 1);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");

  for (int kt = 0; kt < nk; ++kt) {
    if (kt + NBUF - 1 < nk) issue(kt + NBUF - 1);
    const char* la = smem + (kt % NBUF) * STAGE;
    const char* lb = la + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = read_frag<BN, BT>(lb, wn * WTN + 16 * j, kk, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = read_frag<BM, AT>(la, wm * WTM + 16 * i, kk, lane);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    wait_next(kt + NBUF - 1 < nk);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }

  // ---- epilogue per wave through a private 16 x 64 fp32 LDS strip (reuses the staging ring)
  float* strip = (float*)smem + wave * (16 * 68);
  const bool atomic = OF32 && EPI == EPI_STORE && gridDim.y > 1;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) strip[((lane >> 4) * 4 + r) * 68 + 16 * j + (lane & 15)] = acc[i][j][r];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const long rbase = m0 + wm * WTM + 16 * i;
    if (atomic) {
      float* C = (float*)p.C + z * p.sC;
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) {
        const long gm = rbase + rr;
        if (gm < p.M) atomicAdd(C + gm * p.ldc + n0 + wn * WTN + lane, p.alpha * strip[rr * 68 + lane]);
      }
    } else {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int c = lane + 64 * q;
        const int rr = c >> 3, col = (c & 7) * 8;
        const long gm = rbase + rr, gn = n0 + wn * WTN + col;
        float v[8];
        const f32x4 lo = *(const f32x4*)(strip + rr * 68 + col);
        const f32x4 hi = *(const f32x4*)(strip + rr * 68 + col + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = lo[e];
          v[e + 4] = hi[e];
        }
        if (gm < p.M) epi_chunk<EPI, OF32>(p, z, gm, gn, v);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

// ======================================================================== 256 x 256, ping-pong
// Same tile / waves / LDS-DMA staging as gemm256_kernel, scheduled as 4 phases per K-tile with
// the two wave groups (wr = 0: rows 0-127, wr = 1: rows 128-255 of the tile) one barrier apart
// (cdna_hip_programming.md §5 "256² 8-phase template", T3-T5): while one wave of a SIMD runs its
// 16-MFMA quadrant, the other issues the LDS reads and LDS-DMA of its next phase.
//
// The ring holds two K-tiles of four 16-KiB half-tiles (A rows 0-127 | A rows 128-255 | B cols
// 0-127 | B cols 128-255); a wave reads only A half wr and B half wc >> 1.  Per K-tile t
// (stage t & 1), per wave, quadrants (m half of the wave's 128 rows, n half of its 64 columns):
//   phase 0: ds_read A(m0) + B(n0) of t; LDS-DMA A(t+1)          MFMA (m0, n0)
//   phase 1: ds_read B(n1)                                        MFMA (m0, n1)
//   phase 2: ds_read A(m1)                                        MFMA (m1, n1)
//   phase 3: LDS-DMA B(t+2); vmcnt -> all of t+1 landed           MFMA (m1, n0)
// WAR: a half-tile is re-staged only after the barrier that follows the last wave's lgkmcnt on
// its previous contents (B last read in phase 1, A in phase 2, group 1 one barrier later).
// RAW: every wave's vmcnt for tile t+1 precedes (in barrier order) the first read of it.
// FS: frame-strided rows (GemmP::a_fs / b_fs / c_fs) of A (bit 0), B (bit 1), C (bit 2; bf16 STORE)
template <bool AT, bool BT, int EPI, bool OF32, int FS = 0>
__global__ __launch_bounds__(NT8, 1) void gemm_pp_kernel(GemmP p) {
  constexpr bool FA = FS & 1, FB = (FS & 2) != 0, FC = (FS & 4) != 0;
  constexpr int HALF = 128 * BK * 2, STAGE = 4 * HALF;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;

  const int nwg = p.tiles_m * p.tiles_n;
  int bid = blockIdx.x;
  {
    const int q = nwg / 8, r = nwg % 8, x = bid % 8;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
  }
  int tm, tn;
  if (p.group_m > 1) {
    // grouped order: an XCD's co-resident tiles form a group_m x (32 / group_m) block, so the
    // A rows and B columns they read fit its L2 together (row-major order streams all of B)
    const int span = p.group_m * p.tiles_n, g = bid / span, first = g * p.group_m;
    const int gs = p.tiles_m - first < p.group_m ? p.tiles_m - first : p.group_m;
    tm = first + (bid % span) % gs;
    tn = (bid % span) / gs;
  } else {
    tm = bid / p.tiles_n;
    tn = bid % p.tiles_n;
  }
  const long m0 = (long)tm * 256, n0 = (long)tn * 256;
  const long z = blockIdx.z;
  const bf16* A = p.A + z * p.sA;
  const bf16* B = p.B + z * p.sB;
  const long kbeg = (long)blockIdx.y * p.kchunk;
  const long kend = kbeg + p.kchunk < p.K ? kbeg + p.kchunk : p.K;
  const int nk = (int)((kend - kbeg) / BK);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto issueA = [&](int t) {
    char* st = smem + (t & 1) * STAGE;
    glds_tile<128, AT, FA>(st, A, p.lda, m0, kbeg + (long)t * BK, p.M, wave, lane, p.a_fs);
    glds_tile<128, AT, FA>(st + HALF, A, p.lda, m0 + 128, kbeg + (long)t * BK, p.M, wave, lane, p.a_fs);
  };
  auto issueB = [&](int t) {
    char* st = smem + (t & 1) * STAGE + 2 * HALF;
    glds_tile<128, BT, FB>(st, B, p.ldb, n0, kbeg + (long)t * BK, p.N, wave, lane, p.b_fs);
    glds_tile<128, BT, FB>(st + HALF, B, p.ldb, n0 + 128, kbeg + (long)t * BK, p.N, wave, lane, p.b_fs);
  };
  const int bcol = (wc & 1) * 64;  // first column of this wave inside its B half
  auto readA = [&](bf16x8 (&af)[4][2], const char* la, int mh) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i][kk] = read_frag_async<128, AT>(la, 64 * mh + 16 * i, kk, lane);
  };
  auto readB = [&](bf16x8 (&bq)[2][2], const char* lb, int nh) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < 2; ++j) bq[j][kk] = read_frag_async<128, BT>(lb, bcol + 32 * nh + 16 * j, kk, lane);
  };
  auto quad = [&](const bf16x8 (&af)[4][2], const bf16x8 (&bq)[2][2], int mh, int nh) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[4 * mh + i][2 * nh + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][kk], bq[j][kk], acc[4 * mh + i][2 * nh + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
#define OWLK_PP_BAR() asm volatile("s_barrier" ::: "memory")
#define OWLK_PP_SYNC()                                                  \
  do {                                                                  \
    asm volatile("s_barrier\n\ts_waitcnt lgkmcnt(0)" ::: "memory");   \
    __builtin_amdgcn_sched_barrier(0);                                  \
  } while (0)

  issueA(0);
  issueB(0);
  if (nk > 1) {
    issueB(1);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  OWLK_PP_BAR();
  if (wr == 1) OWLK_PP_BAR();  // group 1 runs one barrier behind group 0

  bf16x8 af[4][2], b0[2][2], b1[2][2];
  for (int t = 0; t < nk; ++t) {
    const char* la = smem + (t & 1) * STAGE + wr * HALF;
    const char* lb = smem + (t & 1) * STAGE + (2 + (wc >> 1)) * HALF;
    // phase 0
    readB(b0, lb, 0);
    readA(af, la, 0);
    if (t + 1 < nk) issueA(t + 1);
    OWLK_PP_SYNC();
    quad(af, b0, 0, 0);
    OWLK_PP_BAR();
    // phase 1
    readB(b1, lb, 1);
    OWLK_PP_SYNC();
    quad(af, b1, 0, 1);
    OWLK_PP_BAR();
    // phase 2
    readA(af, la, 1);
    OWLK_PP_SYNC();
    quad(af, b1, 1, 1);
    OWLK_PP_BAR();
    // phase 3
    if (t + 2 < nk) {
      issueB(t + 2);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    OWLK_PP_SYNC();
    quad(af, b0, 1, 0);
    OWLK_PP_BAR();
  }
  if (wr == 0) OWLK_PP_BAR();  // pairs with group 1's final barrier: every MFMA / LDS read done
#undef OWLK_PP_BAR
#undef OWLK_PP_SYNC
#ifdef OWLK_GEMM_EXP_NOEPI  // timing experiment only (tools/build_variant.sh -DOWLK_GEMM_EXP_NOEPI)
  {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) t += acc[i][j][0];
    if (t == 1234.5f) ((float*)p.C)[threadIdx.x] = t;
    return;
  }
#endif

  // ---- epilogue per wave through a private 16 x 64 fp32 LDS strip (reuses the staging ring).
  // Each lane owns one 8-column chunk (fixed for the whole tile): its bias is loaded once, and the
  // aux / resid / gate inputs of strip i + 1 are loaded while strip i is formatted and stored, so
  // no strip waits a full global-load latency (per-strip loads cost ~10 us per tile-round).
  const long wrow0 = m0 + 128 * wr, wcol0 = n0 + 64 * wc;
  float* strip = (float*)smem + wave * (16 * 68);
  const bool atomic = OF32 && EPI == EPI_STORE && gridDim.y > 1;
  const int ccol = (lane & 7) * 8;
  const long gn = wcol0 + ccol;
  float bb[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bb[e] = 0.f;
  if (!atomic && p.bias) {
    const f32x4 lo = *(const f32x4*)(p.bias + gn), hi = *(const f32x4*)(p.bias + gn + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      bb[e] = rb(lo[e]);
      bb[e + 4] = rb(hi[e]);
    }
  }
  constexpr bool HAS_X = EPI == EPI_GATE_RESID || EPI == EPI_DSILU || EPI == EPI_AXPBY || EPI == EPI_DELTA;
  constexpr bool HAS_G = EPI == EPI_GATE_RESID;
  static_assert((EPI != EPI_DELTA && EPI != EPI_QKROPE) || OWLK_GEMM_EPI2,
                "EPI_DELTA / EPI_QKROPE are built in the paired epilogue only");
  // prefetch depth (strips): every input of the tile up front where registers allow
  constexpr int PD = (EPI == EPI_DSILU || EPI == EPI_AXPBY || EPI == EPI_DELTA) ? 8 : (EPI == EPI_GATE_RESID ? 4 : 1);
  bf16x8 xin[8][2], gin[8][2];  // [strip][q]
  // OWLK_GEMM_EPI2: per-lane element offsets of row wrow0 + (lane >> 3) in C / aux / resid; the row
  // chunks of the tile are wave-uniform steps d = 16 i + 8 q from them (frame-strided C: the chunk
  // stays inside the lane's 64-row frame block, as wrow0 % 128 == 0 and (d & 63) + 7 < 64)
  const int l8 = lane >> 3;
  const bool full = m0 + 256 <= p.M;
  const long cbase = z * p.sC + row_off<FC>(wrow0 + l8, p.ldc, p.c_fs) + gn;
  const long abase = z * p.sAux + (wrow0 + l8) * p.ldaux + gn;
  const long rbase0 = z * p.sRes + (wrow0 + l8) * p.ldres + gn;
  auto c_step = [&](int d) { return FC ? (long)(d >> 6) * p.c_fs + (long)(d & 63) * p.ldc : (long)d * p.ldc; };
  auto load_in = [&](int i, bf16x8 (&x)[2], bf16x8 (&g)[2]) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      long gm = wrow0 + 16 * i + 8 * q + (lane >> 3);
      gm = gm < p.M ? gm : p.M - 1;
      if (HAS_X && OWLK_GEMM_EPI2) {
        const int d = 16 * i + 8 * q;
        const long xo = EPI == EPI_GATE_RESID ? (full ? rbase0 + d * p.ldres : z * p.sRes + gm * p.ldres + gn)
                                              : (full ? abase + d * p.ldaux : z * p.sAux + gm * p.ldaux + gn);
        x[q] = *(const bf16x8*)((EPI == EPI_GATE_RESID ? p.resid : p.aux) + xo);
      } else if (HAS_X) {
        const bf16* src = EPI == EPI_GATE_RESID ? p.resid + z * p.sRes + gm * p.ldres
                                                 : p.aux + z * p.sAux + gm * p.ldaux;
        x[q] = *(const bf16x8*)(src + gn);
      }
      if (HAS_G) g[q] = *(const bf16x8*)(p.gate + z * p.sGate + (long)frame_of(p, (unsigned)gm) * p.ldgate + gn);
    }
  };
  if (!atomic) {
#pragma unroll
    for (int i = 0; i < PD; ++i) load_in(i, xin[i], gin[i]);
  }
  float cs[8];  // fused column sums of the stored outputs (EPI_DSILU with p.colsum)
#pragma unroll
  for (int e = 0; e < 8; ++e) cs[e] = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (!atomic && i + PD < 8) load_in(i + PD, xin[i + PD], gin[i + PD]);
    // EPI_QKROPE: this strip's rope table rows, loaded before the strip is staged through LDS so their
    // latency hides behind it (the rotation of row chunk q reads rcv[q] / rsv[q])
    f32x4 rcv[2], rsv[2];
    if constexpr (EPI == EPI_QKROPE) {
      if (wcol0 < p.qk_cols) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          long gm = wrow0 + 16 * i + 8 * q + (lane >> 3);
          gm = gm < p.M ? gm : p.M - 1;
          const long pos = p.tab_off + (p.tpos_div > 0 ? gm % p.tpos_div : gm);
          rcv[q] = *(const f32x4*)(p.rcos + pos * p.ld_tab + (lane & 7) * 4);
          rsv[q] = *(const f32x4*)(p.rsin + pos * p.ld_tab + (lane & 7) * 4);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) strip[((lane >> 4) * 4 + r) * 68 + 16 * j + (lane & 15)] = acc[i][j][r];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const long rbase = wrow0 + 16 * i;
    if (atomic && p.ws) {
      // this split's partial, unscaled: 16 B per lane, 4 rows x 256 B per wave-instruction
      float* W = p.ws + (long)blockIdx.y * p.M * p.N;
#pragma unroll
      for (int rq = 0; rq < 4; ++rq) {
        const int rr = 4 * rq + (lane >> 4);
        const long gm = rbase + rr;
        if (gm < p.M)
          *(f32x4*)(W + gm * p.N + wcol0 + 4 * (lane & 15)) = *(const f32x4*)(strip + rr * 68 + 4 * (lane & 15));
      }
    } else if (atomic) {
      float* C = (float*)p.C + z * p.sC;
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) {
        const long gm = rbase + rr;
        if (gm < p.M) atomicAdd(C + gm * p.ldc + wcol0 + lane, p.alpha * strip[rr * 68 + lane]);
      }
    } else {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int rr = 8 * q + (lane >> 3);
        const long gm = rbase + rr;
        float v[8];
        const f32x4 lo = *(const f32x4*)(strip + rr * 68 + ccol);
        const f32x4 hi = *(const f32x4*)(strip + rr * 68 + ccol + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = lo[e];
          v[e + 4] = hi[e];
        }
        if (OWLK_GEMM_EPI2) {
          const int d = 16 * i + 8 * q;
          if (gm < p.M)
            epi_apply2<EPI, OF32>(p, cbase + c_step(d), abase + d * p.ldaux, rbase0 + d * p.ldres, v, bb, xin[i][q],
                                  gin[i][q], cs);
          if constexpr (EPI == EPI_QKROPE) {  // the row's 64 columns (one q / k head) on 8 neighbouring lanes
            if (wcol0 < p.qk_cols) {
              float ss = 0.f;
#pragma unroll
              for (int e = 0; e < 8; ++e) ss += cs[e] * cs[e];
              ss = gm < p.M ? ss : 0.f;
              ss += __shfl_xor(ss, 1, 64);
              ss += __shfl_xor(ss, 2, 64);
              ss += __shfl_xor(ss, 4, 64);
              const float r = rsqrtf(ss / 64 + QK_RMS_EPS);
              if (gm < p.M) {
                const int j = lane & 7;
                const long wh = wcol0 >> 6;
                if (j == 0 && p.rstd) p.rstd[gm * (p.qk_cols >> 6) + wh] = r;
                const f32x4 cv = rcv[q], sv = rsv[q];
                bf16x4 y0, y1;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  const float x0 = rb(cs[2 * e] * r), x1 = rb(cs[2 * e + 1] * r);
                  y0[e] = (bf16)(x0 * cv[e] - x1 * sv[e]);
                  y1[e] = (bf16)(x1 * cv[e] + x0 * sv[e]);
                }
                // lane pairs (j, j ^ 1) share the row: swap halves so each lane stores 16 B, the even lane
                // both y0 quads (q positions 8 m .. 8 m + 7), the odd lane both y1 quads (32 + 8 m ..)
                const uint2 w0 = __builtin_bit_cast(uint2, y0), w1 = __builtin_bit_cast(uint2, y1);
                const bool odd = j & 1;
                const uint2 snd = odd ? w0 : w1;
                const uint2 rcv{(unsigned)__shfl_xor((int)snd.x, 1, 64), (unsigned)__shfl_xor((int)snd.y, 1, 64)};
                const u32x4 ow = odd ? u32x4{rcv.x, rcv.y, w1.x, w1.y} : u32x4{w0.x, w0.y, rcv.x, rcv.y};
                *(u32x4*)(p.aux + gm * p.ldaux + wh * 64 + (odd ? 32 : 0) + 8 * (j >> 1)) = ow;
              }
            }
          }
          if constexpr (EPI == EPI_DELTA) {  // the row's 64 columns (one head) sit on 8 neighbouring lanes
            float sd = gm < p.M ? cs[0] : 0.f;
            sd += __shfl_xor(sd, 1, 64);
            sd += __shfl_xor(sd, 2, 64);
            sd += __shfl_xor(sd, 4, 64);
            if ((lane & 7) == 0 && gm < p.M) {
              const long b = gm / p.dl;
              p.delta[(b * (p.N >> 6) + (gn >> 6)) * p.dl + (gm - b * p.dl)] = sd;
            }
          }
        } else if (gm < p.M) {
          if constexpr (EPI != EPI_DELTA && EPI != EPI_QKROPE)
            epi_apply<EPI, OF32, FC>(p, z, gm, gn, v, bb, xin[i][q], gin[i][q], cs);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if (EPI == EPI_DSILU && p.colsum) {
    // lanes l, l + 8, ..., l + 56 hold the same 8 columns: butterfly over lane bits 3..5, then
    // one fp32 atomic per column per wave (2 waves x tiles_m adders per column)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      cs[e] += __shfl_xor(cs[e], 8, 64);
      cs[e] += __shfl_xor(cs[e], 16, 64);
      cs[e] += __shfl_xor(cs[e], 32, 64);
    }
    if (lane < 8) {
      if (p.cs_part) {  // this wave's partial row; colsum_reduce adds the rows in order afterwards
        float* dst = p.cs_part + (long)(2 * tm + wr) * p.N + gn;
        *(f32x4*)dst = f32x4{cs[0], cs[1], cs[2], cs[3]};
        *(f32x4*)(dst + 4) = f32x4{cs[4], cs[5], cs[6], cs[7]};
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) atomicAdd(p.colsum + gn + e, cs[e]);
      }
    }
  }
}

template <int BM, int BN, bool AT, bool BT, int EPI, bool OF32>
int launch(GemmP& p, long batch, hipStream_t s) {
  p.tiles_m = (int)((p.M + BM - 1) / BM);
  p.tiles_n = (int)((p.N + BN - 1) / BN);
  const int splits = (int)((p.K + p.kchunk - 1) / p.kchunk);
  dim3 grid(p.tiles_m * p.tiles_n, (unsigned)splits, (unsigned)batch);
  hipLaunchKernelGGL((gemm_kernel<BM, BN, AT, BT, EPI, OF32>), grid, dim3(NT), 0, s, p);
  return owlk::check_launch("gemm");
}

template <int BM, int BN, int EPI, bool OF32>
int dispatch_t(GemmP& p, int at, int bt, long batch, hipStream_t s) {
  if (!at && !bt) return launch<BM, BN, false, false, EPI, OF32>(p, batch, s);
  if (!at && bt) return launch<BM, BN, false, true, EPI, OF32>(p, batch, s);
  if (at && bt) return launch<BM, BN, true, true, EPI, OF32>(p, batch, s);
  return launch<BM, BN, true, false, EPI, OF32>(p, batch, s);
}

template <int BM, int BN>
int dispatch_e(GemmP& p, int at, int bt, int epi, int cf32, long batch, hipStream_t s) {
  switch (epi) {
    case EPI_STORE:
      return cf32 ? dispatch_t<BM, BN, EPI_STORE, true>(p, at, bt, batch, s)
                  : dispatch_t<BM, BN, EPI_STORE, false>(p, at, bt, batch, s);
    case EPI_SILU: return dispatch_t<BM, BN, EPI_SILU, false>(p, at, bt, batch, s);
    case EPI_GATE_RESID: return dispatch_t<BM, BN, EPI_GATE_RESID, false>(p, at, bt, batch, s);
    case EPI_DSILU: return dispatch_t<BM, BN, EPI_DSILU, false>(p, at, bt, batch, s);
    case EPI_AXPBY: return dispatch_t<BM, BN, EPI_AXPBY, false>(p, at, bt, batch, s);
    case EPI_SCALE2:  // X X^T only: both operands k-contiguous
      if (at || bt) break;
      return launch<BM, BN, false, false, EPI_SCALE2, false>(p, batch, s);
  }
  owlk::set_error("gemm: unknown epilogue %d", epi);
  return 1;
}


template <bool AT, bool BT, int EPI, bool OF32>
int launch256(GemmP& p, long batch, hipStream_t s) {
  p.tiles_m = (int)((p.M + 255) / 256);
  p.tiles_n = (int)((p.N + 255) / 256);
  const int splits = (int)((p.K + p.kchunk - 1) / p.kchunk);
  dim3 grid(p.tiles_m * p.tiles_n, (unsigned)splits, (unsigned)batch);
  static const int pp = getenv("OWLK_GEMM_PP") ? atoi(getenv("OWLK_GEMM_PP")) : 1;
  static const int fuse_cs = getenv("OWLK_GEMM_COLSUM") ? atoi(getenv("OWLK_GEMM_COLSUM")) : 1;
  if (pp && EPI == EPI_DSILU && batch == 1 && fuse_cs) p.colsum = p.colsum_req;
  // grouped tile order for the short-K GEMMs (K <= 4096: -2..4 % at dit_v4's K = 1536 shapes, -2..6 %
  // at dit_v4_5B's K = 2560, profiles/r5z_gemm_group_5b_ab.txt); at K >= 4608 and for split-K weight
  // gradients row-major order measured equal or better
  static const int group_m = getenv("OWLK_GEMM_GROUP") ? atoi(getenv("OWLK_GEMM_GROUP")) : -1;
  p.group_m = group_m >= 0 ? group_m : (splits == 1 && p.kchunk <= 4096 ? 4 : 0);
  const int fs = (p.a_fs ? 1 : 0) | (p.b_fs ? 2 : 0) | (p.c_fs ? 4 : 0);
  if (fs) {
    // frame-strided rows: only the combinations the MMDiT block uses are built
    bool ok = false;
    if constexpr (!AT && !BT && EPI == EPI_STORE && !OF32) {  // video qkv projection into the joint rows
      if (fs == 4) {
        hipLaunchKernelGGL((gemm_pp_kernel<AT, BT, EPI, OF32, 4>), grid, dim3(NT8), 0, s, p);
        ok = true;
      }
    }
    if constexpr (!AT && !BT && EPI == EPI_GATE_RESID) {  // out-projection reading the joint attention output
      if (fs == 1) {
        hipLaunchKernelGGL((gemm_pp_kernel<AT, BT, EPI, OF32, 1>), grid, dim3(NT8), 0, s, p);
        ok = true;
      }
    }
    if constexpr (!AT && BT && EPI == EPI_STORE && !OF32) {  // dX into the joint dO / from the joint dqkv
      if (fs == 4) {
        hipLaunchKernelGGL((gemm_pp_kernel<AT, BT, EPI, OF32, 4>), grid, dim3(NT8), 0, s, p);
        ok = true;
      }
      if (fs == 1) {
        hipLaunchKernelGGL((gemm_pp_kernel<AT, BT, EPI, OF32, 1>), grid, dim3(NT8), 0, s, p);
        ok = true;
      }
    }
    if constexpr (AT && BT && EPI == EPI_STORE && OF32) {  // weight gradients over joint rows
      if (fs == 1) {
        hipLaunchKernelGGL((gemm_pp_kernel<AT, BT, EPI, OF32, 1>), grid, dim3(NT8), 0, s, p);
        ok = true;
      }
      if (fs == 2) {
        hipLaunchKernelGGL((gemm_pp_kernel<AT, BT, EPI, OF32, 2>), grid, dim3(NT8), 0, s, p);
        ok = true;
      }
    }
    OWLK_REQUIRE(ok && pp, "gemm: frame-strided rows (mask %d) not built for this operand layout / epilogue", fs);
    return owlk::check_launch("gemm256");
  }
  if constexpr (EPI == EPI_DELTA || EPI == EPI_QKROPE) {
    OWLK_REQUIRE(pp && splits == 1 && batch == 1, "gemm: the delta / rope epilogues run in the unsplit ping-pong kernel");
    hipLaunchKernelGGL((gemm_pp_kernel<AT, BT, EPI, OF32>), grid, dim3(NT8), 0, s, p);
  } else if (pp) {
    hipLaunchKernelGGL((gemm_pp_kernel<AT, BT, EPI, OF32>), grid, dim3(NT8), 0, s, p);
  } else {
    hipLaunchKernelGGL((gemm256_kernel<256, AT, BT, EPI, OF32>), grid, dim3(NT8), 0, s, p);
  }
  return owlk::check_launch("gemm256");
}

template <int EPI, bool OF32>
int dispatch256_t(GemmP& p, int at, int bt, long batch, hipStream_t s) {
  if (!at && !bt) return launch256<false, false, EPI, OF32>(p, batch, s);
  if (!at && bt) return launch256<false, true, EPI, OF32>(p, batch, s);
  if (at && bt) return launch256<true, true, EPI, OF32>(p, batch, s);
  return launch256<true, false, EPI, OF32>(p, batch, s);
}

int dispatch256(GemmP& p, int at, int bt, int epi, int cf32, long batch, hipStream_t s) {
  switch (epi) {
    case EPI_STORE:
      return cf32 ? dispatch256_t<EPI_STORE, true>(p, at, bt, batch, s)
                  : dispatch256_t<EPI_STORE, false>(p, at, bt, batch, s);
    case EPI_SILU: return dispatch256_t<EPI_SILU, false>(p, at, bt, batch, s);
    case EPI_GATE_RESID: return dispatch256_t<EPI_GATE_RESID, false>(p, at, bt, batch, s);
    case EPI_DSILU: return dispatch256_t<EPI_DSILU, false>(p, at, bt, batch, s);
    case EPI_AXPBY: return dispatch256_t<EPI_AXPBY, false>(p, at, bt, batch, s);
    case EPI_SCALE2:
      if (at || bt) break;
      return launch256<false, false, EPI_SCALE2, false>(p, batch, s);
    case EPI_DELTA:  // the out-projection dX layout only: dO = dY W (W [out, in], k-contiguous rows of dY)
      if (at || !bt) break;
      return launch256<false, true, EPI_DELTA, false>(p, batch, s);
    case EPI_QKROPE:  // the qkv projection's layout only: qkv = h W^T + b
      if (at || bt) break;
      return launch256<false, false, EPI_QKROPE, false>(p, batch, s);
  }
  owlk::set_error("gemm: unknown epilogue %d", epi);
  return 1;
}
// C[m, n] = alpha sum_s W[s][m, n] + beta C[m, n] (beta 0: C is not read); N % 4 == 0
__global__ __launch_bounds__(256) void splitk_reduce_k(const float* __restrict__ W, int splits, long M, long N,
                                                       float* C, long ldc, float alpha, float beta) {
  const long nq = N / 4, total = M * nq, MN = M * N;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long m = i / nq, n = (i - m * nq) * 4;
    const float* w = W + m * N + n;
    f32x4 a = __builtin_nontemporal_load((const f32x4*)w);
    for (int sp = 1; sp < splits; ++sp) {
      const f32x4 b = __builtin_nontemporal_load((const f32x4*)(w + sp * MN));
#pragma unroll
      for (int e = 0; e < 4; ++e) a[e] += b[e];
    }
    f32x4* c = (f32x4*)(C + m * ldc + n);
    f32x4 o;
    if (beta != 0.f) {
      const f32x4 old = *c;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = alpha * a[e] + beta * old[e];
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = alpha * a[e];
    }
    *c = o;
  }
}

// skinny split-K reduce: v = sum_s W[s][m, n .. n + 8) in split order, then the GEMM's own
// epilogue (bias, SiLU + aux, gate + residual) on the bf16 output
template <int EPI>
__global__ __launch_bounds__(256) void splitk_epi_k(GemmP p, int splits) {
  const long n8 = p.N / 8, total = p.M * n8, MN = p.M * p.N;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long m = i / n8, n = (i - m * n8) * 8;
    const float* w = p.ws + m * p.N + n;
    float v[8];
    {
      const f32x4 lo = __builtin_nontemporal_load((const f32x4*)w), hi = __builtin_nontemporal_load((const f32x4*)(w + 4));
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = lo[e];
        v[e + 4] = hi[e];
      }
    }
    // unrolled so the loads of several splits are in flight at once (the reduce is latency-bound
    // at decode sizes: M = 1..64 rows, a few hundred threads); the adds stay in split order
#pragma unroll 8
    for (int sp = 1; sp < splits; ++sp) {
      const f32x4 lo = __builtin_nontemporal_load((const f32x4*)(w + sp * MN));
      const f32x4 hi = __builtin_nontemporal_load((const f32x4*)(w + sp * MN + 4));
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] += lo[e];
        v[e + 4] += hi[e];
      }
    }
    epi_chunk<EPI, false>(p, 0, m, n, v);
  }
}

// ---------------------------------------------------------------- decode GEMM (M <= 128)
// One 64-token frame (or a CFG pair of them) against full weight matrices: a weight stream.  A
// workgroup owns a 64-row x 64-column output tile and one K chunk of nsub x 256: per 256-deep
// sub-chunk its 4 waves stage the 64 weight rows and 64 activation rows into LDS by LDS-DMA in
// whole 512-B rows (full cache lines; fragment-shaped global loads were TA-bound), then each wave
// multiplies its 16 activation rows against all 64 columns from LDS.  With several K chunks
// (gridDim.y) each workgroup stores its fp32 partial tile and the last one to arrive at the tile
// (arrival counter, agent-scope release/acquire) adds the partials in chunk order and applies the
// epilogue: one launch, deterministic.
// ws = [tile counters: kDecodeCounterBytes, zero on entry, left zero][partials: S x M_pad x N fp32].
constexpr int DEC_T = 64;              // tile rows = tile columns
constexpr int DEC_KC = 256;            // K per staged sub-chunk
constexpr int DEC_ROWB = DEC_KC * 2;   // bytes per staged row
constexpr int DEC_LD = DEC_T + 4;      // fp32 output tile row stride (floats)
constexpr long kDecodeCounterBytes = 4096;

template <int EPI>
__global__ __launch_bounds__(256, 1) void gemm_decode_k(GemmP p, int* counters, int nsub) {
  // two stages of [W rows 0-63 | X rows 64-127] x 512 B, 16-B chunks XOR-swizzled by (row & 31)
  // (conflict-free fragment reads); afterwards stage 0 holds the fp32 tile and the last-arriver
  // flag (one __shared__ object)
  constexpr int STAGE = 2 * DEC_T * DEC_ROWB;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  float* tilef = (float*)smem;
  int* flag = (int*)(smem + DEC_T * DEC_LD * 4);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int tile = blockIdx.x, split = blockIdx.y, S = gridDim.y, mt = blockIdx.z;
  const int tiles = gridDim.x;
  const long n0 = (long)tile * DEC_T, m0 = (long)mt * DEC_T;
  const int r16 = lane & 15, g = lane >> 4;
  const long kfirst = (long)split * nsub * DEC_KC;
  const int nst = (int)((p.K - kfirst + DEC_KC - 1) / DEC_KC < nsub ? (p.K - kfirst + DEC_KC - 1) / DEC_KC : nsub);
  // stage i: waves 0-1 move the 64 weight rows, waves 2-3 the 64 activation rows; a
  // wave-instruction moves 2 rows x 32 chunks (lane -> row + (lane >> 5), LDS slot lane & 31)
  const bool isw = wave < 2;
  const bf16* rowp[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int r = (wave & 1) * 32 + 2 * j + (lane >> 5);
    if (isw) {
      rowp[j] = p.B + (n0 + r) * p.ldb;
    } else {
      const long m = m0 + r < p.M ? m0 + r : p.M - 1;
      rowp[j] = p.A + m * p.lda;
    }
  }
  const int ldsrow0 = (isw ? 0 : DEC_T) + (wave & 1) * 32;
  auto issue = [&](int i) {
    const long kbeg = kfirst + (long)i * DEC_KC;
    const int nch = (int)((p.K - kbeg < DEC_KC ? p.K - kbeg : DEC_KC) / 8);
    char* buf = smem + (i & 1) * STAGE + ldsrow0 * DEC_ROWB;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int r = 2 * j + (lane >> 5);
      int ch = (lane & 31) ^ r;  // (staged row & 31) == r
      ch = ch < nch ? ch : nch - 1;  // past a short last chunk: a valid address, never read
      __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)(rowp[j] + kbeg + ch * 8),
                                       (void __attribute__((address_space(3)))*)(buf + 2 * j * DEC_ROWB), 16, 0, 0);
    }
  };
  f32x4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int xr = DEC_T + 16 * wave + r16;  // this lane's staged activation row
  issue(0);
  if (nst > 1) issue(1);
  for (int sc = 0; sc < nst; ++sc) {
    // raw barriers: __syncthreads() would make hipcc drain the next stage's DMA (vmcnt(0)) too
    if (sc + 1 < nst)
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // stage sc landed, sc + 1 still in flight
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_barrier" ::: "memory");
    const long kbeg = kfirst + (long)sc * DEC_KC;
    const int kc = (int)(p.K - kbeg < DEC_KC ? p.K - kbeg : DEC_KC);  // multiple of 32
    const char* buf = smem + (sc & 1) * STAGE;
    for (int st = 0; st < kc / 32; ++st) {
      const int c = 4 * st + g;
      const bf16x8 a = *(const bf16x8*)(buf + xr * DEC_ROWB + ((c ^ (xr & 31)) << 4));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int wr = 16 * j + r16;
        const bf16x8 b = *(const bf16x8*)(buf + wr * DEC_ROWB + ((c ^ (wr & 31)) << 4));
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[j], 0, 0, 0);
      }
    }
    if (sc + 2 < nst) {
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // every wave is done reading it
      issue(sc + 2);
    }
  }
  __syncthreads();  // staging reads done: the LDS now takes the fp32 tile
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) tilef[(16 * wave + 4 * g + r) * DEC_LD + 16 * j + r16] = acc[j][r];
  __syncthreads();
  const long rows = p.M - m0 < DEC_T ? p.M - m0 : DEC_T;
  // partials [mt][split][tile][64 x 64] fp32 through a buffer descriptor (byte offsets < 2^31)
  const long pstride = (long)tiles * DEC_T * DEC_T * 4;  // bytes between K chunks
  const long mbase = (long)mt * S * pstride + (long)tile * DEC_T * DEC_T * 4;
  const __amdgpu_buffer_rsrc_t prs =
      __builtin_amdgcn_make_buffer_rsrc(p.ws, (short)0, S > 1 ? (int)(S * pstride * gridDim.z) : 0, 0x00020000);
  for (int it = threadIdx.x; it < DEC_T * (DEC_T / 8); it += 256) {
    const int row = it >> 3, c = (it & 7) * 8;
    if (row >= rows) continue;
    const f32x4 lo = *(const f32x4*)(tilef + row * DEC_LD + c), hi = *(const f32x4*)(tilef + row * DEC_LD + c + 4);
    if (S == 1) {
      float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      epi_chunk<EPI, false>(p, 0, m0 + row, n0 + c, v);
    } else {  // write-through (sc1) stores: visible to any XCD without a release fence
      const int off = (int)(mbase + split * pstride + (row * DEC_T + c) * 4);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, lo), prs, off, 0, 16);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, hi), prs, off + 16, 0, 16);
    }
  }
  if (S == 1) return;
  // hand-off (cdna_hip_programming.md Guideline 16, R1 with a counter): every wave drains its sc1
  // partial stores, then lane 0 adds to the tile's arrival counter; the last arriver reads every
  // partial with sc1 loads (past this CU's L1), so neither side needs an agent fence.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* cnt = counters + mt * tiles + tile;
  if (threadIdx.x == 0) *flag = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (*flag != S - 1) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the ticket
  for (int it = threadIdx.x; it < DEC_T * (DEC_T / 8); it += 256) {
    const int row = it >> 3, c = (it & 7) * 8;
    if (row >= rows) continue;
    const int off = (int)(mbase + (row * DEC_T + c) * 4);
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = 0.f;
#pragma unroll 4
    for (int sp = 0; sp < S; ++sp) {
      const f32x4 lo = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(prs, off + sp * (int)pstride, 0, 16));
      const f32x4 hi =
          __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(prs, off + sp * (int)pstride + 16, 0, 16));
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] += lo[e];
        v[e + 4] += hi[e];
      }
    }
    epi_chunk<EPI, false>(p, 0, m0 + row, n0 + c, v);
  }
  if (threadIdx.x == 0) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// (K chunks, sub-chunks per chunk) of the decode plan
void decode_split(long M, long N, long K, long& S, long& nsub) {
  const long mtiles = (M + DEC_T - 1) / DEC_T, tiles = N / DEC_T, subs = (K + DEC_KC - 1) / DEC_KC;
  // one workgroup per CU (128 KiB of LDS): split K only as far as it fills the 256 CUs
  static const int force = getenv("OWLK_DECODE_NSUB") ? atoi(getenv("OWLK_DECODE_NSUB")) : 0;
  long sp = 256 / (tiles * mtiles);
  if (sp < 1) sp = 1;
  nsub = force > 0 ? force : (subs + sp - 1) / sp;
  if (nsub > subs) nsub = subs;
  S = (subs + nsub - 1) / nsub;
}

int launch_decode(GemmP& p, int epi, void* ws, hipStream_t s) {
  long S, nsub;
  decode_split(p.M, p.N, p.K, S, nsub);
  const long tiles = p.N / DEC_T, mtiles = (p.M + DEC_T - 1) / DEC_T;
  int* counters = (int*)ws;
  p.ws = S > 1 ? (float*)((char*)ws + kDecodeCounterBytes) : nullptr;
  const dim3 grid((unsigned)tiles, (unsigned)S, (unsigned)mtiles);
  switch (epi) {
    case EPI_STORE: hipLaunchKernelGGL(gemm_decode_k<EPI_STORE>, grid, dim3(256), 0, s, p, counters, (int)nsub); break;
    case EPI_SILU: hipLaunchKernelGGL(gemm_decode_k<EPI_SILU>, grid, dim3(256), 0, s, p, counters, (int)nsub); break;
    default: hipLaunchKernelGGL(gemm_decode_k<EPI_GATE_RESID>, grid, dim3(256), 0, s, p, counters, (int)nsub); break;
  }
  return owlk::check_launch("gemm_decode");
}

// split-K factor for long reductions onto few 256^2 tiles (weight gradients, K = tokens): at one
// workgroup per CU (128 KiB LDS) the grid runs in ceil(tiles * s / 256) rounds, so pick s to fill
// the last round (e.g. 144 tiles: s = 4 -> 2.25 rounds, 75 % of the third idle; s = 7 -> 3.94);
// >= 2 rounds of work, chunks >= 2048 deep, and a small preference for fewer splits (each adds
// an fp32 atomic pass over the output).
long pick_splits(long tiles, long K) {
  constexpr long CUS = 256;
  long best = 1;
  double best_score = -1.0;
  for (long sp = 2; sp <= 64 && K / sp >= 2048; ++sp) {
    const long wg = tiles * sp;
    if (wg < 2 * CUS) continue;
    const long rounds = (wg + CUS - 1) / CUS;
    const double score = (double)wg / (double)(rounds * CUS) - 0.004 * (double)sp;
    if (score > best_score) {
      best_score = score;
      best = sp;
    }
  }
  return best;
}
}  // namespace

// The 256^2 split-K plan for an fp32 output (weight gradients): number of K splits (1 = none).
// Shared by the launch and by owlk_gemm_splitk_bytes, so the caller sizes the workspace exactly.
static bool fits256(long M, long N, long K, int a_trans, int b_trans, int c_f32, float beta) {
  static const int use256 = getenv("OWLK_GEMM_NO256") ? 0 : 1;
  return use256 && K % 64 == 0 && N % 256 == 0 && (!a_trans || M % 256 == 0) && (!b_trans || N % 256 == 0) &&
         !(c_f32 && beta != 0.f && beta != 1.f);
}
// fewest 256^2 tiles that take the ping-pong kernel (one partial round of 256 CUs beats 3+ rounds of the
// 128^2 kernel: the per-frame modulation GEMM [1,536 x 9,216 x 1,536] has 216); OWLK_GEMM_MIN256 for A/B
static long min_tiles256() {
  static const long v = getenv("OWLK_GEMM_MIN256") ? atol(getenv("OWLK_GEMM_MIN256")) : 192;
  return v;
}
// Skinny-M GEMMs (decode: one 64-token frame against the full weights) give few 64x64 tiles; split K
// so the grid streams the weights from every CU: bf16 output with STORE (beta 0) / SILU / GATE_RESID
// epilogues, applied after a fixed-order reduce of the fp32 partials (deterministic).
static long skinny_splits(long M, long N, long K, long batch, int c_f32, int epi, float beta) {
  if (batch != 1 || c_f32 || M > 256 || K < 512 || K % BK) return 1;
  if (!(epi == EPI_SILU || epi == EPI_GATE_RESID || (epi == EPI_STORE && beta == 0.f))) return 1;
  const long tiles = ((M + 63) / 64) * ((N + 63) / 64);
  if (tiles >= 256) return 1;
  long sp = (768 + tiles - 1) / tiles;         // ~3 workgroups per CU
  const long maxsp = K / (2 * BK);             // >= 2 K-steps per split
  if (sp > maxsp) sp = maxsp;
  if (sp < 2) return 1;
  const long kchunk = ((K + sp - 1) / sp + BK - 1) / BK * BK;
  return (K + kchunk - 1) / kchunk;
}

// Split-K plans (one function, shared by the launch and the workspace query):
//   SKINNY  M <= 256 bf16 outputs with few 64^2 tiles (decode): partials + splitk_epi_k
//   S256    fp32 weight gradients on 256^2 tiles: partials + splitk_reduce_k
//   S128    fp32 long reductions that do not tile by 256 (e.g. proj_in dW, N = 128): 128^2 tiles,
//           partials + splitk_reduce_k (fp32 atomics only without a workspace)
//   DECODE  M <= 128 rows of bf16 output against k-contiguous weights (decode): gemm_decode_k,
//           K chunks summed by the last workgroup of each 64-column tile
enum SplitKind { SPLIT_NONE = 0, SPLIT_SKINNY, SPLIT_256, SPLIT_128, SPLIT_DECODE };
struct SplitPlan {
  int kind;
  long splits, kchunk;
  bool opt = false;  // taken only with a workspace (deterministic partials); else the unsplit plan
};

// frames: frame-strided operand rows (owlk_gemm_frames) -- only the 256^2 kernel reads them, so
// neither the decode plan nor the skinny split-K plan may be taken
static SplitPlan split_plan(long M, long N, long K, long batch, int a_trans, int b_trans, int c_f32, int epi,
                            float beta, bool frames = false, bool allow_opt = true) {
  SplitPlan pl{SPLIT_NONE, 1, K, false};
  static const int use_decode = getenv("OWLK_GEMM_DECODE") ? atoi(getenv("OWLK_GEMM_DECODE")) : 1;
  if (use_decode && !frames && M <= 128 && batch == 1 && !a_trans && !b_trans && !c_f32 && N % DEC_T == 0 && K % 32 == 0 &&
      ((M + DEC_T - 1) / DEC_T) * (N / DEC_T) <= kDecodeCounterBytes / 4 &&
      (epi == EPI_SILU || epi == EPI_GATE_RESID || epi == EPI_STORE)) {
    decode_split(M, N, K, pl.splits, pl.kchunk);  // kchunk field: sub-chunks per chunk
    pl.kind = SPLIT_DECODE;
    return pl;
  }
  auto chunk = [&](long sp) { return ((K + sp - 1) / sp + BK - 1) / BK * BK; };
  const long sk = frames ? 1 : skinny_splits(M, N, K, batch, c_f32, epi, beta);
  if (sk > 1) {
    pl.kchunk = chunk(sk);
    pl.splits = (K + pl.kchunk - 1) / pl.kchunk;
    pl.kind = SPLIT_SKINNY;
    return pl;
  }
  const long tiles128 = ((M + 127) / 128) * ((N + 127) / 128) * batch;
  const long tiles256 = ((M + 255) / 256) * ((N + 255) / 256) * batch;
  if (fits256(M, N, K, a_trans, b_trans, c_f32, beta)) {
    if (c_f32 && epi == EPI_STORE && batch == 1 && (beta == 0.f || beta == 1.f) && K >= 8192 && tiles256 < 1024) {
      const long sp = pick_splits(tiles256, K);
      if (sp > 1) {
        pl.kchunk = chunk(sp);
        pl.splits = (K + pl.kchunk - 1) / pl.kchunk;
        pl.kind = SPLIT_256;
        return pl;
      }
    }
    if (allow_opt && c_f32 && epi == EPI_STORE && batch == 1 && (beta == 0.f || beta == 1.f) && K >= 8192 &&
        K < 16384 && tiles256 < 128) {
      // few tiles, mid K (the per-frame cond gradient [1,536 x 1,536 x 9,216]: 108 -> 62 us): one round
      // of 256^2 splits of >= 1,024 instead of the 128^2 kernel's two, with a workspace only (without:
      // the unsplit plan, deterministic, rather than fp32 atomics).  At K = 1,536 (the modulation
      // weight gradients) the same plan measured equal ([3,072 x 1,536]) or slower ([1,536 x 1,536]:
      // 25 -> 34 us) than the 64^2 kernel (profiles/r5w_small_gemm_ab.txt)
      long sp = 256 / tiles256;
      if (sp > K / 1024) sp = K / 1024;
      if (sp > 1) {
        pl.kchunk = chunk(sp);
        pl.splits = (K + pl.kchunk - 1) / pl.kchunk;
        pl.kind = SPLIT_256;
        pl.opt = true;
        return pl;
      }
    }
    if (tiles256 >= min_tiles256()) return pl;
  }
  if (c_f32 && epi == EPI_STORE && (beta == 1.f || (beta == 0.f && batch == 1)) && K >= 8192 && tiles128 < 1024) {
    long sp = (1024 + tiles128 - 1) / tiles128;
    if (sp > K / 4096) sp = K / 4096;
    if (sp > 1) {
      pl.kchunk = chunk(sp);
      pl.splits = (K + pl.kchunk - 1) / pl.kchunk;
      pl.kind = SPLIT_128;
    }
  }
  return pl;
}

// workspace bytes of a plan's per-split partials (0: the plan does not split or cannot use them)
static long split_ws_bytes(const SplitPlan& pl, long M, long N, long batch) {
  if (pl.kind == SPLIT_NONE || (pl.kind == SPLIT_128 && batch != 1)) return 0;
  if (pl.kind == SPLIT_DECODE)
    return pl.splits > 1 ? kDecodeCounterBytes + pl.splits * ((M + DEC_T - 1) / DEC_T) * DEC_T * N * (long)sizeof(float)
                         : 0;
  return pl.splits * M * N * (long)sizeof(float);
}

static int gemm_dispatch(GemmP& p, long M, long N, long K, long batch,
                         const void* A, long lda, long sA, int a_trans,
                         const void* B, long ldb, long sB, int b_trans,
                         void* C, long ldc, long sC, int c_f32,
                         int epi, float alpha, float beta, const float* bias,
                         void* aux, long ldaux, long sAux,
                         const void* gate, long ldgate, long sGate, long tpf,
                         const void* resid, long ldres, long sRes,
                         void* ws, long ws_bytes, void* stream) {
  OWLK_REQUIRE(M > 0 && N > 0 && K > 0 && batch > 0, "gemm: bad sizes M=%ld N=%ld K=%ld b=%ld", M, N, K, batch);
  OWLK_REQUIRE(N % 8 == 0, "gemm: N=%ld must be a multiple of 8", N);
  OWLK_REQUIRE(a_trans ? (M % 8 == 0) : (K % 8 == 0), "gemm: A contiguous dim must be a multiple of 8");
  OWLK_REQUIRE(b_trans ? (N % 8 == 0) : (K % 8 == 0), "gemm: B contiguous dim must be a multiple of 8");
  OWLK_REQUIRE(lda % 8 == 0 && ldb % 8 == 0 && ldc % 8 == 0, "gemm: leading dims must be multiples of 8");
  OWLK_REQUIRE(((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) % 16 == 0, "gemm: operands must be 16-byte aligned");
  OWLK_REQUIRE(!c_f32 || epi == EPI_STORE, "gemm: fp32 output only with EPI_STORE");
  OWLK_REQUIRE(epi != EPI_GATE_RESID || (gate && resid && tpf > 0), "gemm: gate epilogue needs gate/resid/tpf");
  OWLK_REQUIRE(epi != EPI_GATE_RESID || M < (1L << 31), "gemm: gate epilogue rows must stay below 2^31");
  OWLK_REQUIRE(!(epi == EPI_SILU || epi == EPI_DSILU || epi == EPI_AXPBY || epi == EPI_SCALE2) || aux,
               "gemm: epilogue needs aux");
  OWLK_REQUIRE(epi != EPI_SCALE2 || (!a_trans && !b_trans), "gemm: SCALE2 epilogue needs k-contiguous operands");
  p.M = M; p.N = N; p.K = K;
  p.A = (const bf16*)A; p.lda = lda; p.sA = sA;
  p.B = (const bf16*)B; p.ldb = ldb; p.sB = sB;
  p.C = C; p.ldc = ldc; p.sC = sC;
  p.alpha = alpha; p.beta = beta; p.bias = bias;
  p.aux = (bf16*)aux; p.ldaux = ldaux; p.sAux = sAux;
  p.gate = (const bf16*)gate; p.ldgate = ldgate; p.sGate = sGate; p.tpf = tpf > 0 ? tpf : 1;
  {
    int sh = 0;
    while ((2L << sh) <= p.tpf) ++sh;
    p.tpf_shift = sh;
    p.tpf_mul = (p.tpf & (p.tpf - 1)) ? (unsigned)(((1ULL << (32 + sh)) + p.tpf - 1) / p.tpf) : 0u;
  }
  p.resid = (const bf16*)resid; p.ldres = ldres; p.sRes = sRes;
  hipStream_t s = (hipStream_t)stream;
  const long tiles128 = ((M + 127) / 128) * ((N + 127) / 128) * batch;
  const long tiles256 = ((M + 255) / 256) * ((N + 255) / 256) * batch;
  p.kchunk = K;
  const bool frames = p.a_fs || p.b_fs || p.c_fs;
  SplitPlan pl = split_plan(M, N, K, batch, a_trans, b_trans, c_f32, epi, beta, frames);
  const long pws = split_ws_bytes(pl, M, N, batch);
  bool have_ws = ws && (uintptr_t)ws % 16 == 0 && pws > 0 && ws_bytes >= pws;
  static const int atomic_splitk = getenv("OWLK_GEMM_ATOMIC") ? atoi(getenv("OWLK_GEMM_ATOMIC")) : 0;
  if (pl.opt && (!have_ws || atomic_splitk)) {
    // the opt plan needs its workspace: with fp32 atomics asked for (OWLK_GEMM_ATOMIC), or a
    // workspace that covers the 128^2 plan, take the plan the shape had before it; else unsplit
    // (deterministic) rather than atomics nobody asked for
    const SplitPlan p128 = split_plan(M, N, K, batch, a_trans, b_trans, c_f32, epi, beta, frames, false);
    const long w128 = split_ws_bytes(p128, M, N, batch);
    const bool ws128 = ws && (uintptr_t)ws % 16 == 0 && w128 > 0 && ws_bytes >= w128;
    pl = (atomic_splitk || ws128) ? p128 : SplitPlan{SPLIT_NONE, 1, K, false};
    have_ws = ws128;
  }
  if (pl.kind == SPLIT_DECODE && (pl.splits == 1 || have_ws)) return launch_decode(p, epi, ws, s);
  {
    const long sk = pl.splits;
    if (pl.kind == SPLIT_SKINNY && have_ws) {
      p.kchunk = pl.kchunk;
      p.ws = (float*)ws;
      if (int e = dispatch_e<64, 64>(p, a_trans, b_trans, epi, c_f32, batch, s)) return e;
      const long work = M * (N / 8);
      const unsigned grid = (unsigned)std::min<long>((work + 255) / 256, 2048);
      switch (epi) {
        case EPI_STORE: hipLaunchKernelGGL(splitk_epi_k<EPI_STORE>, dim3(grid), dim3(256), 0, s, p, (int)sk); break;
        case EPI_SILU: hipLaunchKernelGGL(splitk_epi_k<EPI_SILU>, dim3(grid), dim3(256), 0, s, p, (int)sk); break;
        default: hipLaunchKernelGGL(splitk_epi_k<EPI_GATE_RESID>, dim3(grid), dim3(256), 0, s, p, (int)sk); break;
      }
      return owlk::check_launch("splitk_epi");
    }
  }
  // split-K onto an fp32 output: partials into the caller's workspace + one fixed-order reduce
  // (any beta, deterministic); without a large enough workspace (or OWLK_GEMM_ATOMIC=1) fp32
  // atomics onto C, cleared first when beta = 0
  OWLK_REQUIRE(!frames || (fits256(M, N, K, a_trans, b_trans, c_f32, beta) && batch == 1 &&
                           (pl.kind == SPLIT_256 || pl.kind == SPLIT_NONE) &&
                           (pl.kind != SPLIT_256 || (have_ws && !atomic_splitk)) && pl.kchunk % FRAME_ROWS == 0),
               "gemm: frame-strided rows need the 256^2 kernel (M=%ld N=%ld K=%ld)", M, N, K);
  if (frames && pl.kind == SPLIT_NONE) return dispatch256(p, a_trans, b_trans, epi, c_f32, batch, s);
  if (fits256(M, N, K, a_trans, b_trans, c_f32, beta)) {
    const long nsp = pl.kind == SPLIT_256 ? pl.splits : 1;
    if (nsp > 1) {
      p.kchunk = pl.kchunk;
      if (atomic_splitk || !have_ws) {
        if (beta == 0.f)
          OWLK_REQUIRE(hipMemset2DAsync(C, ldc * sizeof(float), 0, N * sizeof(float), M, s) == hipSuccess,
                       "gemm: clearing the split-K output failed");
        return dispatch256(p, a_trans, b_trans, epi, c_f32, batch, s);
      }
      {
        p.ws = (float*)ws;
        if (int e = dispatch256(p, a_trans, b_trans, epi, c_f32, batch, s)) return e;
        const long work = M * (N / 4);
        const unsigned grid = (unsigned)std::min<long>((work + 255) / 256, 2048);
        hipLaunchKernelGGL(splitk_reduce_k, dim3(grid), dim3(256), 0, s, p.ws, (int)nsp, M, N, (float*)C, ldc,
                           alpha, beta);
        return owlk::check_launch("splitk_reduce");
      }
    }
    if (tiles256 >= min_tiles256()) return dispatch256(p, a_trans, b_trans, epi, c_f32, batch, s);
  }
  // long reductions onto small outputs (weight gradients, K = tokens) that do not tile by 256:
  // 128x128 tiles, K split so the grid covers ~4 workgroups per CU; per-split partials + a
  // fixed-order reduce with a workspace, else fp32 atomics onto a cleared (beta 0) or kept (beta 1) C
  if (pl.kind == SPLIT_128) {
    p.kchunk = pl.kchunk;
    if (have_ws && !atomic_splitk) {
      p.ws = (float*)ws;
      if (int e = dispatch_e<128, 128>(p, a_trans, b_trans, epi, c_f32, batch, s)) return e;
      const long work = M * (N / 4);
      const unsigned grid = (unsigned)std::min<long>((work + 255) / 256, 2048);
      hipLaunchKernelGGL(splitk_reduce_k, dim3(grid), dim3(256), 0, s, p.ws, (int)pl.splits, M, N, (float*)C, ldc,
                         alpha, beta);
      return owlk::check_launch("splitk_reduce");
    }
    if (beta == 0.f) {  // the atomics add onto C: clear it first
      OWLK_REQUIRE(hipMemset2DAsync(C, ldc * sizeof(float), 0, N * sizeof(float), M, s) == hipSuccess,
                   "gemm: clearing the split-K output failed");
      p.beta = 1.f;
    }
    return dispatch_e<128, 128>(p, a_trans, b_trans, epi, c_f32, batch, s);
  }
  // small outputs (per-frame modulation, Newton-Schulz) use 64x64 tiles to fill the chip
  if (tiles128 < 512) return dispatch_e<64, 64>(p, a_trans, b_trans, epi, c_f32, batch, s);
  return dispatch_e<128, 128>(p, a_trans, b_trans, epi, c_f32, batch, s);
}

extern "C" int owlk_colsum(const void* x, int x_f32, long R, long N, long ld, float* out, void* ws, long ws_bytes,
                           void* stream);
extern "C" long owlk_colsum_ws_bytes(long R, long N);

// column-sum partials of the fused DSILU epilogue: [tiles_m * 2][N] fp32
static long fused_colsum_bytes(long M, long N) { return ((M + 255) / 256) * 2 * N * (long)sizeof(float); }

extern "C" int owlk_gemm(long M, long N, long K, long batch,
                         const void* A, long lda, long sA, int a_trans,
                         const void* B, long ldb, long sB, int b_trans,
                         void* C, long ldc, long sC, int c_f32,
                         int epi, float alpha, float beta, const float* bias,
                         void* aux, long ldaux, long sAux,
                         const void* gate, long ldgate, long sGate, long tpf,
                         const void* resid, long ldres, long sRes,
                         float* colsum, void* ws, long ws_bytes, void* stream) {
  OWLK_REQUIRE(!colsum || (batch == 1 && !c_f32), "gemm: colsum needs batch 1 and a bf16 output");
  GemmP p{};
  p.colsum_req = colsum;
  if (colsum && ws && (uintptr_t)ws % 16 == 0 && ws_bytes >= fused_colsum_bytes(M, N)) p.cs_part = (float*)ws;
  if (int e = gemm_dispatch(p, M, N, K, batch, A, lda, sA, a_trans, B, ldb, sB, b_trans, C, ldc, sC, c_f32, epi,
                            alpha, beta, bias, aux, ldaux, sAux, gate, ldgate, sGate, tpf, resid, ldres, sRes, ws,
                            ws_bytes, stream))
    return e;
  if (colsum && p.colsum && p.cs_part)  // fused, deterministic: add the per-wave partial rows in order
    return owlk::colsum_reduce(p.cs_part, (int)(((M + 255) / 256) * 2), N, colsum, (hipStream_t)stream);
  if (colsum && !p.colsum)  // not fused by this kernel: a separate (workspace: deterministic) pass
    return owlk_colsum(C, 0, M, N, ldc, colsum, ws, ws_bytes, stream);
  return 0;
}

extern "C" int owlk_attn_delta(const void* o, const void* dout, long ld, long B, long L, int H, int D, float* delta,
                               void* stream);

// dO = dY W (bf16) and the attention backward's delta = rowsum(dO * O) per (sample, head, token): in the
// ping-pong kernel's epilogue when the shape takes it (EPI_DELTA: the head's 64 columns are one wave's
// strip columns, so dO is not read back), else the GEMM and owlk_attn_delta -- the same bits either way
extern "C" int owlk_gemm_attn_delta(long M, long N, long K, const void* dY, long lddy, const void* W, long ldw,
                                    void* dO, long ldc, const void* o, long ldo, long L, int H, int D,
                                    float* delta, void* stream) {
  OWLK_REQUIRE(L > 0 && M % L == 0 && H > 0 && D > 0 && N == (long)H * D && o && delta,
               "gemm_attn_delta: bad shape M=%ld N=%ld L=%ld H=%d D=%d", M, N, L, H, D);
  static const int pp = getenv("OWLK_GEMM_PP") ? atoi(getenv("OWLK_GEMM_PP")) : 1;
  static const int fuse_env = getenv("OWLK_GEMM_DELTA") ? atoi(getenv("OWLK_GEMM_DELTA")) : 1;
  const long tiles256 = ((M + 255) / 256) * ((N + 255) / 256);
  const SplitPlan pl = split_plan(M, N, K, 1, 0, 1, 0, EPI_DELTA, 0.f);
  if (fuse_env && pp && D == 64 && fits256(M, N, K, 0, 1, 0, 0.f) && tiles256 >= min_tiles256() &&
      pl.kind == SPLIT_NONE && ldo % 8 == 0 && (uintptr_t)o % 16 == 0) {
    GemmP p{};
    p.delta = delta;
    p.dl = L;
    return gemm_dispatch(p, M, N, K, 1, dY, lddy, 0, 0, W, ldw, 0, 1, dO, ldc, 0, 0, EPI_DELTA, 1.f, 0.f, nullptr,
                         const_cast<void*>(o), ldo, 0, nullptr, 0, 0, 0, nullptr, 0, 0, nullptr, 0, stream);
  }
  OWLK_REQUIRE(ldo == ldc, "gemm_attn_delta: the unfused form needs O and dO with one row stride");
  if (int e = owlk_gemm(M, N, K, 1, dY, lddy, 0, 0, W, ldw, 0, 1, dO, ldc, 0, 0, EPI_STORE, 1.f, 0.f, nullptr,
                        nullptr, 0, 0, nullptr, 0, 0, 0, nullptr, 0, 0, nullptr, nullptr, 0, stream))
    return e;
  return owlk_attn_delta(o, dO, ldc, M / L, L, H, D, delta, stream);
}

extern "C" int owlk_qk_rope_fwd(const void* qkv, long ldq, long T, int H, int D, const float* cosb,
                                const float* sinb, long ld_tab, long n_tab, long tab_off, long tpos_div, void* out,
                                long ldo, float* rstd, void* stream);

// qkv = h W^T + b (bf16) and the QK-RMSNorm + RoPE rows of its q | k columns: in the ping-pong kernel's
// epilogue when the shape takes it (EPI_QKROPE: a head's 64 columns are one wave's strip columns, so
// qkv is not read back), else the GEMM and owlk_qk_rope_fwd -- the same bits either way
extern "C" int owlk_gemm_qk_rope(long M, long N, long K, const void* A, long lda, const void* W, long ldw,
                                 const float* bias, void* qkv, long ldq, int H, int D, const float* cosb,
                                 const float* sinb, long ld_tab, long n_tab, long tab_off, long tpos_div, void* out,
                                 long ldo, float* rstd, void* stream) {
  OWLK_REQUIRE(H > 0 && (D == 64 || D == 128) && N == 3L * H * D && out && cosb && sinb,
               "gemm_qk_rope: bad shape N=%ld H=%d D=%d", N, H, D);
  {
    const long span = tpos_div > 0 ? (M < tpos_div ? M : tpos_div) : M;
    OWLK_REQUIRE(n_tab > 0 && tab_off >= 0 && tab_off + span <= n_tab,
                 "gemm_qk_rope: positions %ld.. past the %ld-row rope table", tab_off, n_tab);
  }
  static const int pp = getenv("OWLK_GEMM_PP") ? atoi(getenv("OWLK_GEMM_PP")) : 1;
  static const int fuse_env = getenv("OWLK_GEMM_ROPE") ? atoi(getenv("OWLK_GEMM_ROPE")) : 1;
  const long tiles256 = ((M + 255) / 256) * ((N + 255) / 256);
  const SplitPlan pl = split_plan(M, N, K, 1, 0, 0, 0, EPI_QKROPE, 0.f);
  if (fuse_env && pp && D == 64 && fits256(M, N, K, 0, 0, 0, 0.f) && tiles256 >= min_tiles256() &&
      pl.kind == SPLIT_NONE && ldo % 8 == 0 && ld_tab % 4 == 0 && (uintptr_t)out % 16 == 0 &&
      (uintptr_t)cosb % 16 == 0 && (uintptr_t)sinb % 16 == 0) {
    GemmP p{};
    p.rcos = cosb;
    p.rsin = sinb;
    p.ld_tab = ld_tab;
    p.tab_off = tab_off;
    p.tpos_div = tpos_div;
    p.rstd = rstd;
    p.qk_cols = 2L * H * D;
    return gemm_dispatch(p, M, N, K, 1, A, lda, 0, 0, W, ldw, 0, 0, qkv, ldq, 0, 0, EPI_QKROPE, 1.f, 0.f, bias, out,
                         ldo, 0, nullptr, 0, 0, 0, nullptr, 0, 0, nullptr, 0, stream);
  }
  if (int e = owlk_gemm(M, N, K, 1, A, lda, 0, 0, W, ldw, 0, 0, qkv, ldq, 0, 0, EPI_STORE, 1.f, 0.f, bias, nullptr,
                        0, 0, nullptr, 0, 0, 0, nullptr, 0, 0, nullptr, nullptr, 0, stream))
    return e;
  return owlk_qk_rope_fwd(qkv, ldq, M, H, D, cosb, sinb, ld_tab, n_tab, tab_off, tpos_div, out, ldo, rstd, stream);
}

extern "C" int owlk_gemm_frames(long M, long N, long K, const void* A, long lda, long a_fs, int a_trans,
                                const void* B, long ldb, long b_fs, int b_trans, void* C, long ldc, long c_fs,
                                int c_f32, int epi, float alpha, float beta, const float* bias, void* aux, long ldaux,
                                const void* gate, long ldgate, long tpf, const void* resid, long ldres, void* ws,
                                long ws_bytes, void* stream) {
  OWLK_REQUIRE(a_fs >= 0 && b_fs >= 0 && c_fs >= 0 && a_fs % 8 == 0 && b_fs % 8 == 0 && c_fs % 8 == 0,
               "gemm_frames: frame strides must be non-negative multiples of 8");
  OWLK_REQUIRE(!c_fs || (!c_f32 && epi == EPI_STORE), "gemm_frames: frame-strided C only for a bf16 STORE");
  OWLK_REQUIRE((!a_fs || (a_trans ? K : M) % FRAME_ROWS == 0) && (!b_fs || (b_trans ? K : N) % FRAME_ROWS == 0) &&
                   (!c_fs || M % FRAME_ROWS == 0),
               "gemm_frames: frame-strided dims must be whole frames of %d rows", FRAME_ROWS);
  GemmP p{};
  p.a_fs = a_fs;
  p.b_fs = b_fs;
  p.c_fs = c_fs;
  return gemm_dispatch(p, M, N, K, 1, A, lda, 0, a_trans, B, ldb, 0, b_trans, C, ldc, 0, c_f32, epi, alpha, beta, bias,
                       aux, ldaux, 0, gate, ldgate, 0, tpf, resid, ldres, 0, ws, ws_bytes, stream);
}

extern "C" long owlk_gemm_splitk_bytes(long M, long N, long K, long batch, int a_trans, int b_trans, int c_f32,
                                       int epi, float beta) {
  if (M <= 0 || N <= 0 || K <= 0 || batch <= 0) return 0;
  return split_ws_bytes(split_plan(M, N, K, batch, a_trans, b_trans, c_f32, epi, beta), M, N, batch);
}

extern "C" long owlk_gemm_ws_counter_bytes(long M, long N, long K, long batch, int a_trans, int b_trans, int c_f32,
                                           int epi, float beta) {
  if (M <= 0 || N <= 0 || K <= 0 || batch <= 0) return 0;
  const SplitPlan pl = split_plan(M, N, K, batch, a_trans, b_trans, c_f32, epi, beta);
  return pl.kind == SPLIT_DECODE && pl.splits > 1 ? kDecodeCounterBytes : 0;
}

extern "C" long owlk_gemm_ws_bytes(long M, long N, long K, long batch, int a_trans, int b_trans, int c_f32, int epi,
                                   float beta, int colsum) {
  long b = owlk_gemm_splitk_bytes(M, N, K, batch, a_trans, b_trans, c_f32, epi, beta);
  if (colsum && M > 0 && N > 0) {
    const long c = std::max(fused_colsum_bytes(M, N), owlk_colsum_ws_bytes(M, N));
    b = std::max(b, c);
  }
  return b;
}
