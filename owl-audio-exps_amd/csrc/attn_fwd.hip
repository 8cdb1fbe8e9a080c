// Block-sparse frame-causal flash attention, forward (gfx950, head_dim 64).
//
// Replaces the compiled flex_attention + create_block_mask pair of the reference
// (attn.py:13-16, 24-62, 106-109; mmattn.py:75).  Semantics: softmax(q k^T / sqrt(D)) v over the
// allowed keys of attn_common.hpp, bf16 in / fp32 accumulate / bf16 out, plus the per-row
// log-sum-exp (natural log) for the backward pass.
//
// Workgroup = 4 waves = 128 query rows of one (batch, head); each wave owns 32 rows.  Per 64-key
// tile the wave computes S^T = K Q^T with v_mfma_f32_32x32x16_bf16 (key rows in registers, the
// query on the lane) so the softmax row statistics stay in-lane (+ one lane^32 exchange), then
// feeds the S^T accumulators straight back as the B operand of O^T += V^T P^T (V^T fragments
// through ds_read_b64_tr_b16).  K/V tiles arrive by LDS-DMA into a 3-deep ring.
// lse is written in base 2 of the scaled logits, lse2 = log2 sum_k exp2(scale log2(e) s_k) (=
// natural lse * log2 e): the backward's P = exp2(c s - lse2) then needs no conversion.
#include "attn_common.hpp"

#include <cstdlib>
#include <type_traits>

namespace {

constexpr int D = 64;
constexpr int QT = 128;  // query rows per workgroup
constexpr int KT = 64;   // keys per tile
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

struct FwdP {
  const bf16 *q, *k, *v;
  bf16* o;
  float* lse;           // [B, H, Lq]
  long ldq, ldk, ldv, ldo;      // token row strides (elements)
  long sqb, skb, svb, sob;      // batch strides (elements)
  long Lq, Lkv;
  int H;
  float scale_log2;     // softmax scale * log2(e)
  float bound;          // BOUNDED: |q.k| <= bound for every pair (raw score units)
  MaskP m;
};

// stage one 64x64 bf16 tile (rows r0.., 128-B rows) into registers: 2 chunks per thread
DEV void stage_load(bf16x8 (&r)[2], const bf16* base, long ld, long r0, long R) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = threadIdx.x + 256 * i;
    const long row = r0 + (c >> 3);
    r[i] = row < R ? *(const bf16x8*)(base + row * ld + (c & 7) * 8) : bf16x8{};
  }
}

template <bool TR>
DEV void stage_store(char* lds, const bf16x8 (&r)[2]) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = threadIdx.x + 256 * i;
    const int row = c >> 3, ch = c & 7;
    const int sw = TR ? swz_tr(row) : swz_row(row);
    *(bf16x8*)(lds + row * 128 + ((ch ^ sw) << 4)) = r[i];
  }
}

// GLDS = true: K/V tiles arrive by LDS-DMA into a 3-deep ring with two tiles in flight (no
// staging registers, counted vmcnt + raw s_barrier); false: register-staged double buffer.
// BOUNDED = true: the caller guarantees |q.k| <= p.bound (QK-RMSNorm'd q, k have |q| = |k| =
// sqrt(D), attn.py:84), so every exp2 argument c*s lies in [-c*bound, c*bound] (+-11.8 at D 64):
// p = exp2(c s) needs no running max, no offset and no rescale.  Softmax is shift-invariant, so
// the result is the same function; P keeps bf16's relative precision at any magnitude.
template <bool GLDS, bool BOUNDED>
__global__ __launch_bounds__(256) void attn_fwd_k(FwdP p) {
  constexpr int NBUF = GLDS ? 3 : 2;
  __shared__ __attribute__((aligned(16))) char smem[NBUF * 2 * KT * D * 2];  // [buf][K|V][64][64]
  __shared__ int red_lo;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int h = lane >> 5, ql = lane & 31;
  const long b = blockIdx.z;
  const int head = blockIdx.y;
  const int ntq = (int)((p.Lq + QT - 1) / QT);
  const long q0 = (long)(ntq - 1 - (int)blockIdx.x) * QT;  // heaviest (latest) query tiles first
  const long r0 = q0 + 32 * w;                             // this wave's first row
  const MaskP& m = p.m;

  const bf16* Q = p.q + b * p.sqb + head * D;
  const bf16* K = p.k + b * p.skb + head * D;
  const bf16* V = p.v + b * p.svb + head * D;

  // ---- kv frame range of the whole workgroup
  const long qlast = (q0 + QT < p.Lq ? q0 + QT : p.Lq) - 1;
  const int fq_lo = frame_of(m, q0 + m.q_offset), fq_hi = frame_of(m, qlast + m.q_offset);
  int lo_f;
  if (m.kv_lo) {
    if (threadIdx.x == 0) red_lo = 1 << 30;
    __syncthreads();
    int mn = 1 << 30;
    for (int f = fq_lo + threadIdx.x; f <= fq_hi; f += 256) mn = min(mn, m.kv_lo[b * m.fstride + f]);
    atomicMin(&red_lo, mn);
    __syncthreads();
    lo_f = red_lo;
  } else {
    lo_f = m.window > 0 ? max(0, fq_lo - m.window + 1) : 0;
  }
  int hi_f = m.causal ? fq_hi : (m.window > 0 ? min(m.n_frames - 1, fq_hi + m.window - 1) : m.n_frames - 1);
  long kv_begin = (long)lo_f * m.tpf;
  long kv_end = ((long)hi_f + 1) * m.tpf;
  if (kv_end > p.Lkv) kv_end = p.Lkv;
  kv_begin = (kv_begin / KT) * KT;
  const int ntiles = kv_end > kv_begin ? (int)((kv_end - kv_begin + KT - 1) / KT) : 0;

  // ---- this wave's query fragments (B operand of S^T = K Q^T): Q[row][16s + 8h .. +8]
  const long my_q = r0 + ql;
  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s)
    qf[s] = my_q < p.Lq ? *(const bf16x8*)(Q + my_q * p.ldq + 16 * s + 8 * h) : bf16x8{};
  if constexpr (BOUNDED) {
    // q' = bf16(q * c), c = scale * log2(e): S' = K q'^T is already the exp2 argument.  With
    // |q.k| <= bound, |S'| <= c * bound (checked < 40 on the host), so p = exp2(S') needs no
    // running max and no offset; the one extra rounding of q' is 2^-9 relative per element.
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      float f[8];
      unpack8(qf[s], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] *= p.scale_log2;
      qf[s] = pack8(f);
    }
  }
  const long wlast = (r0 + 31 < p.Lq ? r0 + 31 : p.Lq - 1);
  const bool wave_live = r0 < p.Lq;
  const int wfq0 = frame_of(m, r0 + m.q_offset), wfq1 = frame_of(m, wlast + m.q_offset);
  const int my_fq = frame_of(m, (my_q < p.Lq ? my_q : wlast) + m.q_offset);

  f32x16 o[2];
  o[0] = f32x16{};
  o[1] = f32x16{};
  float mrow = BOUNDED ? 0.f : -INFINITY, lrow = 0.f;

  constexpr int BUFB = 2 * KT * D * 2;
  bf16x8 kr[2], vr[2];
  const GldsOff goff_k = glds_offsets<SW_ROW>(p.ldk, w, lane), goff_v = glds_offsets<SW_TR>(p.ldv, w, lane);
  if (GLDS) {
    if (ntiles > 0) {
      tile_glds<SW_ROW>(smem, K, p.ldk, kv_begin, p.Lkv, w, lane);
      tile_glds<SW_TR>(smem + KT * D * 2, V, p.ldv, kv_begin, p.Lkv, w, lane);
    }
    if (ntiles > 1) {
      tile_glds<SW_ROW>(smem + BUFB, K, p.ldk, kv_begin + KT, p.Lkv, w, lane);
      tile_glds<SW_TR>(smem + BUFB + KT * D * 2, V, p.ldv, kv_begin + KT, p.Lkv, w, lane);
      OWLK_VMCNT(4);
    } else {
      OWLK_VMCNT(0);
    }
    OWLK_BARRIER();
  } else {
    if (ntiles > 0) {
      stage_load(kr, K, p.ldk, kv_begin, p.Lkv);
      stage_load(vr, V, p.ldv, kv_begin, p.Lkv);
      stage_store<false>(smem, kr);
      stage_store<true>(smem + KT * D * 2, vr);
    }
    __syncthreads();
  }

  for (int t = 0; t < ntiles; ++t) {
    const long c0 = kv_begin + (long)t * KT;
    const bool more = t + 1 < ntiles;
    const bool more2 = t + 2 < ntiles;
    if (GLDS) {
      if (more2) {
        char* nb = smem + ((t + 2) % 3) * BUFB;
        const long c2 = c0 + 2 * KT;
        if (c2 + KT <= p.Lkv) {
          tile_glds_fast(nb, K + c2 * p.ldk, goff_k, w);
          tile_glds_fast(nb + KT * D * 2, V + c2 * p.ldv, goff_v, w);
        } else {
          tile_glds<SW_ROW>(nb, K, p.ldk, c2, p.Lkv, w, lane);
          tile_glds<SW_TR>(nb + KT * D * 2, V, p.ldv, c2, p.Lkv, w, lane);
        }
      }
    } else if (more) {
      stage_load(kr, K, p.ldk, c0 + KT, p.Lkv);
      stage_load(vr, V, p.ldv, c0 + KT, p.Lkv);
    }
    const char* lk = smem + (GLDS ? (t % 3) : (t & 1)) * BUFB;
    const char* lv = lk + KT * D * 2;

    const long clast = (c0 + KT - 1 < p.Lkv ? c0 + KT - 1 : p.Lkv - 1);
    int kind = TILE_EMPTY;
    if (wave_live) kind = classify(m, b, wfq0, wfq1, frame_of(m, c0), frame_of(m, clast));
    if (kind == TILE_FULL && c0 + KT > p.Lkv) kind = TILE_PARTIAL;
    kind = __builtin_amdgcn_readfirstlane(kind);  // wave-uniform: scalar branch, no exec masking

    if (kind != TILE_EMPTY) {
      const bool masked = kind == TILE_PARTIAL;
      // S^T[key][q] for two 32-key blocks
      f32x16 st[2];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        st[kb] = f32x16{};
        const int krow = 32 * kb + ql;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const bf16x8 kf = *(const bf16x8*)(lk + krow * 128 + (((2 * s + h) ^ swz_row(krow)) << 4));
          st[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], st[kb], 0, 0, 0);
        }
      }
      if (masked) {  // wave-uniform: only tiles straddling a mask edge
        const unsigned long long bh = tile_bits(m, b, my_q, my_q < p.Lq, c0, p.Lkv, true) >> (4 * h);
        apply_bits<0>(st[0], bh, -INFINITY);
        apply_bits<32>(st[1], bh, -INFINITY);
      }
      float mc = 0.f;
      if constexpr (!BOUNDED) {
        // row max on raw scores; p = exp2(s * c - m * c) is one FMA + one v_exp per score
        float tmax = -INFINITY;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int r = 0; r < 16; ++r) tmax = fmaxf(tmax, st[kb][r]);
        tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
        const float mnew = fmaxf(mrow, tmax);
        mc = mnew == -INFINITY ? 0.f : mnew * p.scale_log2;
        if (__any(mnew > mrow)) {  // some row's max moved: rescale l and O (exactly)
          const float alpha = __builtin_amdgcn_exp2f(mrow * p.scale_log2 - mc);
          lrow *= alpha;
#pragma unroll
          for (int db = 0; db < 2; ++db)
#pragma unroll
            for (int r = 0; r < 16; ++r) o[db][r] *= alpha;
        }
        mrow = mnew;
      }
      float psum = 0.f;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float pv = BOUNDED ? __builtin_amdgcn_exp2f(st[kb][r])
                                   : __builtin_amdgcn_exp2f(fmaf(st[kb][r], p.scale_log2, -mc));
          st[kb][r] = pv;
          psum += pv;
        }
      lrow += psum;

      // O^T[d][q] += V^T[d][key] P^T[key][q]
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const bf16x8 pf = acc_frag(st[kb], s);
#pragma unroll
          for (int db = 0; db < 2; ++db)
            o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_tr<SW_TR>(lv, 32 * kb, s, db, lane), pf, o[db], 0, 0,
                                                            0);
        }
    }
    if (GLDS) {
      if (more2)
        OWLK_VMCNT(4);  // tile t+1 landed (this wave's part); t+2 may stay in flight
      else
        OWLK_VMCNT(0);
      OWLK_BARRIER();
    } else {
      if (more) {
        char* nb = smem + ((t + 1) & 1) * BUFB;
        stage_store<false>(nb, kr);
        stage_store<true>(nb + KT * D * 2, vr);
      }
      __syncthreads();
    }
  }

  // ---- epilogue: O = O^T / l, lse
  const float ltot = lrow + __shfl_xor(lrow, 32, 64);
  if (my_q < p.Lq) {
    const float inv = ltot > 0.f ? 1.f / ltot : 0.f;
    bf16* O = p.o + b * p.sob + my_q * p.ldo + head * D;
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        bf16x4 v4;
#pragma unroll
        for (int e = 0; e < 4; ++e) v4[e] = (bf16)(o[db][4 * gq + e] * inv);
        *(bf16x4*)(O + 32 * db + 8 * gq + 4 * h) = v4;
      }
    if (h == 0)
      p.lse[(b * p.H + head) * p.Lq + my_q] = ltot > 0.f ? mrow * p.scale_log2 + __log2f(ltot) : -INFINITY;
  }
}

}  // namespace

MaskP owlk_make_mask(long tpf, int window, int causal, long q_offset, long Lkv, const int* kv_lo, const int* q_hi,
                     const int* run_start, const int* doc, long fstride) {
  MaskP m;
  m.tpf = tpf;
  m.magic = tpf > 1 ? (unsigned)((1ull << 32) / (unsigned long long)tpf + 1) : 0u;
  m.window = window;
  m.causal = causal;
  m.q_offset = q_offset;
  m.n_frames = (int)((Lkv + tpf - 1) / tpf);
  m.kv_lo = kv_lo;
  m.q_hi = q_hi;
  m.run_start = run_start;
  m.doc = doc;
  m.fstride = fstride;
  return m;
}

extern "C" int owlk_attn_fwd(const void* q, long ldq, long sqb, const void* k, long ldk, long skb, const void* v,
                             long ldv, long svb, void* o, long ldo, long sob, float* lse, long B, int H, long Lq,
                             long Lkv, int head_dim, float scale, float score_bound, long tpf, int window,
                             int causal, long q_offset, const int* kv_lo, const int* q_hi, const int* run_start,
                             const int* doc, long fstride, void* stream) {
  OWLK_REQUIRE(head_dim == D, "attn_fwd: head_dim %d not built (64 only)", head_dim);
  OWLK_REQUIRE(tpf > 0 && Lq > 0 && Lkv > 0 && B > 0 && H > 0, "attn_fwd: bad sizes");
  OWLK_REQUIRE((Lkv + q_offset) < (1L << 31) / (tpf > 1 ? tpf : 1) || tpf == 1, "attn_fwd: sequence too long");
  OWLK_REQUIRE(!doc || (run_start != nullptr), "attn_fwd: doc mask needs run_start");
  OWLK_REQUIRE(((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)o) % 16 == 0 && ldq % 8 == 0 &&
                   ldk % 8 == 0 && ldv % 8 == 0 && ldo % 8 == 0,
               "attn_fwd: q/k/v/o rows must be 16-byte aligned");
  FwdP p;
  p.q = (const bf16*)q; p.k = (const bf16*)k; p.v = (const bf16*)v; p.o = (bf16*)o; p.lse = lse;
  p.ldq = ldq; p.ldk = ldk; p.ldv = ldv; p.ldo = ldo;
  p.sqb = sqb; p.skb = skb; p.svb = svb; p.sob = sob;
  p.Lq = Lq; p.Lkv = Lkv; p.H = H;
  p.scale_log2 = scale * LOG2E;
  p.bound = score_bound;
  OWLK_REQUIRE(score_bound >= 0.f && score_bound * scale < 40.f, "attn_fwd: score_bound out of range");
  p.m = owlk_make_mask(tpf, window, causal, q_offset, Lkv, kv_lo, q_hi, run_start, doc, fstride);
  dim3 grid((unsigned)((Lq + QT - 1) / QT), (unsigned)H, (unsigned)B);
  static const int variant = getenv("OWLK_ATTN_FWD_REGSTAGE") ? 0 : 1;
  const bool bounded = score_bound > 0.f;
  if (variant && bounded)
    hipLaunchKernelGGL((attn_fwd_k<true, true>), grid, dim3(256), 0, (hipStream_t)stream, p);
  else if (variant)
    hipLaunchKernelGGL((attn_fwd_k<true, false>), grid, dim3(256), 0, (hipStream_t)stream, p);
  else if (bounded)
    hipLaunchKernelGGL((attn_fwd_k<false, true>), grid, dim3(256), 0, (hipStream_t)stream, p);
  else
    hipLaunchKernelGGL((attn_fwd_k<false, false>), grid, dim3(256), 0, (hipStream_t)stream, p);
  return owlk::check_launch("attn_fwd");
}
