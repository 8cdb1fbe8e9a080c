// Per-frame conditioning of the DiT (gfx950): the timestep / control embeddings' elementwise
// prologue, the conditioning sum + SiLU, and the small-K weight gradients of the embedding MLPs.
// Replaces the reference's torch elementwise ops (embeddings.py:30-184, gamerft.py:39-48,
// modulation.py:13 silu(cond)) so that the training step runs no ATen arithmetic.
//
// Rounding follows the reference run in bf16 (the golden fixtures: CPU autocast keeps sin / cos /
// atan2 / log1p / norm in the bf16 input dtype): every torch op rounds its result to bf16.
//
//   cond_embed   per row r (one frame of one sample):
//     ts:     e_i = bf16(bf16(ts * mult) * tf_i); ts_in = [bf16 sin e | bf16 cos e]     (SinCosEmbed)
//     mouse:  x = sign(m) * bf16(log1p|m|); ang = bf16(atan2(x1, x0)); mag = bf16(|x|)   (MouseEmbedding)
//             (the inner bf16 roundings only where that input is bf16: an fp32 input runs fp32 ops)
//             ce, se = bf16(cos ang), bf16(sin ang); mouse_in[:, :H] = bf16(Wa ce + Wa' se)
//             (angle_proj, bf16 operands, fp32 sum); mouse_in[:, H:] = SinCos(mag)
//     button: btn_in = 2 b - 1 (zero-padded to a multiple of 8 columns)               (ButtonEmbeddding)
//   cond_silu    cond = bf16(t + (has_controls ? bf16(m + b) : 0)); s = bf16(silu(cond))  (+ backward)
//   small_k_wgrad  dW[n, k] = beta dW + sum_r dy[r, n] x[r, k] for k < K <= 16 (rows in order)
#include "common.hpp"

namespace {

// value as the reference's torch op leaves it: rounded to bf16 when the op ran on a bf16 input, kept
// fp32 when the input (and so the op) was fp32
__device__ __forceinline__ float rt(float v, int f32) { return f32 ? v : rb(v); }

__device__ __forceinline__ float ld_in(const void* p, long i, int f32) {
  return f32 ? ((const float*)p)[i] : bf2f(((const bf16*)p)[i]);
}

// one workgroup per row: threads < ht write the timestep embedding, < hm the mouse magnitude
// embedding, < 2 hm the angle projection, < nbp the button input.  Every output is the bf16 that
// autocast hands the following Linear; tfreq / mfreq are the fp32 frequency tables, rounded here
// when the embedding runs in bf16 (SinCosEmbed's .to(dtype)).
__global__ __launch_bounds__(256) void cond_embed_k(const void* __restrict__ ts, int ts_f32,
                                                    const float* __restrict__ tfreq, int ht, float tmult,
                                                    bf16* __restrict__ ts_in, long ldt, const void* __restrict__ mouse,
                                                    int mouse_f32, long ldm, const float* __restrict__ mfreq, int hm,
                                                    float mmult, const float* __restrict__ wang,
                                                    bf16* __restrict__ mouse_in, long ldmi, bf16* __restrict__ ang,
                                                    const void* __restrict__ btn, int btn_f32, long ldb, int nb,
                                                    int nbp, bf16* __restrict__ btn_in, long ldbi) {
  const long r = blockIdx.x;
  const int tid = threadIdx.x;
  if (ts) {
    const float x = rt(ld_in(ts, r, ts_f32) * tmult, ts_f32);
    for (int i = tid; i < ht; i += 256) {
      const float e = rt(x * rt(tfreq[i], ts_f32), ts_f32);
      ts_in[r * ldt + i] = (bf16)sinf(e);
      ts_in[r * ldt + ht + i] = (bf16)cosf(e);
    }
  }
  if (mouse) {
    const int f = mouse_f32;
    // symlog: sign(x) * log1p(|x|) (the product of +-1 and a rounded value is exact)
    const float m0 = ld_in(mouse, r * ldm, f), m1 = ld_in(mouse, r * ldm + 1, f);
    const float x0 = (m0 > 0.f ? 1.f : (m0 < 0.f ? -1.f : 0.f)) * rt(log1pf(fabsf(m0)), f);
    const float x1 = (m1 > 0.f ? 1.f : (m1 < 0.f ? -1.f : 0.f)) * rt(log1pf(fabsf(m1)), f);
    const float a = rt(atan2f(x1, x0), f);
    const float mag = rt(sqrtf(x0 * x0 + x1 * x1), f);
    // angle_proj's bf16 operands: autocast casts (cos, sin) to bf16 whatever their dtype
    const float ce = rb(rt(cosf(a), f)), se = rb(rt(sinf(a), f));
    if (tid == 0) {
      ang[r * 2] = (bf16)ce;
      ang[r * 2 + 1] = (bf16)se;
    }
    const float xm = rt(mag * mmult, f);
    for (int i = tid; i < hm; i += 256) {
      const float e = rt(xm * rt(mfreq[i], f), f);
      mouse_in[r * ldmi + 2 * hm + i] = (bf16)sinf(e);
      mouse_in[r * ldmi + 3 * hm + i] = (bf16)cosf(e);
    }
    for (int j = tid; j < 2 * hm; j += 256)  // angle_proj: [2 hm, 2] weights, no bias
      mouse_in[r * ldmi + j] = (bf16)(rb(wang[2 * j]) * ce + rb(wang[2 * j + 1]) * se);
  }
  if (btn) {
    for (int k = tid; k < nbp; k += 256)
      btn_in[r * ldbi + k] = k < nb ? (bf16)(2.f * ld_in(btn, r * ldb + k, btn_f32) - 1.f) : (bf16)0.f;
  }
}

// 8 columns per thread; hc: per-sample bool (has_controls), row r is sample r / rows_per; null = all 1
__global__ __launch_bounds__(256) void cond_silu_fwd_k(const bf16* __restrict__ t, const bf16* __restrict__ m,
                                                       const bf16* __restrict__ b, const unsigned char* __restrict__ hc,
                                                       long rows_per, long R, int d, bf16* __restrict__ cond,
                                                       bf16* __restrict__ s) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  const int nch = d / 8;
  if (idx >= R * nch) return;
  const long r = idx / nch;
  const long off = r * d + (idx - r * nch) * 8;
  float tv[8], c[8], o[8];
  unpack8(*(const bf16x8*)(t + off), tv);
  const bool on = m && (!hc || hc[r / rows_per]);
  if (on) {
    float mv[8], bv[8];
    unpack8(*(const bf16x8*)(m + off), mv);
    unpack8(*(const bf16x8*)(b + off), bv);
#pragma unroll
    for (int e = 0; e < 8; ++e) c[e] = rb(tv[e] + rb(mv[e] + bv[e]));
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) c[e] = tv[e];
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = silu_f(c[e]);
  if (cond) *(bf16x8*)(cond + off) = pack8(c);
  *(bf16x8*)(s + off) = pack8(o);
}

// ds (fp32: the summed gradient of s over its consumers, rounded to bf16 as autograd's bf16 sum
// would be; or bf16) -> dcond = bf16(bf16(ds) silu'(cond)), or = ds with cond null (the gradient of
// cond itself); dctrl = has_controls ? dcond : 0.  dcond / dctrl may each be null.
__global__ __launch_bounds__(256) void cond_silu_bwd_k(const void* __restrict__ ds, int ds_bf16,
                                                       const bf16* __restrict__ cond,
                                                       const unsigned char* __restrict__ hc, long rows_per, long R,
                                                       int d, bf16* __restrict__ dcond, bf16* __restrict__ dctrl) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  const int nch = d / 8;
  if (idx >= R * nch) return;
  const long r = idx / nch;
  const long off = r * d + (idx - r * nch) * 8;
  float g[8], o[8];
  if (ds_bf16) {
    unpack8(*(const bf16x8*)((const bf16*)ds + off), g);
  } else {
    const f32x4 g0 = *(const f32x4*)((const float*)ds + off), g1 = *(const f32x4*)((const float*)ds + off + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      g[e] = rb(g0[e]);
      g[e + 4] = rb(g1[e]);
    }
  }
  if (cond) {
    float c[8];
    unpack8(*(const bf16x8*)(cond + off), c);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float sg = sigmoid_f(c[e]);
      o[e] = g[e] * sg * (1.f + c[e] * (1.f - sg));
    }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = g[e];
  }
  const bf16x8 v = pack8(o);
  if (dcond) *(bf16x8*)(dcond + off) = v;
  if (dctrl) {
    // a branch: the vector-typed ?: form of this select wrote zeros into lanes 0-1 of kept rows
    bf16x8 c = v;
    if (hc && !hc[r / rows_per]) {
      const float z[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      c = pack8(z);
    }
    *(bf16x8*)(dctrl + off) = c;
  }
}

// dW[n, k] (ldw) = beta dW + sum_r dy[r, n] x[r, k], k < K: a workgroup = 64 columns n x 4 row
// groups (waves); each lane sums its rows in order, the 4 group sums meet in a fixed order.
template <int KM>
__global__ __launch_bounds__(256) void small_k_wgrad_k(const bf16* __restrict__ dy, long lddy,
                                                       const bf16* __restrict__ x, long ldx, long R, long N, int K,
                                                       float* __restrict__ dw, long ldw, float beta) {
  __shared__ float red[4][64][KM];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long n = (long)blockIdx.x * 64 + lane;
  float acc[KM];
#pragma unroll
  for (int k = 0; k < KM; ++k) acc[k] = 0.f;
  if (n < N) {
    const long per = (R + 3) / 4, r0 = w * per, r1 = r0 + per < R ? r0 + per : R;
    for (long r = r0; r < r1; ++r) {
      const float g = bf2f(dy[r * lddy + n]);
#pragma unroll
      for (int k = 0; k < KM; ++k)
        if (k < K) acc[k] += g * bf2f(x[r * ldx + k]);
    }
  }
#pragma unroll
  for (int k = 0; k < KM; ++k) red[w][lane][k] = acc[k];
  __syncthreads();
  if (w == 0 && n < N) {
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      if (k >= K) break;
      const float s = ((red[0][lane][k] + red[1][lane][k]) + red[2][lane][k]) + red[3][lane][k];
      dw[n * ldw + k] = beta == 0.f ? s : beta * dw[n * ldw + k] + s;
    }
  }
}

}  // namespace

extern "C" int owlk_cond_embed(const void* ts, int ts_f32, const float* tfreq, int ht, float tmult, void* ts_in,
                               long ldt, const void* mouse, int mouse_f32, long ldm, const float* mfreq, int hm,
                               float mmult, const float* wang, void* mouse_in, long ldmi, void* ang, const void* btn,
                               int btn_f32, long ldb, int nb, int nbp, void* btn_in, long ldbi, long R,
                               void* stream) {
  OWLK_REQUIRE(R > 0 && (!ts || (tfreq && ts_in && ht > 0)), "cond_embed: bad timestep arguments");
  OWLK_REQUIRE(!mouse || (mfreq && wang && mouse_in && ang && hm > 0), "cond_embed: bad mouse arguments");
  OWLK_REQUIRE(!btn || (btn_in && nb > 0 && nbp >= nb), "cond_embed: bad button arguments");
  hipLaunchKernelGGL(cond_embed_k, dim3((unsigned)R), dim3(256), 0, (hipStream_t)stream, ts, ts_f32, tfreq, ht, tmult,
                     (bf16*)ts_in, ldt, mouse, mouse_f32, ldm, mfreq, hm, mmult, wang, (bf16*)mouse_in, ldmi,
                     (bf16*)ang, btn, btn_f32, ldb, nb, nbp, (bf16*)btn_in, ldbi);
  return owlk::check_launch("cond_embed");
}

extern "C" int owlk_cond_silu_fwd(const void* t, const void* m, const void* b, const void* hc, long rows_per, long R,
                                  int d, void* cond, void* s, void* stream) {
  OWLK_REQUIRE(d % 8 == 0 && R > 0 && rows_per > 0 && (!m || b), "cond_silu_fwd: bad sizes");
  OWLK_REQUIRE(((uintptr_t)t | (uintptr_t)m | (uintptr_t)b | (uintptr_t)cond | (uintptr_t)s) % 16 == 0,
               "cond_silu_fwd: rows must be 16-byte aligned");
  const long work = R * (d / 8);
  hipLaunchKernelGGL(cond_silu_fwd_k, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)t, (const bf16*)m, (const bf16*)b, (const unsigned char*)hc, rows_per, R, d, (bf16*)cond, (bf16*)s);
  return owlk::check_launch("cond_silu_fwd");
}

extern "C" int owlk_cond_silu_bwd(const void* ds, int ds_bf16, const void* cond, const void* hc, long rows_per, long R,
                                  int d, void* dcond, void* dctrl, void* stream) {
  OWLK_REQUIRE(d % 8 == 0 && R > 0 && rows_per > 0, "cond_silu_bwd: bad sizes");
  OWLK_REQUIRE(((uintptr_t)ds | (uintptr_t)cond | (uintptr_t)dcond | (uintptr_t)dctrl) % 16 == 0,
               "cond_silu_bwd: rows must be 16-byte aligned");
  const long work = R * (d / 8);
  hipLaunchKernelGGL(cond_silu_bwd_k, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, (hipStream_t)stream, ds,
                     ds_bf16, (const bf16*)cond, (const unsigned char*)hc, rows_per, R, d, (bf16*)dcond,
                     (bf16*)dctrl);
  return owlk::check_launch("cond_silu_bwd");
}

extern "C" int owlk_small_k_wgrad(const void* dy, long lddy, const void* x, long ldx, long R, long N, int K, float* dw,
                                  long ldw, float beta, void* stream) {
  OWLK_REQUIRE(R > 0 && N > 0 && K > 0 && K <= 16, "small_k_wgrad: K=%d must be in 1..16", K);
  const dim3 g((unsigned)((N + 63) / 64));
  hipStream_t s = (hipStream_t)stream;
  const bf16* a = (const bf16*)dy;
  const bf16* b = (const bf16*)x;
  if (K <= 2)
    hipLaunchKernelGGL(small_k_wgrad_k<2>, g, dim3(256), 0, s, a, lddy, b, ldx, R, N, K, dw, ldw, beta);
  else if (K <= 8)
    hipLaunchKernelGGL(small_k_wgrad_k<8>, g, dim3(256), 0, s, a, lddy, b, ldx, R, N, K, dw, ldw, beta);
  else
    hipLaunchKernelGGL(small_k_wgrad_k<16>, g, dim3(256), 0, s, a, lddy, b, ldx, R, N, K, dw, ldw, beta);
  return owlk::check_launch("small_k_wgrad");
}
