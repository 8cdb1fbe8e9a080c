// Fused Muon optimizer passes (reference muon.py:66-84), HBM-bound elementwise work.
//
// owlk_muon_momentum: one pass per parameter group does what the reference spends three torch
//   passes on (buf.lerp_(g, 1-m); g.lerp_(buf, m); torch.stack) plus the Frobenius-norm reduction
//   of the Newton-Schulz prologue (sum of bf16(g')^2, muon.py:24-26): reads g and buf, writes buf
//   and the stacked fp32 NS input, and the kNormParts partial sums of ||bf16(g')||^2 per matrix.
// owlk_muon_apply: p = p * (1 - lr*wd) - lr*scale * u (muon.py:80-84, two torch passes) in one,
//   reading u straight from the NS output layout (transposed when rows > cols, 64x64 LDS tiles).
// Each launch takes up to kMaxT same-shaped matrices as a kernel-argument pointer table (grid.y).
#include "common.hpp"

namespace {

constexpr int kMaxT = 16;
struct Ptrs {
  float* a[kMaxT];
  float* b[kMaxT];
};

// torch's lerp (ATen Lerp.h): weight < 0.5 ? self + w (end - self) : end - (end - self)(1 - w)
DEV float lerp_t(float s, float e, float w) {
  const float d = e - s;
  return fabsf(w) < 0.5f ? s + w * d : e - d * (1.f - w);
}

DEV float momentum1(float& b, float g, float m, bool nesterov) {
  b = lerp_t(b, g, 1.f - m);
  return nesterov ? lerp_t(g, b, m) : b;
}

template <bool VEC>
__global__ __launch_bounds__(256) void muon_momentum_k(Ptrs P, long n, float m, int nesterov,
                                                       float* __restrict__ stack, float* __restrict__ sumsq) {
  const int z = blockIdx.y;
  float* __restrict__ g = P.a[z];
  float* __restrict__ buf = P.b[z];
  float* __restrict__ out = stack ? stack + (long)z * n : g;
  const bool nes = nesterov != 0;
  float acc = 0.f;
  if (VEC) {
    const long n4 = n >> 2;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
      const f32x4 gv = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(g) + i);
      f32x4 bv = reinterpret_cast<const f32x4*>(buf)[i];
      f32x4 r;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float b = bv[j];
        r[j] = momentum1(b, gv[j], m, nes);
        bv[j] = b;
        const float a = rb(r[j]);
        acc += a * a;
      }
      reinterpret_cast<f32x4*>(buf)[i] = bv;
      __builtin_nontemporal_store(r, reinterpret_cast<f32x4*>(out) + i);
    }
  } else {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
      float b = buf[i];
      const float r = momentum1(b, g[i], m, nes);
      buf[i] = b;
      out[i] = r;
      const float a = rb(r);
      acc += a * a;
    }
  }
  if (!sumsq) return;
  __shared__ float red[4];
  acc = block_sum256(acc, red);
  if (threadIdx.x == 0) sumsq[(long)z * kNormParts + blockIdx.x] = acc;  // partial, fixed slot
}

// u[z] is [rows, cols] (TR = 0, contiguous) or [cols, rows] (TR = 1, the NS iterate before the
// transpose back); p[z] is [rows, cols] fp32.
__global__ __launch_bounds__(256) void muon_apply_flat_k(Ptrs P, const bf16* __restrict__ u, long n,
                                                          float decay, float alpha) {
  const int z = blockIdx.y;
  float* __restrict__ p = P.a[z];
  const bf16* __restrict__ uz = u + (long)z * n;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    p[i] = fmaf(-alpha, (float)uz[i], __fmul_rn(p[i], decay));
}

__global__ __launch_bounds__(256) void muon_apply_tr_k(Ptrs P, const bf16* __restrict__ u, long rows, long cols,
                                                        float decay, float alpha) {
  __shared__ float tile[64][65];
  const int z = blockIdx.z;
  float* __restrict__ p = P.a[z];
  const bf16* __restrict__ uz = u + (long)z * rows * cols;
  const long r0 = (long)blockIdx.y * 64, c0 = (long)blockIdx.x * 64;
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {  // read u[c][r] along r
    const int cc = i / 64, rr = i % 64;
    const long r = r0 + rr, c = c0 + cc;
    tile[rr][cc] = (r < rows && c < cols) ? (float)uz[c * rows + r] : 0.f;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {  // write p[r][c] along c
    const int rr = i / 64, cc = i % 64;
    const long r = r0 + rr, c = c0 + cc;
    if (r < rows && c < cols) {
      const long o = r * cols + c;
      p[o] = fmaf(-alpha, tile[rr][cc], __fmul_rn(p[o], decay));
    }
  }
}


// AdamW (torch.optim.AdamW, foreach order; rft_trainer.py / muon.py:143-146): per element
//   p = p*(1 - lr wd); m = lerp(m, g, 1 - b1); v = v b2 + (1 - b2) g g;
//   p = p + ss * m / (sqrt(v) / bc2s + eps)       with ss = -lr / (1 - b1^t), bc2s = sqrt(1 - b2^t)
// One launch covers up to kMaxA tensors of any sizes (grid.y = tensor); reads p g m v, writes p m v.
constexpr int kMaxA = 16;
struct AdamPtrs {
  float* p[kMaxA];
  const float* g[kMaxA];
  float* m[kMaxA];
  float* v[kMaxA];
  long n[kMaxA];
};

DEV void adamw1(float& p, float g, float& m, float& v, float decay, float b1, float b2, float ss, float bc2s,
                float eps) {
  p = __fmul_rn(p, decay);
  m = lerp_t(m, g, 1.f - b1);
  v = __fadd_rn(__fmul_rn(v, b2), (1.f - b2) * g * g);
  const float d = __fadd_rn(__fdiv_rn(__fsqrt_rn(v), bc2s), eps);
  p = p + ss * __fdiv_rn(m, d);
}

template <bool VEC>
__global__ __launch_bounds__(256) void adamw_k(AdamPtrs A, float decay, float b1, float b2, float ss, float bc2s,
                                               float eps) {
  const int z = blockIdx.y;
  float* __restrict__ p = A.p[z];
  const float* __restrict__ g = A.g[z];
  float* __restrict__ m = A.m[z];
  float* __restrict__ v = A.v[z];
  const long n = A.n[z];
  if (VEC) {
    const long n4 = n >> 2;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
      f32x4 pv = reinterpret_cast<const f32x4*>(p)[i];
      const f32x4 gv = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(g) + i);
      f32x4 mv = reinterpret_cast<const f32x4*>(m)[i];
      f32x4 vv = reinterpret_cast<const f32x4*>(v)[i];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float pj = pv[j], mj = mv[j], vj = vv[j];
        adamw1(pj, gv[j], mj, vj, decay, b1, b2, ss, bc2s, eps);
        pv[j] = pj;
        mv[j] = mj;
        vv[j] = vj;
      }
      reinterpret_cast<f32x4*>(p)[i] = pv;
      reinterpret_cast<f32x4*>(m)[i] = mv;
      reinterpret_cast<f32x4*>(v)[i] = vv;
    }
  } else {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
      float pj = p[i], mj = m[i], vj = v[i];
      adamw1(pj, g[i], mj, vj, decay, b1, b2, ss, bc2s, eps);
      p[i] = pj;
      m[i] = mj;
      v[i] = vj;
    }
  }
}


// EMA of the weights (ema_pytorch as restated in utils/grad_reducer.py): shadow = lerp(shadow, p, w),
// torch's lerp formula, over up to kMaxA tensors of any sizes per launch.
struct LerpPtrs {
  float* s[kMaxA];
  const float* p[kMaxA];
  long n[kMaxA];
};

template <bool VEC>
__global__ __launch_bounds__(256) void ema_k(LerpPtrs E, float w) {
  const int z = blockIdx.y;
  float* __restrict__ sh = E.s[z];
  const float* __restrict__ p = E.p[z];
  const long n = E.n[z];
  if (VEC) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < (n >> 2); i += (long)gridDim.x * 256) {
      f32x4 a = reinterpret_cast<const f32x4*>(sh)[i];
      const f32x4 b = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p) + i);
#pragma unroll
      for (int j = 0; j < 4; ++j) a[j] = lerp_t(a[j], b[j], w);
      reinterpret_cast<f32x4*>(sh)[i] = a;
    }
  } else {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) sh[i] = lerp_t(sh[i], p[i], w);
  }
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

unsigned flat_blocks(long work, int count) {
  // ~4 waves per CU over the whole launch (256 CUs), at least one block per 256 items
  long b = (work + 255) / 256;
  const long cap = 4096 / (count > 0 ? count : 1) + 1;
  return (unsigned)(b < cap ? (b > 0 ? b : 1) : cap);
}

}  // namespace

extern "C" int owlk_muon_momentum(int count, float* const* g, float* const* buf, long n, float momentum,
                                  int nesterov, float* stack, float* sumsq, void* stream) {
  OWLK_REQUIRE(count >= 0 && n > 0 && g && buf, "muon_momentum: bad args");
  hipStream_t s = (hipStream_t)stream;
  for (int base = 0; base < count; base += kMaxT) {
    const int k = count - base < kMaxT ? count - base : kMaxT;
    Ptrs P{};
    bool vec = (n % 4) == 0 && (!stack || aligned16(stack));
    for (int i = 0; i < k; ++i) {
      OWLK_REQUIRE(g[base + i] && buf[base + i], "muon_momentum: null tensor pointer");
      P.a[i] = g[base + i];
      P.b[i] = buf[base + i];
      vec = vec && aligned16(P.a[i]) && aligned16(P.b[i]);
    }
    float* st = stack ? stack + (long)base * n : nullptr;
    float* sq = sumsq ? sumsq + (long)base * kNormParts : nullptr;
    // with the norm requested: exactly kNormParts blocks per matrix, one partial slot each
    const dim3 grid(sumsq ? (unsigned)kNormParts : flat_blocks(vec ? n / 4 : n, k), (unsigned)k);
    if (vec)
      hipLaunchKernelGGL(muon_momentum_k<true>, grid, dim3(256), 0, s, P, n, momentum, nesterov, st, sq);
    else
      hipLaunchKernelGGL(muon_momentum_k<false>, grid, dim3(256), 0, s, P, n, momentum, nesterov, st, sq);
  }
  return owlk::check_launch("muon_momentum");
}

extern "C" int owlk_muon_apply(int count, float* const* p, const void* u, long rows, long cols, int transpose,
                               float decay, float alpha, void* stream) {
  OWLK_REQUIRE(count >= 0 && rows > 0 && cols > 0 && p && u, "muon_apply: bad args");
  hipStream_t s = (hipStream_t)stream;
  const long n = rows * cols;
  for (int base = 0; base < count; base += kMaxT) {
    const int k = count - base < kMaxT ? count - base : kMaxT;
    Ptrs P{};
    for (int i = 0; i < k; ++i) {
      OWLK_REQUIRE(p[base + i], "muon_apply: null tensor pointer");
      P.a[i] = p[base + i];
    }
    const bf16* ub = (const bf16*)u + (long)base * n;
    if (transpose) {
      const dim3 grid((unsigned)((cols + 63) / 64), (unsigned)((rows + 63) / 64), (unsigned)k);
      hipLaunchKernelGGL(muon_apply_tr_k, grid, dim3(256), 0, s, P, ub, rows, cols, decay, alpha);
    } else {
      const dim3 grid(flat_blocks(n, k), (unsigned)k);
      hipLaunchKernelGGL(muon_apply_flat_k, grid, dim3(256), 0, s, P, ub, n, decay, alpha);
    }
  }
  return owlk::check_launch("muon_apply");
}

extern "C" int owlk_adamw(int count, float* const* p, const float* const* g, float* const* m, float* const* v,
                          const long* n, float lr, float beta1, float beta2, float weight_decay, float eps,
                          float step_size, float bc2_sqrt, void* stream) {
  OWLK_REQUIRE(count >= 0 && p && g && m && v && n && bc2_sqrt > 0.f, "adamw: bad args");
  hipStream_t s = (hipStream_t)stream;
  const float decay = 1.f - lr * weight_decay;
  for (int base = 0; base < count; base += kMaxA) {
    const int k = count - base < kMaxA ? count - base : kMaxA;
    AdamPtrs A{};
    bool vec = true;
    long nmax = 1;
    for (int i = 0; i < k; ++i) {
      const int j = base + i;
      OWLK_REQUIRE(p[j] && g[j] && m[j] && v[j] && n[j] > 0, "adamw: null tensor or empty size");
      A.p[i] = p[j];
      A.g[i] = g[j];
      A.m[i] = m[j];
      A.v[i] = v[j];
      A.n[i] = n[j];
      vec = vec && (n[j] % 4) == 0 && aligned16(p[j]) && aligned16(g[j]) && aligned16(m[j]) && aligned16(v[j]);
      nmax = n[j] > nmax ? n[j] : nmax;
    }
    const dim3 grid(flat_blocks(vec ? nmax / 4 : nmax, k), (unsigned)k);
    if (vec)
      hipLaunchKernelGGL(adamw_k<true>, grid, dim3(256), 0, s, A, decay, beta1, beta2, step_size, bc2_sqrt, eps);
    else
      hipLaunchKernelGGL(adamw_k<false>, grid, dim3(256), 0, s, A, decay, beta1, beta2, step_size, bc2_sqrt, eps);
  }
  return owlk::check_launch("adamw");
}

extern "C" int owlk_ema(int count, float* const* shadow, const float* const* p, const long* n, float weight,
                        void* stream) {
  OWLK_REQUIRE(count >= 0 && shadow && p && n, "ema: bad args");
  hipStream_t s = (hipStream_t)stream;
  for (int base = 0; base < count; base += kMaxA) {
    const int k = count - base < kMaxA ? count - base : kMaxA;
    LerpPtrs E{};
    bool vec = true;
    long nmax = 1;
    for (int i = 0; i < k; ++i) {
      const int j = base + i;
      OWLK_REQUIRE(shadow[j] && p[j] && n[j] > 0, "ema: null tensor or empty size");
      E.s[i] = shadow[j];
      E.p[i] = p[j];
      E.n[i] = n[j];
      vec = vec && (n[j] % 4) == 0 && aligned16(shadow[j]) && aligned16(p[j]);
      nmax = n[j] > nmax ? n[j] : nmax;
    }
    const dim3 grid(flat_blocks(vec ? nmax / 4 : nmax, k), (unsigned)k);
    if (vec)
      hipLaunchKernelGGL(ema_k<true>, grid, dim3(256), 0, s, E, weight);
    else
      hipLaunchKernelGGL(ema_k<false>, grid, dim3(256), 0, s, E, weight);
  }
  return owlk::check_launch("ema");
}
