// MMDiT plumbing kernels (gfx950), HBM-bound, 16-B chunks per lane.
//   frame mux   mmattn.py:54-60 / :77-80: per frame, the video tokens (n0 per frame) and the
//               audio token (n1 per frame) are concatenated into one joint sequence of
//               (n0 + n1)-token frames, and the attention output is split back.  dir 0 gathers
//               two token-major streams into the joint layout, dir 1 scatters it back (the
//               backward of one is the other).
//   layer_norm  normalization.py:6-7, F.layer_norm(x, (d,)) without affine, eps 1e-5, computed
//               in fp32 (autocast's fp32 list) and rounded to the input dtype (bf16).
#include "common.hpp"

namespace {

constexpr float LN_EPS = 1e-5f;

__global__ __launch_bounds__(256) void frame_mux_k(int dir, long rows, int n0, int n1, int nch, bf16* a, long lda,
                                                   bf16* b, long ldb, bf16* j, long ldj) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= rows * nch) return;
  const long r = idx / nch;
  const int c = (int)(idx - r * nch);
  const int per = n0 + n1;
  const long f = r / per;
  const int i = (int)(r - f * per);
  bf16* s = i < n0 ? a + (f * n0 + i) * lda : b + (f * n1 + (i - n0)) * ldb;
  bf16* jp = j + r * ldj;
  if (dir == 0)
    *(bf16x8*)(jp + c * 8) = *(const bf16x8*)(s + c * 8);
  else
    *(bf16x8*)(s + c * 8) = *(const bf16x8*)(jp + c * 8);
}

// one wave per row; the row stays in registers between the mean and variance passes
template <int MAXC>
__global__ __launch_bounds__(256) void layernorm_fwd_k(const bf16* __restrict__ x, long ldx, long T, int d,
                                                       bf16* __restrict__ y, long ldy, float* __restrict__ mean,
                                                       float* __restrict__ rstd) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= T) return;
  const int nch = d / 8;
  float xv[MAXC][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
      unpack8(*(const bf16x8*)(x + row * ldx + c * 8), xv[i]);
#pragma unroll
      for (int e = 0; e < 8; ++e) s += xv[i][e];
    }
  }
  const float mu = wave_sum(s) / d;
  float v = 0.f;
#pragma unroll
  for (int i = 0; i < MAXC; ++i)
    if (lane + 64 * i < nch)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float t = xv[i][e] - mu;
        v += t * t;
      }
  const float r = rsqrtf(wave_sum(v) / d + LN_EPS);
  if (lane == 0) {
    mean[row] = mu;
    rstd[row] = r;
  }
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (xv[i][e] - mu) * r;
      *(bf16x8*)(y + row * ldy + c * 8) = pack8(o);
    }
  }
}

// dx = r * (dy - mean(dy) - xhat * mean(dy * xhat)), xhat = (x - mu) r, all fp32
template <int MAXC>
__global__ __launch_bounds__(256) void layernorm_bwd_k(const bf16* __restrict__ dy, long lddy,
                                                       const bf16* __restrict__ x, long ldx,
                                                       const float* __restrict__ mean,
                                                       const float* __restrict__ rstd, long T, int d,
                                                       bf16* __restrict__ dx, long lddx) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= T) return;
  const int nch = d / 8;
  const float mu = mean[row], r = rstd[row];
  float g[MAXC][8], xh[MAXC][8];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
      unpack8(*(const bf16x8*)(dy + row * lddy + c * 8), g[i]);
      unpack8(*(const bf16x8*)(x + row * ldx + c * 8), xh[i]);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        xh[i][e] = (xh[i][e] - mu) * r;
        s1 += g[i][e];
        s2 += g[i][e] * xh[i][e];
      }
    }
  }
  const float m1 = wave_sum(s1) / d, m2 = wave_sum(s2) / d;
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = r * (g[i][e] - m1 - xh[i][e] * m2);
      *(bf16x8*)(dx + row * lddx + c * 8) = pack8(o);
    }
  }
}

}  // namespace

extern "C" int owlk_frame_mux(int dir, long frames, int n0, int n1, int cols, void* a, long lda, void* b, long ldb,
                              void* joint, long ldj, void* stream) {
  OWLK_REQUIRE((dir == 0 || dir == 1) && frames >= 0 && n0 >= 0 && n1 >= 0 && cols % 8 == 0,
               "frame_mux: bad arguments");
  OWLK_REQUIRE(lda % 8 == 0 && ldb % 8 == 0 && ldj % 8 == 0 &&
                   ((uintptr_t)a | (uintptr_t)b | (uintptr_t)joint) % 16 == 0,
               "frame_mux: rows must be 16-byte aligned");
  const long rows = frames * (n0 + n1), total = rows * (cols / 8);
  if (total == 0) return 0;
  hipLaunchKernelGGL(frame_mux_k, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, dir, rows,
                     n0, n1, cols / 8, (bf16*)a, lda, (bf16*)b, ldb, (bf16*)joint, ldj);
  return owlk::check_launch("frame_mux");
}

extern "C" int owlk_layernorm_fwd(const void* x, long ldx, long T, int d, void* y, long ldy, float* mean, float* rstd,
                                  void* stream) {
  OWLK_REQUIRE(d % 8 == 0 && d <= 64 * 8 * MAXCPL && T >= 0, "layernorm_fwd: bad d=%d", d);
  if (T == 0) return 0;
  OWLK_CPL_DISPATCH(d, layernorm_fwd_k, dim3((unsigned)((T + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
                    (const bf16*)x, ldx, T, d, (bf16*)y, ldy, mean, rstd);
  return owlk::check_launch("layernorm_fwd");
}

extern "C" int owlk_layernorm_bwd(const void* dy, long lddy, const void* x, long ldx, const float* mean,
                                  const float* rstd, long T, int d, void* dx, long lddx, void* stream) {
  OWLK_REQUIRE(d % 8 == 0 && d <= 64 * 8 * MAXCPL && T >= 0, "layernorm_bwd: bad d=%d", d);
  if (T == 0) return 0;
  OWLK_CPL_DISPATCH(d, layernorm_bwd_k, dim3((unsigned)((T + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
                    (const bf16*)dy, lddy, (const bf16*)x, ldx, mean, rstd, T, d, (bf16*)dx, lddx);
  return owlk::check_launch("layernorm_bwd");
}
