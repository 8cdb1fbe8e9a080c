// Newton-Schulz prologue for Muon (muon.py:23-29): X = bf16(G) (transposed when rows > cols),
// X = X / (||X||_F + 1e-7) with the reference's bf16 rounding of the norm and the quotient.
// The five quintic iterations themselves run on the GEMM kernels (epilogue AXPBY) -- see
// owl_wms/muon.py.
#include "common.hpp"

namespace {

template <typename T>
DEV float ld_f(const T* p, long i) { return (float)p[i]; }

template <typename T>
__global__ __launch_bounds__(256) void sumsq_k(const T* __restrict__ g, long n, float* __restrict__ work) {
  const long z = blockIdx.y;
  const T* gz = g + z * n;
  float acc = 0.f;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float x = rb(ld_f(gz, i));
    acc += x * x;
  }
  acc = wave_sum(acc);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(work + z, red[0] + red[1] + red[2] + red[3]);
}

// 64x64 tiled (optionally transposing) scale: x[z][c][r] or x[z][r][c] = bf16(bf16(g) / den)
template <typename T, bool TR>
__global__ __launch_bounds__(256) void scale_k(const T* __restrict__ g, long rows, long cols,
                                               const float* __restrict__ work, bf16* __restrict__ x) {
  __shared__ float tile[64][65];
  const long z = blockIdx.z;
  const float den = rb(rb(sqrtf(work[z])) + 1e-7f);
  const T* gz = g + z * rows * cols;
  bf16* xz = x + z * rows * cols;
  const long r0 = (long)blockIdx.y * 64, c0 = (long)blockIdx.x * 64;
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int rr = i / 64, cc = i % 64;
    const long r = r0 + rr, c = c0 + cc;
    const float v = (r < rows && c < cols) ? rb(rb(ld_f(gz, r * cols + c)) / den) : 0.f;
    if (TR)
      tile[rr][cc] = v;
    else if (r < rows && c < cols)
      xz[r * cols + c] = (bf16)v;
  }
  if (TR) {
    __syncthreads();
    for (int i = threadIdx.x; i < 64 * 64; i += 256) {
      const int cc = i / 64, rr = i % 64;
      const long r = r0 + rr, c = c0 + cc;
      if (r < rows && c < cols) xz[c * rows + r] = (bf16)tile[rr][cc];
    }
  }
}

}  // namespace

extern "C" int owlk_ns_normalize(const void* g, int g_f32, long rows, long cols, long batch, int transpose, void* x,
                                 float* work, void* stream) {
  OWLK_REQUIRE(rows > 0 && cols > 0 && batch > 0 && work && x, "ns_normalize: bad args");
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(work, 0, batch * sizeof(float), s) != hipSuccess) {
    owlk::set_error("ns_normalize: memset failed");
    return 2;
  }
  const long n = rows * cols;
  long blocks = (n + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  dim3 g1((unsigned)blocks, (unsigned)batch);
  dim3 g2((unsigned)((cols + 63) / 64), (unsigned)((rows + 63) / 64), (unsigned)batch);
  if (g_f32) {
    hipLaunchKernelGGL(sumsq_k<float>, g1, dim3(256), 0, s, (const float*)g, n, work);
    if (transpose)
      hipLaunchKernelGGL((scale_k<float, true>), g2, dim3(256), 0, s, (const float*)g, rows, cols, work, (bf16*)x);
    else
      hipLaunchKernelGGL((scale_k<float, false>), g2, dim3(256), 0, s, (const float*)g, rows, cols, work, (bf16*)x);
  } else {
    hipLaunchKernelGGL(sumsq_k<bf16>, g1, dim3(256), 0, s, (const bf16*)g, n, work);
    if (transpose)
      hipLaunchKernelGGL((scale_k<bf16, true>), g2, dim3(256), 0, s, (const bf16*)g, rows, cols, work, (bf16*)x);
    else
      hipLaunchKernelGGL((scale_k<bf16, false>), g2, dim3(256), 0, s, (const bf16*)g, rows, cols, work, (bf16*)x);
  }
  return owlk::check_launch("ns_normalize");
}

// The scale pass alone, for callers that already hold sum(bf16(g)^2) per matrix (owlk_muon_momentum
// accumulates it while it writes g).
extern "C" int owlk_ns_scale(const void* g, int g_f32, long rows, long cols, long batch, int transpose, void* x,
                             const float* sumsq, void* stream) {
  OWLK_REQUIRE(rows > 0 && cols > 0 && batch > 0 && sumsq && x && g, "ns_scale: bad args");
  hipStream_t s = (hipStream_t)stream;
  dim3 g2((unsigned)((cols + 63) / 64), (unsigned)((rows + 63) / 64), (unsigned)batch);
  if (g_f32) {
    if (transpose)
      hipLaunchKernelGGL((scale_k<float, true>), g2, dim3(256), 0, s, (const float*)g, rows, cols, sumsq, (bf16*)x);
    else
      hipLaunchKernelGGL((scale_k<float, false>), g2, dim3(256), 0, s, (const float*)g, rows, cols, sumsq, (bf16*)x);
  } else {
    if (transpose)
      hipLaunchKernelGGL((scale_k<bf16, true>), g2, dim3(256), 0, s, (const bf16*)g, rows, cols, sumsq, (bf16*)x);
    else
      hipLaunchKernelGGL((scale_k<bf16, false>), g2, dim3(256), 0, s, (const bf16*)g, rows, cols, sumsq, (bf16*)x);
  }
  return owlk::check_launch("ns_scale");
}
