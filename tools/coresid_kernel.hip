// A stand-in for an RCCL all-reduce kernel's footprint (tools/coresidency.py): nwg persistent
// workgroups of 256 threads with 8 KiB of LDS, each streaming its share of a buffer (read + write) and
// recording, per workgroup, the 100 MHz real-time clock when it started and when it finished.
#include <hip/hip_runtime.h>

__global__ __launch_bounds__(256) void coresid_copy_k(const float4* __restrict__ src, float4* __restrict__ dst, long n,
                                                      unsigned long long* __restrict__ stamps) {
  __shared__ float4 stage[512];  // 8 KiB, as a collective's staging buffer
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    stage[threadIdx.x] = src[i];
    __syncthreads();
    dst[i] = stage[threadIdx.x ^ 1];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    stamps[2 * blockIdx.x] = t0;
    stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
  }
}

__global__ void coresid_now_k(unsigned long long* out) { *out = __builtin_amdgcn_s_memrealtime(); }

extern "C" int coresid_copy(const void* src, void* dst, long n_float4, int nwg, unsigned long long* stamps,
                            void* stream) {
  hipLaunchKernelGGL(coresid_copy_k, dim3(nwg), dim3(256), 0, (hipStream_t)stream, (const float4*)src, (float4*)dst,
                     n_float4, stamps);
  return hipGetLastError() != hipSuccess;
}
extern "C" int coresid_now(unsigned long long* out, void* stream) {
  hipLaunchKernelGGL(coresid_now_k, dim3(1), dim3(1), 0, (hipStream_t)stream, out);
  return hipGetLastError() != hipSuccess;
}
