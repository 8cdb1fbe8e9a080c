// Micro-benchmark: fp32 no-return atomic-add throughput with the access pattern a fused
// attention backward (dQ accumulated by atomics) would have.  Each workgroup owns one key
// tile j of one head and walks query tiles i = nq-1 .. j, adding a 64 x 64 fp32 tile per step.
//   hipcc --offload-arch=gfx950 -O3 tools/atomic_bench.hip -o /tmp/atomic_bench && /tmp/atomic_bench
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void walk(float* acc, int nq, int heads, int kt_per_q, int mode) {
  const int h = blockIdx.x % heads;  // heads fastest: concurrent WGs of different heads
  const int j = blockIdx.x / heads;  // key tile (in units of query tiles when kt_per_q == 1)
  const int jq = j * kt_per_q;
  float* base = acc + (size_t)h * nq * 64 * 64;
  for (int i = nq - 1; i >= jq; --i) {
    float* t = base + (size_t)i * 64 * 64;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int e = r * 256 + threadIdx.x;
      if (mode == 0)
        __hip_atomic_fetch_add(t + e, 1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else
        t[e] += 1.0f;  // plain RMW (wrong answer, bandwidth reference)
    }
  }
}

int main() {
  const int heads = 24, nq = 1536;
  float* acc;
  const size_t n = (size_t)heads * nq * 64 * 64;
  hipMalloc(&acc, n * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int kt = 1; kt <= 4; kt *= 2) {
    for (int mode = 0; mode < 2; ++mode) {
      const int nk = nq / kt;
      hipMemset(acc, 0, n * 4);
      walk<<<nk * heads, 256>>>(acc, nq, heads, kt, mode);
      hipEventRecord(a);
      walk<<<nk * heads, 256>>>(acc, nq, heads, kt, mode);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      double tiles = 0;
      for (int j = 0; j < nk; ++j) tiles += nq - j * kt;
      tiles *= heads;
      const double bytes = tiles * 64 * 64 * 4;
      printf("key tile %3d rows, %s: %.2f ms, %.1f GB of adds, %.2f TB/s\n", 64 * kt,
             mode ? "plain RMW" : "atomic   ", ms, bytes / 1e9, bytes / ms / 1e9);
    }
  }
  float h0;
  hipMemcpy(&h0, acc, 4, hipMemcpyDeviceToHost);
  printf("acc[0] = %.0f\n", h0);
  return 0;
}
