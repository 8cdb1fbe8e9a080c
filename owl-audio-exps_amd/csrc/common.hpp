// Shared device helpers for libowlk (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define DEV __device__ __forceinline__

// round-to-nearest-even through bf16, as autocast does after every bf16 op.  Integer form on
// purpose: hipcc contracts (float)(__bf16)(a*b) + c into an FMA, silently dropping the rounding.
DEV float rb(float x) {
  unsigned u = __float_as_uint(x);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return __uint_as_float(u & 0xFFFF0000u);
}
DEV float bf2f(bf16 x) { return (float)x; }
// the same rounding for a PAIR by one v_cvt_pk_bf16_f32 (RNE): the packed word (bits 15:0 = a, 31:16 =
// b, the layout of a bf16 vector store) and the two rounded values read back by integer ops, which
// the compiler cannot fold into the neighbouring float arithmetic.  ~1.5 VALU per value against 4
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
DEV unsigned cvt2(float a, float b) {
  const bf16x2 v = {(bf16)a, (bf16)b};
  unsigned w = __builtin_bit_cast(unsigned, v);
  __asm__("" : "+v"(w));  // one conversion of the pair (seen through, hipcc splits it into two plus shifts)
  return w;
}
DEV float bf_lo(unsigned w) { return __uint_as_float(w << 16); }
DEV float bf_hi(unsigned w) { return __uint_as_float(w & 0xFFFF0000u); }
// lanes of one wave handing values to each other through LDS (a staging image written by some lanes,
// read back by others): the compiler's memory model is per thread, so without this it may reorder a
// lane's reads above its own writes when it proves their addresses differ.  Emits no instruction.
DEV void wave_lds_handoff() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// sigmoid with v_rcp_f32 (1 ulp) instead of the IEEE division sequence (~10 VALU per element,
// a tenth of a K = 1536 GEMM tile in the SiLU / dSiLU epilogues)
DEV float sigmoid_f(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
DEV float silu_f(float x) { return x * sigmoid_f(x); }

// LDS pointer helpers
typedef s16x4 __attribute__((address_space(3))) * lds_s16x4_ptr;

DEV s16x4 ds_read_tr16(const void* lds_byte_ptr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_ptr)(lds_byte_ptr));
}

// Same instruction through inline asm: invisible to the waitcnt pass.  The builtin above carries
// no LDS alias scope, so after any LDS-DMA (global_load_lds) hipcc puts an s_waitcnt vmcnt(0)
// before the first such read -- draining a DMA ring that is meant to stay in flight.  The CALLER
// must retire these reads itself (s_waitcnt lgkmcnt(0) + sched_barrier before the consumer).
DEV s16x4 ds_read_tr16_async(const void* lds_byte_ptr) {
  s16x4 r;
  const unsigned a = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)lds_byte_ptr;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a));
  return r;
}

DEV bf16x8 join_tr(s16x4 lo, s16x4 hi) {
  union { s16x4 s[2]; bf16x8 v; } u;
  u.s[0] = lo;
  u.s[1] = hi;
  return u.v;
}

DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Frobenius-norm partials: the sum-of-squares passes write kNormParts per-block partial sums per
// matrix (no atomics) and the consumer adds them in index order, so the norm is bitwise
// reproducible (OWLK_NORM_PARTS in include/owlk.h).
constexpr int kNormParts = 256;

// fixed-order sum of a 256-thread block's values (wave butterflies, then the 4 wave sums in order)
DEV float block_sum256(float v, float* red4) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red4[threadIdx.x >> 6] = v;
  __syncthreads();
  const float r = ((red4[0] + red4[1]) + red4[2]) + red4[3];
  __syncthreads();
  return r;
}

DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// 8 x bf16 <-> 8 x f32
DEV void unpack8(const bf16x8& v, float* f) {
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = (float)v[i];
}
DEV bf16x8 pack8(const float* f) {
  bf16x8 v;
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (bf16)f[i];
  return v;
}

// ---------------------------------------------------------------- host-side error plumbing
#ifdef __cplusplus
#include <cstdio>
#include <string>
namespace owlk {
void set_error(const char* fmt, ...);
int check_launch(const char* what);
// out[n] += sum_s part[s][n], s = 0 .. splits-1 in order (fp32, N % 4 == 0, 16-B aligned)
int colsum_reduce(const float* part, int splits, long N, float* out, hipStream_t s);
}  // namespace owlk
#define OWLK_REQUIRE(cond, ...)             \
  do {                                      \
    if (!(cond)) {                          \
      owlk::set_error(__VA_ARGS__);         \
      return 1;                             \
    }                                       \
  } while (0)

static constexpr int MAXCPL = 8;  // max 16-B chunks per lane (d <= 4096)

// launch helper: pick the chunks-per-lane instantiation for a row width d
#define OWLK_CPL_DISPATCH(d, KERNEL, ...)                     \
  do {                                                        \
    const int cpl_ = ((d) / 8 + 63) / 64;                     \
    switch (cpl_) {                                           \
      case 1: hipLaunchKernelGGL(KERNEL<1>, __VA_ARGS__); break; \
      case 2: hipLaunchKernelGGL(KERNEL<2>, __VA_ARGS__); break; \
      case 3: hipLaunchKernelGGL(KERNEL<3>, __VA_ARGS__); break; \
      case 4: hipLaunchKernelGGL(KERNEL<4>, __VA_ARGS__); break; \
      case 5: hipLaunchKernelGGL(KERNEL<5>, __VA_ARGS__); break; \
      case 6: hipLaunchKernelGGL(KERNEL<6>, __VA_ARGS__); break; \
      default: hipLaunchKernelGGL(KERNEL<8>, __VA_ARGS__); break; \
    }                                                         \
  } while (0)

#endif
