// Newton-Schulz for Muon (muon.py:11-38).
//   prologue (muon.py:23-29): X = bf16(G) (transposed when rows > cols), X = X / (||X||_F + 1e-7)
//     with the reference's bf16 rounding of the norm and the quotient;
//   iterations (muon.py:30-34), in the eager reference's rounding order, on the batched GEMM:
//     A = X X^T and cA = bf16(c A)          (one GEMM, SCALE2 epilogue)
//     B = bf16(b A) + bf16(cA @ A)           (GEMM + AXPBY epilogue, alpha 1)
//     X = bf16(a X) + bf16(B @ X)            (GEMM + AXPBY epilogue, alpha 1)
//   owlk_newton_schulz_bf16 composes all of it behind one C entry (zero-padding dims that are not
//   multiples of 8, which adds nothing to the norm or to any product).
#include "common.hpp"

namespace {

template <typename T>
DEV float ld_f(const T* p, long i) { return (float)p[i]; }

// grid (kNormParts, batch): work[z][blockIdx.x] = this block's share of sum(bf16(g)^2)
template <typename T>
__global__ __launch_bounds__(256) void sumsq_k(const T* __restrict__ g, long n, float* __restrict__ work) {
  const long z = blockIdx.y;
  const T* gz = g + z * n;
  float acc = 0.f;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float x = rb(ld_f(gz, i));
    acc += x * x;
  }
  __shared__ float red[4];
  acc = block_sum256(acc, red);
  if (threadIdx.x == 0) work[z * kNormParts + blockIdx.x] = acc;
}

// 64x64 tiled (optionally transposing) scale: x[z][c][r] or x[z][r][c] = bf16(bf16(g) / den)
template <typename T, bool TR>
__global__ __launch_bounds__(256) void scale_k(const T* __restrict__ g, long rows, long cols,
                                               const float* __restrict__ work, bf16* __restrict__ x, long ldx,
                                               long sx) {
  __shared__ float tile[64][65];
  __shared__ float red[4];
  const long z = blockIdx.z;
  // ||X||_F from the kNormParts partials, added in fixed order (bitwise reproducible)
  const float ss = block_sum256(work[z * kNormParts + threadIdx.x], red);
  const float den = rb(rb(sqrtf(ss)) + 1e-7f);
  const T* gz = g + z * rows * cols;
  bf16* xz = x + z * sx;
  const long r0 = (long)blockIdx.y * 64, c0 = (long)blockIdx.x * 64;
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int rr = i / 64, cc = i % 64;
    const long r = r0 + rr, c = c0 + cc;
    const float v = (r < rows && c < cols) ? rb(rb(ld_f(gz, r * cols + c)) / den) : 0.f;
    if (TR)
      tile[rr][cc] = v;
    else if (r < rows && c < cols)
      xz[r * ldx + c] = (bf16)v;
  }
  if (TR) {
    __syncthreads();
    for (int i = threadIdx.x; i < 64 * 64; i += 256) {
      const int cc = i / 64, rr = i % 64;
      const long r = r0 + rr, c = c0 + cc;
      if (r < rows && c < cols) xz[c * ldx + r] = (bf16)tile[rr][cc];
    }
  }
}

// out[z][r][c] = X[z][c][r] (X [batch][cols_p][rows_p], transposed back) or X[z][r][c] (cropped)
template <bool TR>
__global__ __launch_bounds__(256) void ns_out_k(const bf16* __restrict__ X, long ldx, long sx, long rows, long cols,
                                                bf16* __restrict__ out) {
  __shared__ bf16 tile[64][66];
  const long z = blockIdx.z;
  const bf16* xz = X + z * sx;
  bf16* oz = out + z * rows * cols;
  const long r0 = (long)blockIdx.y * 64, c0 = (long)blockIdx.x * 64;
  if (!TR) {
    for (int i = threadIdx.x; i < 64 * 64; i += 256) {
      const long r = r0 + i / 64, c = c0 + i % 64;
      if (r < rows && c < cols) oz[r * cols + c] = xz[r * ldx + c];
    }
    return;
  }
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {  // read X rows (= out columns) coalesced
    const long c = c0 + i / 64, r = r0 + i % 64;
    if (r < rows && c < cols) tile[i / 64][i % 64] = xz[c * ldx + r];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const long r = r0 + i / 64, c = c0 + i % 64;
    if (r < rows && c < cols) oz[r * cols + c] = tile[i % 64][i / 64];
  }
}

long al256(long b) { return (b + 255) / 256 * 256; }
long up8(long v) { return (v + 7) / 8 * 8; }

}  // namespace

extern "C" int owlk_ns_normalize(const void* g, int g_f32, long rows, long cols, long batch, int transpose, void* x,
                                 float* work, void* stream) {
  OWLK_REQUIRE(rows > 0 && cols > 0 && batch > 0 && work && x, "ns_normalize: bad args");
  hipStream_t s = (hipStream_t)stream;
  const long n = rows * cols;
  dim3 g1((unsigned)kNormParts, (unsigned)batch);
  dim3 g2((unsigned)((cols + 63) / 64), (unsigned)((rows + 63) / 64), (unsigned)batch);
  if (g_f32) {
    hipLaunchKernelGGL(sumsq_k<float>, g1, dim3(256), 0, s, (const float*)g, n, work);
    if (transpose)
      hipLaunchKernelGGL((scale_k<float, true>), g2, dim3(256), 0, s, (const float*)g, rows, cols, work, (bf16*)x,
                         transpose ? rows : cols, rows * cols);
    else
      hipLaunchKernelGGL((scale_k<float, false>), g2, dim3(256), 0, s, (const float*)g, rows, cols, work, (bf16*)x,
                         transpose ? rows : cols, rows * cols);
  } else {
    hipLaunchKernelGGL(sumsq_k<bf16>, g1, dim3(256), 0, s, (const bf16*)g, n, work);
    if (transpose)
      hipLaunchKernelGGL((scale_k<bf16, true>), g2, dim3(256), 0, s, (const bf16*)g, rows, cols, work, (bf16*)x,
                         transpose ? rows : cols, rows * cols);
    else
      hipLaunchKernelGGL((scale_k<bf16, false>), g2, dim3(256), 0, s, (const bf16*)g, rows, cols, work, (bf16*)x,
                         transpose ? rows : cols, rows * cols);
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
      hipLaunchKernelGGL((scale_k<float, true>), g2, dim3(256), 0, s, (const float*)g, rows, cols, sumsq, (bf16*)x,
                         transpose ? rows : cols, rows * cols);
    else
      hipLaunchKernelGGL((scale_k<float, false>), g2, dim3(256), 0, s, (const float*)g, rows, cols, sumsq, (bf16*)x,
                         transpose ? rows : cols, rows * cols);
  } else {
    if (transpose)
      hipLaunchKernelGGL((scale_k<bf16, true>), g2, dim3(256), 0, s, (const bf16*)g, rows, cols, sumsq, (bf16*)x,
                         transpose ? rows : cols, rows * cols);
    else
      hipLaunchKernelGGL((scale_k<bf16, false>), g2, dim3(256), 0, s, (const bf16*)g, rows, cols, sumsq, (bf16*)x,
                         transpose ? rows : cols, rows * cols);
  }
  return owlk::check_launch("ns_scale");
}

extern "C" int owlk_gemm(long M, long N, long K, long batch, const void* A, long lda, long sA, int a_trans,
                         const void* B, long ldb, long sB, int b_trans, void* C, long ldc, long sC, int c_f32,
                         int epi, float alpha, float beta, const float* bias, void* aux, long ldaux, long sAux,
                         const void* gate, long ldgate, long sGate, long tpf, const void* resid, long ldres, long sRes,
                         float* colsum, void* ws, long ws_bytes, void* stream);

extern "C" long owlk_ns_iterate_ws_bytes(long batch, long m, long k) {
  if (batch <= 0 || m <= 0 || k <= 0) return 0;
  return al256(batch * m * k * 2) + 3 * al256(batch * m * m * 2);
}

// In place on x: a normalised bf16 X [batch, m, k] (m <= k, both multiples of 8, contiguous).
extern "C" int owlk_ns_iterate(void* x, long batch, long m, long k, int steps, float a, float b, float c, void* ws,
                               long ws_bytes, void* stream) {
  OWLK_REQUIRE(x && batch > 0 && m > 0 && k > 0 && steps >= 0, "ns_iterate: bad args");
  OWLK_REQUIRE(m % 8 == 0 && k % 8 == 0 && m <= k, "ns_iterate: need m <= k, both multiples of 8 (m=%ld k=%ld)", m, k);
  OWLK_REQUIRE(ws && ws_bytes >= owlk_ns_iterate_ws_bytes(batch, m, k) && (uintptr_t)ws % 16 == 0,
               "ns_iterate: workspace too small (%ld < %ld bytes)", ws_bytes, owlk_ns_iterate_ws_bytes(batch, m, k));
  constexpr int STORE = 0, AXPBY = 4, SCALE2 = 5;
  char* w = (char*)ws;
  bf16* Y = (bf16*)w;
  w += al256(batch * m * k * 2);
  bf16* A = (bf16*)w;
  w += al256(batch * m * m * 2);
  bf16* cA = (bf16*)w;
  w += al256(batch * m * m * 2);
  bf16* Bm = (bf16*)w;
  bf16* X = (bf16*)x;
  const long mk = m * k, mm = m * m;
  (void)STORE;
  for (int it = 0; it < steps; ++it) {
    // A = X X^T (muon.py:32), and c*A as the next product's left operand
    if (int e = owlk_gemm(m, m, k, batch, X, k, mk, 0, X, k, mk, 0, A, m, mm, 0, SCALE2, c, 0.f, nullptr, cA, m, mm,
                          nullptr, 0, 0, 1, nullptr, 0, 0, nullptr, nullptr, 0, stream))
      return e;
    // B = b*A + (c*A) @ A (muon.py:33): right operand A[l][j] read as B(n = j, k = l)
    if (int e = owlk_gemm(m, m, m, batch, cA, m, mm, 0, A, m, mm, 1, Bm, m, mm, 0, AXPBY, 1.f, b, nullptr, A, m, mm,
                          nullptr, 0, 0, 1, nullptr, 0, 0, nullptr, nullptr, 0, stream))
      return e;
    // X = a*X + B @ X (muon.py:34)
    if (int e = owlk_gemm(m, k, m, batch, Bm, m, mm, 0, X, k, mk, 1, Y, k, mk, 0, AXPBY, 1.f, a, nullptr, X, k, mk,
                          nullptr, 0, 0, 1, nullptr, 0, 0, nullptr, nullptr, 0, stream))
      return e;
    bf16* t = X;
    X = Y;
    Y = t;
  }
  if (X != (bf16*)x &&
      hipMemcpyAsync(x, X, batch * mk * 2, hipMemcpyDeviceToDevice, (hipStream_t)stream) != hipSuccess) {
    owlk::set_error("ns_iterate: copy-back failed");
    return 2;
  }
  return 0;
}

extern "C" long owlk_newton_schulz_ws_bytes(long batch, long rows, long cols) {
  if (batch <= 0 || rows <= 0 || cols <= 0) return 0;
  const long m = up8(rows < cols ? rows : cols), k = up8(rows < cols ? cols : rows);
  return al256(batch * m * k * 2) + al256(batch * kNormParts * 4) + owlk_ns_iterate_ws_bytes(batch, m, k);
}

// zeropower_via_newtonschulz5 (muon.py:11-38) for g [batch, rows, cols] (fp32 or bf16) -> out bf16
// [batch, rows, cols].  Coefficients (a, b, c) = (3.4445, -4.7750, 2.0315) in the reference.
extern "C" int owlk_newton_schulz_bf16(const void* g, int g_f32, long batch, long rows, long cols, int steps, float a,
                                       float b, float c, void* out, void* ws, long ws_bytes, void* stream) {
  OWLK_REQUIRE(g && out && batch > 0 && rows > 0 && cols > 0 && steps >= 0, "newton_schulz: bad args");
  OWLK_REQUIRE(ws && ws_bytes >= owlk_newton_schulz_ws_bytes(batch, rows, cols) && (uintptr_t)ws % 16 == 0,
               "newton_schulz: workspace too small (%ld < %ld bytes)", ws_bytes,
               owlk_newton_schulz_ws_bytes(batch, rows, cols));
  hipStream_t s = (hipStream_t)stream;
  const bool tr = rows > cols;
  const long m = up8(tr ? cols : rows), k = up8(tr ? rows : cols);
  char* w = (char*)ws;
  bf16* X = (bf16*)w;
  w += al256(batch * m * k * 2);
  float* work = (float*)w;
  w += al256(batch * kNormParts * 4);
  const bool padded = m != (tr ? cols : rows) || k != (tr ? rows : cols);
  if (padded && hipMemsetAsync(X, 0, batch * m * k * 2, s) != hipSuccess) {
    owlk::set_error("newton_schulz: memset failed");
    return 2;
  }
  const long n = rows * cols;
  dim3 g1((unsigned)kNormParts, (unsigned)batch);
  dim3 g2((unsigned)((cols + 63) / 64), (unsigned)((rows + 63) / 64), (unsigned)batch);
  if (g_f32) {
    hipLaunchKernelGGL(sumsq_k<float>, g1, dim3(256), 0, s, (const float*)g, n, work);
    if (tr)
      hipLaunchKernelGGL((scale_k<float, true>), g2, dim3(256), 0, s, (const float*)g, rows, cols, work, X, k, m * k);
    else
      hipLaunchKernelGGL((scale_k<float, false>), g2, dim3(256), 0, s, (const float*)g, rows, cols, work, X, k, m * k);
  } else {
    hipLaunchKernelGGL(sumsq_k<bf16>, g1, dim3(256), 0, s, (const bf16*)g, n, work);
    if (tr)
      hipLaunchKernelGGL((scale_k<bf16, true>), g2, dim3(256), 0, s, (const bf16*)g, rows, cols, work, X, k, m * k);
    else
      hipLaunchKernelGGL((scale_k<bf16, false>), g2, dim3(256), 0, s, (const bf16*)g, rows, cols, work, X, k, m * k);
  }
  if (int e = owlk::check_launch("newton_schulz normalize")) return e;
  if (int e = owlk_ns_iterate(X, batch, m, k, steps, a, b, c, w, ws_bytes - (w - (char*)ws), stream)) return e;
  if (tr)
    hipLaunchKernelGGL((ns_out_k<true>), g2, dim3(256), 0, s, X, k, m * k, rows, cols, (bf16*)out);
  else
    hipLaunchKernelGGL((ns_out_k<false>), g2, dim3(256), 0, s, X, k, m * k, rows, cols, (bf16*)out);
  return owlk::check_launch("newton_schulz out");
}
