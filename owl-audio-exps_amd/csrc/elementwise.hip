// HBM-bound fused kernels of the DiT block (gfx950).  Every kernel moves bf16 rows as 16-B
// chunks (8 elements per lane) and reproduces the reference's bf16 autocast rounding order:
//   AdaLN      modulation.py:7-26 / cond_adaln :46-55   y = bf16(bf16(bf16(rms(x)) * bf16(1+a)) + b)
//   Gate       modulation.py:28-43 / cond_gate :57-63   (fwd fused into the GEMM epilogue)
//   QK-norm    attn.py:84 + rope.py:43-51               fp32 rotation of bf16(rms(q)), [even||odd]
//   flow noise gamerft.py:92-95,107-111                 x_t = bf16(bf16(x*bf16(1-t)) + bf16(z*t))
#include "common.hpp"

namespace {

constexpr float RMS_EPS = 1.1920928955078125e-07f;  // finfo(float32).eps, F.rms_norm default

// ------------------------------------------------------------------ AdaLN forward
// one wave per token row; lane owns chunks c = lane + 64*i
template <int MAXC>
__global__ __launch_bounds__(256) void adaln_fwd_k(const bf16* __restrict__ x, long ldx,
                                                   const bf16* __restrict__ sc, const bf16* __restrict__ sh,
                                                   long ldm, long tpf, long T, int d, bf16* __restrict__ y,
                                                   long ldy, float* __restrict__ rstd, bf16* __restrict__ yact) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= T) return;
  const int nch = d / 8;
  bf16x8 xv[MAXC];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
      xv[i] = *(const bf16x8*)(x + row * ldx + c * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float f = (float)xv[i][e];
        ss += f * f;
      }
    }
  }
  ss = wave_sum(ss);
  const float r = rsqrtf(ss / d + RMS_EPS);
  if (lane == 0 && rstd) rstd[row] = r;
  const long f = row / tpf;
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
      float a[8], b[8], o[8];
      unpack8(*(const bf16x8*)(sc + f * ldm + c * 8), a);
      unpack8(*(const bf16x8*)(sh + f * ldm + c * 8), b);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float xn = rb((float)xv[i][e] * r);
        o[e] = rb(rb(xn * rb(1.f + a[e])) + b[e]);
      }
      *(bf16x8*)(y + row * ldy + c * 8) = pack8(o);
      if (yact) {
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = silu_f(o[e]);
        *(bf16x8*)(yact + row * ldy + c * 8) = pack8(o);
      }
    }
  }
}

// ------------------------------------------------------------------ AdaLN backward
// one workgroup per frame (tpf token rows); wave w takes rows w, w+4, ...; each lane keeps the
// per-column partial sums of its chunks, combined across the 4 waves through LDS at the end.
// GATE: the gate backward of the block's attention branch on the dx rows just formed (gate_bwd_k's
// products in its order: the same rows per wave, the same lane partials and LDS combine), so dx is
// not read back: dyg = bf16(dx * g[frame]), dg[frame] = sum_t dx*y, dbf[frame] = sum_t dyg.
struct GateBwdArgs {
  const bf16* y;
  long ldy;
  const bf16* g;
  long ldgg;
  bf16* dyg;
  long lddyg;
  float* dg;
  long lddg;
  int dg_bf16;
  float* dbf;
  long ldr;
};

template <int MAXC, bool GATE = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MAXC <= 3 ? 2 : 1))) void adaln_bwd_k(const bf16* __restrict__ dy, long lddy,
                                                   const bf16* __restrict__ x, long ldx,
                                                   const float* __restrict__ rstd,
                                                   const bf16* __restrict__ sc, long ldm, long tpf, int d,
                                                   const bf16* __restrict__ dres, long ldres,
                                                   bf16* __restrict__ dx, long lddx,
                                                   float* __restrict__ dsc, float* __restrict__ dsh, long ldg,
                                                   const bf16* __restrict__ ypre, int mod_bf16, GateBwdArgs ga = {}) {
  extern __shared__ float red[];  // [4][2][d]
  const long f = blockIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nch = d / 8;
  float pa[MAXC][8], pb[MAXC][8];
  float t1[MAXC][8];
  // GATE: each lane's gate partials live in its wave's slice of the LDS buffer (only that lane
  // touches them until the combine), registers stay below occupancy 2's 256
  bf16x8 gv[GATE ? MAXC : 1];  // the frame's gate row, packed
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = lane + 64 * i;
#pragma unroll
    for (int e = 0; e < 8; ++e) pa[i][e] = pb[i][e] = 0.f;
    if constexpr (GATE) {
      if (c < nch) {
        gv[i] = *(const bf16x8*)(ga.g + f * ga.ldgg + c * 8);
        float4* q = (float4*)(red + (w * 2 + 0) * d + c * 8);
        float4* b = (float4*)(red + (w * 2 + 1) * d + c * 8);
        q[0] = q[1] = b[0] = b[1] = float4{0.f, 0.f, 0.f, 0.f};
      }
    }
    if (c < nch) {
      float a[8];
      unpack8(*(const bf16x8*)(sc + f * ldm + c * 8), a);
#pragma unroll
      for (int e = 0; e < 8; ++e) t1[i][e] = rb(1.f + a[e]);
    }
  }
  // the wave's next row (dy, x, dres, rstd) is loaded while the current one is reduced and stored:
  // two rows of 16-B loads in flight per lane instead of one
  bf16x8 ndy[MAXC], nx[MAXC], nres[MAXC];
  float nr = 0.f;
  auto load = [&](long t) {
    const long row = f * tpf + t;
    nr = rstd[row];
#pragma unroll
    for (int i = 0; i < MAXC; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
        ndy[i] = *(const bf16x8*)(dy + row * lddy + c * 8);
        nx[i] = *(const bf16x8*)(x + row * ldx + c * 8);
        if (dres) nres[i] = *(const bf16x8*)(dres + row * ldres + c * 8);
      }
    }
  };
  if (w < tpf) load(w);
  for (long t = w; t < tpf; t += 4) {
    const long row = f * tpf + t;
    const float r = nr;
    bf16x8 cdy[MAXC], cx[MAXC], cres[MAXC];
#pragma unroll
    for (int i = 0; i < MAXC; ++i) {
      cdy[i] = ndy[i];
      cx[i] = nx[i];
      cres[i] = nres[i];
    }
    if (t + 4 < tpf) load(t + 4);
    bf16x8 cyg[GATE ? MAXC : 1];  // GATE: this row of y, loaded now so its latency hides behind the reduction
    if constexpr (GATE) {
#pragma unroll
      for (int i = 0; i < MAXC; ++i)
        if (lane + 64 * i < nch) cyg[i] = *(const bf16x8*)(ga.y + row * ga.ldy + (lane + 64 * i) * 8);
    }
    // g = dy * (1 + scale) and xh = x * rstd are formed twice (for the row's dot product, then for
    // dx) instead of kept: the rows stay packed in registers
    float dot = 0.f;
#pragma unroll
    for (int i = 0; i < MAXC; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
        float dv[8], xv[8];
        unpack8(cdy[i], dv);
        unpack8(cx[i], xv);
        if (ypre) {  // FinalLayer: dy arrives as d silu(y); silu backward in bf16 like autocast
          float yp[8];
          unpack8(*(const bf16x8*)(ypre + row * lddy + c * 8), yp);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float sg = sigmoid_f(yp[e]);
            dv[e] = rb(dv[e] * sg * (1.f + yp[e] * (1.f - sg)));
          }
          cdy[i] = pack8(dv);  // exact: dv is bf16-rounded
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float xh = xv[e] * r;
          const float xn = rb(xh);
          pa[i][e] += dv[e] * xn;
          pb[i][e] += dv[e];
          dot += (dv[e] * t1[i][e]) * xh;
        }
      }
    }
    dot = wave_sum(dot) / d;
#pragma unroll
    for (int i = 0; i < MAXC; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
        float o[8], rs[8], dv[8], xv[8];
        unpack8(cdy[i], dv);
        unpack8(cx[i], xv);
        if (dres) unpack8(cres[i], rs);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = r * (dv[e] * t1[i][e] - (xv[e] * r) * dot) + (dres ? rs[e] : 0.f);
        const bf16x8 ov = pack8(o);
        *(bf16x8*)(dx + row * lddx + c * 8) = ov;
        if constexpr (GATE) {
          float dv[8], yv[8], og[8], gf[8], qg[8], qb[8];
          unpack8(ov, dv);
          unpack8(cyg[i], yv);
          unpack8(gv[i], gf);
          float4* q = (float4*)(red + (w * 2 + 0) * d + c * 8);
          float4* b = (float4*)(red + (w * 2 + 1) * d + c * 8);
          *(float4*)qg = q[0];
          *(float4*)(qg + 4) = q[1];
          *(float4*)qb = b[0];
          *(float4*)(qb + 4) = b[1];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            qg[e] += dv[e] * yv[e];
            og[e] = rb(dv[e] * gf[e]);
            qb[e] += og[e];
          }
          q[0] = *(float4*)qg;
          q[1] = *(float4*)(qg + 4);
          b[0] = *(float4*)qb;
          b[1] = *(float4*)(qb + 4);
          *(bf16x8*)(ga.dyg + row * ga.lddyg + c * 8) = pack8(og);
        }
      }
    }
  }
  if constexpr (GATE) {  // the gate's partials: already in LDS, one slice per wave
    __syncthreads();
    for (int j = threadIdx.x; j < d; j += 256) {
      float sa = 0.f, sb = 0.f;
#pragma unroll
      for (int ww = 0; ww < 4; ++ww) {
        sa += red[(ww * 2 + 0) * d + j];
        sb += red[(ww * 2 + 1) * d + j];
      }
      if (ga.dg_bf16)
        ((bf16*)ga.dg)[f * ga.lddg + j] = (bf16)sa;
      else
        ga.dg[f * ga.lddg + j] = sa;
      if (ga.dbf) ga.dbf[f * ga.ldr + j] = sb;
    }
    __syncthreads();
  }
  // combine the 4 waves' column partials
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = lane + 64 * i;
    if (c < nch)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[(w * 2 + 0) * d + c * 8 + e] = pa[i][e];
        red[(w * 2 + 1) * d + c * 8 + e] = pb[i][e];
      }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < d; j += 256) {
    float sa = 0.f, sb = 0.f;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) {
      sa += red[(ww * 2 + 0) * d + j];
      sb += red[(ww * 2 + 1) * d + j];
    }
    if (mod_bf16) {  // straight into the bf16 modulation-gradient matrix (fused.CondModFn)
      ((bf16*)dsc)[f * ldg + j] = (bf16)sa;
      ((bf16*)dsh)[f * ldg + j] = (bf16)sb;
    } else {
      dsc[f * ldg + j] = sa;
      dsh[f * ldg + j] = sb;
    }
  }
}

// ------------------------------------------------------------------ Gate backward
// forward: out = resid + bf16(g[frame] * y)  (fused in the GEMM epilogue)
// backward: dy = bf16(dout * g); dg[frame] = sum_t dout*y; dyf[frame] = sum_t dy (bias partials)
template <int MAXC>
__global__ __launch_bounds__(256) void gate_bwd_k(const bf16* __restrict__ dout, long ldo,
                                                  const bf16* __restrict__ y, long ldy,
                                                  const bf16* __restrict__ g, long ldg, long tpf, int d,
                                                  bf16* __restrict__ dy, long lddy,
                                                  float* __restrict__ dg, float* __restrict__ dbf, long ldr,
                                                  int dg_bf16, long lddg) {
  extern __shared__ float red[];
  const long f = blockIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nch = d / 8;
  float pg[MAXC][8], pb[MAXC][8], gv[MAXC][8];
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = lane + 64 * i;
#pragma unroll
    for (int e = 0; e < 8; ++e) pg[i][e] = pb[i][e] = 0.f;
    if (c < nch) unpack8(*(const bf16x8*)(g + f * ldg + c * 8), gv[i]);
  }
  // the wave's next row is loaded while the current one is processed (two rows in flight)
  bf16x8 nd[MAXC], ny[MAXC];
  auto load = [&](long t) {
    const long row = f * tpf + t;
#pragma unroll
    for (int i = 0; i < MAXC; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
        nd[i] = *(const bf16x8*)(dout + row * ldo + c * 8);
        ny[i] = *(const bf16x8*)(y + row * ldy + c * 8);
      }
    }
  };
  if (w < tpf) load(w);
  for (long t = w; t < tpf; t += 4) {
    const long row = f * tpf + t;
    bf16x8 cd[MAXC], cy[MAXC];
#pragma unroll
    for (int i = 0; i < MAXC; ++i) {
      cd[i] = nd[i];
      cy[i] = ny[i];
    }
    if (t + 4 < tpf) load(t + 4);
#pragma unroll
    for (int i = 0; i < MAXC; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
        float dv[8], yv[8], o[8];
        unpack8(cd[i], dv);
        unpack8(cy[i], yv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          pg[i][e] += dv[e] * yv[e];
          o[e] = rb(dv[e] * gv[i][e]);
          pb[i][e] += o[e];
        }
        *(bf16x8*)(dy + row * lddy + c * 8) = pack8(o);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = lane + 64 * i;
    if (c < nch)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[(w * 2 + 0) * d + c * 8 + e] = pg[i][e];
        red[(w * 2 + 1) * d + c * 8 + e] = pb[i][e];
      }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < d; j += 256) {
    float sa = 0.f, sb = 0.f;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) {
      sa += red[(ww * 2 + 0) * d + j];
      sb += red[(ww * 2 + 1) * d + j];
    }
    if (dg_bf16)
      ((bf16*)dg)[f * lddg + j] = (bf16)sa;
    else
      dg[f * lddg + j] = sa;
    if (dbf) dbf[f * ldr + j] = sb;
  }
}

// ------------------------------------------------------------------ QK RMSNorm + RoPE
// one (token, q|k, head) row of D = 8*CPR elements per CPR lanes; lane owns 4 rotation pairs.
// qkv row layout (attn.py:83): [q(h d) | k(h d) | v(h d)]; out row: [q_rot(h d) | k_rot(h d)]
template <int D>
__global__ __launch_bounds__(256) void qk_rope_fwd_k(const bf16* __restrict__ qkv, long ldq, long T, int H,
                                                     const float* __restrict__ cosb, const float* __restrict__ sinb,
                                                     long ld_tab, long tab_off, long tpos_div,
                                                     bf16* __restrict__ out, long ldo, float* __restrict__ rstd) {
  constexpr int CPR = D / 8;
  const long gid = (long)blockIdx.x * 256 + threadIdx.x;
  const long rowid = gid / CPR;  // (token, which, head)
  const int j = gid % CPR;
  if (rowid >= T * 2 * H) return;
  const long tok = rowid / (2 * H);
  const int wh = rowid % (2 * H);  // which*H + head
  const bf16x8 v = *(const bf16x8*)(qkv + tok * ldq + (long)wh * D + j * 8);
  float xv[8];
  unpack8(v, xv);
  float ss = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) ss += xv[e] * xv[e];
#pragma unroll
  for (int o = 1; o < CPR; o <<= 1) ss += __shfl_xor(ss, o, 64);
  const float r = rsqrtf(ss / D + RMS_EPS);
  if (j == 0 && rstd) rstd[tok * 2 * H + wh] = r;
  const long pos = tab_off + (tpos_div > 0 ? tok % tpos_div : tok);
  const f32x4 c = *(const f32x4*)(cosb + pos * ld_tab + j * 4);
  const f32x4 s = *(const f32x4*)(sinb + pos * ld_tab + j * 4);
  bf16x4 y0, y1;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float x0 = rb(xv[2 * i] * r), x1 = rb(xv[2 * i + 1] * r);
    y0[i] = (bf16)(x0 * c[i] - x1 * s[i]);
    y1[i] = (bf16)(x1 * c[i] + x0 * s[i]);
  }
  bf16* o = out + tok * ldo + (long)wh * D;
  *(bf16x4*)(o + j * 4) = y0;
  *(bf16x4*)(o + D / 2 + j * 4) = y1;
}

// decode form: the same q / k rotation with q, k and a copy of v written to three destinations with
// their own row and batch strides (token t of batch t / L, row t % L) -- k and v straight into the
// KV cache's slots behind the cached window, so the decode step needs no separate cache copies
template <int D>
__global__ __launch_bounds__(256) void qk_rope_kv_k(const bf16* __restrict__ qkv, long ldq, long T, long L, int H,
                                                    const float* __restrict__ cosb, const float* __restrict__ sinb,
                                                    long ld_tab, long tab_off, bf16* __restrict__ qo, long ldqo,
                                                    long sqo, bf16* __restrict__ ko, long ldko, long sko,
                                                    bf16* __restrict__ vo, long ldvo, long svo,
                                                    const long* __restrict__ state, long n_tab, long cap) {
  constexpr int CPR = D / 8;
  const long gid = (long)blockIdx.x * 256 + threadIdx.x;
  const long rowid = gid / CPR;  // (token, which, head)
  const int j = gid % CPR;
  if (rowid >= T * 3 * H) return;
  const long tok = rowid / (3 * H);
  const int wh = rowid % (3 * H);  // which * H + head
  const long bb = tok / L, t = tok - bb * L;
  if (state) {  // {start, cached tokens, rope offset}: k / v rows go behind the window of the buffers
    const long start = state[0], cached = state[1], off = state[2];
    if (start < 0 || cached < 0 || start + cached + L > cap || off < 0 || off + L > n_tab) {
      // a position past the cache buffers or the rope table (the host checks every position it
      // sets; this guards the replayed graph): touch neither, poison this row of q with NaN
      if (wh < H) {
        const bf16x4 nan4 = {(bf16)NAN, (bf16)NAN, (bf16)NAN, (bf16)NAN};
        bf16* o = qo + bb * sqo + t * ldqo + (long)wh * D;
        *(bf16x4*)(o + j * 4) = nan4;
        *(bf16x4*)(o + D / 2 + j * 4) = nan4;
      }
      return;
    }
    ko += (start + cached) * ldko;
    vo += (start + cached) * ldvo;
    tab_off = off;
  }
  const bf16x8 v = *(const bf16x8*)(qkv + tok * ldq + (long)wh * D + j * 8);
  if (wh >= 2 * H) {  // v: copied as is
    *(bf16x8*)(vo + bb * svo + t * ldvo + (long)(wh - 2 * H) * D + j * 8) = v;
    return;
  }
  float xv[8];
  unpack8(v, xv);
  float ss = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) ss += xv[e] * xv[e];
#pragma unroll
  for (int o = 1; o < CPR; o <<= 1) ss += __shfl_xor(ss, o, 64);
  const float r = rsqrtf(ss / D + RMS_EPS);
  const long pos = tab_off + t;
  const f32x4 c = *(const f32x4*)(cosb + pos * ld_tab + j * 4);
  const f32x4 s = *(const f32x4*)(sinb + pos * ld_tab + j * 4);
  bf16x4 y0, y1;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float x0 = rb(xv[2 * i] * r), x1 = rb(xv[2 * i + 1] * r);
    y0[i] = (bf16)(x0 * c[i] - x1 * s[i]);
    y1[i] = (bf16)(x1 * c[i] + x0 * s[i]);
  }
  bf16* o = wh < H ? qo + bb * sqo + t * ldqo + (long)wh * D : ko + bb * sko + t * ldko + (long)(wh - H) * D;
  *(bf16x4*)(o + j * 4) = y0;
  *(bf16x4*)(o + D / 2 + j * 4) = y1;
}

// backward: d(q_rot) -> inverse rotation -> rms_norm backward (recomputing xhat from raw qkv)
template <int D>
__global__ __launch_bounds__(256) void qk_rope_bwd_k(const bf16* __restrict__ dqk, long ldd,
                                                     const bf16* __restrict__ qkv, long ldq, long T, int H,
                                                     const float* __restrict__ cosb, const float* __restrict__ sinb,
                                                     long ld_tab, long tab_off, long tpos_div,
                                                     const float* __restrict__ rstd,
                                                     bf16* __restrict__ dqkv, long ldg) {
  constexpr int CPR = D / 8;
  const long gid = (long)blockIdx.x * 256 + threadIdx.x;
  const long rowid = gid / CPR;
  const int j = gid % CPR;
  if (rowid >= T * 2 * H) return;
  const long tok = rowid / (2 * H);
  const int wh = rowid % (2 * H);
  const bf16* dp = dqk + tok * ldd + (long)wh * D;
  const bf16x4 d0 = *(const bf16x4*)(dp + j * 4);
  const bf16x4 d1 = *(const bf16x4*)(dp + D / 2 + j * 4);
  const long pos = tab_off + (tpos_div > 0 ? tok % tpos_div : tok);
  const f32x4 c = *(const f32x4*)(cosb + pos * ld_tab + j * 4);
  const f32x4 s = *(const f32x4*)(sinb + pos * ld_tab + j * 4);
  float dxn[8], xh[8];
  const float r = rstd[tok * 2 * H + wh];
  float xv[8];
  unpack8(*(const bf16x8*)(qkv + tok * ldq + (long)wh * D + j * 8), xv);
  float dot = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float a = (float)d0[i], b = (float)d1[i];
    dxn[2 * i] = a * c[i] + b * s[i];
    dxn[2 * i + 1] = b * c[i] - a * s[i];
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    xh[e] = xv[e] * r;
    dot += dxn[e] * xh[e];
  }
#pragma unroll
  for (int o = 1; o < CPR; o <<= 1) dot += __shfl_xor(dot, o, 64);
  dot /= D;
  float o[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = r * (dxn[e] - xh[e] * dot);
  *(bf16x8*)(dqkv + tok * ldg + (long)wh * D + j * 8) = pack8(o);
}

#ifndef OWLK_RB_UNROLL
#define OWLK_RB_UNROLL 2
#endif
#ifndef OWLK_RB_MAXBLK
#define OWLK_RB_MAXBLK 1024
#endif
// qk_rope_bwd_k with the column sums of its output fused (the q / k part of the qkv bias gradient,
// attn.py:90's Linear bias): a workgroup is one row of 2 H D / 8 threads (8 columns each) walking
// `rows_per` tokens, so every thread owns fixed columns and adds its bf16-rounded outputs; the
// per-workgroup partial rows are summed in order by colsum_reduce (deterministic).  Saves the
// separate colsum pass's re-read of the 2 H D columns (604 MB per dit_v4 layer).
template <int D>
__global__ __launch_bounds__(1024) void qk_rope_bwd_cs_k(const bf16* __restrict__ dqk, long ldd,
                                                         const bf16* __restrict__ qkv, long ldq, long T, int H,
                                                         const float* __restrict__ cosb,
                                                         const float* __restrict__ sinb, long ld_tab, long tab_off,
                                                         long tpos_div, const float* __restrict__ rstd,
                                                         bf16* __restrict__ dqkv, long ldg, long rows_per,
                                                         float* __restrict__ part) {
  constexpr int CPR = D / 8;
  const int wh = threadIdx.x / CPR, j = threadIdx.x % CPR;
  const long N = 2L * H * D;
  const long t0 = (long)blockIdx.x * rows_per, t1 = t0 + rows_per < T ? t0 + rows_per : T;
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll OWLK_RB_UNROLL
  for (long tok = t0; tok < t1; ++tok) {
    const bf16* dp = dqk + tok * ldd + (long)wh * D;
    const bf16x4 d0 = *(const bf16x4*)(dp + j * 4);
    const bf16x4 d1 = *(const bf16x4*)(dp + D / 2 + j * 4);
    const long pos = tab_off + (tpos_div > 0 ? tok % tpos_div : tok);
    const f32x4 c = *(const f32x4*)(cosb + pos * ld_tab + j * 4);
    const f32x4 s = *(const f32x4*)(sinb + pos * ld_tab + j * 4);
    float dxn[8], xh[8], xv[8];
    const float r = rstd[tok * 2 * H + wh];
    unpack8(*(const bf16x8*)(qkv + tok * ldq + (long)wh * D + j * 8), xv);
    float dot = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float a = (float)d0[i], b = (float)d1[i];
      dxn[2 * i] = a * c[i] + b * s[i];
      dxn[2 * i + 1] = b * c[i] - a * s[i];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      xh[e] = xv[e] * r;
      dot += dxn[e] * xh[e];
    }
#pragma unroll
    for (int o = 1; o < CPR; o <<= 1) dot += __shfl_xor(dot, o, 64);
    dot /= D;
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = r * (dxn[e] - xh[e] * dot);
    const bf16x8 ob = pack8(o);
    *(bf16x8*)(dqkv + tok * ldg + (long)wh * D + j * 8) = ob;
    float ov[8];
    unpack8(ob, ov);
#pragma unroll
    for (int e = 0; e < 8; ++e) cs[e] += ov[e];
  }
  float* dst = part + (long)blockIdx.x * N + (long)wh * D + j * 8;
  *(f32x4*)dst = f32x4{cs[0], cs[1], cs[2], cs[3]};
  *(f32x4*)(dst + 4) = f32x4{cs[4], cs[5], cs[6], cs[7]};
}

// ------------------------------------------------------------------ flow noise + patchify
// x, z: [B, N, C, P] (P = h*w pixels); ts_raw: [B, N] fp32 (pre-sigmoid draw, bf16-valued)
// out: xt_tok, tgt_tok: [B, N*P, C] bf16 token-major (gamerft.py:52 'b n c h w -> b (n h w) c')
__global__ __launch_bounds__(256) void flow_noise_k(const bf16* __restrict__ x, const bf16* __restrict__ z,
                                                    const float* __restrict__ ts_raw, int C, int P, long BN,
                                                    bf16* __restrict__ xt, bf16* __restrict__ tgt,
                                                    float* __restrict__ ts_out) {
  extern __shared__ float tile[];  // [2][C][P+1]
  const long fr = blockIdx.x;
  if (fr >= BN) return;
  const float t = rb(1.f / (1.f + __expf(-rb(ts_raw[fr]))));  // bf16 sigmoid of the bf16 draw
  if (threadIdx.x == 0 && ts_out) ts_out[fr] = t;
  const float omt = rb(1.f - t);
  const long base = fr * (long)C * P;
  for (int i = threadIdx.x; i < C * P; i += 256) {
    const float xv = (float)x[base + i], zv = (float)z[base + i];
    const int c = i / P, pp = i % P;
    tile[c * (P + 1) + pp] = rb(rb(xv * omt) + rb(zv * t));
    tile[C * (P + 1) + c * (P + 1) + pp] = rb(zv - xv);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < C * P; i += 256) {
    const int pp = i / C, c = i % C;
    const long o = (fr * P + pp) * (long)C + c;
    xt[o] = (bf16)tile[c * (P + 1) + pp];
    tgt[o] = (bf16)tile[C * (P + 1) + c * (P + 1) + pp];
  }
}

// token-major [B, N*P, C] -> [B, N, C, P] (unpatchify, gamerft.py:58)
__global__ __launch_bounds__(256) void unpatchify_k(const bf16* __restrict__ tok, int C, int P, long BN,
                                                    bf16* __restrict__ out) {
  extern __shared__ float tile[];
  const long fr = blockIdx.x;
  if (fr >= BN) return;
  for (int i = threadIdx.x; i < C * P; i += 256) {
    const int pp = i / C, c = i % C;
    tile[c * (P + 1) + pp] = (float)tok[(fr * P + pp) * (long)C + c];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < C * P; i += 256) out[fr * (long)C * P + i] = (bf16)tile[(i / P) * (P + 1) + i % P];
}

// ------------------------------------------------------------------ gate + residual (recompute)
// out = bf16(x + bf16(g[t / tpf] * y)): the GATE_RESID GEMM epilogue's output rebuilt from its
// kept inputs (the lean block backward), bit for bit
__global__ __launch_bounds__(256) void gate_resid_k(const bf16* __restrict__ x, long ldx, const bf16* __restrict__ y,
                                                    long ldy, const bf16* __restrict__ g, long ldg, long tpf, long T,
                                                    int d, bf16* __restrict__ out, long ldo) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  const int nch = d / 8;
  if (idx >= T * nch) return;
  const long t = idx / nch;
  const int c = (int)(idx - t * nch) * 8;
  float xv[8], yv[8], gv[8], o[8];
  unpack8(*(const bf16x8*)(x + t * ldx + c), xv);
  unpack8(*(const bf16x8*)(y + t * ldy + c), yv);
  unpack8(*(const bf16x8*)(g + (t / tpf) * ldg + c), gv);
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = xv[e] + rb(gv[e] * yv[e]);
  *(bf16x8*)(out + t * ldo + c) = pack8(o);
}

// ------------------------------------------------------------------ MSE loss + gradient
// partial[block] = sum (pred - tgt)^2 over the block's elements; dpred = bf16(scale*(pred-tgt))
__global__ __launch_bounds__(256) void mse_k(const bf16* __restrict__ pred, const bf16* __restrict__ tgt, long n8,
                                             float gscale, bf16* __restrict__ dpred, float* __restrict__ partial) {
  __shared__ float red[4];
  float acc = 0.f;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    float p[8], t[8], g[8];
    unpack8(((const bf16x8*)pred)[i], p);
    unpack8(((const bf16x8*)tgt)[i], t);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float df = p[e] - t[e];
      acc += df * df;
      g[e] = gscale * df;
    }
    if (dpred) ((bf16x8*)dpred)[i] = pack8(g);
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// loss = (float)(sum of the partials in double, in block order) / n: one workgroup, fixed order
__global__ __launch_bounds__(64) void mse_finish_k(const float* __restrict__ partial, int nb, long n,
                                                   float* __restrict__ loss) {
  __shared__ double red[64];
  double acc = 0.0;
  for (int i = threadIdx.x; i < nb; i += 64) acc += (double)partial[i];
  red[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int i = 0; i < 64; ++i) s += red[i];
    loss[0] = (float)s / (float)n;
  }
}

// backward of F.mse_loss (fp32 math under autocast): dpred = bf16((gscale (pred - tgt)) g), g the
// loss gradient read on the device (null: 1)
__global__ __launch_bounds__(256) void mse_grad_k(const bf16* __restrict__ pred, const bf16* __restrict__ tgt, long n8,
                                                  float gscale, const float* __restrict__ gout,
                                                  bf16* __restrict__ dpred) {
  const float go = gout ? gout[0] : 1.f;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    float p[8], t[8], g[8];
    unpack8(((const bf16x8*)pred)[i], p);
    unpack8(((const bf16x8*)tgt)[i], t);
#pragma unroll
    for (int e = 0; e < 8; ++e) g[e] = (gscale * (p[e] - t[e])) * go;
    ((bf16x8*)dpred)[i] = pack8(g);
  }
}

// ------------------------------------------------------------------ column sums (bias grads)
// out[n] (+)= sum_r x[r, n]; x bf16 or fp32; grid.y splits the rows.  With a workspace each split
// stores its partial row (part[split][n]) and colsum_reduce_k adds them onto out in split order
// (bitwise reproducible); without one, fp32 atomics combine the splits.
// fs > 0: frame-strided rows, row r at (r / 64) * fs + (r % 64) * ld (owlk_colsum_frames)
template <typename T, int U>
__global__ __launch_bounds__(256) void colsum_k(const T* __restrict__ x, long R, long N, long ld, long rows_per,
                                                float* __restrict__ out, float* __restrict__ part, long fs) {
  const long col = ((long)blockIdx.x * 256 + threadIdx.x) * 8;
  if (col >= N) return;
  const long r0 = (long)blockIdx.y * rows_per, r1 = r0 + rows_per < R ? r0 + rows_per : R;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  auto add_row = [&](long r) {
    const long ro = fs ? (r >> 6) * fs + (r & 63) * ld : r * ld;
    if constexpr (sizeof(T) == 2) {
      float v[8];
      unpack8(__builtin_nontemporal_load((const bf16x8*)(x + ro + col)), v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += v[e];
    } else {
      const f32x4 a = *(const f32x4*)(x + ro + col), b = *(const f32x4*)(x + ro + col + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[e] += a[e];
        acc[e + 4] += b[e];
      }
    }
  };
  long r = r0;
  // U rows per iteration: U independent 16-B loads in flight per lane (latency-bound otherwise)
  for (; r + U <= r1; r += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) add_row(r + u);
  }
  for (; r < r1; ++r) add_row(r);
  if (part) {
    float* dst = part + (long)blockIdx.y * N + col;
    *(f32x4*)dst = f32x4{acc[0], acc[1], acc[2], acc[3]};
    *(f32x4*)(dst + 4) = f32x4{acc[4], acc[5], acc[6], acc[7]};
    return;
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) atomicAdd(out + col + e, acc[e]);
}

// out[n] += sum_s part[s][n] (N % 4 == 0); shared with the GEMM's fused column sums.  A block is 64
// columns (16 quads) x 16 split lanes: lane sl adds splits sl, sl + 16, ... in order with 8 loads in
// flight (a single thread walking hundreds of splits is latency-bound), then the 16 lane sums meet
// in a fixed LDS tree -- the result depends only on (splits, N), never on timing.
__global__ __launch_bounds__(256) void colsum_reduce_k(const float* __restrict__ part, int splits, long N,
                                                       float* __restrict__ out) {
  __shared__ f32x4 red[16][16];
  const int cq = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const long n = ((long)blockIdx.x * 16 + cq) * 4;
  f32x4 a = {0.f, 0.f, 0.f, 0.f};
  if (n < N) {
    int sp = sl;
    for (; sp + 16 * 7 < splits; sp += 16 * 8) {
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *(const f32x4*)(part + (long)(sp + 16 * u) * N + n);
#pragma unroll
      for (int u = 0; u < 8; ++u) a += v[u];
    }
    for (; sp < splits; sp += 16) a += *(const f32x4*)(part + (long)sp * N + n);
  }
  red[sl][cq] = a;
  __syncthreads();
#pragma unroll
  for (int w = 8; w >= 1; w >>= 1) {
    if (sl < w) red[sl][cq] += red[sl + w][cq];
    __syncthreads();
  }
  if (sl == 0 && n < N) {
    f32x4 o = *(f32x4*)(out + n);
    o += red[0][cq];
    *(f32x4*)(out + n) = o;
  }
}

// ------------------------------------------------------------------ attention-bwd preprocess
// delta[b, h, t] = sum_d dO[t, h, d] * O[t, h, d]   (fp32; D = 64/128 -> 8/16 lanes per row)
template <int D>
__global__ __launch_bounds__(256) void attn_delta_k(const bf16* __restrict__ o, const bf16* __restrict__ dout,
                                                    long ld, long L, int H, long nrows, float* __restrict__ delta) {
  constexpr int CPR = D / 8;
  const long gid = (long)blockIdx.x * 256 + threadIdx.x;
  const long rowid = gid / CPR;  // (b, t, h) in token-major order
  const int j = gid % CPR;
  if (rowid >= nrows) return;
  const long bt = rowid / H;
  const int h = rowid % H;
  float a[8], b[8];
  unpack8(*(const bf16x8*)(o + bt * ld + (long)h * D + j * 8), a);
  unpack8(*(const bf16x8*)(dout + bt * ld + (long)h * D + j * 8), b);
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) s += a[e] * b[e];
#pragma unroll
  for (int off = 1; off < CPR; off <<= 1) s += __shfl_xor(s, off, 64);
  if (j == 0) {
    const long bb = bt / L, t = bt % L;
    delta[(bb * H + h) * L + t] = s;
  }
}

}  // namespace

// ======================================================================== C ABI
extern "C" int owlk_adaln_fwd(const void* x, long ldx, const void* scale, const void* shift, long ldm, long tpf,
                              long T, int d, void* y, long ldy, float* rstd, void* yact, void* stream) {
  OWLK_REQUIRE(d % 8 == 0 && d <= 64 * 8 * MAXCPL && tpf > 0 && T % tpf == 0, "adaln_fwd: bad d=%d tpf=%ld T=%ld", d,
               tpf, T);
  OWLK_CPL_DISPATCH(d, adaln_fwd_k, dim3((unsigned)((T + 3) / 4)), dim3(256), 0, (hipStream_t)stream, (const bf16*)x,
                     ldx, (const bf16*)scale, (const bf16*)shift, ldm, tpf, T, d, (bf16*)y, ldy, rstd, (bf16*)yact);
  return owlk::check_launch("adaln_fwd");
}

extern "C" int owlk_adaln_bwd(const void* dy, long lddy, const void* x, long ldx, const float* rstd,
                              const void* scale, long ldm, long tpf, long T, int d, const void* dres, long ldres,
                              void* dx, long lddx, void* dscale, void* dshift, long ldg, const void* ypre,
                              int mod_bf16, void* stream) {
  OWLK_REQUIRE(d % 8 == 0 && d <= 64 * 8 * MAXCPL && tpf > 0 && T % tpf == 0, "adaln_bwd: bad d=%d tpf=%ld T=%ld", d,
               tpf, T);
  OWLK_CPL_DISPATCH(d, adaln_bwd_k, dim3((unsigned)(T / tpf)), dim3(256), 8 * d * sizeof(float), (hipStream_t)stream,
                     (const bf16*)dy, lddy, (const bf16*)x, ldx, rstd, (const bf16*)scale, ldm, tpf, d,
                     (const bf16*)dres, ldres, (bf16*)dx, lddx, (float*)dscale, (float*)dshift, ldg, (const bf16*)ypre,
                     mod_bf16);
  return owlk::check_launch("adaln_bwd");
}

extern "C" int owlk_adaln_gate_bwd(const void* dy, long lddy, const void* x, long ldx, const float* rstd,
                                   const void* scale, long ldm, long tpf, long T, int d, const void* dres, long ldres,
                                   void* dx, long lddx, void* dscale, void* dshift, long ldg, int mod_bf16,
                                   const void* y, long ldy, const void* g, long ldgg, void* dyg, long lddyg, void* dg,
                                   long lddg, int dg_bf16, float* dbias_frames, long ldr, void* stream) {
  OWLK_REQUIRE(d % 8 == 0 && d <= 64 * 8 * MAXCPL && tpf > 0 && T % tpf == 0,
               "adaln_gate_bwd: bad d=%d tpf=%ld T=%ld", d, tpf, T);
  OWLK_REQUIRE(y && g && dyg && dg, "adaln_gate_bwd: y, g, dyg and dg are required");
  const GateBwdArgs ga{(const bf16*)y, ldy, (const bf16*)g, ldgg, (bf16*)dyg, lddyg, (float*)dg, lddg, dg_bf16,
                       dbias_frames, ldr};
  const dim3 grid((unsigned)(T / tpf));
  const size_t lds = 8 * d * sizeof(float);
  hipStream_t s = (hipStream_t)stream;
#define OWLK_AGB(C)                                                                                                  \
  hipLaunchKernelGGL((adaln_bwd_k<C, true>), grid, dim3(256), lds, s, (const bf16*)dy, lddy, (const bf16*)x, ldx,    \
                     rstd, (const bf16*)scale, ldm, tpf, d, (const bf16*)dres, ldres, (bf16*)dx, lddx, (float*)dscale, \
                     (float*)dshift, ldg, (const bf16*)nullptr, mod_bf16, ga)
  switch ((d / 8 + 63) / 64) {
    case 1: OWLK_AGB(1); break;
    case 2: OWLK_AGB(2); break;
    case 3: OWLK_AGB(3); break;
    case 4: OWLK_AGB(4); break;
    case 5: OWLK_AGB(5); break;
    case 6: OWLK_AGB(6); break;
    default: OWLK_AGB(8); break;
  }
#undef OWLK_AGB
  return owlk::check_launch("adaln_gate_bwd");
}

extern "C" int owlk_gate_bwd(const void* dout, long ldo, const void* y, long ldy, const void* g, long ldg, long tpf,
                             long T, int d, void* dy, long lddy, void* dg, long lddg, int dg_bf16,
                             float* dbias_frames, long ldr, void* stream) {
  OWLK_REQUIRE(d % 8 == 0 && d <= 64 * 8 * MAXCPL && tpf > 0 && T % tpf == 0, "gate_bwd: bad d=%d tpf=%ld T=%ld", d,
               tpf, T);
  OWLK_CPL_DISPATCH(d, gate_bwd_k, dim3((unsigned)(T / tpf)), dim3(256), 8 * d * sizeof(float), (hipStream_t)stream,
                     (const bf16*)dout, ldo, (const bf16*)y, ldy, (const bf16*)g, ldg, tpf, d, (bf16*)dy, lddy,
                     (float*)dg, dbias_frames, ldr, dg_bf16, lddg);
  return owlk::check_launch("gate_bwd");
}

// every table row a launch reads lies inside the [n_tab, ld_tab] cos / sin tables (the reference
// slices cos[offset:offset + n] and fails on a short slice, rope.py:46-49; a kernel would read past
// the buffer instead)
static bool rope_rows_ok(long T, long n_tab, long tab_off, long tpos_div) {
  const long span = tpos_div > 0 ? (T < tpos_div ? T : tpos_div) : T;
  return n_tab > 0 && tab_off >= 0 && tab_off + span <= n_tab;
}

extern "C" int owlk_qk_rope_fwd(const void* qkv, long ldq, long T, int H, int D, const float* cosb,
                                const float* sinb, long ld_tab, long n_tab, long tab_off, long tpos_div, void* out,
                                long ldo, float* rstd, void* stream) {
  OWLK_REQUIRE(D == 64 || D == 128, "qk_rope_fwd: head_dim %d unsupported", D);
  OWLK_REQUIRE(rope_rows_ok(T, n_tab, tab_off, tpos_div), "qk_rope_fwd: positions %ld.. past the %ld-row rope table",
               tab_off, n_tab);
  const long threads = T * 2 * H * (D / 8);
  dim3 g((unsigned)((threads + 255) / 256));
  if (D == 64)
    hipLaunchKernelGGL(qk_rope_fwd_k<64>, g, dim3(256), 0, (hipStream_t)stream, (const bf16*)qkv, ldq, T, H, cosb,
                       sinb, ld_tab, tab_off, tpos_div, (bf16*)out, ldo, rstd);
  else
    hipLaunchKernelGGL(qk_rope_fwd_k<128>, g, dim3(256), 0, (hipStream_t)stream, (const bf16*)qkv, ldq, T, H, cosb,
                       sinb, ld_tab, tab_off, tpos_div, (bf16*)out, ldo, rstd);
  return owlk::check_launch("qk_rope_fwd");
}

static int qk_rope_kv_launch(const void* qkv, long ldq, long T, long L, int H, int D, const float* cosb,
                             const float* sinb, long ld_tab, long n_tab, long tab_off, void* qo, long ldqo, long sqo,
                             void* ko, long ldko, long sko, void* vo, long ldvo, long svo, const long* state,
                             long cap, void* stream);


extern "C" int owlk_qk_rope_fwd_kv(const void* qkv, long ldq, long T, long L, int H, int D, const float* cosb,
                                   const float* sinb, long ld_tab, long n_tab, long tab_off, void* qo, long ldqo,
                                   long sqo, void* ko, long ldko, long sko, void* vo, long ldvo, long svo,
                                   void* stream) {
  OWLK_REQUIRE(L > 0 && rope_rows_ok(L, n_tab, tab_off, 0), "qk_rope_fwd_kv: positions %ld.. past the %ld-row rope table",
               tab_off, n_tab);
  return qk_rope_kv_launch(qkv, ldq, T, L, H, D, cosb, sinb, ld_tab, n_tab, tab_off, qo, ldqo, sqo, ko, ldko, sko, vo,
                           ldvo, svo, nullptr, 0, stream);
}

extern "C" int owlk_qk_rope_fwd_kv_dev(const void* qkv, long ldq, long T, long L, int H, int D, const float* cosb,
                                       const float* sinb, long ld_tab, long n_tab, const long* state, void* qo,
                                       long ldqo, long sqo, void* kbuf, long ldk, long skb, void* vbuf, long ldv,
                                       long svb, long cap, void* stream) {
  OWLK_REQUIRE(state, "qk_rope_fwd_kv_dev: state pointer required");
  OWLK_REQUIRE(n_tab > 0 && cap > 0, "qk_rope_fwd_kv_dev: rope table rows / cache capacity required");
  return qk_rope_kv_launch(qkv, ldq, T, L, H, D, cosb, sinb, ld_tab, n_tab, 0, qo, ldqo, sqo, kbuf, ldk, skb, vbuf, ldv,
                           svb, state, cap, stream);
}

static int qk_rope_kv_launch(const void* qkv, long ldq, long T, long L, int H, int D, const float* cosb,
                             const float* sinb, long ld_tab, long n_tab, long tab_off, void* qo, long ldqo, long sqo,
                             void* ko, long ldko, long sko, void* vo, long ldvo, long svo, const long* state,
                             long cap, void* stream) {
  OWLK_REQUIRE(D == 64 || D == 128, "qk_rope_fwd_kv: head_dim %d unsupported", D);
  OWLK_REQUIRE(L > 0 && T % L == 0, "qk_rope_fwd_kv: T=%ld is not a whole number of L=%ld rows", T, L);
  OWLK_REQUIRE(((uintptr_t)qo | (uintptr_t)ko | (uintptr_t)vo) % 16 == 0 && ldqo % 8 == 0 && ldko % 8 == 0 &&
                   ldvo % 8 == 0 && sqo % 8 == 0 && sko % 8 == 0 && svo % 8 == 0,
               "qk_rope_fwd_kv: destinations must be 16-byte aligned");
  const long threads = T * 3 * H * (D / 8);
  dim3 g((unsigned)((threads + 255) / 256));
  if (D == 64)
    hipLaunchKernelGGL(qk_rope_kv_k<64>, g, dim3(256), 0, (hipStream_t)stream, (const bf16*)qkv, ldq, T, L, H, cosb,
                       sinb, ld_tab, tab_off, (bf16*)qo, ldqo, sqo, (bf16*)ko, ldko, sko, (bf16*)vo, ldvo, svo, state,
                       n_tab, cap);
  else
    hipLaunchKernelGGL(qk_rope_kv_k<128>, g, dim3(256), 0, (hipStream_t)stream, (const bf16*)qkv, ldq, T, L, H, cosb,
                       sinb, ld_tab, tab_off, (bf16*)qo, ldqo, sqo, (bf16*)ko, ldko, sko, (bf16*)vo, ldvo, svo, state,
                       n_tab, cap);
  return owlk::check_launch("qk_rope_fwd_kv");
}

extern "C" int owlk_qk_rope_bwd(const void* dqk, long ldd, const void* qkv, long ldq, long T, int H, int D,
                                const float* cosb, const float* sinb, long ld_tab, long n_tab, long tab_off,
                                long tpos_div, const float* rstd, void* dqkv, long ldg, void* stream) {
  OWLK_REQUIRE(D == 64 || D == 128, "qk_rope_bwd: head_dim %d unsupported", D);
  OWLK_REQUIRE(rope_rows_ok(T, n_tab, tab_off, tpos_div), "qk_rope_bwd: positions %ld.. past the %ld-row rope table",
               tab_off, n_tab);
  const long threads = T * 2 * H * (D / 8);
  dim3 g((unsigned)((threads + 255) / 256));
  if (D == 64)
    hipLaunchKernelGGL(qk_rope_bwd_k<64>, g, dim3(256), 0, (hipStream_t)stream, (const bf16*)dqk, ldd,
                       (const bf16*)qkv, ldq, T, H, cosb, sinb, ld_tab, tab_off, tpos_div, rstd, (bf16*)dqkv, ldg);
  else
    hipLaunchKernelGGL(qk_rope_bwd_k<128>, g, dim3(256), 0, (hipStream_t)stream, (const bf16*)dqk, ldd,
                       (const bf16*)qkv, ldq, T, H, cosb, sinb, ld_tab, tab_off, tpos_div, rstd, (bf16*)dqkv, ldg);
  return owlk::check_launch("qk_rope_bwd");
}

// row-blocks of the fused-bias qk_rope backward: ~1024 workgroups, >= 16 tokens each; 0 = shape not
// supported by the fused form (one row of 2 H D / 8 threads must be whole waves, <= 1024 threads)
static long qk_rope_bwd_blocks(long T, int H, int D, long* rows_per) {
  const long thr = 2L * H * D / 8;
  if ((D != 64 && D != 128) || T <= 0 || thr % 64 || thr > 1024) return 0;
  long nb = T / 16 < OWLK_RB_MAXBLK ? T / 16 : OWLK_RB_MAXBLK;
  if (nb < 1) nb = 1;
  const long rp = (T + nb - 1) / nb;
  if (rows_per) *rows_per = rp;
  return (T + rp - 1) / rp;
}

extern "C" long owlk_qk_rope_bwd_ws_bytes(long T, int H, int D) {
  return qk_rope_bwd_blocks(T, H, D, nullptr) * 2L * H * D * (long)sizeof(float);
}

extern "C" int owlk_qk_rope_bwd_bias(const void* dqk, long ldd, const void* qkv, long ldq, long T, int H, int D,
                                     const float* cosb, const float* sinb, long ld_tab, long n_tab, long tab_off,
                                     long tpos_div, const float* rstd, void* dqkv, long ldg, float* dbias, void* ws,
                                     long ws_bytes, void* stream) {
  OWLK_REQUIRE(rope_rows_ok(T, n_tab, tab_off, tpos_div),
               "qk_rope_bwd_bias: positions %ld.. past the %ld-row rope table", tab_off, n_tab);
  long rows_per = 0;
  const long nb = qk_rope_bwd_blocks(T, H, D, &rows_per);
  const long N = 2L * H * D;
  OWLK_REQUIRE(nb > 0, "qk_rope_bwd_bias: H=%d D=%d not supported by the fused form", H, D);
  OWLK_REQUIRE(ws && ws_bytes >= nb * N * (long)sizeof(float) && ((uintptr_t)ws & 15) == 0,
               "qk_rope_bwd_bias: workspace too small or misaligned (owlk_qk_rope_bwd_ws_bytes)");
  OWLK_REQUIRE(dbias && ((uintptr_t)dbias & 15) == 0, "qk_rope_bwd_bias: dbias must be 16-byte aligned");
  hipStream_t s = (hipStream_t)stream;
  const dim3 g((unsigned)nb), blk((unsigned)(N / 8));
  if (D == 64)
    hipLaunchKernelGGL(qk_rope_bwd_cs_k<64>, g, blk, 0, s, (const bf16*)dqk, ldd, (const bf16*)qkv, ldq, T, H, cosb,
                       sinb, ld_tab, tab_off, tpos_div, rstd, (bf16*)dqkv, ldg, rows_per, (float*)ws);
  else
    hipLaunchKernelGGL(qk_rope_bwd_cs_k<128>, g, blk, 0, s, (const bf16*)dqk, ldd, (const bf16*)qkv, ldq, T, H, cosb,
                       sinb, ld_tab, tab_off, tpos_div, rstd, (bf16*)dqkv, ldg, rows_per, (float*)ws);
  if (int e = owlk::check_launch("qk_rope_bwd_bias")) return e;
  return owlk::colsum_reduce((const float*)ws, (int)nb, N, dbias, s);
}

extern "C" int owlk_flow_noise(const void* x, const void* z, const float* ts_raw, int C, int P, long BN, void* xt,
                               void* tgt, float* ts_out, void* stream) {
  OWLK_REQUIRE(C * P <= 16384 && C > 0 && P > 0, "flow_noise: C*P too large");
  hipLaunchKernelGGL(flow_noise_k, dim3((unsigned)BN), dim3(256), 2 * C * (P + 1) * sizeof(float),
                     (hipStream_t)stream, (const bf16*)x, (const bf16*)z, ts_raw, C, P, BN, (bf16*)xt, (bf16*)tgt,
                     ts_out);
  return owlk::check_launch("flow_noise");
}

extern "C" int owlk_unpatchify(const void* tok, int C, int P, long BN, void* out, void* stream) {
  OWLK_REQUIRE(C * P <= 16384, "unpatchify: C*P too large");
  hipLaunchKernelGGL(unpatchify_k, dim3((unsigned)BN), dim3(256), C * (P + 1) * sizeof(float), (hipStream_t)stream,
                     (const bf16*)tok, C, P, BN, (bf16*)out);
  return owlk::check_launch("unpatchify");
}

extern "C" int owlk_gate_resid(const void* x, long ldx, const void* y, long ldy, const void* g, long ldg, long tpf,
                               long T, int d, void* out, long ldo, void* stream) {
  OWLK_REQUIRE(d % 8 == 0 && T > 0 && tpf > 0 && T % tpf == 0, "gate_resid: bad sizes");
  OWLK_REQUIRE((((uintptr_t)x | (uintptr_t)y | (uintptr_t)g | (uintptr_t)out) % 16 == 0) &&
                   (ldx | ldy | ldg | ldo) % 8 == 0,
               "gate_resid: rows must be 16-byte aligned");
  const long work = T * (d / 8);
  hipLaunchKernelGGL(gate_resid_k, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)x, ldx, (const bf16*)y, ldy, (const bf16*)g, ldg, tpf, T, d, (bf16*)out, ldo);
  return owlk::check_launch("gate_resid");
}

extern "C" int owlk_mse(const void* pred, const void* tgt, long n, float gscale, void* dpred, float* partial,
                        int nblocks, float* loss, void* stream) {
  OWLK_REQUIRE(n % 8 == 0 && nblocks > 0, "mse: n=%ld must be a multiple of 8", n);
  hipLaunchKernelGGL(mse_k, dim3(nblocks), dim3(256), 0, (hipStream_t)stream, (const bf16*)pred, (const bf16*)tgt,
                     n / 8, gscale, (bf16*)dpred, partial);
  if (loss) {
    if (int rc = owlk::check_launch("mse")) return rc;
    hipLaunchKernelGGL(mse_finish_k, dim3(1), dim3(64), 0, (hipStream_t)stream, partial, nblocks, n, loss);
  }
  return owlk::check_launch("mse");
}

extern "C" int owlk_mse_grad(const void* pred, const void* tgt, long n, float gscale, const float* gout, void* dpred,
                             void* stream) {
  OWLK_REQUIRE(n % 8 == 0 && dpred, "mse_grad: n=%ld must be a multiple of 8", n);
  const long n8 = n / 8;
  const long nb = (n8 + 255) / 256 < 2048 ? (n8 + 255) / 256 : 2048;
  hipLaunchKernelGGL(mse_grad_k, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, (const bf16*)pred,
                     (const bf16*)tgt, n8, gscale, gout, (bf16*)dpred);
  return owlk::check_launch("mse_grad");
}

// enough row splits to fill the chip (~2k workgroups), but >= 16 rows per workgroup: in the atomic
// form every split adds N atomics onto the same N outputs, and short splits turn into same-address
// contention (<= 512 adders per output: 2048 splits onto N = 1536 ran at 0.66 TB/s)
static long colsum_splits(long R, long N, long* rows_per) {
  const long cols_blocks = (N / 8 + 255) / 256;
  long splits = 2048 / cols_blocks;
  if (splits > 512) splits = 512;
  if (splits > R / 16) splits = R / 16;
  if (splits < 1) splits = 1;
  const long rp = (R + splits - 1) / splits;
  if (rows_per) *rows_per = rp;
  return (R + rp - 1) / rp;
}

extern "C" long owlk_colsum_ws_bytes(long R, long N) {
  if (R <= 0 || N <= 0) return 0;
  return colsum_splits(R, N, nullptr) * N * (long)sizeof(float);
}

extern "C" int owlk_colsum_frames(const void* x, int x_f32, long R, long N, long ld, long fs, float* out, void* ws,
                                  long ws_bytes, void* stream);

extern "C" int owlk_colsum(const void* x, int x_f32, long R, long N, long ld, float* out, void* ws, long ws_bytes,
                           void* stream) {
  return owlk_colsum_frames(x, x_f32, R, N, ld, 0, out, ws, ws_bytes, stream);
}

extern "C" int owlk_colsum_frames(const void* x, int x_f32, long R, long N, long ld, long fs, float* out, void* ws,
                                  long ws_bytes, void* stream) {
  OWLK_REQUIRE(N % 8 == 0 && ld % 8 == 0, "colsum: N, ld must be multiples of 8");
  OWLK_REQUIRE(fs == 0 || (fs > 0 && fs % 8 == 0 && R % 64 == 0), "colsum: frame-strided rows need whole 64-row frames");
  OWLK_REQUIRE(((uintptr_t)out & 15) == 0, "colsum: out must be 16-byte aligned");
  long rows_per;
  const long splits = colsum_splits(R, N, &rows_per);
  const long cols_blocks = (N / 8 + 255) / 256;
  float* part = (ws && ws_bytes >= splits * N * (long)sizeof(float) && ((uintptr_t)ws & 15) == 0) ? (float*)ws
                                                                                                   : nullptr;
  dim3 g((unsigned)cols_blocks, (unsigned)splits);
  hipStream_t s = (hipStream_t)stream;
  if (x_f32)
    hipLaunchKernelGGL((colsum_k<float, 4>), g, dim3(256), 0, s, (const float*)x, R, N, ld, rows_per, out, part, fs);
  else
    hipLaunchKernelGGL((colsum_k<bf16, 8>), g, dim3(256), 0, s, (const bf16*)x, R, N, ld, rows_per, out, part, fs);
  if (part) return owlk::colsum_reduce(part, (int)splits, N, out, s);
  return owlk::check_launch("colsum");
}

int owlk::colsum_reduce(const float* part, int splits, long N, float* out, hipStream_t s) {
  hipLaunchKernelGGL(colsum_reduce_k, dim3((unsigned)((N + 63) / 64)), dim3(256), 0, s, part, splits, N, out);
  return owlk::check_launch("colsum_reduce");
}

extern "C" int owlk_attn_delta(const void* o, const void* dout, long ld, long B, long L, int H, int D, float* delta,
                               void* stream) {
  OWLK_REQUIRE(D == 64 || D == 128, "attn_delta: head_dim %d unsupported", D);
  const long nrows = B * L * H;
  const long threads = nrows * (D / 8);
  dim3 g((unsigned)((threads + 255) / 256));
  if (D == 64)
    hipLaunchKernelGGL(attn_delta_k<64>, g, dim3(256), 0, (hipStream_t)stream, (const bf16*)o, (const bf16*)dout, ld,
                       L, H, nrows, delta);
  else
    hipLaunchKernelGGL(attn_delta_k<128>, g, dim3(256), 0, (hipStream_t)stream, (const bf16*)o, (const bf16*)dout,
                       ld, L, H, nrows, delta);
  return owlk::check_launch("attn_delta");
}
