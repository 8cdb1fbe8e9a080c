// Block-sparse frame-causal flash attention, backward (gfx950, head_dim 64 and 128).
//
// Gradient of the reference's flex_attention (attn.py:106-109; autograd of torch's flex
// template): with P recomputed from the forward log-sum-exp,
//   dV = P^T dO,  dS = P o (dP - delta),  dP = dO V^T,  delta = rowsum(dO o O),
//   dK = scale * dS^T Q,  dQ = scale * dS K.
// lse is the forward's base-2 log-sum-exp of the scaled logits, so P = exp2(c s - lse).
// Two deterministic kernels (no float atomics):
//   dkdv : workgroup = 4 waves x 32 keys; sweeps 64-query tiles; S, dP with the key on the lane
//          (Q/dO rows x K/V in registers), then dV^T += dO^T P and dK^T += Q^T dS take P / dS
//          straight from the accumulators as B operands.
//   dq   : workgroup = 4 waves x 32 queries; sweeps 64-key tiles like the forward (query on the
//          lane), dQ^T += K^T dS^T with K^T fragments through ds_read_b64_tr_b16.
#include "attn_common.hpp"


namespace {

constexpr int TB = 128;              // rows owned by a workgroup (4 waves x 32)
constexpr int TL = 64;               // rows per swept tile
constexpr int SUB = TL * 64 * 2;     // one 64-row x 64-column bf16 sub-tile (128-B rows): 8 KiB
constexpr float LOG2E = 1.4426950408889634f;

// head_dim D as D/64 column sub-tiles (see attn_fwd.hip); ring depth 3 at D 64, 2 at D 128
template <int D>
struct Cfg {
  static constexpr int NSUB = D / 64, NS = D / 16, NDB = D / 32;
  static constexpr int NBUF = D == 64 ? 3 : 2;
  static constexpr int OPS = 4 * NSUB;  // LDS-DMA wave-instructions per tile per wave (two tiles)
};

struct BwdP {
  const bf16 *q, *k, *v, *dout;
  const float *lse, *delta;  // [B, H, Lq]; lse in base 2 (attn_fwd)
  bf16 *dq, *dk, *dv;
  long ldq, ldk, ldv, ldo, lddq, lddk, lddv;  // token row strides
  long sqb, skb, svb, sob, sdqb, sdkb, sdvb;  // batch strides
  long Lq, Lkv;
  int H;
  float scale, scale_log2;
  MaskP m;
};

template <int N>
DEV void vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int NDB>
DEV void store_rowT(bf16* dst, const f32x16 (&acc)[NDB], float mul, int h) {
#pragma unroll
  for (int db = 0; db < NDB; ++db)
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      bf16x4 v4;
#pragma unroll
      for (int e = 0; e < 4; ++e) v4[e] = (bf16)(acc[db][4 * gq + e] * mul);
      *(bf16x4*)(dst + 32 * db + 8 * gq + 4 * h) = v4;
    }
}

// ======================================================================== dK, dV
// Query tiles of QT x 64 rows per ring slot.  QT = 2 (D 64, unwindowed masks: two-slot ring,
// 66 KiB per workgroup, two workgroups per CU) pays the per-tile fixed costs (DMA issue, ring
// bookkeeping, the workgroup barrier) once per 64 MFMAs: global layers -2.5 %.  Windowed (local)
// layers keep QT = 1 and the three-slot ring: their short sweeps are dominated by mask-edge
// tiles, which QT = 2 makes twice as large (+60 % measured there).
template <int D, int QT_>
struct DkdvCfg {
  static constexpr int QT = QT_;
  static constexpr int NBUF = QT == 2 ? 2 : Cfg<D>::NBUF;
  static constexpr int TLQ = TL * QT;  // query rows per tile
};

// FULL tiles (no mask bits): the 2 QT blocks of 32 query rows x this wave's 32 keys run as a
// software pipeline in one branch-free region, so the S / dP MFMAs of block i+1 issue while the
// VALU turns block i's scores into P and dS (exp2, multiply, bf16 packing).  For the one-wave-
// per-SIMD D 128 kernel, whose MFMA pipe has no partner wave to cover the softmax; at D 64 the
// two co-resident waves already do that (+1 % measured there, so not used).
template <class C, int QT>
DEV void dkdv_full_pipelined(const char* tb, const float* l2, const float* dlt, const bf16x8 (&kf)[C::NS],
                             const bf16x8 (&vf)[C::NS], f32x16 (&dk)[C::NDB], f32x16 (&dv)[C::NDB], int lane) {
  const int h = lane >> 5;
  constexpr int NB = 2 * QT;  // 32-row blocks per tile
  auto chains = [&](int blk, f32x16& st, f32x16& dp) {
    const int sq = blk >> 1, qb = blk & 1;
    const char* lq = tb + sq * C::NSUB * SUB;
    const char* ld = tb + (QT + sq) * C::NSUB * SUB;
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int rowb = 64 * sq + 32 * qb + 8 * g4 + 4 * h;
      const f32x4 L = *(const f32x4*)(l2 + rowb);
      const f32x4 Dl = *(const f32x4*)(dlt + rowb);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        st[4 * g4 + e] = L[e];
        dp[4 * g4 + e] = Dl[e];
      }
    }
#pragma unroll
    for (int s = 0; s < C::NS; ++s) {
      st = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_row<SW_DUAL>(lq + (s >> 2) * SUB, 32 * qb, s & 3, lane),
                                                   kf[s], st, 0, 0, 0);
      dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_row<SW_DUAL>(ld + (s >> 2) * SUB, 32 * qb, s & 3, lane),
                                                   vf[s], dp, 0, 0, 0);
    }
  };
  auto softmax = [&](f32x16& st, f32x16& dp, bf16x8 (&pf)[2], bf16x8 (&sf)[2]) {
#pragma unroll
    for (int r = 0; r < 16; ++r) st[r] = __builtin_amdgcn_exp2f(-st[r]);
#pragma unroll
    for (int r = 0; r < 16; ++r) dp[r] *= st[r];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      pf[s] = acc_frag(st, s);
      sf[s] = acc_frag(dp, s);
    }
  };
  auto grads = [&](int blk, const bf16x8 (&pf)[2], const bf16x8 (&sf)[2]) {
    const int sq = blk >> 1, qb = blk & 1;
    const char* lq = tb + sq * C::NSUB * SUB;
    const char* ld = tb + (QT + sq) * C::NSUB * SUB;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int db = 0; db < C::NDB; ++db) {
        dv[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_tr<SW_DUAL>(ld + (db >> 1) * SUB, 32 * qb, s, db & 1, lane),
                                                         pf[s], dv[db], 0, 0, 0);
        dk[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_tr<SW_DUAL>(lq + (db >> 1) * SUB, 32 * qb, s, db & 1, lane),
                                                         sf[s], dk[db], 0, 0, 0);
      }
  };
  f32x16 sa, da, sb, db_;
  bf16x8 pf[2], sf[2];
  chains(0, sa, da);
#pragma unroll
  for (int blk = 0; blk < NB; blk += 2) {
    chains(blk + 1, sb, db_);  // even block in (sa, da), odd block in (sb, db_)
    softmax(sa, da, pf, sf);
    __builtin_amdgcn_sched_barrier(0);
    grads(blk, pf, sf);
    __builtin_amdgcn_sched_barrier(0);
    if (blk + 2 < NB) chains(blk + 2, sa, da);
    softmax(sb, db_, pf, sf);
    __builtin_amdgcn_sched_barrier(0);
    grads(blk + 1, pf, sf);
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int D, int QT_, bool PIPE = false>
__global__ __launch_bounds__(256, D == 64 ? 2 : 1) void attn_bwd_dkdv_k(BwdP p) {
  using C = Cfg<D>;
  using G = DkdvCfg<D, QT_>;
  constexpr int QT = G::QT, TLQ = G::TLQ, NBUF = G::NBUF;
  constexpr int BUF = 2 * QT * C::NSUB * SUB + 2 * TLQ * 4;  // Q [QT] | dO [QT] | lse2 | delta
  constexpr int LSEW = TLQ / 64;                              // waves moving one 256-B lse2 row each
  // ONE __shared__ object (the reduction slot sits past the ring): with a second one hipcc tags
  // the LDS-DMA with an alias scope and drains the ring (vmcnt(0)) before the first ds_read of
  // every tile (cdna_hip_programming.md §5 item 4(a))
  __shared__ __attribute__((aligned(16))) char smem[NBUF * BUF + 16];
  int& red_hi = *(int*)(smem + NBUF * BUF);
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int h = lane >> 5, ql = lane & 31;
  const BlockIds bid = xcd_block_ids();
  const long b = bid.z;
  const int head = bid.y;
  const long k0 = (long)bid.x * TB;
  const long kw0 = k0 + 32 * w;
  const MaskP& m = p.m;

  const bf16* Q = p.q + b * p.sqb + head * D;
  const bf16* K = p.k + b * p.skb + head * D;
  const bf16* V = p.v + b * p.svb + head * D;
  const bf16* dO = p.dout + b * p.sob + head * D;
  const float* LSE = p.lse + (b * p.H + head) * p.Lq;
  const float* DLT = p.delta + (b * p.H + head) * p.Lq;

  // ---- query range that can see this key block
  const long klast = (k0 + TB < p.Lkv ? k0 + TB : p.Lkv) - 1;
  const int fk_lo = frame_of(m, k0), fk_hi = frame_of(m, klast);
  int fq_end;
  if (m.q_hi) {
    if (threadIdx.x == 0) red_hi = -1;
    __syncthreads();
    int mx = -1;
    for (int f = fk_lo + threadIdx.x; f <= fk_hi; f += 256) mx = max(mx, m.q_hi[b * m.fstride + f]);
    atomicMax(&red_hi, mx);
    __syncthreads();
    fq_end = red_hi;
  } else {
    fq_end = m.window > 0 ? min(m.n_frames - 1, fk_hi + m.window - 1) : m.n_frames - 1;
  }
  const int fq_start = m.causal ? fk_lo : (m.window > 0 ? max(0, fk_lo - m.window + 1) : 0);
  long qbeg = ((long)fq_start * m.tpf / TL) * TL;
  long qend = ((long)fq_end + 1) * m.tpf;
  if (qend > p.Lq) qend = p.Lq;
  const int ntiles = qend > qbeg ? (int)((qend - qbeg + TLQ - 1) / TLQ) : 0;

  // ---- this wave's K and V as B operands (key on the lane): X[key][16 s + 8 h ..]
  const long my_k = kw0 + ql;
  bf16x8 kf[C::NS], vf[C::NS];
#pragma unroll
  for (int s = 0; s < C::NS; ++s) {
    kf[s] = my_k < p.Lkv ? *(const bf16x8*)(K + my_k * p.ldk + 16 * s + 8 * h) : bf16x8{};
    vf[s] = my_k < p.Lkv ? *(const bf16x8*)(V + my_k * p.ldv + 16 * s + 8 * h) : bf16x8{};
  }
  // Row constants ride in the accumulators: k' = bf16(-c k), v' = -v, and the S / dP chains start
  // from lse2 / delta, so  acc_s = lse2 - c s  (P = exp2(-acc_s), the negation a free input
  // modifier of v_exp) and  acc_p = delta - dP = -(dP - delta).  That removes the per-score FMA
  // and subtraction; dK = scale dS^T Q picks up the sign (stored with -scale).  k' rounds c k to
  // bf16 once (the forward rounded c q instead: the same 2^-9 relative level).
#pragma unroll
  for (int s = 0; s < C::NS; ++s) {
    float f[8], g[8];
    unpack8(kf[s], f);
    unpack8(vf[s], g);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      f[j] *= -p.scale_log2;
      g[j] = -g[j];
    }
    kf[s] = pack8(f);
    vf[s] = pack8(g);
  }
  const bool wave_live = kw0 < p.Lkv;
  const long wklast = (kw0 + 31 < p.Lkv ? kw0 + 31 : p.Lkv - 1);
  const int wfk0 = frame_of(m, kw0), wfk1 = frame_of(m, wklast);
  TileRange full = full_range_q(m, b, wfk0, wfk1, qbeg, p.Lq, TLQ);
  if (!wave_live || kw0 + 32 > p.Lkv) full = TileRange{1, 0};
  full.lo = __builtin_amdgcn_readfirstlane(full.lo);
  full.hi = __builtin_amdgcn_readfirstlane(full.hi);

  f32x16 dk[C::NDB], dv[C::NDB];
#pragma unroll
  for (int db = 0; db < C::NDB; ++db) dk[db] = dv[db] = f32x16{};

  // Q / dO sub-tiles + the lse2 / delta rows arrive by LDS-DMA into the ring: per 64-row sub-tile
  // every wave issues 2 x 1 KiB per column sub-tile of Q and of dO (its 16 rows); waves
  // 0 .. 2 LSEW - 1 one 256-B row of lse2 / delta each; offsets are per-lane constants.
  const GldsOff go_q = glds_offsets<SW_DUAL>(p.ldq, w, lane), go_d = glds_offsets<SW_DUAL>(p.ldo, w, lane);
  auto issue = [&](char* buf, long q0) {
#pragma unroll
    for (int sq = 0; sq < QT; ++sq) {
      const long r = q0 + 64 * sq;
      char* bq = buf + sq * C::NSUB * SUB;
      char* bd = buf + (QT + sq) * C::NSUB * SUB;
#pragma unroll
      for (int sb = 0; sb < C::NSUB; ++sb) {
        if (r + TL <= p.Lq) {
          tile_glds_fast(bq + sb * SUB, Q + r * p.ldq + 64 * sb, go_q, w);
          tile_glds_fast(bd + sb * SUB, dO + r * p.ldo + 64 * sb, go_d, w);
        } else {
          tile_glds<SW_DUAL>(bq + sb * SUB, Q + 64 * sb, p.ldq, r, p.Lq, w, lane);
          tile_glds<SW_DUAL>(bd + sb * SUB, dO + 64 * sb, p.ldo, r, p.Lq, w, lane);
        }
      }
    }
    if (w < 2 * LSEW) {
      const int part = w >> 1;  // 64-row part of the lse2 / delta vectors
      const long r = q0 + 64 * part;
      const long n = p.Lq - r;
      const int i = r + 64 <= p.Lq ? lane : (lane < n ? lane : (n > 0 ? (int)n - 1 : 0));  // ragged: clamp
      const long src = r + i < p.Lq ? r + i : p.Lq - 1;
      glds_f32(buf + 2 * QT * C::NSUB * SUB + ((w & 1) * TLQ + 64 * part) * 4, ((w & 1) ? DLT : LSE) + src);
    }
  };
  constexpr int OPS = 4 * QT * C::NSUB;  // 16-B LDS-DMA wave-instructions per tile per wave
  auto wait_oldest = [&](int younger) {  // this wave's share of the oldest issued tile landed
    if (younger <= 0)
      vmcnt<0>();
    else if (w < 2 * LSEW)
      vmcnt<OPS + 1>();
    else
      vmcnt<OPS>();
  };
#pragma unroll
  for (int i = 0; i < NBUF - 1; ++i)
    if (i < ntiles) issue(smem + i * BUF, qbeg + (long)i * TLQ);
  wait_oldest(min(NBUF - 2, ntiles - 1));
  OWLK_BARRIER();

  for (int t = 0; t < ntiles; ++t) {
    const long q0 = qbeg + (long)t * TLQ;
    if (t + NBUF - 1 < ntiles) issue(smem + ((t + NBUF - 1) % NBUF) * BUF, q0 + (long)(NBUF - 1) * TLQ);
    const char* tb = smem + (t % NBUF) * BUF;
    const float* l2 = (const float*)(tb + 2 * QT * C::NSUB * SUB);
    const float* dlt = l2 + TLQ;

    int kind = TILE_FULL;
    if (t < full.lo || t >= full.hi) {
      const long qlast = (q0 + TLQ - 1 < p.Lq ? q0 + TLQ - 1 : p.Lq - 1);
      kind = TILE_EMPTY;
      if (wave_live) kind = classify(m, b, frame_of(m, q0), frame_of(m, qlast), wfk0, wfk1);
      if (kind == TILE_FULL && (q0 + TLQ > p.Lq || kw0 + 32 > p.Lkv)) kind = TILE_PARTIAL;
    }
    kind = __builtin_amdgcn_readfirstlane(kind);

    if constexpr (PIPE) {
      if (kind == TILE_FULL) {
        dkdv_full_pipelined<C, QT>(tb, l2, dlt, kf, vf, dk, dv, lane);
        kind = TILE_EMPTY;  // done
      }
    }
    if (kind != TILE_EMPTY) {
      const bool masked = kind == TILE_PARTIAL;
#pragma unroll
      for (int sq = 0; sq < QT; ++sq) {
        const char* lq = tb + sq * C::NSUB * SUB;
        const char* ld = tb + (QT + sq) * C::NSUB * SUB;
        unsigned long long bh = 0ull;
        if (masked) bh = tile_bits(m, b, my_k, my_k < p.Lkv, q0 + 64 * sq, p.Lq, false) >> (4 * h);
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
          f32x16 st, dp;
#pragma unroll
          for (int g4 = 0; g4 < 4; ++g4) {  // rows acc_row(4 g4 + e, h) = rowb + e
            const int rowb = 64 * sq + 32 * qb + 8 * g4 + 4 * h;
            const f32x4 L = *(const f32x4*)(l2 + rowb);
            const f32x4 Dl = *(const f32x4*)(dlt + rowb);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              st[4 * g4 + e] = L[e];
              dp[4 * g4 + e] = Dl[e];
            }
          }
#pragma unroll
          for (int s = 0; s < C::NS; ++s) {
            st = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_row<SW_DUAL>(lq + (s >> 2) * SUB, 32 * qb, s & 3, lane),
                                                         kf[s], st, 0, 0, 0);
            dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_row<SW_DUAL>(ld + (s >> 2) * SUB, 32 * qb, s & 3, lane),
                                                         vf[s], dp, 0, 0, 0);
          }
#pragma unroll
          for (int r = 0; r < 16; ++r) st[r] = __builtin_amdgcn_exp2f(-st[r]);
          if (masked) {
            if (qb == 0)
              apply_bits<0>(st, bh, 0.f);
            else
              apply_bits<32>(st, bh, 0.f);
          }
#pragma unroll
          for (int r = 0; r < 16; ++r) dp[r] *= st[r];
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const bf16x8 pf = acc_frag(st, s), sf = acc_frag(dp, s);
#pragma unroll
            for (int db = 0; db < C::NDB; ++db) {
              dv[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                  frag_tr<SW_DUAL>(ld + (db >> 1) * SUB, 32 * qb, s, db & 1, lane), pf, dv[db], 0, 0, 0);
              dk[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                  frag_tr<SW_DUAL>(lq + (db >> 1) * SUB, 32 * qb, s, db & 1, lane), sf, dk[db], 0, 0, 0);
            }
          }
        }
      }
    }
    wait_oldest(min(NBUF - 2, ntiles - 2 - t));
    OWLK_BARRIER();
  }

  if (my_k < p.Lkv) {
    store_rowT<C::NDB>(p.dk + b * p.sdkb + my_k * p.lddk + head * D, dk, -p.scale, h);  // dS was accumulated negated
    store_rowT<C::NDB>(p.dv + b * p.sdvb + my_k * p.lddv + head * D, dv, 1.f, h);
  }
}

// ======================================================================== dK, dV on 16x16x32 MFMAs
// The same workgroup, ring and tile classes as attn_bwd_dkdv_k (D 64), with every product on
// v_mfma_f32_16x16x32_bf16: the chip holds a higher clock on that shape than on 32x32x16 at the same
// cycles per FLOP (MI355X_MICROARCH.md, DVFS give-back item 7).  Per wave 32 keys as two 16-key
// column tiles (lane column c = lane & 15, k-group g = lane >> 4); per 32-query block two 16-row
// tiles.  S and dP put the key on the lane column and the query on rows 4 g + r, so their
// accumulators are the B operands of dV^T += dO^T P and dK^T += Q^T dS with the k (query) order
// permuted: slot j of group g is query 4 g + j (j < 4) or 16 + 4 g + (j - 4); the A operands dO^T
// and Q^T are read in that order by two ds_read_b64_tr_b16 per fragment (rows 4 g .. 4 g + 3 and
// 16 + 4 g .. + 3 of the tile, columns 16 ds + 4 (c & 3) .. + 3).
template <int QT_>
__global__ __launch_bounds__(256, 2) void attn_bwd_dkdv16_k(BwdP p) {
  constexpr int D = 64;
  using G = DkdvCfg<D, QT_>;
  constexpr int QT = G::QT, TLQ = G::TLQ, NBUF = G::NBUF;
  constexpr int BUF = 2 * QT * SUB + 2 * TLQ * 4;  // Q [QT] | dO [QT] | lse2 | delta
  constexpr int LSEW = TLQ / 64;
  __shared__ __attribute__((aligned(16))) char smem[NBUF * BUF + 16];
  int& red_hi = *(int*)(smem + NBUF * BUF);
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = lane & 15, g = lane >> 4;
  const BlockIds bid = xcd_block_ids();
  const long b = bid.z;
  const int head = bid.y;
  const long k0 = (long)bid.x * TB;
  const long kw0 = k0 + 32 * w;
  const MaskP& m = p.m;

  const bf16* Q = p.q + b * p.sqb + head * D;
  const bf16* K = p.k + b * p.skb + head * D;
  const bf16* V = p.v + b * p.svb + head * D;
  const bf16* dO = p.dout + b * p.sob + head * D;
  const float* LSE = p.lse + (b * p.H + head) * p.Lq;
  const float* DLT = p.delta + (b * p.H + head) * p.Lq;

  const long klast = (k0 + TB < p.Lkv ? k0 + TB : p.Lkv) - 1;
  const int fk_lo = frame_of(m, k0), fk_hi = frame_of(m, klast);
  int fq_end;
  if (m.q_hi) {
    if (threadIdx.x == 0) red_hi = -1;
    __syncthreads();
    int mx = -1;
    for (int f = fk_lo + threadIdx.x; f <= fk_hi; f += 256) mx = max(mx, m.q_hi[b * m.fstride + f]);
    atomicMax(&red_hi, mx);
    __syncthreads();
    fq_end = red_hi;
  } else {
    fq_end = m.window > 0 ? min(m.n_frames - 1, fk_hi + m.window - 1) : m.n_frames - 1;
  }
  const int fq_start = m.causal ? fk_lo : (m.window > 0 ? max(0, fk_lo - m.window + 1) : 0);
  long qbeg = ((long)fq_start * m.tpf / TL) * TL;
  long qend = ((long)fq_end + 1) * m.tpf;
  if (qend > p.Lq) qend = p.Lq;
  const int ntiles = qend > qbeg ? (int)((qend - qbeg + TLQ - 1) / TLQ) : 0;

  // this lane's two keys (column c of the wave's two 16-key tiles) as B operands, k' = bf16(-c k),
  // v' = -v (row constants in the accumulators, as attn_bwd_dkdv_k)
  long my_k[2];
  bf16x8 kf[2][2], vf[2][2];  // [key tile][k step of 32 d]
#pragma unroll
  for (int t2 = 0; t2 < 2; ++t2) {
    my_k[t2] = kw0 + 16 * t2 + c;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 kv = my_k[t2] < p.Lkv ? *(const bf16x8*)(K + my_k[t2] * p.ldk + 32 * ks + 8 * g) : bf16x8{};
      bf16x8 vv = my_k[t2] < p.Lkv ? *(const bf16x8*)(V + my_k[t2] * p.ldv + 32 * ks + 8 * g) : bf16x8{};
      float f[8], h8[8];
      unpack8(kv, f);
      unpack8(vv, h8);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        f[j] *= -p.scale_log2;
        h8[j] = -h8[j];
      }
      kf[t2][ks] = pack8(f);
      vf[t2][ks] = pack8(h8);
    }
  }
  const bool wave_live = kw0 < p.Lkv;
  const long wklast = (kw0 + 31 < p.Lkv ? kw0 + 31 : p.Lkv - 1);
  const int wfk0 = frame_of(m, kw0), wfk1 = frame_of(m, wklast);
  TileRange full = full_range_q(m, b, wfk0, wfk1, qbeg, p.Lq, TLQ);
  if (!wave_live || kw0 + 32 > p.Lkv) full = TileRange{1, 0};
  full.lo = __builtin_amdgcn_readfirstlane(full.lo);
  full.hi = __builtin_amdgcn_readfirstlane(full.hi);

  f32x4 dk[4][2], dv[4][2];  // [16-column d tile][key tile]
#pragma unroll
  for (int ds = 0; ds < 4; ++ds)
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) dk[ds][t2] = dv[ds][t2] = f32x4{0.f, 0.f, 0.f, 0.f};

  const GldsOff go_q = glds_offsets<SW_DUAL>(p.ldq, w, lane), go_d = glds_offsets<SW_DUAL>(p.ldo, w, lane);
  auto issue = [&](char* buf, long q0) {
#pragma unroll
    for (int sq = 0; sq < QT; ++sq) {
      const long r = q0 + 64 * sq;
      char* bq = buf + sq * SUB;
      char* bd = buf + (QT + sq) * SUB;
      if (r + TL <= p.Lq) {
        tile_glds_fast(bq, Q + r * p.ldq, go_q, w);
        tile_glds_fast(bd, dO + r * p.ldo, go_d, w);
      } else {
        tile_glds<SW_DUAL>(bq, Q, p.ldq, r, p.Lq, w, lane);
        tile_glds<SW_DUAL>(bd, dO, p.ldo, r, p.Lq, w, lane);
      }
    }
    if (w < 2 * LSEW) {
      const int part = w >> 1;
      const long r = q0 + 64 * part;
      const long n = p.Lq - r;
      const int i = r + 64 <= p.Lq ? lane : (lane < n ? lane : (n > 0 ? (int)n - 1 : 0));
      const long src = r + i < p.Lq ? r + i : p.Lq - 1;
      glds_f32(buf + 2 * QT * SUB + ((w & 1) * TLQ + 64 * part) * 4, ((w & 1) ? DLT : LSE) + src);
    }
  };
  constexpr int OPS = 4 * QT;
  auto wait_oldest = [&](int younger) {
    if (younger <= 0)
      vmcnt<0>();
    else if (w < 2 * LSEW)
      vmcnt<OPS + 1>();
    else
      vmcnt<OPS>();
  };
#pragma unroll
  for (int i = 0; i < NBUF - 1; ++i)
    if (i < ntiles) issue(smem + i * BUF, qbeg + (long)i * TLQ);
  wait_oldest(min(NBUF - 2, ntiles - 1));
  OWLK_BARRIER();

  for (int t = 0; t < ntiles; ++t) {
    const long q0 = qbeg + (long)t * TLQ;
    if (t + NBUF - 1 < ntiles) issue(smem + ((t + NBUF - 1) % NBUF) * BUF, q0 + (long)(NBUF - 1) * TLQ);
    const char* tb = smem + (t % NBUF) * BUF;
    const float* l2 = (const float*)(tb + 2 * QT * SUB);
    const float* dlt = l2 + TLQ;

    int kind = TILE_FULL;
    if (t < full.lo || t >= full.hi) {
      const long qlast = (q0 + TLQ - 1 < p.Lq ? q0 + TLQ - 1 : p.Lq - 1);
      kind = TILE_EMPTY;
      if (wave_live) kind = classify(m, b, frame_of(m, q0), frame_of(m, qlast), wfk0, wfk1);
      if (kind == TILE_FULL && (q0 + TLQ > p.Lq || kw0 + 32 > p.Lkv)) kind = TILE_PARTIAL;
    }
    kind = __builtin_amdgcn_readfirstlane(kind);

    if (kind != TILE_EMPTY) {
      const bool masked = kind == TILE_PARTIAL;
#pragma unroll
      for (int sq = 0; sq < QT; ++sq) {
        const char* lq = tb + sq * SUB;
        const char* ld = tb + (QT + sq) * SUB;
        unsigned long long bh[2] = {0ull, 0ull};
        if (masked) {
#pragma unroll
          for (int t2 = 0; t2 < 2; ++t2)
            bh[t2] = tile_bits(m, b, my_k[t2], my_k[t2] < p.Lkv, q0 + 64 * sq, p.Lq, false) >> (4 * g);
        }
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
          f32x4 st[2][2], dp[2][2];  // [16-row query tile][key tile]
#pragma unroll
          for (int qs = 0; qs < 2; ++qs) {
            const int rowb = 64 * sq + 32 * qb + 16 * qs + 4 * g;
            const f32x4 L = *(const f32x4*)(l2 + rowb);
            const f32x4 Dl = *(const f32x4*)(dlt + rowb);
            st[qs][0] = st[qs][1] = L;
            dp[qs][0] = dp[qs][1] = Dl;
          }
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int qs = 0; qs < 2; ++qs) {
              const bf16x8 aq = frag_row16(lq, 32 * qb + 16 * qs, ks, lane);
              const bf16x8 ad = frag_row16(ld, 32 * qb + 16 * qs, ks, lane);
#pragma unroll
              for (int t2 = 0; t2 < 2; ++t2) {
                st[qs][t2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aq, kf[t2][ks], st[qs][t2], 0, 0, 0);
                dp[qs][t2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ad, vf[t2][ks], dp[qs][t2], 0, 0, 0);
              }
            }
#pragma unroll
          for (int qs = 0; qs < 2; ++qs)
#pragma unroll
            for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
              for (int r = 0; r < 4; ++r) st[qs][t2][r] = __builtin_amdgcn_exp2f(-st[qs][t2][r]);
          if (masked) {
#pragma unroll
            for (int t2 = 0; t2 < 2; ++t2) {
              if (qb == 0) {
                apply_bits4<0>(st[0][t2], bh[t2], 0.f);
                apply_bits4<16>(st[1][t2], bh[t2], 0.f);
              } else {
                apply_bits4<32>(st[0][t2], bh[t2], 0.f);
                apply_bits4<48>(st[1][t2], bh[t2], 0.f);
              }
            }
          }
          bf16x8 pf[2], sf[2];
#pragma unroll
          for (int t2 = 0; t2 < 2; ++t2) {
#pragma unroll
            for (int qs = 0; qs < 2; ++qs)
#pragma unroll
              for (int r = 0; r < 4; ++r) dp[qs][t2][r] *= st[qs][t2][r];
            pf[t2] = pack_perm(st[0][t2], st[1][t2]);
            sf[t2] = pack_perm(dp[0][t2], dp[1][t2]);
          }
#pragma unroll
          for (int ds = 0; ds < 4; ++ds) {
            const bf16x8 ado = frag_tr16(ld, 32 * qb, ds, lane);
            const bf16x8 aqt = frag_tr16(lq, 32 * qb, ds, lane);
#pragma unroll
            for (int t2 = 0; t2 < 2; ++t2) {
              dv[ds][t2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ado, pf[t2], dv[ds][t2], 0, 0, 0);
              dk[ds][t2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aqt, sf[t2], dk[ds][t2], 0, 0, 0);
            }
          }
        }
      }
    }
    wait_oldest(min(NBUF - 2, ntiles - 2 - t));
    OWLK_BARRIER();
  }

  // dK[key][d], dV[key][d]: this lane holds d = 16 ds + 4 g + r of its two keys
#pragma unroll
  for (int t2 = 0; t2 < 2; ++t2) {
    if (my_k[t2] >= p.Lkv) continue;
    bf16* pk = p.dk + b * p.sdkb + my_k[t2] * p.lddk + head * D + 4 * g;
    bf16* pv = p.dv + b * p.sdvb + my_k[t2] * p.lddv + head * D + 4 * g;
#pragma unroll
    for (int ds = 0; ds < 4; ++ds) {
      bf16x4 a4, b4;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a4[e] = (bf16)(dk[ds][t2][e] * -p.scale);  // dS was accumulated negated
        b4[e] = (bf16)dv[ds][t2][e];
      }
      *(bf16x4*)(pk + 16 * ds) = a4;
      *(bf16x4*)(pv + 16 * ds) = b4;
    }
  }
}

// ======================================================================== dQ
// Key tiles of QT x 64 rows per ring slot: QT = 2 (D 64, unwindowed masks; two-slot ring) pays the
// per-tile fixed costs once per 48 MFMAs, as in the dK/dV kernel.
#ifndef OWLK_DQ_INIT
#define OWLK_DQ_INIT 1
#endif
template <int D, int QT>
__global__ __launch_bounds__(256, D == 64 ? (OWLK_DQ_INIT ? 2 : 3) : 2) void attn_bwd_dq_k(BwdP p) {
  constexpr bool INIT = OWLK_DQ_INIT && D == 64;
  using C = Cfg<D>;
  constexpr int NBUF = QT == 2 ? 2 : C::NBUF, TLK = TL * QT;
  constexpr int BUF = 2 * QT * C::NSUB * SUB;  // K [QT] | V [QT]
  __shared__ __attribute__((aligned(16))) char smem[NBUF * BUF + 16];  // + reduction slot (one object)
  int& red_lo = *(int*)(smem + NBUF * BUF);
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int h = lane >> 5, ql = lane & 31;
  const BlockIds bid = xcd_block_ids();
  const long b = bid.z;
  const int head = bid.y;
  const int ntq = (int)((p.Lq + TB - 1) / TB);
  const long q0 = (long)(ntq - 1 - bid.x) * TB;
  const long r0 = q0 + 32 * w;
  const MaskP& m = p.m;

  const bf16* Q = p.q + b * p.sqb + head * D;
  const bf16* K = p.k + b * p.skb + head * D;
  const bf16* V = p.v + b * p.svb + head * D;
  const bf16* dO = p.dout + b * p.sob + head * D;

  const long qlast = (q0 + TB < p.Lq ? q0 + TB : p.Lq) - 1;
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
  const int hi_f = m.causal ? fq_hi : (m.window > 0 ? min(m.n_frames - 1, fq_hi + m.window - 1) : m.n_frames - 1);
  long kv_begin = ((long)lo_f * m.tpf / TL) * TL;
  long kv_end = ((long)hi_f + 1) * m.tpf;
  if (kv_end > p.Lkv) kv_end = p.Lkv;
  const int ntiles = kv_end > kv_begin ? (int)((kv_end - kv_begin + TLK - 1) / TLK) : 0;

  const long my_q = r0 + ql;
  const bool qok = my_q < p.Lq;
  bf16x8 qf[C::NS], df[C::NS];
#pragma unroll
  for (int s = 0; s < C::NS; ++s) {
    qf[s] = qok ? *(const bf16x8*)(Q + my_q * p.ldq + 16 * s + 8 * h) : bf16x8{};
    df[s] = qok ? *(const bf16x8*)(dO + my_q * p.ldo + 16 * s + 8 * h) : bf16x8{};
  }
  const float L2 = qok ? p.lse[(b * p.H + head) * p.Lq + my_q] : 0.f;  // base-2 lse (attn_fwd)
  const float Dl = qok ? p.delta[(b * p.H + head) * p.Lq + my_q] : 0.f;
  // OWLK_DQ_INIT: q' = bf16(c q) and constant accumulator-init registers -lse2 / -delta (the
  // first MFMA of each chain reads them as C), so S' arrives as the exp2 argument and dP - delta
  // needs no subtraction: 2 VALU per score instead of 4, for 32 more VGPRs (2 waves / SIMD)
  f32x16 sinit, pinit;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    sinit[r] = -L2;
    pinit[r] = -Dl;
  }
  if (INIT) {
#pragma unroll
    for (int s = 0; s < C::NS; ++s) {
      float f[8];
      unpack8(qf[s], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] *= p.scale_log2;
      qf[s] = pack8(f);
    }
  }
  const bool wave_live = r0 < p.Lq;
  const long wlast = (r0 + 31 < p.Lq ? r0 + 31 : p.Lq - 1);
  const int wfq0 = frame_of(m, r0 + m.q_offset), wfq1 = frame_of(m, wlast + m.q_offset);
  TileRange full = full_range_kv(m, b, wfq0, wfq1, kv_begin, p.Lkv, TLK);
  if (!wave_live) full = TileRange{1, 0};
  full.lo = __builtin_amdgcn_readfirstlane(full.lo);
  full.hi = __builtin_amdgcn_readfirstlane(full.hi);

  f32x16 dq[C::NDB];
#pragma unroll
  for (int db = 0; db < C::NDB; ++db) dq[db] = f32x16{};

  // K / V tiles by LDS-DMA into the ring (as in the forward)
  const GldsOff go_k = glds_offsets<SW_DUAL>(p.ldk, w, lane), go_v = glds_offsets<SW_ROW>(p.ldv, w, lane);
  auto issue = [&](char* buf, long c0) {
#pragma unroll
    for (int sk = 0; sk < QT; ++sk) {
      const long c = c0 + 64 * sk;
      char* bk = buf + sk * C::NSUB * SUB;
      char* bv = buf + (QT + sk) * C::NSUB * SUB;
#pragma unroll
      for (int sb = 0; sb < C::NSUB; ++sb) {
        if (c + TL <= p.Lkv) {
          tile_glds_fast(bk + sb * SUB, K + c * p.ldk + 64 * sb, go_k, w);
          tile_glds_fast(bv + sb * SUB, V + c * p.ldv + 64 * sb, go_v, w);
        } else {
          tile_glds<SW_DUAL>(bk + sb * SUB, K + 64 * sb, p.ldk, c, p.Lkv, w, lane);
          tile_glds<SW_ROW>(bv + sb * SUB, V + 64 * sb, p.ldv, c, p.Lkv, w, lane);
        }
      }
    }
  };
  constexpr int OPS = 4 * QT * C::NSUB;  // 16-B LDS-DMA wave-instructions per tile per wave
  auto wait_oldest = [&](int younger) {
    if (younger > 0)
      vmcnt<OPS>();
    else
      vmcnt<0>();
  };
#pragma unroll
  for (int i = 0; i < NBUF - 1; ++i)
    if (i < ntiles) issue(smem + i * BUF, kv_begin + (long)i * TLK);
  wait_oldest(min(NBUF - 2, ntiles - 1));
  OWLK_BARRIER();

  for (int t = 0; t < ntiles; ++t) {
    const long c0 = kv_begin + (long)t * TLK;
    if (t + NBUF - 1 < ntiles) issue(smem + ((t + NBUF - 1) % NBUF) * BUF, c0 + (long)(NBUF - 1) * TLK);
    const char* tb = smem + (t % NBUF) * BUF;
    int kind = TILE_FULL;
    if (t < full.lo || t >= full.hi) {
      const long clast = (c0 + TLK - 1 < p.Lkv ? c0 + TLK - 1 : p.Lkv - 1);
      kind = TILE_EMPTY;
      if (wave_live) kind = classify(m, b, wfq0, wfq1, frame_of(m, c0), frame_of(m, clast));
      if (kind == TILE_FULL && c0 + TLK > p.Lkv) kind = TILE_PARTIAL;
    }
    kind = __builtin_amdgcn_readfirstlane(kind);

    if (kind != TILE_EMPTY) {
      const bool masked = kind == TILE_PARTIAL;
#pragma unroll
      for (int sk = 0; sk < QT; ++sk) {
      const char* lk = tb + sk * C::NSUB * SUB;
      const char* lv = tb + (QT + sk) * C::NSUB * SUB;
      unsigned long long bh = 0ull;
      if (masked) bh = tile_bits(m, b, my_q, qok, c0 + 64 * sk, p.Lkv, true) >> (4 * h);
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        f32x16 st = INIT ? sinit : f32x16{}, dp = INIT ? pinit : f32x16{};
#pragma unroll
        for (int s = 0; s < C::NS; ++s) {
          st = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_row<SW_DUAL>(lk + (s >> 2) * SUB, 32 * kb, s & 3, lane),
                                                       qf[s], st, 0, 0, 0);
          dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_row<SW_ROW>(lv + (s >> 2) * SUB, 32 * kb, s & 3, lane),
                                                       df[s], dp, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r)
          st[r] = INIT ? __builtin_amdgcn_exp2f(st[r]) : __builtin_amdgcn_exp2f(fmaf(st[r], p.scale_log2, -L2));
        if (masked) {
          if (kb == 0)
            apply_bits<0>(st, bh, 0.f);
          else
            apply_bits<32>(st, bh, 0.f);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) dp[r] = INIT ? st[r] * dp[r] : st[r] * (dp[r] - Dl);
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const bf16x8 sf = acc_frag(dp, s);
#pragma unroll
          for (int db = 0; db < C::NDB; ++db)
            dq[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                frag_tr<SW_DUAL>(lk + (db >> 1) * SUB, 32 * kb, s, db & 1, lane), sf, dq[db], 0, 0, 0);
        }
      }
      }  // sk
    }
    wait_oldest(min(NBUF - 2, ntiles - 2 - t));
    OWLK_BARRIER();
  }
  if (qok) store_rowT<C::NDB>(p.dq + b * p.sdqb + my_q * p.lddq + head * D, dq, p.scale, h);
}

// ======================================================================== dQ on 16x16x32 MFMAs
// attn_bwd_dq_k (D 64, accumulator-init form) with every product on v_mfma_f32_16x16x32_bf16
// (see attn_bwd_dkdv16_k): per wave 32 queries as two 16-query column tiles (lane column c), per
// 32-key block two 16-row key tiles; S and dP take K / V rows from LDS as A and q' = bf16(c q) /
// dO from registers as B, so their accumulators (key on rows 4 g + r) are the B operands of
// dQ^T += K^T dS in the permuted key order, K^T read by two ds_read_b64_tr_b16 per fragment.
// D 128 (dit_v4_5B): two 64-column LDS sub-tiles per K / V tile, QT = 1 with a two-slot ring
// (64 KiB per workgroup, two workgroups per CU).
// NT 16-query column tiles per wave (2: 32 queries, 3: 48): with 48, every K / V fragment read from
// LDS and every tile's fixed costs feed 1.5x the MFMAs (as the forward's 64-query waves); 48 fits
// two waves per SIMD only with the 32-key blocks taken as 16-key halves (the D 128 form), 64 does not.
template <int D, int QT, int NT = 2>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq16_k(BwdP p) {
  constexpr int TBQ = 4 * 16 * NT;  // queries per workgroup
  constexpr int NSUB = D / 64, NKD = D / 32, NDS = D / 16;
  constexpr int NBUF = (QT == 2 || D == 128) ? 2 : Cfg<D>::NBUF, TLK = TL * QT;
  constexpr int BUF = 2 * QT * NSUB * SUB;  // K [QT][NSUB] | V [QT][NSUB]
  __shared__ __attribute__((aligned(16))) char smem[NBUF * BUF + 16];
  int& red_lo = *(int*)(smem + NBUF * BUF);
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = lane & 15, g = lane >> 4;
  const BlockIds bid = xcd_block_ids();
  const long b = bid.z;
  const int head = bid.y;
  const int ntq = (int)((p.Lq + TBQ - 1) / TBQ);
  const long q0 = (long)(ntq - 1 - bid.x) * TBQ;
  const long r0 = q0 + 16 * NT * w;
  const MaskP& m = p.m;

  const bf16* Q = p.q + b * p.sqb + head * D;
  const bf16* K = p.k + b * p.skb + head * D;
  const bf16* V = p.v + b * p.svb + head * D;
  const bf16* dO = p.dout + b * p.sob + head * D;

  const long qlast = (q0 + TBQ < p.Lq ? q0 + TBQ : p.Lq) - 1;
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
  const int hi_f = m.causal ? fq_hi : (m.window > 0 ? min(m.n_frames - 1, fq_hi + m.window - 1) : m.n_frames - 1);
  long kv_begin = ((long)lo_f * m.tpf / TL) * TL;
  long kv_end = ((long)hi_f + 1) * m.tpf;
  if (kv_end > p.Lkv) kv_end = p.Lkv;
  const int ntiles = kv_end > kv_begin ? (int)((kv_end - kv_begin + TLK - 1) / TLK) : 0;

  long my_q[NT];
  bool qok[NT];
  bf16x8 qf[NT][NKD], df[NT][NKD];  // [query tile][k step of 32 d]
  f32x4 sinit[NT], pinit[NT];
#pragma unroll
  for (int t2 = 0; t2 < NT; ++t2) {
    my_q[t2] = r0 + 16 * t2 + c;
    qok[t2] = my_q[t2] < p.Lq;
#pragma unroll
    for (int ks = 0; ks < NKD; ++ks) {
      bf16x8 qv = qok[t2] ? *(const bf16x8*)(Q + my_q[t2] * p.ldq + 32 * ks + 8 * g) : bf16x8{};
      df[t2][ks] = qok[t2] ? *(const bf16x8*)(dO + my_q[t2] * p.ldo + 32 * ks + 8 * g) : bf16x8{};
      float f[8];
      unpack8(qv, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] *= p.scale_log2;
      qf[t2][ks] = pack8(f);
    }
    const float L2 = qok[t2] ? p.lse[(b * p.H + head) * p.Lq + my_q[t2]] : 0.f;
    const float Dl = qok[t2] ? p.delta[(b * p.H + head) * p.Lq + my_q[t2]] : 0.f;
    sinit[t2] = f32x4{-L2, -L2, -L2, -L2};
    pinit[t2] = f32x4{-Dl, -Dl, -Dl, -Dl};
  }
  const bool wave_live = r0 < p.Lq;
  const long wlast = (r0 + 16 * NT - 1 < p.Lq ? r0 + 16 * NT - 1 : p.Lq - 1);
  const int wfq0 = frame_of(m, r0 + m.q_offset), wfq1 = frame_of(m, wlast + m.q_offset);
  TileRange full = full_range_kv(m, b, wfq0, wfq1, kv_begin, p.Lkv, TLK);
  if (!wave_live) full = TileRange{1, 0};
  full.lo = __builtin_amdgcn_readfirstlane(full.lo);
  full.hi = __builtin_amdgcn_readfirstlane(full.hi);

  f32x4 dq[NDS][NT];  // [16-row d tile][query tile]
#pragma unroll
  for (int ds = 0; ds < NDS; ++ds)
#pragma unroll
    for (int t2 = 0; t2 < NT; ++t2) dq[ds][t2] = f32x4{0.f, 0.f, 0.f, 0.f};

  const GldsOff go_k = glds_offsets<SW_DUAL>(p.ldk, w, lane), go_v = glds_offsets<SW_ROW>(p.ldv, w, lane);
  auto issue = [&](char* buf, long c0) {
#pragma unroll
    for (int sk = 0; sk < QT; ++sk)
#pragma unroll
      for (int sb = 0; sb < NSUB; ++sb) {
        const long cc = c0 + 64 * sk;
        char* bk = buf + (sk * NSUB + sb) * SUB;
        char* bv = buf + ((QT + sk) * NSUB + sb) * SUB;
        if (cc + TL <= p.Lkv) {
          tile_glds_fast(bk, K + cc * p.ldk + 64 * sb, go_k, w);
          tile_glds_fast(bv, V + cc * p.ldv + 64 * sb, go_v, w);
        } else {
          tile_glds<SW_DUAL>(bk, K + 64 * sb, p.ldk, cc, p.Lkv, w, lane);
          tile_glds<SW_ROW>(bv, V + 64 * sb, p.ldv, cc, p.Lkv, w, lane);
        }
      }
  };
  constexpr int OPS = 4 * QT * NSUB;
  auto wait_oldest = [&](int younger) {
    if (younger > 0)
      vmcnt<OPS>();
    else
      vmcnt<0>();
  };
#pragma unroll
  for (int i = 0; i < NBUF - 1; ++i)
    if (i < ntiles) issue(smem + i * BUF, kv_begin + (long)i * TLK);
  wait_oldest(min(NBUF - 2, ntiles - 1));
  OWLK_BARRIER();

  for (int t = 0; t < ntiles; ++t) {
    const long c0 = kv_begin + (long)t * TLK;
    if (t + NBUF - 1 < ntiles) issue(smem + ((t + NBUF - 1) % NBUF) * BUF, c0 + (long)(NBUF - 1) * TLK);
    const char* tb = smem + (t % NBUF) * BUF;
    int kind = TILE_FULL;
    if (t < full.lo || t >= full.hi) {
      const long clast = (c0 + TLK - 1 < p.Lkv ? c0 + TLK - 1 : p.Lkv - 1);
      kind = TILE_EMPTY;
      if (wave_live) kind = classify(m, b, wfq0, wfq1, frame_of(m, c0), frame_of(m, clast));
      if (kind == TILE_FULL && c0 + TLK > p.Lkv) kind = TILE_PARTIAL;
    }
    kind = __builtin_amdgcn_readfirstlane(kind);

    if (kind != TILE_EMPTY) {
      const bool masked = kind == TILE_PARTIAL;
#pragma unroll
      for (int sk = 0; sk < QT; ++sk) {
        const char* lk = tb + sk * NSUB * SUB;
        const char* lv = tb + (QT + sk) * NSUB * SUB;
        unsigned long long bh[NT] = {};
        if (masked) {
#pragma unroll
          for (int t2 = 0; t2 < NT; ++t2)
            bh[t2] = tile_bits(m, b, my_q[t2], qok[t2], c0 + 64 * sk, p.Lkv, true) >> (4 * g);
        }
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          if constexpr (D == 128 || NT >= 3) {
            // one 16-key row tile at a time (its S / dP chains over the four k steps, exp2, mask,
            // dS, half of the permuted B fragment): the 32-key form spills at two waves per SIMD
            bf16x8 sf[NT];
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
              f32x4 st[NT], dp[NT];
#pragma unroll
              for (int t2 = 0; t2 < NT; ++t2) {
                st[t2] = sinit[t2];
                dp[t2] = pinit[t2];
              }
#pragma unroll
              for (int kd = 0; kd < NKD; ++kd) {
                const bf16x8 ak = frag_row16<SW_DUAL>(lk + (kd >> 1) * SUB, 32 * kb + 16 * ks, kd & 1, lane);
                const bf16x8 av = frag_row16<SW_ROW>(lv + (kd >> 1) * SUB, 32 * kb + 16 * ks, kd & 1, lane);
#pragma unroll
                for (int t2 = 0; t2 < NT; ++t2) {
                  st[t2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ak, qf[t2][kd], st[t2], 0, 0, 0);
                  dp[t2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, df[t2][kd], dp[t2], 0, 0, 0);
                }
              }
#pragma unroll
              for (int t2 = 0; t2 < NT; ++t2)
#pragma unroll
                for (int r = 0; r < 4; ++r) st[t2][r] = __builtin_amdgcn_exp2f(st[t2][r]);
              if (masked) {
#pragma unroll
                for (int t2 = 0; t2 < NT; ++t2) {
                  if (kb == 0 && ks == 0) apply_bits4<0>(st[t2], bh[t2], 0.f);
                  if (kb == 0 && ks == 1) apply_bits4<16>(st[t2], bh[t2], 0.f);
                  if (kb == 1 && ks == 0) apply_bits4<32>(st[t2], bh[t2], 0.f);
                  if (kb == 1 && ks == 1) apply_bits4<48>(st[t2], bh[t2], 0.f);
                }
              }
#pragma unroll
              for (int t2 = 0; t2 < NT; ++t2)
#pragma unroll
                for (int r = 0; r < 4; ++r) sf[t2][4 * ks + r] = (bf16)(dp[t2][r] * st[t2][r]);
              __builtin_amdgcn_sched_barrier(0);  // register budget: one 16-key tile's S / dP live at a time
            }
#pragma unroll
            for (int ds = 0; ds < NDS; ++ds) {
              const bf16x8 akt = frag_tr16(lk + (ds >> 2) * SUB, 32 * kb, ds & 3, lane);
#pragma unroll
              for (int t2 = 0; t2 < NT; ++t2)
                dq[ds][t2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(akt, sf[t2], dq[ds][t2], 0, 0, 0);
            }
            continue;
          }
          f32x4 st[2][NT], dp[2][NT];  // [16-row key tile][query tile]
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int t2 = 0; t2 < NT; ++t2) {
              st[ks][t2] = sinit[t2];
              dp[ks][t2] = pinit[t2];
            }
#pragma unroll
          for (int kd = 0; kd < NKD; ++kd)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
              const bf16x8 ak = frag_row16<SW_DUAL>(lk + (kd >> 1) * SUB, 32 * kb + 16 * ks, kd & 1, lane);
              const bf16x8 av = frag_row16<SW_ROW>(lv + (kd >> 1) * SUB, 32 * kb + 16 * ks, kd & 1, lane);
#pragma unroll
              for (int t2 = 0; t2 < NT; ++t2) {
                st[ks][t2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ak, qf[t2][kd], st[ks][t2], 0, 0, 0);
                dp[ks][t2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, df[t2][kd], dp[ks][t2], 0, 0, 0);
              }
            }
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int t2 = 0; t2 < NT; ++t2)
#pragma unroll
              for (int r = 0; r < 4; ++r) st[ks][t2][r] = __builtin_amdgcn_exp2f(st[ks][t2][r]);
          if (masked) {
#pragma unroll
            for (int t2 = 0; t2 < NT; ++t2) {
              if (kb == 0) {
                apply_bits4<0>(st[0][t2], bh[t2], 0.f);
                apply_bits4<16>(st[1][t2], bh[t2], 0.f);
              } else {
                apply_bits4<32>(st[0][t2], bh[t2], 0.f);
                apply_bits4<48>(st[1][t2], bh[t2], 0.f);
              }
            }
          }
          bf16x8 sf[NT];
#pragma unroll
          for (int t2 = 0; t2 < NT; ++t2) {
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
#pragma unroll
              for (int r = 0; r < 4; ++r) dp[ks][t2][r] *= st[ks][t2][r];
            sf[t2] = pack_perm(dp[0][t2], dp[1][t2]);
          }
#pragma unroll
          for (int ds = 0; ds < NDS; ++ds) {
            const bf16x8 akt = frag_tr16(lk + (ds >> 2) * SUB, 32 * kb, ds & 3, lane);
#pragma unroll
            for (int t2 = 0; t2 < NT; ++t2)
              dq[ds][t2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(akt, sf[t2], dq[ds][t2], 0, 0, 0);
          }
        }
      }
    }
    wait_oldest(min(NBUF - 2, ntiles - 2 - t));
    OWLK_BARRIER();
  }
#pragma unroll
  for (int t2 = 0; t2 < NT; ++t2) {
    if (!qok[t2]) continue;
    bf16* pq = p.dq + b * p.sdqb + my_q[t2] * p.lddq + head * D + 4 * g;
#pragma unroll
    for (int ds = 0; ds < NDS; ++ds) {
      bf16x4 a4;
#pragma unroll
      for (int e = 0; e < 4; ++e) a4[e] = (bf16)(dq[ds][t2][e] * p.scale);
      *(bf16x4*)(pq + 16 * ds) = a4;
    }
  }
}

// 128-row swept tiles (QT 2) pay the per-tile fixed costs once per two 64-row tiles; windowed sweeps
// that are only a few tiles long lose more to their doubled mask-edge tiles (window 16 x 64 tokens:
// +60 %), so QT 2 is taken for unwindowed masks and for windows of at least OWLK_BWD_QT2_MIN tokens
// (default 4096: mmdit_v2's 256-frame layers)
static bool long_sweep(const MaskP& m) {
  static const long qt2_min = getenv("OWLK_BWD_QT2_MIN") ? atol(getenv("OWLK_BWD_QT2_MIN")) : 4096;
  return m.window <= 0 || (long)m.window * m.tpf >= qt2_min;
}

template <int D>
int launch_bwd(int phases, const BwdP& p, long B, int H, long Lq, long Lkv, hipStream_t s) {
  if (phases & 1) {
    const dim3 grid((unsigned)((Lkv + TB - 1) / TB), (unsigned)H, (unsigned)B);
    if constexpr (D == 64) {
      // the 16x16x32-MFMA variant by default (OWLK_DKDV16 = 0: 32x32x16): -7 % at the dit_v4 shape
      static const int v16 = getenv("OWLK_DKDV16") ? atoi(getenv("OWLK_DKDV16")) : 1;
      if (v16) {
        if (long_sweep(p.m))
          hipLaunchKernelGGL((attn_bwd_dkdv16_k<2>), grid, dim3(256), 0, s, p);
        else
          hipLaunchKernelGGL((attn_bwd_dkdv16_k<1>), grid, dim3(256), 0, s, p);
      } else if (p.m.window <= 0) {
        hipLaunchKernelGGL((attn_bwd_dkdv_k<D, 2>), grid, dim3(256), 0, s, p);
      } else {
        hipLaunchKernelGGL((attn_bwd_dkdv_k<D, 1>), grid, dim3(256), 0, s, p);
      }
    } else {
      // D 128 (one wave per SIMD): OWLK_DKDV128 = 0 plain, 1 pipelined FULL tiles, 2 128-row
      // query tiles (two-slot ring, 130 KiB), 3 both (default; global 134.7 -> 99.6 ms, local
      // 3.24 -> 2.70 ms at 20 heads x 98,304 tokens)
      static const int v128 = getenv("OWLK_DKDV128") ? atoi(getenv("OWLK_DKDV128")) : 3;
      const int v = p.m.window <= 0 ? v128 : (v128 & 1);
      if (v == 3)
        hipLaunchKernelGGL((attn_bwd_dkdv_k<D, 2, true>), grid, dim3(256), 0, s, p);
      else if (v == 2)
        hipLaunchKernelGGL((attn_bwd_dkdv_k<D, 2, false>), grid, dim3(256), 0, s, p);
      else if (v == 1)
        hipLaunchKernelGGL((attn_bwd_dkdv_k<D, 1, true>), grid, dim3(256), 0, s, p);
      else
        hipLaunchKernelGGL((attn_bwd_dkdv_k<D, 1>), grid, dim3(256), 0, s, p);
    }
    if (int e = owlk::check_launch("attn_bwd_dkdv")) return e;
  }
  if (phases & 2) {
    const dim3 grid((unsigned)((Lq + TB - 1) / TB), (unsigned)H, (unsigned)B);
    if constexpr (D == 64) {
      static const int v16 = getenv("OWLK_DQ16") ? atoi(getenv("OWLK_DQ16")) : 1;  // 16x16x32 variant (0: 32x32x16)
      // long sweeps: 48 queries per wave (3 x 16-query tiles, 192 per workgroup): global dQ 36.7 ->
      // 34.2 ms at the dit_v4 shape; window 16 keeps 32 (1.07 -> 1.13 ms with 48).  OWLK_DQ_NT = 2
      // forces 32 everywhere.
      static const int nt = getenv("OWLK_DQ_NT") ? atoi(getenv("OWLK_DQ_NT")) : 3;
      const dim3 grid3((unsigned)((Lq + 191) / 192), (unsigned)H, (unsigned)B);
      if (v16 && nt == 3 && long_sweep(p.m)) {
        hipLaunchKernelGGL((attn_bwd_dq16_k<64, 2, 3>), grid3, dim3(256), 0, s, p);
      } else if (v16) {
        if (long_sweep(p.m))
          hipLaunchKernelGGL((attn_bwd_dq16_k<64, 2>), grid, dim3(256), 0, s, p);
        else
          hipLaunchKernelGGL((attn_bwd_dq16_k<64, 1>), grid, dim3(256), 0, s, p);
      } else if (p.m.window <= 0) {
        hipLaunchKernelGGL((attn_bwd_dq_k<D, 2>), grid, dim3(256), 0, s, p);
      } else {
        hipLaunchKernelGGL((attn_bwd_dq_k<D, 1>), grid, dim3(256), 0, s, p);
      }
    } else {
      // D 128: the 16x16x32 form (32 queries per wave, two waves per SIMD) by default;
      // OWLK_DQ16_128 = 0 the 32x32x16 attn_bwd_dq_k
      static const int v16 = getenv("OWLK_DQ16_128") ? atoi(getenv("OWLK_DQ16_128")) : 1;
      if (v16)
        hipLaunchKernelGGL((attn_bwd_dq16_k<128, 1>), grid, dim3(256), 0, s, p);
      else
        hipLaunchKernelGGL((attn_bwd_dq_k<D, 1>), grid, dim3(256), 0, s, p);
    }
    if (int e = owlk::check_launch("attn_bwd_dq")) return e;
  }
  return 0;
}

}  // namespace

static int attn_bwd_impl(int phases, const void* q, long ldq, long sqb, const void* k, long ldk, long skb,
                         const void* v, long ldv, long svb, const void* dout, long ldo, long sob, const float* lse,
                         const float* delta, void* dq, long lddq, long sdqb, void* dk, long lddk, long sdkb, void* dv,
                         long lddv, long sdvb, long B, int H, long Lq, long Lkv, int head_dim, float scale, long tpf,
                         int window, int causal, const int* kv_lo, const int* q_hi, const int* run_start,
                         const int* doc, long fstride, void* stream) {
  OWLK_REQUIRE(head_dim == 64 || head_dim == 128, "attn_bwd: head_dim %d not built (64, 128)", head_dim);
  OWLK_REQUIRE(tpf > 0 && Lq > 0 && Lkv > 0 && B > 0 && H > 0 && Lq == Lkv, "attn_bwd: training shapes only");
  OWLK_REQUIRE(!doc || run_start, "attn_bwd: doc mask needs run_start");
  OWLK_REQUIRE(((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)dout | (uintptr_t)dq | (uintptr_t)dk |
                (uintptr_t)dv) % 16 == 0,
               "attn_bwd: operands must be 16-byte aligned");
  BwdP p;
  p.q = (const bf16*)q; p.k = (const bf16*)k; p.v = (const bf16*)v; p.dout = (const bf16*)dout;
  p.lse = lse; p.delta = delta;
  p.dq = (bf16*)dq; p.dk = (bf16*)dk; p.dv = (bf16*)dv;
  p.ldq = ldq; p.ldk = ldk; p.ldv = ldv; p.ldo = ldo; p.lddq = lddq; p.lddk = lddk; p.lddv = lddv;
  p.sqb = sqb; p.skb = skb; p.svb = svb; p.sob = sob; p.sdqb = sdqb; p.sdkb = sdkb; p.sdvb = sdvb;
  p.Lq = Lq; p.Lkv = Lkv; p.H = H;
  p.scale = scale;
  p.scale_log2 = scale * LOG2E;
  p.m = owlk_make_mask(tpf, window, causal, 0, Lkv, kv_lo, q_hi, run_start, doc, fstride);
  hipStream_t s = (hipStream_t)stream;
  return head_dim == 64 ? launch_bwd<64>(phases, p, B, H, Lq, Lkv, s) : launch_bwd<128>(phases, p, B, H, Lq, Lkv, s);
}

#define OWLK_BWD_ARGS                                                                                            \
  const void *q, long ldq, long sqb, const void *k, long ldk, long skb, const void *v, long ldv, long svb,      \
      const void *dout, long ldo, long sob, const float *lse, const float *delta, void *dq, long lddq, long sdqb, \
      void *dk, long lddk, long sdkb, void *dv, long lddv, long sdvb, long B, int H, long Lq, long Lkv,          \
      int head_dim, float scale, long tpf, int window, int causal, const int *kv_lo, const int *q_hi,            \
      const int *run_start, const int *doc, long fstride, void *stream
#define OWLK_BWD_FWD                                                                                          \
  q, ldq, sqb, k, ldk, skb, v, ldv, svb, dout, ldo, sob, lse, delta, dq, lddq, sdqb, dk, lddk, sdkb, dv, lddv, \
      sdvb, B, H, Lq, Lkv, head_dim, scale, tpf, window, causal, kv_lo, q_hi, run_start, doc, fstride, stream

extern "C" int owlk_attn_bwd(OWLK_BWD_ARGS) { return attn_bwd_impl(3, OWLK_BWD_FWD); }
extern "C" int owlk_attn_bwd_dkdv(OWLK_BWD_ARGS) { return attn_bwd_impl(1, OWLK_BWD_FWD); }
extern "C" int owlk_attn_bwd_dq(OWLK_BWD_ARGS) { return attn_bwd_impl(2, OWLK_BWD_FWD); }
