// Frame-masked flash attention backward in ONE pass (gfx950, head_dim 64, causal / windowed frame masks
// without documents).
//
// Reference: the single compiled flex_attention backward behind attn.py:13-16, 106-109 (torch's
// flex template forms dQ, dK and dV in one kernel).  Same math as attn_bwd.hip:
//   dV = P^T dO,  dS = P o (dP - delta),  dK = scale dS^T Q,  dQ = scale dS K,
// but every (key block, query tile) pair forms S and dP ONCE: 10 D FLOP executed per allowed pair
// instead of the 14 D of the two-kernel form (its dQ kernel recomputes S and dP).
//
// Work item = 256 keys of one (batch, head) chain, held by an 8-wave workgroup (wave w: keys
// 32 w .. 32 w + 31, as attn_bwd_dkdv16_k: S / dP with the key on the lane column, dK^T / dV^T
// in registers).  The workgroup sweeps the 64-row query tiles its keys see in DECREASING order.
// Per tile, dS goes to LDS as a [key][query] bf16 image; one tile later the 8 waves form
// dQ^T[64 d x 64 q] = K^T dS^T over the item's 256 keys (K image in LDS, both operands read by
// ds_read_b64_tr_b16) and add it to the tile's fp32 accumulator: an ORDERED hand-off -- key block
// j adds to query tile i only after block j - 1 has (flag[i] >= j), so every tile receives its
// partial sums in key-block order (bitwise reproducible, no float atomics).  The last contributor
// of a tile (j == jhi(i)) writes bf16 dQ instead of the fp32 sum.
//
// Hand-off (cdna_hip_programming.md Guideline 16, R1 with a flag): every wave stores its part of
// the accumulator write-through (sc1), drains it (s_waitcnt vmcnt(0)) before the workgroup barrier,
// then ONE lane stores the flag (sc1).  Each consumer wave polls the flag with sc1 loads and reads
// the accumulator with sc1 loads only after its own poll matched.  Variant bit 0 ("local") instead
// keeps a chain's items on one XCD (per-XCD queues chosen by HW_REG_XCC_ID, no stealing) and stores
// the accumulator with plain stores, so the sums stay in that XCD's L2; the A/B between the two is
// the reason the variant exists.
//
// Pipelining: the accumulator of tile t + 1 is loaded in step t (issued mid-step, consumed as the
// MFMA chain's initial value after the tile's dK/dV work), its new value is stored at the top of
// step t - 1 and drained by that step's barrier; the flag goes out after it.  A successor block
// therefore runs two tiles behind its predecessor.
//
// Forward progress: items are dequeued in increasing key-block order per chain from per-XCD atomic
// queues; an item waits only on its chain predecessor, which a running workgroup dequeued earlier.
// A workgroup claims its next item during its current item's epilogue: the held claim is later in
// its queue than the holder's running item, so the running item earliest in its queue always has a
// predecessor that is done or running.
// Spins are bounded by the real-time clock (error word in the workspace header).

#include <algorithm>
#include <atomic>

#include "attn_fused_common.hpp"


// timing-only experiment builds (tools/build_variant.sh -DOWLK_FUSED_EXP=n; results are WRONG):
// bit 0: no hand-off (no flag polls, no sum loads); bit 1: no dQ products / stores either;
// bit 2: no dS image writes
#ifndef OWLK_FUSED_EXP
#define OWLK_FUSED_EXP 0
#endif
// timing-only statistics build: workspace int32 words 10 / 11 count the hand-offs that found the
// flag down at mid-step (blocking poll at the next step's top) / all hand-offs, per wave
#ifndef OWLK_FUSED_STATS
#define OWLK_FUSED_STATS 0
#endif
// timing-only profile build: per-phase shader-clock cycles of the sweep, summed over waves, as uint64
// at workspace bytes 128.. : [dQ waves | other waves] x {dQ part, main, end-of-step vmcnt, barrier}
#ifndef OWLK_FUSED_PROF
#define OWLK_FUSED_PROF 0
#endif
// software-pipeline depth of the 32x32 dQ products (k-steps of reads in flight ahead of the MFMA)
// values formed from an opaque lane id at each use instead of kept across the sweep (bits: 1 the
// ring's DMA offsets, 2 the dS image addresses, 4 the operand read addresses, 8 the mask rows and
// the epilogue's keys); 0 = all kept (hipcc spills some of them)
#ifndef OWLK_FUSED_REMAT
#define OWLK_FUSED_REMAT 0
#endif
#ifndef OWLK_FUSED_KV_STAGE  // 1: dK / dV stored as whole rows through LDS
#define OWLK_FUSED_KV_STAGE 1
#endif
#ifndef OWLK_FUSED_DEQ_PF  // 1: an item's successor is claimed during its epilogue
#define OWLK_FUSED_DEQ_PF 1
#endif
#ifndef OWLK_FUSED_DQ_PF
#define OWLK_FUSED_DQ_PF 3
#endif
#ifndef OWLK_FUSED_DMA47  // 1: the ring's LDS-DMA is issued by waves 4-7 only (no dQ work), 0: by all 8
#define OWLK_FUSED_DMA47 1
#endif

namespace {

using namespace owlk_fused;

// packed documents: each query tile's first contributing key block (tile_jlo of the runs form)
__global__ void fused_jlo_k(FusedP p, int B) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x, b = blockIdx.y;
  if (b >= B || i >= p.jlo_stride) return;
  int v = 0;
  if (i < p.ntiles) v = (int)((long)p.kv_lo[b * p.fstride + frame(p, i * FQT)] * p.tpf / FKB);
  p.jlo[(long)b * p.jlo_stride + i] = v;
}

template <bool LOCAL, bool COUNTING, bool RUNS = false>
__global__ __launch_bounds__(512, 2) void attn_bwd_fused_k(FusedP p) {
  // ONE __shared__ object (see attn_bwd.hip: a second one makes hipcc drain the DMA ring)
  __shared__ __attribute__((aligned(16))) char smem[SMEM_BYTES];
  int* sh_item = (int*)(smem + MISC_OFF);
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = lane & 15, g = lane >> 4;
  constexpr bool local = LOCAL, counting = COUNTING;
  const unsigned xcc = xcc_id();
  const int L = p.L;
  char* kimg = smem + KIMG_OFF;
  // dQ^T of a tile: waves 0-3, one 32 x 32 tile each (d tile dt32, query tile qt32)
  const bool dq_wave = DQ16 || w < 4;
  const int dt32 = w & 1, qt32 = (w >> 1) & 1;
  // DQ16: this wave's quarter of dQ^T: d tile dt (16), query tiles qt0, qt0 + 1 (16 each)
  const int dt = w & 3, qt0 = 2 * (w >> 2);
  const unsigned offk = tr16_lane_off(dt, lane), offs0 = ds_tr16_off(qt0, lane), offs1 = ds_tr16_off(qt0 + 1, lane);
  const unsigned acc_lane = (unsigned)(w * NACC * 1024 + lane * 16);  // + e * 1024, + tile * 16 KiB
  int ok32a, ok32b, os32a, os32b;
  tr32_lane_off(dt32, lane, ok32a, ok32b);
  ds_tr32_off(qt32, lane, os32a, os32b);
  // per-lane LDS byte offsets in a ring slot (row0 a multiple of 16 in the immediate): frag_row16
  // of k-step 0 / 1, frag_tr16 of column group ds, the lse2 / delta rows of lane group g
  const unsigned ro0 = ring_row16_off(0, lane), ro1 = ring_row16_off(1, lane);
  // dS^T image pieces (8 B): row r = 32 w + 16 t2 + c, 8-B unit u = 8 qb + 4 e + g, at
  // r * 128 + 8 (u ^ swz_ds8(r)) = dsl + 2048 t2 + ((64 qb + 32 e) ^ dsx), as swz_ds8(r) = swz_ds8(c)
  // (it repeats every 16 rows) and 64 qb + 32 e has only bits 5-6, 8 g bits 3-4
  const unsigned dsl = (unsigned)((32 * w + c) * 128);
  const unsigned dsx = (unsigned)(8 * (g ^ swz_ds8(c)));
  const unsigned tro0 = ring_tr16_off(0, lane), tro1 = ring_tr16_off(1, lane), tro2 = ring_tr16_off(2, lane),
                 tro3 = ring_tr16_off(3, lane);
  if (blockIdx.x == 0 && threadIdx.x == 0) p.hdr[9] = FKB;  // for readers of the workspace (tests)

  // per-lane LDS-DMA source offsets of a 64-row tile (wave w: rows 8 w .. 8 w + 7, one 1-KiB
  // wave-instruction, swizzled source chunk)
  const int drow = 8 * w + (lane >> 3);
  const int dch = (lane & 7) ^ swz_ring(drow);
  // (formed from an opaque lane id at each use: kept live across the sweep they were spilled, and
  // each reload's vmcnt(0) drained the dQ stores before the ring's DMA)
  // OWLK_FUSED_DMA47: waves 4-7 move rows 16 (w - 4) + 8 h + (lane >> 3) instead (h = 0, 1)
  auto row_off = [&](int ld, int h = 0) {
    const int ln = (int)opaque<1>((unsigned)lane);
    const int r = OWLK_FUSED_DMA47 ? 16 * (w - 4) + 8 * h + (ln >> 3) : 8 * w + (ln >> 3);
    return (unsigned)((r * ld + (((ln & 7) ^ swz_ring(r)) * 8)) * 2);
  };

  // OWLK_FUSED_PROF: per-step phases {dq, main, vmwait, barrier} and per-item {dequeue, prologue,
  // epilogue} (s_memtime cycles)
  unsigned long long prof[8] = {0ull, 0ull, 0ull, 0ull, 0ull, 0ull, 0ull, 0ull};
  // the item of the n-th claim on queue x: the queue's chains in groups of p.group (j-major inside
  // a group): fewer chains at a time give each chain more workgroups, so a key block's successor
  // follows closer behind and the chain's sums and Q / dO tiles are re-read fewer times (each
  // generation of concurrent blocks re-sweeps the chain)
  auto item_of = [&](int x, int n, int& chain, int& jj) {
    const int cx = p.nchain > x ? (p.nchain - x + 7) / 8 : 0;
    if (n < 0 || (long)n >= (long)cx * p.nkb) return false;  // the host keeps cx * nkb < 2^31
    const int grp = p.group < cx ? p.group : cx;               // group 1 << 20 = "all": no overflow
    const int gfull = grp * p.nkb, gi = n / gfull, m = n - gi * gfull;
    const int gsz = cx - gi * grp < grp ? cx - gi * grp : grp;
    chain = x + 8 * (gi * grp + m % gsz);
    jj = m / gsz;
    return true;
  };
  // a claim on the queues of XCDs xcc + d0, xcc + d0 + 1, ... (only this XCD's when local)
  auto claim = [&](int d0, int& chain, int& jj) {
    chain = -1;
    jj = 0;
    for (int d = d0; d < (local ? 1 : 8) && chain < 0; ++d) {
      const int x = (int)((xcc + d) & 7);
      const int cx = p.nchain > x ? (p.nchain - x + 7) / 8 : 0;
      if (cx == 0) continue;
      if ((long)__hip_atomic_load(p.hdr + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (long)cx * p.nkb) continue;
      item_of(x, __hip_atomic_fetch_add(p.hdr + x, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), chain, jj);
    }
  };
  if (OWLK_FUSED_DEQ_PF && threadIdx.x == 0) claim(0, sh_item[0], sh_item[1]);
  for (;;) {
    const unsigned long long ca = OWLK_FUSED_PROF ? __builtin_amdgcn_s_memtime() : 0ull;
    // ---- dequeue: the next item of this XCD's queue (others' when it is empty, unless local);
    // OWLK_FUSED_DEQ_PF: claimed during the previous item's epilogue
    if (!OWLK_FUSED_DEQ_PF && threadIdx.x == 0) {
      int chain, jj;
      claim(0, chain, jj);
      sh_item[0] = chain;
      sh_item[1] = jj;
    }
    __syncthreads();
    const int chain = __builtin_amdgcn_readfirstlane(sh_item[0]);
    const int j = __builtin_amdgcn_readfirstlane(sh_item[1]);
    const unsigned long long cb = OWLK_FUSED_PROF ? __builtin_amdgcn_s_memtime() : 0ull;
    if (chain < 0) {
      if (OWLK_FUSED_PROF && lane == 0) {
        unsigned long long* pp = (unsigned long long*)((char*)p.hdr + 128) + (w < 4 ? 0 : 8);
#pragma unroll
        for (int e = 0; e < 7; ++e) __hip_atomic_fetch_add(pp + e, prof[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return;
    }

    const int b = chain / p.H;
    const int head = chain % p.H;
    const bf16* Q = p.q + b * p.sqb + head * 64;
    const bf16* K = p.k + b * p.skb + head * 64;
    const bf16* V = p.v + b * p.svb + head * 64;
    const bf16* dO = p.dout + b * p.sob + head * 64;
    const float* LSE = p.lse + (long)chain * L;
    const float* DLT = p.delta + (long)chain * L;
    int* flg = p.flags + (long)chain * p.ntiles * FLAG_STRIDE;
    const __amdgpu_buffer_rsrc_t ars = __builtin_amdgcn_make_buffer_rsrc(
        p.acc + (long)chain * p.ntiles * ACC_TILE_BYTES, (short)0, p.ntiles * ACC_TILE_BYTES, 0x00020000);
    const int k0 = j * FKB, kw0 = k0 + 32 * w;
    const int* qh = RUNS ? p.q_hi + b * p.fstride : nullptr;  // this chain's sample
    const int* jlo_row = RUNS ? p.jlo + (long)b * p.jlo_stride : nullptr;
    int t_hi = sweep_hi(p, j);
    if (RUNS) {
      const int k1 = k0 + FKB - 1 < L ? k0 + FKB - 1 : L - 1;
      t_hi = (int)((q_hi_end_runs(p, qh, frame(p, k1)) - 1) / FQT);
    }
    const int t_lo = sweep_lo(p, j);
    // the tile's first contributor: packed documents read it from the tile's ring slot (landed with
    // the tile; a slot is re-filled only after its tile's last use)
    auto jlo_at = [&](int i) {
      if constexpr (RUNS) return __builtin_amdgcn_readfirstlane(*(const int*)(smem + JLO_OFF + (i & 1) * 256));
      else return tile_jlo(p, i);
    };

    // ---- K image of the item (unscaled K: the dQ^T A operand), 4 wave-instructions per wave
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 32 * w + 8 * i + (lane >> 3);
      const int ch = (lane & 7) ^ swz_dual(row);
      int gr = k0 + row;
      gr = gr < L ? gr : L - 1;
      dma16(lds_addr(kimg + (32 * w + 8 * i) * 128), K + (long)k0 * p.ldk, (unsigned)(((gr - k0) * p.ldk + ch * 8) * 2));
    }
    // ring: Q and dO 64-row tiles + the lse2 / delta rows (waves 0 / 1)
    auto issue = [&](int t) {
      char* buf = smem + (t & 1) * RING_SLOT;
      const int q0 = t * FQT;
      if (OWLK_FUSED_DMA47) {
        // the waves without dQ work issue the whole tile (the dQ waves are each step's critical path)
        if (w < 4) return;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          char* dst = buf + (16 * (w - 4) + 8 * h) * 128;
          if (q0 + FQT <= L) {
            dma16(lds_addr(dst), Q + (long)q0 * p.ldq, row_off(p.ldq, h));
            dma16(lds_addr(dst + TILE_BYTES), dO + (long)q0 * p.ldo, row_off(p.ldo, h));
          } else {
            const int r = 16 * (w - 4) + 8 * h + (lane >> 3), ch = (lane & 7) ^ swz_ring(r);
            int gr = q0 + r;
            gr = gr < L ? gr : L - 1;
            dma16(lds_addr(dst), Q + (long)q0 * p.ldq, (unsigned)(((gr - q0) * p.ldq + ch * 8) * 2));
            dma16(lds_addr(dst + TILE_BYTES), dO + (long)q0 * p.ldo, (unsigned)(((gr - q0) * p.ldo + ch * 8) * 2));
          }
        }
        if (w < 6) {
          const int src = q0 + lane < L ? lane : L - 1 - q0;
          dma4(lds_addr(buf + 2 * TILE_BYTES + (w - 4) * FQT * 4), (w == 5 ? DLT : LSE) + q0, (unsigned)(src * 4));
        }
        if (RUNS && w == 6) dma4(lds_addr(smem + JLO_OFF + (t & 1) * 256), jlo_row + t, (unsigned)(lane * 4));
        return;
      }
      if (q0 + FQT <= L) {
        dma16(lds_addr(buf + 8 * w * 128), Q + (long)q0 * p.ldq, row_off(p.ldq));
        dma16(lds_addr(buf + TILE_BYTES + 8 * w * 128), dO + (long)q0 * p.ldo, row_off(p.ldo));
      } else {
        int gr = q0 + drow;
        gr = gr < L ? gr : L - 1;
        dma16(lds_addr(buf + 8 * w * 128), Q + (long)q0 * p.ldq, (unsigned)(((gr - q0) * p.ldq + dch * 8) * 2));
        dma16(lds_addr(buf + TILE_BYTES + 8 * w * 128), dO + (long)q0 * p.ldo, (unsigned)(((gr - q0) * p.ldo + dch * 8) * 2));
      }
      if (w < 2) {
        const int src = q0 + lane < L ? lane : L - 1 - q0;
        dma4(lds_addr(buf + 2 * TILE_BYTES + w * FQT * 4), (w ? DLT : LSE) + q0, (unsigned)(src * 4));
      }
      if (RUNS && w == 2) dma4(lds_addr(smem + JLO_OFF + (t & 1) * 256), jlo_row + t, (unsigned)(lane * 4));
    };

    // this lane's two keys (column c of the wave's two 16-key tiles): k' = bf16(-c k), v' = -v
    // (row constants in the accumulators, as attn_bwd_dkdv16_k)
    int my_k[2];
    bf16x8 kf[2][2], vf[2][2];
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) {
      my_k[t2] = kw0 + 16 * t2 + c;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 kv = my_k[t2] < L ? *(const bf16x8*)(K + (long)my_k[t2] * p.ldk + 32 * ks + 8 * g) : bf16x8{};
        bf16x8 vv = my_k[t2] < L ? *(const bf16x8*)(V + (long)my_k[t2] * p.ldv + 32 * ks + 8 * g) : bf16x8{};
        float f[8], h8[8];
        unpack8(kv, f);
        unpack8(vv, h8);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          f[e] *= -p.scale_log2;
          h8[e] = -h8[e];
        }
        kf[t2][ks] = pack8(f);
        vf[t2][ks] = pack8(h8);
      }
    }
    // tile classes of this wave's 32 keys (frames wfk0 .. wfk1): FULL on the whole tiles every one
    // of its keys sees entirely (rows from q_lo_frame(wfk1) tpf to q_hi_end(wfk0)), EMPTY on tiles
    // none of them sees, else PARTIAL
    const bool wave_live = kw0 < L;
    const int wfk0 = frame(p, kw0), wfk1 = frame(p, kw0 + 31 < L ? kw0 + 31 : L - 1);
    const int seen_lo = __builtin_amdgcn_readfirstlane((int)((long)q_lo_frame(p, wfk0) * p.tpf)),
              seen_hi = __builtin_amdgcn_readfirstlane((int)(RUNS ? q_hi_end_runs(p, qh, wfk1) : q_hi_end(p, wfk1)));
    int full_lo = (int)(((long)q_lo_frame(p, wfk1) * p.tpf + FQT - 1) / FQT);
    int full_hi = (int)((RUNS ? q_hi_end_runs(p, qh, wfk0) : q_hi_end(p, wfk0)) / FQT);  // exclusive: whole tiles only
    // packed documents: this lane's keys' row ends, for the PARTIAL tiles' masks
    int khi[2] = {0, 0};
    if (RUNS) {
#pragma unroll
      for (int t2 = 0; t2 < 2; ++t2) {
        const int k = kw0 + 16 * t2 + c;
        khi[t2] = k < L ? (int)q_hi_end_runs(p, qh, frame(p, k)) : 0;
      }
    }
    if (full_hi > L / FQT) full_hi = L / FQT;
    if (!wave_live || kw0 + 32 > L) full_lo = full_hi = 0;
    full_lo = __builtin_amdgcn_readfirstlane(full_lo);
    full_hi = __builtin_amdgcn_readfirstlane(full_hi);

    f32x4 dk[4][2], dv[4][2];
#pragma unroll
    for (int ds = 0; ds < 4; ++ds)
#pragma unroll
      for (int t2 = 0; t2 < 2; ++t2) dk[ds][t2] = dv[ds][t2] = f32x4{0.f, 0.f, 0.f, 0.f};

    // a finished dQ^T tile of this wave: bf16 dQ by the tile's last contributor (lane: query
    // 32 qt32 + (lane & 31); register 4 rr + e: d 32 dt32 + 8 rr + 4 h + e), else the fp32 sum
    // (sc1 write-through; plain in the local variant)
    f32x16 qacc;
    f32x4 qa[2];  // DQ16
    auto store_dq = [&](int i) {
      const bool last = j >= tile_jhi(p, i);
      if constexpr (DQ16) {
        if (last && !counting) {
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int qrow = i * FQT + 16 * (qt0 + e) + c;
            if (qrow < L) {
              bf16x4 o4;
#pragma unroll
              for (int r = 0; r < 4; ++r) o4[r] = (bf16)(qa[e][r] * -p.scale);  // dS accumulated negated
              *(bf16x4*)(p.dq + b * p.sdqb + (long)qrow * p.lddq + head * 64 + 16 * dt + 4 * g) = o4;
            }
          }
        } else {
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int off = (int)(i * ACC_TILE_BYTES + acc_lane + e * 1024);
            if constexpr (local)
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, qa[e]), ars, off, 0, 0);
            else
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, qa[e]), ars, off, 0, 16);
          }
        }
        return;
      }
      if (last && !counting) {
        const int qrow = i * FQT + 32 * qt32 + (lane & 31);
        if (qrow < L) {
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            bf16x4 o4;
#pragma unroll
            for (int r = 0; r < 4; ++r) o4[r] = (bf16)(qacc[4 * rr + r] * -p.scale);  // dS accumulated negated
            *(bf16x4*)(p.dq + b * p.sdqb + (long)qrow * p.lddq + head * 64 + 32 * dt32 + 8 * rr + 4 * (lane >> 5)) = o4;
          }
        }
      } else {
#pragma unroll
        for (int e = 0; e < NACC; ++e) {
          const int off = (int)(i * ACC_TILE_BYTES + acc_lane + e * 1024);
          const f32x4 v4 = {qacc[4 * e], qacc[4 * e + 1], qacc[4 * e + 2], qacc[4 * e + 3]};
          if constexpr (local)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v4), ars, off, 0, 0);
          else
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v4), ars, off, 0, 16);
        }
      }
    };
    const char* accp = p.acc + (long)chain * p.ntiles * ACC_TILE_BYTES;  // + acc_lane per lane
    char* accl = smem + ACC_OFF + w * NACC * 1024;  // this wave's landing zone (lane-linear, as acc_lane)
    char* flagl = smem + FLAGL_OFF + w * 256;
    auto load_acc = [&](int i) {  // -> accl, read back after vm_wait
#pragma unroll
      for (int e = 0; e < NACC; ++e) dma16_sc1(lds_addr(accl + e * 1024), accp + (long)i * ACC_TILE_BYTES + e * 1024, acc_lane);
    };

    // dQ^T[32 d x 32 q] of tile i += K^T[32 d x 16 keys] dS^T[16 keys x 32 q] over the item's keys,
    // from the K image and the tile's dS image (written in the tile's own step); both fragments in
    // frag_tr's permuted row order (the same for A and B), software-pipelined OWLK_FUSED_DQ_PF
    // k-steps deep
    auto dq_mfma = [&](int i) {
      if constexpr (counting) {
#pragma unroll
        for (int e = 0; e < 16; ++e) qacc[e] += 1.f;
#pragma unroll
        for (int e = 0; e < 2; ++e)
#pragma unroll
          for (int r = 0; r < 4; ++r) qa[e][r] += 1.f;
        return;
      }
      if constexpr (DQ16) {
        // dQ^T[16 d x 16 q] (two query tiles) += K^T[16 d x 32 keys] dS^T[32 keys x 16 q]: frag_tr16 at
        // row0 = 32 kk (immediate kk * 4 KiB, + 2 KiB for the second 4-row group), pipelined as below
        constexpr int NK = FKB / 32, PF = OWLK_FUSED_DQ_PF;
        const unsigned sb0 = lds_addr(smem + DS_OFF + (i & 1) * DS_BYTES);
        const unsigned ka = lds_addr(kimg) + offk, s0 = sb0 + offs0, s1 = sb0 + offs1;
        s16x4 r[PF + 1][6];
        auto rd = [&](auto kc) {
          constexpr int k2 = decltype(kc)::value, sl = k2 % (PF + 1);
          r[sl][0] = tr_rd<4096 * k2>(ka);
          r[sl][1] = tr_rd<4096 * k2 + 2048>(ka);
          r[sl][2] = tr_rd<4096 * k2>(s0);
          r[sl][3] = tr_rd<4096 * k2 + 2048>(s0);
          r[sl][4] = tr_rd<4096 * k2>(s1);
          r[sl][5] = tr_rd<4096 * k2 + 2048>(s1);
        };
        static_for<PF>(rd);
        static_for<NK>([&](auto kc) {
          constexpr int k2 = decltype(kc)::value, sl = k2 % (PF + 1);
          if constexpr (k2 + PF < NK) rd(std::integral_constant<int, k2 + PF>{});
          constexpr int younger = 6 * (PF < NK - 1 - k2 ? PF : NK - 1 - k2);
          lgkm6<younger>(r[sl][0], r[sl][1], r[sl][2], r[sl][3], r[sl][4], r[sl][5]);
          const bf16x8 ak = join_tr(r[sl][0], r[sl][1]);
          qa[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ak, join_tr(r[sl][2], r[sl][3]), qa[0], 0, 0, 0);
          qa[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ak, join_tr(r[sl][4], r[sl][5]), qa[1], 0, 0, 0);
        });
        return;
      }
      constexpr int NK = FKB / 16, PF = OWLK_FUSED_DQ_PF;
      const unsigned kb0 = lds_addr(kimg), sb0 = lds_addr(smem + DS_OFF + (i & 1) * DS_BYTES);
      const unsigned ka = kb0 + ok32a, kb = kb0 + ok32b, sa = sb0 + os32a, sb = sb0 + os32b;
      s16x4 r[PF + 1][4];
      auto rd = [&](auto kc) {
        constexpr int k2 = decltype(kc)::value, sl = k2 % (PF + 1);
        r[sl][0] = tr_rd<2048 * k2>(ka);
        r[sl][1] = tr_rd<2048 * k2>(kb);
        r[sl][2] = tr_rd<2048 * k2>(sa);
        r[sl][3] = tr_rd<2048 * k2>(sb);
      };
      static_for<PF>(rd);
      static_for<NK>([&](auto kc) {
        constexpr int k2 = decltype(kc)::value, sl = k2 % (PF + 1);
        if constexpr (k2 + PF < NK) rd(std::integral_constant<int, k2 + PF>{});
        constexpr int younger = 4 * (PF < NK - 1 - k2 ? PF : NK - 1 - k2);
        lgkm4<younger>(r[sl][0], r[sl][1], r[sl][2], r[sl][3]);
        qacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(join_tr(r[sl][0], r[sl][1]), join_tr(r[sl][2], r[sl][3]), qacc,
                                                       0, 0, 0);
      });
    };

    issue(t_hi);
    vm_wait<0>();
    __syncthreads();
    const unsigned long long cc = OWLK_FUSED_PROF ? __builtin_amdgcn_s_memtime() : 0ull;

    // ready: the predecessor's sum of the tile whose dQ is formed next was found published at
    // mid-step of the tile's own step and is in flight to this wave's landing zone (waited for at
    // the top of the next step); else it is polled and loaded there.  Zeros for the chain's first block
    bool ready = true;
    auto dq_begin = [&](int i) {
      f32x4 a[NACC];
#pragma unroll
      for (int e = 0; e < NACC; ++e) a[e] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (j > jlo_at(i) && !(OWLK_FUSED_EXP & 1)) {
        if (OWLK_FUSED_STATS && lane == 0) {
          __hip_atomic_fetch_add(p.hdr + 11, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (!ready) __hip_atomic_fetch_add(p.hdr + 10, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (!ready) {
          if (wait_flag(flg + i * FLAG_STRIDE, fail_at(p, chain, j) ? 1 << 30 : j, p.hdr + 8)) {
            load_acc(i);
          } else {
            // the predecessor's sum never arrived (the error word is set): this tile's dQ is void,
            // and NaN carries that into every later part of it and into the stored dQ rows
#pragma unroll
            for (int e = 0; e < NACC; ++e) *(f32x4*)(accl + e * 1024 + lane * 16) = f32x4{NAN, NAN, NAN, NAN};
          }
        }
        vm_wait<0>();  // the sum's loads are this wave's only vector-memory ops in flight here
#pragma unroll
        for (int e = 0; e < NACC; ++e) a[e] = *(const f32x4*)(accl + e * 1024 + lane * 16);
      }
      if constexpr (DQ16) {
        qa[0] = a[0];
        qa[1] = a[1];
      } else {
#pragma unroll
        for (int rr = 0; rr < NACC; ++rr)
#pragma unroll
          for (int r = 0; r < 4; ++r) qacc[4 * rr + r] = a[rr][r];
      }
    };

    for (int t = t_hi; t >= t_lo; --t) {
      const int q0 = t * FQT;
      const unsigned long long c0 = OWLK_FUSED_PROF ? __builtin_amdgcn_s_memtime() : 0ull;
      const bool dq_on = !(OWLK_FUSED_EXP & 2) && t + 1 <= t_hi && dq_wave;
      // the predecessor's sum of tile t + 1 (waits for this wave's vector memory: before any DMA)
      if (dq_on) dq_begin(t + 1);
      const bool poll = j > jlo_at(t) && dq_wave && !(OWLK_FUSED_EXP & 1);

      int kind = TILE_FULL;
      if (t < full_lo || t >= full_hi) {
        const int r1 = q0 + FQT < L ? q0 + FQT : L;
        kind = !wave_live || r1 <= seen_lo || q0 >= seen_hi ? TILE_EMPTY : TILE_PARTIAL;
      }
      kind = __builtin_amdgcn_readfirstlane(kind);
      const bool masked = kind == TILE_PARTIAL;

      // a tile's S / dP operands of query rows 32 qb .. + 31 (lse2, delta rows, Q and dO
      // fragments), by asm in the order they are consumed: 12 LDS reads
      const unsigned sbase = lds_addr(smem + (t & 1) * RING_SLOT);
      const unsigned a_r0 = sbase + opaque<4>(ro0), a_r1 = sbase + opaque<4>(ro1), a_l = sbase + 16 * (opaque<4>((unsigned)lane) >> 4);
      f32x4 lr[2], dr[2];
      bf16x8 aq[2][2], ad[2][2];  // [k step][16-row query tile]
      auto issue_a = [&](auto qbc) {
        constexpr int qb = decltype(qbc)::value;
        static_for<2>([&](auto qsc) {
          constexpr int qs = decltype(qsc)::value, row = 32 * qb + 16 * qs;
          lr[qs] = rd128<2 * TILE_BYTES + 4 * row, f32x4>(a_l);
          dr[qs] = rd128<2 * TILE_BYTES + 4 * FQT + 4 * row, f32x4>(a_l);
        });
        static_for<2>([&](auto qsc) {
          constexpr int qs = decltype(qsc)::value, row = 32 * qb + 16 * qs;
          aq[0][qs] = rd128<128 * row, bf16x8>(a_r0);
          ad[0][qs] = rd128<TILE_BYTES + 128 * row, bf16x8>(a_r0);
        });
        static_for<2>([&](auto qsc) {
          constexpr int qs = decltype(qsc)::value, row = 32 * qb + 16 * qs;
          aq[1][qs] = rd128<128 * row, bf16x8>(a_r1);
          ad[1][qs] = rd128<TILE_BYTES + 128 * row, bf16x8>(a_r1);
        });
      };

      // dQ of tile t + 1 from its dS image (step t + 1), stored at once; this step's barrier drains
      // the stores, then the flag goes out
      if (dq_on) {
        dq_mfma(t + 1);
        store_dq(t + 1);
      }
      // in issue order: the dQ stores, the ring's LDS-DMA of tile t - 1, the flag poll
      const unsigned long long c1 = OWLK_FUSED_PROF ? __builtin_amdgcn_s_memtime() : 0ull;
      const bool dma = t - 1 >= t_lo;
      if (dma) issue(t - 1);
      if (poll) dma4_sc1(lds_addr(flagl), flg + t * FLAG_STRIDE, 0u);

      const unsigned dsw = lds_addr(smem + DS_OFF + (t & 1) * DS_BYTES) + dsl;
      auto ds_put = [&](int t2, int qb, int e, bf16x4 v) {
        *(AS3 bf16x4*)(uintptr_t)(dsw + 2048 * t2 + ((unsigned)(64 * qb + 32 * e) ^ opaque<2>(dsx))) = v;
      };
      unsigned bh[2] = {0u, 0u};  // bit 4 m + r: query row q0 + 16 m + 4 g + r of key t2
      if (masked) {  // query rows [frame(key) tpf, L) (causal) / [0, L) of the tile, per key
#pragma unroll
        for (int t2 = 0; t2 < 2; ++t2) {
          // the key from an opaque lane id: its row range is formed here, not kept across the sweep
          const int k = kw0 + 16 * t2 + (int)(opaque<8>((unsigned)lane) & 15), fk = frame(p, k);
          const int lo = q_lo_frame(p, fk) * p.tpf - q0, hi = (RUNS ? khi[t2] : (int)q_hi_end(p, fk)) - q0;
          const unsigned long long b64 = k < L ? range_bits(lo, hi) >> (4 * g) : 0ull;
          bh[t2] = (unsigned)(b64 & 0xF) | (unsigned)((b64 >> 12) & 0xF0) | (unsigned)((b64 >> 24) & 0xF00) |
                   (unsigned)((b64 >> 36) & 0xF000);
        }
      }
      bool loads_out = false;
      static_for<2>([&](auto qbc) {
        constexpr int qb = decltype(qbc)::value;
        if (kind == TILE_EMPTY) {
          // no allowed pair for this wave's keys: its rows of the dS image are zero
#pragma unroll
          for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
            for (int e = 0; e < 2; ++e) ds_put(t2, qb, e, bf16x4{});
        } else {
          // S / dP (12 reads in flight, oldest first: lse2 / delta rows, then k step 0, 1).  Issued
          // here, not earlier: holding them across the step's control flow overflows the 256-VGPR
          // budget (tried: 100-200 VGPRs spilled)
          issue_a(qbc);
          f32x4 st[2][2], dp[2][2];  // [16-row query tile][key tile]
          lgkm4<8>(lr[0], dr[0], lr[1], dr[1]);
          // the lse2 / delta rows are the first MFMA's C operand (no accumulator-init copies)
          static_for<2>([&](auto ksc) {
            constexpr int ks = decltype(ksc)::value;
            static_for<2>([&](auto qsc) {
              constexpr int qs = decltype(qsc)::value;
              lgkm2<6 - 4 * ks - 2 * qs>(aq[ks][qs], ad[ks][qs]);
#pragma unroll
              for (int t2 = 0; t2 < 2; ++t2) {
                st[qs][t2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aq[ks][qs], kf[t2][ks], ks ? st[qs][t2] : lr[qs], 0, 0, 0);
                dp[qs][t2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ad[ks][qs], vf[t2][ks], ks ? dp[qs][t2] : dr[qs], 0, 0, 0);
              }
            });
          });
          // the dV / dK operands (dO^T, Q^T of these 32 rows): 16 reads, landing under the
          // softmax-gradient VALU work below
          s16x4 tq[4][4];  // [column group ds][dO^T lo, hi, Q^T lo, hi]
          auto rd_t = [&](auto dsc, unsigned a) {
            constexpr int ds = decltype(dsc)::value;
            tq[ds][0] = tr_rd<TILE_BYTES + 128 * 32 * qb>(a);
            tq[ds][1] = tr_rd<TILE_BYTES + 128 * 32 * qb + 2048>(a);
            tq[ds][2] = tr_rd<128 * 32 * qb>(a);
            tq[ds][3] = tr_rd<128 * 32 * qb + 2048>(a);
          };
          rd_t(std::integral_constant<int, 0>{}, sbase + opaque<4>(tro0));
          rd_t(std::integral_constant<int, 1>{}, sbase + opaque<4>(tro1));
          rd_t(std::integral_constant<int, 2>{}, sbase + opaque<4>(tro2));
          rd_t(std::integral_constant<int, 3>{}, sbase + opaque<4>(tro3));
#pragma unroll
          for (int qs = 0; qs < 2; ++qs)
#pragma unroll
            for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
              for (int r = 0; r < 4; ++r) st[qs][t2][r] = __builtin_amdgcn_exp2f(-st[qs][t2][r]);
          if (masked) {
#pragma unroll
            for (int t2 = 0; t2 < 2; ++t2) {
              apply_bits4<8 * qb>(st[0][t2], bh[t2], 0.f);
              apply_bits4<8 * qb + 4>(st[1][t2], bh[t2], 0.f);
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
          // -dS of this wave's keys into the [key][query] image: lane (c, g) holds queries
          // 32 qb + 4 g .. + 3 (elements 0..3) and 32 qb + 16 + 4 g .. + 3 (elements 4..7) of key c
#pragma unroll
          for (int t2 = 0; t2 < 2; ++t2) {
            if (!(OWLK_FUSED_EXP & 4)) {
              ds_put(t2, qb, 0, __builtin_shufflevector(sf[t2], sf[t2], 0, 1, 2, 3));
              ds_put(t2, qb, 1, __builtin_shufflevector(sf[t2], sf[t2], 4, 5, 6, 7));
            }
          }
          // dV / dK (the dS stores above are younger than every read waited for: the counts
          // only over-wait)
          static_for<4>([&](auto dsc) {
            constexpr int ds = decltype(dsc)::value;
            lgkm4<4 * (3 - ds)>(tq[ds][0], tq[ds][1], tq[ds][2], tq[ds][3]);
            const bf16x8 ado = join_tr(tq[ds][0], tq[ds][1]), aqt = join_tr(tq[ds][2], tq[ds][3]);
#pragma unroll
            for (int t2 = 0; t2 < 2; ++t2) {
              dv[ds][t2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ado, pf[t2], dv[ds][t2], 0, 0, 0);
              dk[ds][t2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aqt, sf[t2], dk[ds][t2], 0, 0, 0);
            }
          });
        }
        if constexpr (qb == 0) {
          if (poll) {  // the flag polled at the top has had half a tile to arrive
            vm_wait<0>();  // the dQ stores and the flag poll, in issue order (the dQ waves issue no ring DMA)
            ready = __builtin_amdgcn_readfirstlane(*(const int*)flagl) >= (fail_at(p, chain, j) ? 1 << 30 : j);
            if (ready) {
              load_acc(t);
              loads_out = true;
            }
          }
        }
      });
      // every wave: its dQ(t + 1) stores and the ring's tile t - 1 have landed (vmcnt counts in
      // issue order; the sum's loads of tile t, issued last, stay in flight to the next step's top)
      const unsigned long long c2 = OWLK_FUSED_PROF ? __builtin_amdgcn_s_memtime() : 0ull;
      if (loads_out)
        vm_wait<NACC>();
      else
        vm_wait<0>();
      const unsigned long long c3 = OWLK_FUSED_PROF ? __builtin_amdgcn_s_memtime() : 0ull;
      __syncthreads();
      if (OWLK_FUSED_PROF) {
        const unsigned long long c4 = __builtin_amdgcn_s_memtime();
        prof[0] += c1 - c0;
        prof[1] += c2 - c1;
        prof[2] += c3 - c2;
        prof[3] += c4 - c3;
      }
      if (t + 1 <= t_hi && threadIdx.x == 0)
        __hip_atomic_store(flg + (t + 1) * FLAG_STRIDE, j + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }

    // ---- epilogue: dQ of tile t_lo (its dS image is in LDS)
    const unsigned long long cd = OWLK_FUSED_PROF ? __builtin_amdgcn_s_memtime() : 0ull;
    const bool dq_epi = !(OWLK_FUSED_EXP & 2) && dq_wave;
    if (dq_epi) dq_begin(t_lo);
    // the next item's claim on this XCD's queue: its return is waited for with the dQ stores
    int npf = 0;
    if (OWLK_FUSED_DEQ_PF && threadIdx.x == 0)
      npf = __hip_atomic_fetch_add(p.hdr + xcc, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (dq_epi) {
      dq_mfma(t_lo);
      store_dq(t_lo);
    }
    vm_wait<0>();
    __syncthreads();  // also: every wave is done with the LDS before the next item's DMA
    if (threadIdx.x == 0) {
      __hip_atomic_store(flg + t_lo * FLAG_STRIDE, j + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (OWLK_FUSED_DEQ_PF) {
        int nc = -1, nj = 0;
        if (!item_of((int)xcc, npf, nc, nj)) claim(1, nc, nj);
        sh_item[0] = nc;  // read after the next item's first barrier
        sh_item[1] = nj;
      }
    }

#if OWLK_FUSED_KV_STAGE
    // dK, dV through this wave's 8 KiB of the (now free) dS images, stored as whole 128-B rows with
    // 16-B stores (lane-held 8-B pieces were 16 stores per lane, whose tail the next item's
    // prologue waits for: vmcnt counts stores).  Row r = key kw0 + r, 16-B chunk x at x ^ (r & 7)
    {
      char* stg = smem + DS_OFF + w * 8192;
#pragma unroll
      for (int t2 = 0; t2 < 2; ++t2) {
        const int r = 16 * t2 + c;
#pragma unroll
        for (int ds = 0; ds < 4; ++ds) {  // this lane: d = 16 ds + 4 g + e of key r
          bf16x4 a4, b4;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            a4[e] = (bf16)(dk[ds][t2][e] * -p.scale);  // dS was accumulated negated
            b4[e] = (bf16)dv[ds][t2][e];
          }
          const int off = r * 128 + (((2 * ds + (g >> 1)) ^ (r & 7)) << 4) + 8 * (g & 1);
          *(bf16x4*)(stg + off) = a4;
          *(bf16x4*)(stg + 4096 + off) = b4;
        }
      }
      wave_lds_handoff();  // the rows were staged by other lanes of this wave
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int r = 8 * it + (lane >> 3), x = lane & 7, k = kw0 + r;
        const int off = r * 128 + ((x ^ (r & 7)) << 4);
        const bf16x8 vk = *(const bf16x8*)(stg + off), vv = *(const bf16x8*)(stg + 4096 + off);
        if (k < L) {
          *(bf16x8*)(p.dk + b * p.sdkb + (long)k * p.lddk + head * 64 + 8 * x) = vk;
          *(bf16x8*)(p.dv + b * p.sdvb + (long)k * p.lddv + head * 64 + 8 * x) = vv;
        }
      }
    }
#else
    // dK[key][d], dV[key][d]: this lane holds d = 16 ds + 4 g + r of its two keys
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) {
      const int k = kw0 + 16 * t2 + (int)(opaque<8>((unsigned)lane) & 15);
      if (k >= L) continue;
      bf16* pk = p.dk + b * p.sdkb + (long)k * p.lddk + head * 64 + 4 * g;
      bf16* pv = p.dv + b * p.sdvb + (long)k * p.lddv + head * 64 + 4 * g;
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
#endif
    if (OWLK_FUSED_PROF) {
      const unsigned long long ce = __builtin_amdgcn_s_memtime();
      prof[4] += cb - ca;
      prof[5] += cc - cb;
      prof[6] += ce - cd;
    }
  }
}

// XCD-local form: every per-XCD queue must have been drained by workgroups running on that XCD.  A
// queue no workgroup reached (an XCD left without workgroups, e.g. by a CU-masked stream) would leave
// its chains' dK / dV / dQ unwritten with no sign.  One small launch after the sweep finds such a
// queue, sets the error word (2) and writes NaN over every row of its chains' dQ, dK and dV.
__global__ __launch_bounds__(256) void fused_drain_check_k(FusedP p) {
  const int x = blockIdx.y;
  const int cx = p.nchain > x ? (p.nchain - x + 7) / 8 : 0;
  if ((long)__hip_atomic_load(p.hdr + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (long)cx * p.nkb) return;
  if (blockIdx.x == 0 && threadIdx.x == 0) __hip_atomic_store(p.hdr + 8, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  bf16x8 nan8;
#pragma unroll
  for (int e = 0; e < 8; ++e) nan8[e] = (bf16)NAN;
  for (int ch = x; ch < p.nchain; ch += 8) {
    const int b = ch / p.H, head = ch % p.H;
    for (long r = (long)blockIdx.x * 32 + (threadIdx.x >> 3); r < p.L; r += (long)gridDim.x * 32) {
      const int col = head * 64 + 8 * (threadIdx.x & 7);
      *(bf16x8*)(p.dq + b * p.sdqb + r * p.lddq + col) = nan8;
      *(bf16x8*)(p.dk + b * p.sdkb + r * p.lddk + col) = nan8;
      *(bf16x8*)(p.dv + b * p.sdvb + r * p.lddv + col) = nan8;
    }
  }
}

// CUs left to other streams' kernels (owlk_set_cu_reserve): the persistent grid shrinks by that many
// CUs' workgroups, so an all-reduce launched beside it finds free CUs instead of waiting for its end
std::atomic<int> g_cu_reserve{0};

int fused_grid(int dev, bool w4) {
  static int cached[64][2][2] = {};  // {CUs, workgroups per CU}
  if (dev < 0 || dev >= 64) dev = 0;
  if (!cached[dev][w4][0]) {
    int cus = 0, per = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (w4)
      per = fused4_occupancy();
    else
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, attn_bwd_fused_k<false, false>, 512, 0);
    cached[dev][w4][1] = per > 0 ? per : 1;
    cached[dev][w4][0] = cus > 0 ? cus : 256;
  }
  const int cus = cached[dev][w4][0], per = cached[dev][w4][1];
  // workgroups reach the XCDs round-robin: (CUs - k) keeps every XCD's queue drained as long as at
  // least one workgroup per XCD remains (8 CUs)
  const int keep = std::max(std::min(cus, 8), cus - g_cu_reserve.load(std::memory_order_relaxed));
  return keep * per;
}

// the XCD-local hand-off needs a workgroup on every one of the 8 per-XCD queues' XCDs (an XCC id
// no workgroup reports would leave its queue undrained): only on a device of 8 XCCs (SPX mode;
// workgroups reach the XCCs round-robin)
bool all_xcds_present(int dev) {
  static int cached[64] = {};  // 0 unknown, 1 yes, -1 no
  if (dev < 0 || dev >= 64) return false;
  if (!cached[dev]) {
    int n = 0;
    cached[dev] = hipDeviceGetAttribute(&n, hipDeviceAttributeNumberOfXccs, dev) == hipSuccess && n == 8 ? 1 : -1;
  }
  return cached[dev] > 0;
}

}  // namespace

static long fused_tiles(long L) { return (L + FQT - 1) / FQT; }

extern "C" int owlk_set_cu_reserve(int cus) {
  OWLK_REQUIRE(cus >= 0, "owlk_set_cu_reserve: negative CU count %d", cus);
  g_cu_reserve.store(cus, std::memory_order_relaxed);
  return 0;
}

extern "C" long owlk_attn_bwd_fused_ws_bytes(long B, int H, long L, int head_dim) {
  if (head_dim != 64 || B <= 0 || H <= 0 || L <= 0) return 0;
  const long nchain = B * H, nt = fused_tiles(L);
  // header | flags | fp32 sums | packed documents' first contributor per (sample, tile), 64 words of
  // slack per sample (the ring's 256-B DMA of a tile's word)
  return HDR_BYTES + nchain * nt * (long)(FLAG_STRIDE * 4) + nchain * nt * (long)ACC_TILE_BYTES + B * (nt + 64) * 4L;
}

extern "C" int owlk_attn_bwd_fused(const void* q, long ldq, long sqb, const void* k, long ldk, long skb,
                                   const void* v, long ldv, long svb, const void* dout, long ldo, long sob,
                                   const float* lse, const float* delta, void* dq, long lddq, long sdqb, void* dk,
                                   long lddk, long sdkb, void* dv, long lddv, long sdvb, long B, int H, long L,
                                   int head_dim, float scale, long tpf, int window, int causal, const int* kv_lo,
                                   const int* q_hi, const int* run_start, const int* doc, long fstride, void* ws,
                                   long ws_bytes, int variant, void* stream) {
  OWLK_REQUIRE(head_dim == 64, "attn_bwd_fused: head_dim %d not built (64)", head_dim);
  OWLK_REQUIRE(tpf > 0 && L > 0 && B > 0 && H > 0, "attn_bwd_fused: bad sizes");
  OWLK_REQUIRE(ldq < (1L << 31) && ldk < (1L << 31) && ldv < (1L << 31) && ldo < (1L << 31) && lddq < (1L << 31) &&
                   lddk < (1L << 31) && lddv < (1L << 31),
               "attn_bwd_fused: row strides too large");
  const bool runs = kv_lo || q_hi;
  OWLK_REQUIRE(!run_start && !doc && (!runs || (kv_lo && q_hi && causal && fstride > 0)),
               "attn_bwd_fused: document masks only as packed runs (kv_lo / q_hi, causal)");
  OWLK_REQUIRE(L < (1L << 31) / (tpf > 1 ? tpf : 1) || tpf == 1, "attn_bwd_fused: sequence too long");
  OWLK_REQUIRE(fused_tiles(L) * (long)ACC_TILE_BYTES < (1L << 31), "attn_bwd_fused: sequence too long");
  OWLK_REQUIRE(B * H < (1L << 24), "attn_bwd_fused: too many heads");
  OWLK_REQUIRE((B * H / 8 + 1) * ((L + FKB - 1) / FKB) < (1L << 31), "attn_bwd_fused: too many work items per queue");
  const long need = owlk_attn_bwd_fused_ws_bytes(B, H, L, head_dim);
  OWLK_REQUIRE(ws && ws_bytes >= need && (uintptr_t)ws % 256 == 0, "attn_bwd_fused: workspace (%ld bytes, 256-B aligned) needed",
               need);
  OWLK_REQUIRE(((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)dout | (uintptr_t)dq | (uintptr_t)dk |
                (uintptr_t)dv) % 16 == 0,
               "attn_bwd_fused: operands must be 16-byte aligned");
  FusedP p;
  p.q = (const bf16*)q; p.k = (const bf16*)k; p.v = (const bf16*)v; p.dout = (const bf16*)dout;
  p.lse = lse; p.delta = delta;
  p.dq = (bf16*)dq; p.dk = (bf16*)dk; p.dv = (bf16*)dv;
  p.ldq = (int)ldq; p.ldk = (int)ldk; p.ldv = (int)ldv; p.ldo = (int)ldo;
  p.lddq = (int)lddq; p.lddk = (int)lddk; p.lddv = (int)lddv;
  p.sqb = sqb; p.skb = skb; p.svb = svb; p.sob = sob; p.sdqb = sdqb; p.sdkb = sdkb; p.sdvb = sdvb;
  p.L = (int)L;
  p.H = H;
  p.nchain = (int)(B * H);
  p.ntiles = (int)fused_tiles(L);
  p.nkb = (int)((L + FKB - 1) / FKB);
  p.tpf = (int)tpf;
  p.causal = causal ? 1 : 0;
  p.window = window > 0 ? window : 0;
  p.magic = tpf > 1 ? (unsigned)((1ull << 32) / (unsigned long long)tpf + 1) : 0u;
  p.scale = scale;
  p.scale_log2 = scale * 1.4426950408889634f;
  p.hdr = (int*)ws;
  p.flags = (int*)((char*)ws + HDR_BYTES);
  p.acc = (char*)ws + HDR_BYTES + (long)p.nchain * p.ntiles * FLAG_STRIDE * 4;
  p.variant = variant;
  p.group = (variant >> 2) & 15 ? (variant >> 2) & 15 : 1 << 20;  // variant bits 2-5; 0 = all of the queue's chains
  p.kv_lo = kv_lo;
  p.q_hi = q_hi;
  p.fstride = fstride;
  p.jlo_stride = p.ntiles + 64;
  p.jlo = (int*)(p.acc + (long)p.nchain * p.ntiles * ACC_TILE_BYTES);
  p.fail_chain = (variant & 64) ? 0 : -1;  // test mode: chain 0's block-1 hand-off waits time out
  hipStream_t s = (hipStream_t)stream;
  // counters, error word and flags are zero on entry (one memset node, 16-B multiple from the start)
  if (hipMemsetAsync(ws, 0, (size_t)(HDR_BYTES + (long)p.nchain * p.ntiles * FLAG_STRIDE * 4), s) != hipSuccess)
    return owlk::check_launch("attn_bwd_fused memset");
  int dev = 0;
  (void)hipGetDevice(&dev);
  // variant bit 7: one wave per SIMD (attn_bwd_fused4_k, the hand-placed main step)
  // (its bf16 dQ rows are stored through a buffer resource: L * lddq * 2 must stay below 2^31)
  const bool w4 = (variant & 128) != 0 && L * lddq * 2 < (1L << 31);
  const dim3 grid((unsigned)fused_grid(dev, w4));
  // the XCD-local hand-off only on an 8-XCC device (else: write-through)
  if ((variant & 1) && !all_xcds_present(dev)) variant &= ~1;
  if (runs) {
    OWLK_REQUIRE(!(variant & 2), "attn_bwd_fused: no counting mode with documents");
    const dim3 gj((unsigned)((p.jlo_stride + 255) / 256), (unsigned)B);
    hipLaunchKernelGGL(fused_jlo_k, gj, dim3(256), 0, s, p, (int)B);
    if (w4)
      fused4_launch(p, variant & 3, true, grid, s);
    else if (variant & 1)
      hipLaunchKernelGGL((attn_bwd_fused_k<true, false, true>), grid, dim3(512), 0, s, p);
    else
      hipLaunchKernelGGL((attn_bwd_fused_k<false, false, true>), grid, dim3(512), 0, s, p);
  } else if (w4) {
    fused4_launch(p, variant & 3, false, grid, s);
  } else {
    switch (variant & 3) {
      case 0: hipLaunchKernelGGL((attn_bwd_fused_k<false, false>), grid, dim3(512), 0, s, p); break;
      case 1: hipLaunchKernelGGL((attn_bwd_fused_k<true, false>), grid, dim3(512), 0, s, p); break;
      case 2: hipLaunchKernelGGL((attn_bwd_fused_k<false, true>), grid, dim3(512), 0, s, p); break;
      default: hipLaunchKernelGGL((attn_bwd_fused_k<true, true>), grid, dim3(512), 0, s, p); break;
    }
  }
  if (int e = owlk::check_launch("attn_bwd_fused")) return e;
  // the XCD-local form relies on workgroups reaching all 8 XCDs: check every queue was drained
  if (variant & 1) {
    hipLaunchKernelGGL(fused_drain_check_k, dim3(64, 8), dim3(256), 0, s, p);
    return owlk::check_launch("attn_bwd_fused drain check");
  }
  return 0;
}
