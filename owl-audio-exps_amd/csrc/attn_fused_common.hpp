// Shared pieces of the single-pass attention backward kernels (attn_bwd_fused.hip: 8 waves x 32
// keys; attn_bwd_fused4.hip: 4 waves x 64 keys with the hand-placed main step): the LDS layout,
// the work-item geometry of the frame mask, the hand-off helpers and the inline-asm memory forms.
#pragma once
#include <utility>

#include "attn_common.hpp"

#define AS1 __attribute__((address_space(1)))
#define AS3 __attribute__((address_space(3)))
#ifndef OWLK_FUSED_REMAT
#define OWLK_FUSED_REMAT 0
#endif
#ifndef OWLK_FUSED_DQ_PF
#define OWLK_FUSED_DQ_PF 3
#endif

namespace owlk_fused {


constexpr int FKB = 256;                                // keys per work item (8 waves x 32)
constexpr int FQT = 64;                                 // query rows per swept tile
constexpr int TILE_BYTES = 64 * 128;                    // 64 rows x 64 bf16, 128-B rows
constexpr int RING_SLOT = 2 * TILE_BYTES + 2 * FQT * 4;  // Q | dO | lse2 | delta
constexpr int NSLOT = 2;
constexpr int KIMG_OFF = NSLOT * RING_SLOT;    // K of the item: 256 rows x 128 B
constexpr int DS_OFF = KIMG_OFF + FKB * 128;   // two dS^T images [key][64 q] bf16
constexpr int DS_BYTES = FKB * 128;
constexpr int ACC_OFF = DS_OFF + 2 * DS_BYTES;  // per wave 2 KiB: its part of a tile's fp32 sum
constexpr int FLAGL_OFF = ACC_OFF + 8 * 2048;    // per wave 256 B: a polled flag word (64 copies)
constexpr int MISC_OFF = FLAGL_OFF + 8 * 256;
constexpr int JLO_OFF = MISC_OFF + 16;          // packed documents: per ring slot, its tile's first contributor
constexpr int SMEM_BYTES = JLO_OFF + 2 * 256;
constexpr int FLAG_STRIDE = 16;                // ints: one 64-B line per query-tile flag
constexpr long HDR_BYTES = 256;  // [0, 8) dequeue counters, [8] error word, [9] keys per item
constexpr int ACC_TILE_BYTES = FQT * 64 * 4;   // fp32 accumulator of one query tile
// dQ^T products: 0 = 32x32x16 MFMAs on waves 0-3 (one 32 d x 32 q tile each); 1 = 16x16x32 MFMAs
// on all 8 waves (one 16 d x 32 q quarter each: 50 % more LDS bytes, no idle waves)
#ifndef OWLK_FUSED_DQ16
#define OWLK_FUSED_DQ16 0
#endif
constexpr bool DQ16 = OWLK_FUSED_DQ16;
constexpr int NACC = DQ16 ? 2 : 4;  // 16-B words per lane of a wave's part of a tile's sum

struct FusedP {
  const bf16 *q, *k, *v, *dout;
  const float *lse, *delta;  // [B, H, L]; lse in base 2 (attn_fwd)
  bf16 *dq, *dk, *dv;
  int ldq, ldk, ldv, ldo, lddq, lddk, lddv;  // token row strides (elements)
  long sqb, skb, svb, sob, sdqb, sdkb, sdvb;  // batch strides
  int L;                                      // Lq == Lkv
  int H, nchain, ntiles, nkb;
  int tpf, causal;    // the mask: frame = token / tpf; causal or not, window (frames; <= 0: none); no documents
  int window;
  unsigned magic;     // floor(2^32 / tpf) + 1 (exact frame division below 2^32 / tpf); 0 if tpf == 1
  float scale, scale_log2;
  int* hdr;    // dequeue counters / error word
  int* flags;  // [nchain][ntiles] x FLAG_STRIDE
  char* acc;   // [nchain][ntiles][ACC_TILE_BYTES]
  int variant;
  int group;  // chains of a queue taken at a time (>= 1)
  // packed documents (causal, every document one run of frames; attn_common.hpp runs_mode): key
  // frame fk is seen by query frames fk .. q_hi[fk], query frame fq sees key frames kv_lo[fq] .. fq
  const int *kv_lo, *q_hi;  // [B][fstride], window folded in
  long fstride;
  int* jlo;                  // [B][jlo_stride]: each query tile's first contributing key block
  int jlo_stride;
  int fail_chain;            // test mode (variant bit 6): chain 0's block-1 hand-off waits time out; else -1
};

DEV unsigned xcc_id() {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
  return x;
}

// per-lane byte offset of frag_tr16(lds, row0, ds, lane) for any row0 that is a multiple of 16
// (swz_dual repeats every 16 rows); the second ds_read_b64_tr_b16 of the fragment is 2 KiB further
// per-lane byte offsets of frag_tr<SW_DUAL>(lds, row0, 0, cb, lane) (32x32x16 fragment of column
// group cb) for any row0 that is a multiple of 16: its two ds_read_b64_tr_b16 (rows 4 h + qq and
// 8 + 4 h + qq); the swizzle repeats every 16 rows
DEV void tr32_lane_off(int cb, int lane, int& oa, int& ob) {
  const int g = lane >> 4, h = lane >> 5, qq = (lane & 15) >> 2, pp = lane & 3;
  const int ra = 4 * h + qq, rb = ra + 8;
  const int ch = 4 * cb + 2 * (g & 1) + (pp >> 1);
  oa = ra * 128 + ((ch ^ swz_dual(ra)) << 4) + 8 * (pp & 1);
  ob = rb * 128 + ((ch ^ swz_dual(rb)) << 4) + 8 * (pp & 1);
}

// per-lane byte offset of frag_row16(lds, row0, ks, lane) for any row0 that is a multiple of 16
DEV unsigned row16_lane_off(int ks, int lane) {
  const int r = lane & 15;
  return (unsigned)(r * 128 + (((4 * ks + (lane >> 4)) ^ swz_dual(r)) << 4));
}

DEV unsigned tr16_lane_off(int ds, int lane) {
  const int c = lane & 15, g = lane >> 4;
  const int x = 4 * g + (c >> 2);
  const int ch = 2 * ds + ((c & 3) >> 1);
  return (unsigned)(x * 128 + ((ch ^ swz_dual(x)) << 4) + 8 * (c & 1));
}

// LDS swizzles of the single-pass kernels' Q / dO ring and -dS^T images, chosen against the gfx950 lane groups
// (ds_read_b128: 4 x 16 lanes {0-3,12-15,20-27} ..; ds_write_b64: 4 x 16 contiguous lanes on 32
// banks; ds_read_b64_tr_b16: 2 x 32) so that every ring read (row fragments and transposed), every
// -dS row write and every dS^T read is conflict-free (swz_dual, shared with the 8-wave kernel, left
// the ring's row reads and the -dS writes 2-way conflicted: a quarter of the LDS-array cycles).
// Ring: 16-B chunk c of row r at c ^ (r & 6).  -dS^T image: 8-B unit u (4 queries) of key row r at
// u ^ swz_ds8(r).  The K image keeps swz_dual (its reads are conflict-free with it).
DEV int swz_ring(int r) { return r & 6; }
DEV int swz_ds8(int r) { return (r & 1) | ((r & 2) << 2) | ((r & 12) >> 1); }
DEV unsigned ring_row16_off(int ks, int lane) {  // frag_row16 of rows row0 + (lane & 15), row0 % 16 == 0
  const int r = lane & 15;
  return (unsigned)(r * 128 + (((4 * ks + (lane >> 4)) ^ swz_ring(r)) << 4));
}
DEV unsigned ring_tr16_off(int ds, int lane) {  // frag_tr16 (dO^T / Q^T) of column group ds
  const int c = lane & 15, g = lane >> 4;
  const int x = 4 * g + (c >> 2);
  const int ch = 2 * ds + ((c & 3) >> 1);
  return (unsigned)(x * 128 + ((ch ^ swz_ring(x)) << 4) + 8 * (c & 1));
}
DEV void ds_tr32_off(int cb, int lane, int& oa, int& ob) {  // dS^T fragment of query group cb (rows 4 h + qq, + 8)
  const int g = lane >> 4, h = lane >> 5, qq = (lane & 15) >> 2, pp = lane & 3;
  const int ra = 4 * h + qq, rb = ra + 8, u = 8 * cb + 4 * (g & 1) + pp;
  oa = ra * 128 + 8 * (u ^ swz_ds8(ra));
  ob = rb * 128 + 8 * (u ^ swz_ds8(rb));
}
DEV unsigned ds_tr16_off(int ds, int lane) {  // frag_tr16 of the dS^T image (OWLK_FUSED_DQ16; 2-way conflicted)
  const int c = lane & 15, g = lane >> 4;
  const int x = 4 * g + (c >> 2);
  return (unsigned)(x * 128 + 8 * ((4 * ds + (c & 3)) ^ swz_ds8(x)));
}

// Every vector-memory access of the sweep goes through inline asm, and the waits are counted by
// hand (vmcnt counts loads, LDS-DMA and stores in issue order).  A compiler-visible LDS-DMA makes
// hipcc drain it (vmcnt(0)) before every ds_read_b64_tr_b16 (the builtin carries no memory operand),
// which here would also drain the accumulator loads in flight; asm outputs get their waits through
// "+v" operands of the s_waitcnt, so no consumer is scheduled above it.  The kernel uses m0 only
// here (no other LDS-DMA, no dynamic register indexing).
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
DEV unsigned lds_addr(const void* p) { return (unsigned)(uintptr_t)(const AS3 void*)p; }
// one LDS-DMA wave-instruction (16 or 4 B per lane) to the wave-uniform LDS byte address `lds`
// from the wave-uniform base `base` (SGPRs) + a 32-bit per-lane byte offset, so no 64-bit per-lane
// address is kept live across the sweep.  No instruction offset: it would move the LDS
// destination too (M0 + offset + lane * size)
DEV void dma16(unsigned lds, const void* base, unsigned off) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(lds), "v"(off), "s"(base)
               : "memory", "m0");
}
DEV void dma4(unsigned lds, const void* base, unsigned off) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dword %1, %2" ::"s"(lds), "v"(off), "s"(base)
               : "memory", "m0");
}
// the hand-off's loads (sc1: past this CU's L1, cdna_hip_programming.md Guideline 16) land in LDS
// too: a register destination of an asm load whose wait is a separate statement could be copied
// by the compiler before the data arrives; these are read back by ds_read after vm_wait
DEV void dma16_sc1(unsigned lds, const void* base, unsigned off) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 sc1" ::"s"(lds), "v"(off), "s"(base)
               : "memory", "m0");
}
DEV void dma4_sc1(unsigned lds, const void* base, unsigned off) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dword %1, %2 sc1" ::"s"(lds), "v"(off), "s"(base)
               : "memory", "m0");
}
#pragma clang diagnostic pop
// a copy the compiler cannot see through: values formed from it are formed where they are used
// (hoisted out of the sweep, the dS image's 16 per-lane piece addresses were kept live and spilled)
template <int BIT = 0>
DEV unsigned opaque(unsigned x) {
  if (!BIT || (OWLK_FUSED_REMAT & BIT)) asm volatile("" : "+v"(x));
  return x;
}
template <int N>
DEV void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// Every LDS read of the sweep's MFMA operands is inline asm, software-pipelined by hand (left to
// itself hipcc reads each MFMA's operands right before it into one register set and waits
// lgkmcnt(0)); retired by lgkm2 / lgkm4, whose "+v" operands keep every consumer below the wait.
// LDS operations complete in order and the sweep has no scalar loads, so a count N waits for all
// but the N youngest LDS operations: counting only the asm reads issued after the awaited ones is
// exact or over-waits (compiler-issued LDS stores / reads in between only add younger operations)
template <int OFF>
DEV s16x4 tr_rd(unsigned lds) {
  s16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(lds), "n"(OFF) : "memory");
  return r;
}
template <int OFF, typename T>
DEV T rd128(unsigned lds) {
  T r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(lds), "n"(OFF) : "memory");
  return r;
}
template <int N, typename A, typename B>
DEV void lgkm2(A& a, B& b) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "n"(N) : "memory");
}
template <int N, typename A, typename B, typename C>
DEV void lgkm3(A& a, B& b, C& c) {
  asm volatile("s_waitcnt lgkmcnt(%3)" : "+v"(a), "+v"(b), "+v"(c) : "n"(N) : "memory");
}
template <int N, typename A, typename B, typename C, typename D>
DEV void lgkm4(A& a, B& b, C& c, D& d) {
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "n"(N) : "memory");
}
template <int N, typename T>
DEV void lgkm6(T& a, T& b, T& c, T& d, T& e, T& f) {
  asm volatile("s_waitcnt lgkmcnt(%6)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f) : "n"(N) : "memory");
}
template <typename F, int... I>
DEV void static_for_(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
DEV void static_for(F&& f) {
  static_for_(f, std::make_integer_sequence<int, N>{});
}

DEV int frame(const FusedP& p, int idx) { return p.magic ? (int)__umulhi((unsigned)idx, p.magic) : idx; }

// The frame mask without documents (attn.py:24-62): query frame fq sees key frame fk iff fk <= fq
// (causal) and |fq - fk| < window (window > 0).  Key frame fk is seen by query tokens
// [q_lo_frame(fk) tpf, q_hi_end(fk)).
DEV int q_lo_frame(const FusedP& p, int fk) {
  return p.causal ? fk : (p.window > 0 && fk - p.window + 1 > 0 ? fk - p.window + 1 : 0);
}
DEV long q_hi_end(const FusedP& p, int fk) {
  if (p.window <= 0) return p.L;
  const long e = (long)(fk + p.window) * p.tpf;
  return e < p.L ? e : p.L;
}
// key block j sweeps query tiles sweep_lo(j) .. sweep_hi(j), both non-decreasing in j, so the
// blocks that sweep tile i are the contiguous range tile_jlo(i) .. tile_jhi(i): the closed forms
// of min{j : sweep_hi(j) >= i} and max{j : sweep_lo(j) <= i} (tests/test_attn_fused_gpu.py checks
// them against those definitions, and the counting mode checks the kernel's hand-offs against them)
DEV int sweep_lo(const FusedP& p, int j) { return (int)((long)q_lo_frame(p, frame(p, j * FKB)) * p.tpf / FQT); }
DEV int sweep_hi(const FusedP& p, int j) {
  const int k1 = j * FKB + FKB - 1 < p.L ? j * FKB + FKB - 1 : p.L - 1;
  return (int)((q_hi_end(p, frame(p, k1)) - 1) / FQT);
}
DEV int tile_jlo(const FusedP& p, int i) {
  if (p.window <= 0) return 0;
  const long x = (long)(frame(p, i * FQT) - p.window + 1) * p.tpf;
  return x > 0 ? (int)(x / FKB) : 0;
}
DEV int tile_jhi(const FusedP& p, int i) {
  const int ql = i * FQT + FQT - 1 < p.L ? i * FQT + FQT - 1 : p.L - 1;
  long f = frame(p, ql);
  if (!p.causal) {
    if (p.window <= 0) return p.nkb - 1;
    f += p.window - 1;
  }
  const long kend = (f + 1) * p.tpf;
  const long ke = kend < p.L ? kend : p.L;
  const int j = (int)((ke - 1) / FKB);
  return j < p.nkb - 1 ? j : p.nkb - 1;
}

// Packed documents: q_hi is non-decreasing (runs are contiguous, the window end is fq + W - 1), so
// block j's sweep still ends at its last key's q_hi, and q_hi[fk] >= fq <=> fk >= kv_lo[fq] makes
// min{j : sweep_hi(j) >= i} the block of key kv_lo[frame(i FQT)] tpf (fused_jlo_k, read per tile
// from the ring slot: no global load inside the sweep)
DEV long q_hi_end_runs(const FusedP& p, const int* qh, int fk) {
  const long e = (long)(qh[fk] + 1) * p.tpf;
  return e < p.L ? e : p.L;
}

// test mode (variant bit 6): chain 0's block 1 waits for a flag value no block stores, so its hand-off
// waits time out (after the spin bound) and take the error path
DEV bool fail_at(const FusedP& p, int chain, int j) { return chain == p.fail_chain && j == 1; }

// bounded poll of a flag word (every lane loads the same word: one request), sc1 loads
DEV bool wait_flag(const int* f, int want, int* err) {
  if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >= want)
    return true;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    __builtin_amdgcn_s_sleep(2);
    if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >= want)
      return true;
    if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {  // >= 2 s at the 100 MHz clock
      __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    // after any timeout every later wait gives up at once (results are void; the word says so)
    if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != 0)
      return false;
  }
}

// attn_bwd_fused4.hip (one wave per SIMD): resident workgroups per CU, and the launch of
// attn_bwd_fused4_k<variant bit 0 (local), bit 1 (counting), runs> on 256-thread workgroups
int fused4_occupancy();
void fused4_launch(const FusedP& p, int variant, bool runs, dim3 grid, hipStream_t s);

}  // namespace owlk_fused
