#!/usr/bin/env python3
"""Generate the hand-placed main step of the one-wave-per-SIMD single-pass attention backward.

    python tools/gen_fused4_asm.py            # writes owl-audio-exps_amd/csrc/attn_bwd_fused4_step.inc
    python tools/gen_fused4_asm.py --stats    # schedule / register / wait statistics only

The step (one 64-row query tile against one wave's 64 keys, attn_bwd_fused.hip `attn_bwd_fused4_k`)
is four blocks of 32 `v_mfma_f32_16x16x32_bf16`: S / dP of query half 0 (M1_0), S / dP of half 1
(M1_1), dV / dK of half 0 (M2_0), dV / dK of half 1 (M2_1).  Everything else rides in the gaps
between them at a fixed place:

* the Q / dO row fragments of the S / dP products through a three-slot AGPR ring, two groups ahead;
* the lse2 / delta rows straight into the registers the S / dP chains start from;
* the softmax-gradient VALU of half 0 (exp2, dP * P, bf16 packing, in place) under M1_1 and M2_0,
  that of half 1 under M2_0 and M2_1 (M2 runs key tile by key tile, so a tile's packing is due
  only at its own MFMAs);
* the -dS rows into the [key][query] LDS image right after their packing;
* the transposed dO^T / Q^T fragments of the dV / dK products.

Registers are fixed here, not by hipcc: the statement clobbers v[112:255] and the AGPR file; the
accumulators dK^T / dV^T and the K' / V' fragments are compiler-allocated AGPR operands (they
stay in a[0:191]).  The generator counts every LDS operation (in-order completion; lgkmcnt is
4 bits, so counts above 15 over-wait) and pads the MFMA hazards with s_nop:
  VALU write -> MFMA read: 2 wait states; 16x16x32 MFMA write -> VALU / LDS read: 8 (hipcc's own
  padding on gfx950); MFMA read or write -> VALU / LDS-load write of that register: 12 (margin).
"""
import argparse
import re
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "owl-audio-exps_amd", "csrc", "attn_bwd_fused4_step.inc")
# schedule knobs for A/B builds (tools/build_f4_variants.sh): the 16x16x32 MFMA the hand-off check goes
# before, the first MFMA of the ring DMA pieces and their spacing
KNOB = {k: int(os.environ.get("F4_" + k.upper(), v))
        for k, v in (("check", 96), ("dma0", 3), ("dmastep", 4), ("pro", 0), ("dqslots", 4), ("xnodma", 0),
                     ("xnodqr", 0), ("ringv", 0), ("rvl", 49), ("flagall", 0), ("xprep", 0), ("xend", 0),
                     ("xbar", 0), ("xexp", 0), ("pollpos", 0), ("xdmaconst", 0), ("chkpoll", 0))}  # x*: timing-only experiments (results wrong)

TILE_BYTES = 64 * 128
VLO = 96  # the statement's VGPRs: v[VLO:255]
FQT = 64
MF = "v_mfma_f32_16x16x32_bf16"


class Ins:
    __slots__ = ("text", "kind", "reads", "writes", "lds", "cost", "mfma_c", "passes")

    def __init__(self, text, kind, reads=(), writes=(), lds=False, cost=4, mfma_c=(), passes=4):
        self.text = text
        self.kind = kind  # mfma | valu | exp | ldsr | ldsw | cmp | nop | wait | salu
        self.reads = list(reads)  # physical registers ('v', n) / ('a', n)
        self.writes = list(writes)
        self.lds = lds
        self.cost = cost
        self.mfma_c = list(mfma_c)  # registers read as the accumulator input (chain)
        self.passes = passes


def vr(lo, n):
    return [("v", lo + i) for i in range(n)]


def ar(lo, n):
    return [("a", lo + i) for i in range(n)]


def rng(f, lo, n):
    return f"{f}[{lo}:{lo + n - 1}]" if n > 1 else f"{f}{lo}"


# ---------------------------------------------------------------- register plan
# VGPR temporaries
def ST(h, t4, qs):  # S^T accumulator tile (16 q x 16 keys) of half h, key tile t4, query sub-tile qs
    return 128 + 64 * h + 8 * t4 + 4 * qs


def DP(h, t4, qs):
    return 128 + 64 * h + 32 + 8 * t4 + 4 * qs


def LR(h, qs):  # lse2 rows (the S chain's initial value); half 1's reuse half 0's registers
    return 112 + 4 * qs


def DR(h, qs):  # delta rows
    return 112 + 8 + 4 * qs


# Persistent AGPRs (the whole work item; only this file's statements touch the AGPR file, the
# kernel's translation unit is built with -amdgpu-mfma-vgpr-form -amdgpu-spill-vgpr-to-agpr=0):
# dK^T[4 ds + t4] a[4 i : 4 i + 3], dV^T a[64 + 4 i ..], K'[2 t4 + ks] a[128 + 4 i ..], V' a[160 + 4 i ..]
def DK(i):
    return 4 * i


def DV(i):
    return 64 + 4 * i


def KF(i):
    return 128 + 4 * i


def VF(i):
    return 160 + 4 * i


# AGPR temporaries: the Q / dO row-fragment ring (3 slots x 8), the dO^T / Q^T fragments of half 0
# (4 x 8) and of half 1 (4 x 8, in the ring's registers once M1 is done + 8 spare)
def RING(s):
    return 192 + 8 * s


def TQ(h, ds):
    return (216 + 8 * ds) if h == 0 else (192, 200, 208, 248)[ds]


QA = 96  # the dQ^T accumulator (32 d x 32 q, v_mfma_f32_32x32x16_bf16): v[96:111]
MF32 = "v_mfma_f32_32x32x16_bf16"


def DQR(s):  # dQ operand ring (4 or 5 slots x 8): K^T fragment +0..3, dS^T fragment +4..7; tq_0's
    return (216, 224, 232, 240, 248)[s]  # registers (+ tq_1's last group), free until M1_1


def stamp(i):
    return Ins(f"s_memtime %[ts{i}]", "raw")


RING_SLOT = 2 * TILE_BYTES + 2 * FQT * 4
DS_BYTES = 256 * 128


def build(kind, local, prof=False, P=0):
    """Program order of one step: list of Ins (operand names in %[...]).  kind: 'full', 'masked' (PARTIAL
    tiles: the allowed query range of each key applied after the exponentials) or 'empty' (no key of
    the wave sees the tile: only the dQ products, zero -dS rows, the stores and the check)."""
    masked = kind == "masked"
    SL = P * RING_SLOT  # this tile's ring slot (t & 1 = P), the next tile's DMA goes to the other
    SN = (1 - P) * RING_SLOT
    pro = []  # before the first MFMA
    mf = []  # 128 16x16x32 MFMAs
    # ---- MFMA stream
    # M1_h: for ks, qs, t4: S, dP  (group (ks, qs) = ring group 4h + 2ks + qs)
    for h in range(2):
        for ks in range(2):
            for qs in range(2):
                g = 4 * h + 2 * ks + qs
                slot = RING(g % 3)
                for t4 in range(4):
                    d = ST(h, t4, qs)
                    c = LR(h, qs) if ks == 0 else d
                    mf.append(Ins(f"{MF} {rng('v', d, 4)}, {rng('a', slot, 4)}, {rng('a', KF(2 * t4 + ks), 4)}, {rng('v', c, 4)}",
                                  "mfma", reads=ar(slot, 4) + vr(c, 4), writes=vr(d, 4), mfma_c=vr(c, 4)))
                    d = DP(h, t4, qs)
                    c = DR(h, qs) if ks == 0 else d
                    mf.append(Ins(f"{MF} {rng('v', d, 4)}, {rng('a', slot + 4, 4)}, {rng('a', VF(2 * t4 + ks), 4)}, {rng('v', c, 4)}",
                                  "mfma", reads=ar(slot + 4, 4) + vr(c, 4), writes=vr(d, 4), mfma_c=vr(c, 4)))
    # M2_h: dV^T[ds][t4] += dO^T[ds] P^T[t4], dK^T[ds][t4] += Q^T[ds] (-dS)^T[t4]; key tile outer
    for h in range(2):
        for t4 in range(4):
            for ds in range(4):
                tq = TQ(h, ds)
                pf, sf = ST(h, t4, 0), DP(h, t4, 0)
                i = 4 * ds + t4
                mf.append(Ins(f"{MF} {rng('a', DV(i), 4)}, {rng('a', tq, 4)}, {rng('v', pf, 4)}, {rng('a', DV(i), 4)}",
                              "mfma", reads=ar(tq, 4) + vr(pf, 4) + ar(DV(i), 4), writes=ar(DV(i), 4), mfma_c=ar(DV(i), 4)))
                mf.append(Ins(f"{MF} {rng('a', DK(i), 4)}, {rng('a', tq + 4, 4)}, {rng('v', sf, 4)}, {rng('a', DK(i), 4)}",
                              "mfma", reads=ar(tq + 4, 4) + vr(sf, 4) + ar(DK(i), 4), writes=ar(DK(i), 4), mfma_c=ar(DK(i), 4)))
    assert len(mf) == 128
    # the previous tile's dQ^T[32 d x 32 q] += K^T[32 d x 16 keys] dS^T[16 keys x 32 q] over the item's
    # 256 keys (attn_bwd_fused_k's dq_mfma, same order): 16 MFMAs, one between every two of M1_0's
    dq = []
    NS = KNOB["dqslots"]
    for k2 in range(16):
        r = DQR(k2 % NS)
        dq.append(Ins(f"{MF32} {rng('v', QA, 16)}, {rng('a', r, 4)}, {rng('a', r + 4, 4)}, {rng('v', QA, 16)}", "mfma",
                      reads=ar(r, 8) + vr(QA, 16), writes=vr(QA, 16), mfma_c=vr(QA, 16), passes=8))
    stream = []  # (Ins, small index or None)
    for i in range(128):
        if i < 32 and i % 2 == KNOB["pro"]:
            stream.append((dq[i // 2], None))
        stream.append((mf[i], i))
    pos = {i: n for n, (_, i) in enumerate(stream) if i is not None}
    dpos = [n for n, (x, i) in enumerate(stream) if i is None]

    # ---- LDS reads
    def rd_group(g):  # Q row fragment (A of S) and dO row fragment (A of dP) of ring group g
        h, ks, qs = g // 4, (g // 2) & 1, g & 1
        row = 32 * h + 16 * qs
        slot = RING(g % 3)
        return [Ins(f"ds_read_b128 {rng('a', slot, 4)}, %[ar{ks}] offset:{SL + 128 * row}", "ldsr", writes=ar(slot, 4), lds=True),
                Ins(f"ds_read_b128 {rng('a', slot + 4, 4)}, %[ar{ks}] offset:{SL + TILE_BYTES + 128 * row}", "ldsr",
                    writes=ar(slot + 4, 4), lds=True)]

    def rd_rows(h):
        out = []
        for qs in range(2):
            row = 32 * h + 16 * qs
            out.append(Ins(f"ds_read_b128 {rng('v', LR(h, qs), 4)}, %[al] offset:{SL + 2 * TILE_BYTES + 4 * row}", "ldsr",
                           writes=vr(LR(h, qs), 4), lds=True))
            out.append(Ins(f"ds_read_b128 {rng('v', DR(h, qs), 4)}, %[al] offset:{SL + 2 * TILE_BYTES + 4 * FQT + 4 * row}",
                           "ldsr", writes=vr(DR(h, qs), 4), lds=True))
        return out

    def rd_tr(h, ds):  # dO^T (A of dV^T) and Q^T (A of dK^T) of column group ds, permuted k order
        tq = TQ(h, ds)
        o = SL + 4096 * h
        return [Ins(f"ds_read_b64_tr_b16 {rng('a', tq, 2)}, %[tr{ds}] offset:{TILE_BYTES + o}", "ldsr", writes=ar(tq, 2), lds=True),
                Ins(f"ds_read_b64_tr_b16 {rng('a', tq + 2, 2)}, %[tr{ds}] offset:{TILE_BYTES + o + 2048}", "ldsr",
                    writes=ar(tq + 2, 2), lds=True),
                Ins(f"ds_read_b64_tr_b16 {rng('a', tq + 4, 2)}, %[tr{ds}] offset:{o}", "ldsr", writes=ar(tq + 4, 2), lds=True),
                Ins(f"ds_read_b64_tr_b16 {rng('a', tq + 6, 2)}, %[tr{ds}] offset:{o + 2048}", "ldsr",
                    writes=ar(tq + 6, 2), lds=True)]

    def rd_dq(k2):  # K^T (image rows 16 k2 ..) and dS^T fragments of dQ k-step k2 (frag_tr of attn_bwd_fused_k)
        r = DQR(k2 % NS)
        # (the dS image of tile t + 1: the other one)
        # K^T fragment: one ds_read_b128 of the lane-linear fragment image (attn_bwd_fused4.hip)
        return [Ins(f"ds_read_b128 {rng('a', r, 4)}, %[kf] offset:{1024 * k2}", "ldsr", writes=ar(r, 4), lds=True)] + \
            [Ins(f"ds_read_b64_tr_b16 {rng('a', r + 2 * i, 2)}, %[{nm}] offset:{2048 * k2 + (1 - P) * DS_BYTES}",
                 "ldsr", writes=ar(r + 2 * i, 2), lds=True) for i, nm in ((2, "sa"), (3, "sb"))]

    def rd_qacc():  # the dQ sum so far (predecessor's, zeros or NaN), lane-linear in the landing zone
        return [Ins(f"ds_read_b128 {rng('v', QA + 4 * e, 4)}, %[qa] offset:{1024 * e}", "ldsr", writes=vr(QA + 4 * e, 4),
                    lds=True) for e in range(4)]

    # ---- softmax-gradient VALU of (h, t4), then its two -dS row writes
    def chunk(h, t4):
        out = []
        st0, dp0 = ST(h, t4, 0), DP(h, t4, 0)
        for i in range(8):  # P = exp2(-(lse2 - c s))
            out.append(Ins(f"v_exp_f32_e64 v{st0 + i}, -v{st0 + i}" if not KNOB["xexp"] else f"v_mov_b32 v{st0 + i}, v{st0 + i}",
                           "exp", reads=vr(st0 + i, 1), writes=vr(st0 + i, 1), cost=8))
        if masked:
            # query row 32 h + 16 qs + 4 g + r of the tile is allowed for key tile t4 iff lo <= . < hi,
            # with %[mlo{t4}] / %[mhi{t4}] = bound - 4 g (per lane)
            for qs in range(2):
                for r in range(4):
                    q = 32 * h + 16 * qs + r
                    reg = st0 + 4 * qs + r
                    out.append(Ins(f"v_cmp_ge_i32_e32 vcc, {q}, %[mlo{t4}]", "cmp"))
                    out.append(Ins("s_nop 1", "nop", cost=8))
                    out.append(Ins(f"v_cndmask_b32_e32 v{reg}, 0, v{reg}, vcc", "valu", reads=vr(reg, 1), writes=vr(reg, 1)))
                    out.append(Ins(f"v_cmp_lt_i32_e32 vcc, {q}, %[mhi{t4}]", "cmp"))
                    out.append(Ins("s_nop 1", "nop", cost=8))
                    out.append(Ins(f"v_cndmask_b32_e32 v{reg}, 0, v{reg}, vcc", "valu", reads=vr(reg, 1), writes=vr(reg, 1)))
        for i in range(8):  # dP - delta (accumulated as delta - dO v') times P: -dS
            out.append(Ins(f"v_mul_f32_e32 v{dp0 + i}, v{dp0 + i}, v{st0 + i}", "valu", reads=vr(dp0 + i, 1) + vr(st0 + i, 1),
                           writes=vr(dp0 + i, 1)))
        for base in (st0, dp0):  # pack_perm in place: word w = bf16(x[2w]) | bf16(x[2w + 1]) << 16
            for wd in range(4):
                out.append(Ins(f"v_cvt_pk_bf16_f32 v{base + wd}, v{base + 2 * wd}, v{base + 2 * wd + 1}", "valu",
                               reads=vr(base + 2 * wd, 2), writes=vr(base + wd, 1)))
        # -dS rows of keys 16 t4 + c into the image: queries 32 h + 4 g .. (e 0), 32 h + 16 + 4 g .. (e 1)
        out.append(Ins(f"ds_write_b64 %[ds{2 * h}], {rng('v', dp0, 2)} offset:{P * DS_BYTES + 2048 * t4}", "ldsw",
                       reads=vr(dp0, 2), lds=True, cost=8))
        out.append(Ins(f"ds_write_b64 %[ds{2 * h + 1}], {rng('v', dp0 + 2, 2)} offset:{P * DS_BYTES + 2048 * t4}", "ldsw",
                       reads=vr(dp0 + 2, 2), lds=True, cost=8))
        return out

    # ---- the dQ stores (after the last dQ MFMA): mode 0 = the fp32 sum (4 x 16 B per lane into the
    # chain's accumulator, lane-linear; write-through unless local), 1 = the tile's last contributor's
    # bf16 dQ rows (-scale folded in; 4 x 8 B per lane, rows past L addressed out of the buffer's range)
    def stores():
        pol = "" if local else " sc1"
        t = ["s_bitcmp1_b32 %[fl], 0", "s_cbranch_scc1 .Lf4bf%="]
        t += [f"buffer_store_dwordx4 {rng('v', QA + 4 * e, 4)}, %[soffa], %[rsrc], %[soffs] offen offset:{1024 * e}{pol}"
              for e in range(4)]
        t += ["s_branch .Lf4st%=", ".Lf4bf%=:"]
        t += [f"v_mul_f32_e32 v{QA + i}, %[nscale], v{QA + i}" for i in range(16)]
        t += [f"v_cvt_pk_bf16_f32 v{QA + i}, v{QA + 2 * i}, v{QA + 2 * i + 1}" for i in range(8)]
        t += [f"buffer_store_dwordx2 {rng('v', QA + 2 * rr, 2)}, %[soffr], %[rsrc], %[soffs] offen offset:{16 * rr}"
              for rr in range(4)]
        t += [".Lf4st%=:"]
        return [Ins("\n".join(t), "raw", reads=vr(QA, 16), writes=vr(QA, 16))]

    # ---- the hand-off check of the tile this step sweeps: its flag (polled by LDS-DMA before the
    # statement) against want (INT_MAX when the tile has no predecessor to wait for); on a match the predecessor's sum goes to the landing zone (4 LDS-DMA
    # pieces, sc1), to be consumed by the next step.  The dQ stores are the 4 youngest vector-memory
    # operations here, so vmcnt(4) waits for the poll (and the ring's DMA, issued before it)
    def check(ringw=False):
        tmp = LR(0, 0)
        # (a poll placed after the dQ stores: nothing younger than it at the check)
        out = [Ins("s_waitcnt vmcnt(0)" if KNOB["pollpos"] > 32 and kind != "empty" else "s_waitcnt vmcnt(4)", "raw")]
        if KNOB["chkpoll"] and kind != "empty" and not KNOB["pollpos"]:
            # wait for the poll alone: the ring's DMA (4 or 5 pieces, flags bit 1) and the dQ stores
            # after it may still fly (the end of the step waits for them)
            out = [Ins("s_bitcmp1_b32 %[fl], 1\ns_cbranch_scc0 .Lf4c4%=\ns_waitcnt vmcnt(8)\ns_branch .Lf4c5%=\n"
                       ".Lf4c4%=:\ns_waitcnt vmcnt(4)\n.Lf4c5%=:", "raw")]
        if ringw:  # the next tile's ring rows, staged in v[112:127] / v96 since rvl, into the other slot
            t = ["s_waitcnt vmcnt(0)", "s_bitcmp1_b32 %[fl], 1", "s_cbranch_scc0 .Lf4rw%="]
            t += [f"ds_write_b128 %[rq], {rng('v', 112 + 4 * i, 4)} offset:{SN + (TILE_BYTES if i >= 2 else 0) + 1024 * (i % 2)}"
                  for i in range(4)]
            t += ["s_bitcmp1_b32 %[fl], 2", "s_cbranch_scc0 .Lf4rw%=", f"ds_write_b32 %[rl], v96 offset:{SN}", ".Lf4rw%=:"]
            out = [Ins("\n".join(t), "raw", reads=vr(112, 16) + vr(96, 1))]  # (LDS ops not counted: later waits over-wait)
        out += [
               Ins(f"ds_read_b32 v{tmp}, %[flagv]", "ldsr", writes=vr(tmp, 1), lds=True),
               Ins(f"v_readfirstlane_b32 %[tmp], v{tmp}", "valu", reads=vr(tmp, 1))]
        t = ["s_nop 3", "s_mov_b32 %[lout], 0",
             "s_cmp_lt_i32 %[tmp], %[want]", "s_cbranch_scc1 .Lf4np%=", "s_mov_b32 %[lout], 1",
             "s_mov_b32 m0, %[m0a]", "s_nop 0"]
        t += [f"global_load_lds_dwordx4 %[soffa], %[sumbase] offset:{1024 * e} sc1" for e in range(4)]
        t += [".Lf4np%=:"]
        out.append(Ins("\n".join(t), "raw"))
        return out

    # the flag of this step's tile, polled by LDS-DMA (sc1) at the statement's top: every lane loads the
    # word into its slot of the wave's flag area; checked at the top of M2_0
    poll = [Ins("s_mov_b32 m0, %[m0f]\ns_nop 0\nglobal_load_lds_dword %[zero], %[fb] sc1", "raw")]

    # the ring's LDS-DMA of the next tile (t - 1, into the other slot): 2 Q + 2 dO rows-pieces per wave
    # (rows 16 w + 8 h ..), the lse2 (wave 0) / delta (wave 1) row; flags bit 1 / bit 2
    def dma_piece(i):
        if KNOB["xnodma"]:
            return Ins("s_nop 0", "raw")
        if i < 4:
            src, off = ("qb", f"qo{i % 2}") if i < 2 else ("ob", f"oo{i % 2}")
            dst = SN + (TILE_BYTES if i >= 2 else 0) + 1024 * (i % 2)
            t = ["s_bitcmp1_b32 %[fl], 1", f"s_cbranch_scc0 .Lf4d{i}%=", f"s_add_u32 m0, %[m0q], {dst}", "s_nop 0",
                 f"global_load_lds_dwordx4 %[{off}], %[{src}]", f".Lf4d{i}%=:"]
        else:
            t = ["s_bitcmp1_b32 %[fl], 2", f"s_cbranch_scc0 .Lf4d{i}%=", f"s_add_u32 m0, %[m0l], {SN}", "s_nop 0",
                 "global_load_lds_dword %[lo], %[lb]", f".Lf4d{i}%=:"]
        return Ins("\n".join(t), "raw")

    if kind == "empty":
        zero = [Ins("v_mov_b32 v112, 0", "valu", writes=vr(112, 1)), Ins("v_mov_b32 v113, 0", "valu", writes=vr(113, 1))]
        zero += [Ins(f"ds_write_b64 %[ds{i}], v[112:113] offset:{P * DS_BYTES + 2048 * t4}", "ldsw", reads=vr(112, 2), lds=True)
                 for t4 in range(4) for i in range(4)]
        fill = [[] for _ in range(17)]
        for k2 in range(13):
            fill[k2 + 1] += rd_dq(k2 + 3)
        fill[1] += zero[:2]
        for n in range(8):
            fill[n + 1] += zero[2 + 2 * n:4 + 2 * n]
        for i in range(5):
            fill[2 + 2 * i].append(dma_piece(i))
        prog = [Ins("s_waitcnt lgkmcnt(0)", "wait"), Ins("s_nop 3", "nop")] + poll + rd_qacc() + rd_dq(0) + rd_dq(1) + rd_dq(2)
        for n in range(16):
            prog += fill[n]
            prog.append(dq[n])
        prog += fill[16] + stores() + check()
        return prog

    # ---- placement: fill[n] = instructions issued right before stream entry n
    N = len(stream)
    fill = [[] for _ in range(N + 1)]
    # prologue: the dQ sum, dQ k-step 0, rows and ring group 0 of half 0, k-step 1, ring group 1, k-step 2
    # (pro 1: the first S / dP operands first, and the stream opens with two 16x16x32 MFMAs)
    ahead = NS - 1
    if KNOB["pro"]:
        pro += rd_rows(0)[0:2] + rd_group(0) + rd_qacc() + rd_dq(0) + rd_rows(0)[2:4] + rd_group(1)
        pro += sum((rd_dq(k) for k in range(1, ahead)), [])
    else:
        pro += rd_qacc() + rd_dq(0) + rd_rows(0)[0:2] + rd_group(0) + rd_rows(0)[2:4] + rd_dq(1) + rd_group(1)
        pro += sum((rd_dq(k) for k in range(2, ahead)), [])
    # dQ k-step k2 + NS - 1 right after dQ MFMA k2 (NS-slot ring)
    for k2 in range(16 - ahead):
        fill[dpos[k2] + 1] += rd_dq(k2 + ahead)
    # ring groups 2 .. 7, two groups ahead of their first MFMA (group g's MFMAs are 8 g .. 8 g + 7)
    for g in range(2, 8):
        fill[pos[8 * (g - 2) + 1]] += rd_group(g)
    # lse2 / delta rows of half 1 (for MFMA 32), into half 0's row registers once its chains have
    # read them (MFMAs 0 .. 15)
    fill[pos[19]] += rd_rows(1)
    # the dQ stores after M1_0 (12 wait states after the last 32x32x16 MFMA, padded by finalize)
    fill[pos[32]] += stores()
    # dO^T / Q^T of half 0 (first use MFMA 64) during M1_1, in the dQ ring's registers (free after M1_0);
    # of half 1 (ring registers, free after MFMA 63) during M2_0 (first use 96)
    for ds in range(4):
        fill[pos[36 + 6 * ds]] += rd_tr(0, ds)
        fill[pos[66 + 6 * ds]] += rd_tr(1, ds)
    if KNOB["ringv"]:  # the ring rows by plain loads into v[112:127] (free after half 1's first chains) / v96
        t = ["s_bitcmp1_b32 %[fl], 1", "s_cbranch_scc0 .Lf4rv%="]
        t += [f"global_load_dwordx4 {rng('v', 112 + 4 * i, 4)}, %[{('qo', 'oo')[i // 2]}{i % 2}], %[{('qb', 'ob')[i // 2]}]"
              for i in range(4)]
        t += ["s_bitcmp1_b32 %[fl], 2", "s_cbranch_scc0 .Lf4rv%=", "global_load_dword v96, %[lo], %[lb]", ".Lf4rv%=:"]
        fill[pos[KNOB["rvl"]]].append(Ins("\n".join(t), "raw", writes=vr(112, 16) + vr(96, 1)))
        fill[pos[KNOB["check"]]] = check(True) + fill[pos[KNOB["check"]]]
    else:
        fill[pos[KNOB["check"]]] = check() + fill[pos[KNOB["check"]]]
        for i in range(5):  # the ring's DMA between the MFMAs of M1_0 + dQ (no VALU there)
            fill[pos[KNOB["dma0"] + KNOB["dmastep"] * i]].append(dma_piece(i))
    if prof:  # s_memtime at the block boundaries (SMEM: one outstanding keeps every lgkmcnt wait safe)
        fill[pos[32]].append(stamp(1))
        fill[pos[64]].insert(0, stamp(2))  # (after a check placed at 64)
        fill[pos[96]].insert(0, stamp(3))
    # VALU: half 0 chunks paced over MFMAs 33 .., half 1 after; chunk (h, t4) due before MFMA 64 + 32 h + 8 t4
    vstream = []
    for h in range(2):
        for t4 in range(4):
            vstream.append(((h, t4), chunk(h, t4)))
    lo_gap, hi_gap = 33, 118
    total = sum(len(c) for _, c in vstream)
    k = 0
    for (h, t4), ins in vstream:
        due = 64 + 32 * h + 8 * t4 - 1
        first = 33 if h == 0 else 65
        for x in ins:
            gap = lo_gap + (k * (hi_gap - lo_gap)) // total
            gap = max(gap, first)
            gap = min(gap, due)
            fill[pos[gap]].append(x)
            k += 1
    if KNOB["pollpos"]:
        fill[pos[KNOB["pollpos"]]] += poll
    prog = [Ins("s_waitcnt lgkmcnt(0)", "wait"), Ins("s_nop 3", "nop")] + ([stamp(0)] if prof else []) + \
        ([] if KNOB["pollpos"] else poll) + pro
    for n in range(N):
        prog += fill[n]
        prog.append(stream[n][0])
    prog += fill[N]
    if prof:
        prog += [stamp(4), Ins("s_waitcnt lgkmcnt(0)", "wait")]
    return prog


def finalize(prog, allow_pending=False):
    """Insert lgkmcnt waits and hazard nops; returns the instruction texts and statistics.  allow_pending:
    LDS loads may still fly at the end (the caller drains them with lgkmcnt(0) before their use)."""
    out = []
    # LDS bookkeeping
    issued = 0          # LDS ops issued so far
    done_upto = 0       # all LDS ops with index < done_upto are known complete
    pending = {}        # register -> LDS op index that writes it (loads not yet waited for)
    # hazard bookkeeping: per register (position in wait states) of last write / MFMA access
    pos = 0
    last_w = {}   # reg -> (pos, kind)
    last_mfma = {}  # reg -> pos of the last MFMA reading it as the accumulator or writing it
    last_ab = {}    # reg -> pos of the last MFMA reading it as the A / B operand
    nops = waits = 0

    def ws_since(p):
        return pos - p - 1  # instructions strictly between

    for ins in prog:
        if ins.kind == "wait":
            out.append(ins.text)
            pos += 1
            if "lgkmcnt(0)" in ins.text:
                done_upto = issued
                pending.clear()
            continue
        # 1. LDS results this instruction consumes
        need = -1
        for r in ins.reads:
            if r in pending:
                need = max(need, pending[r])
        if ins.lds and ins.kind == "ldsr":
            # WAR on its destination against an older LDS read of the same registers is ordered (in-order)
            pass
        if need >= done_upto:
            cnt = issued - need - 1
            cnt = min(cnt, 15)
            out.append(f"s_waitcnt lgkmcnt({cnt})")
            waits += 1
            pos += 1
            done_upto = issued - cnt
            for r in list(pending):
                if pending[r] < done_upto:
                    del pending[r]
        # 2. hazards
        pad = 0
        if ins.kind == "mfma":
            for r in ins.reads:
                if r in ins.mfma_c and last_w.get(r, (-99, "", 0))[1] == "mfma":
                    continue  # accumulate chain
                w = last_w.get(r)
                if w and w[1] in ("valu", "exp"):
                    pad = max(pad, 2 - ws_since(w[0]))
                if w and w[1] == "mfma":
                    pad = max(pad, w[2] + 4 - ws_since(w[0]))
            for r in ins.writes:
                w = last_w.get(r)
                if w and w[1] in ("valu", "exp"):
                    pad = max(pad, 2 - ws_since(w[0]))
        else:
            for r in ins.reads:
                w = last_w.get(r)
                if w and w[1] == "mfma":
                    pad = max(pad, w[2] - ws_since(w[0]))
            for r in ins.writes:
                m = last_mfma.get(r)
                if m is not None:
                    pad = max(pad, 12 - ws_since(m))
                m = last_ab.get(r)
                if m is not None:
                    pad = max(pad, 2 - ws_since(m))
        while pad > 0:
            n = min(pad, 8)
            out.append(f"s_nop {n - 1}")
            pos += n
            pad -= n
            nops += 1
        # 3. issue (a raw block -- branches, stores -- counts as one wait state: its shortest path)
        out += ins.text.split("\n")
        if ins.lds:
            idx = issued
            issued += 1
            if ins.kind == "ldsr":
                for r in ins.writes:
                    pending[r] = idx
        for r in ins.writes:
            last_w[r] = (pos, "mfma" if ins.kind == "mfma" else ("ld" if ins.kind == "ldsr" else "valu"),
                         12 if ins.passes == 8 else 8)
        if ins.kind == "mfma":
            for r in ins.mfma_c + ins.writes:
                last_mfma[r] = pos
            for r in ins.reads:
                if r not in ins.mfma_c:
                    last_ab[r] = pos
        m = re.match(r"s_nop (\d+)", ins.text)
        pos += int(m.group(1)) + 1 if m else 1
    # end: the last MFMAs' results / operands are the compiler's again after the statement
    out.append("s_nop 7")
    out.append("s_nop 3")
    assert allow_pending or not pending, "LDS loads never waited for"
    return out, dict(nops=nops, waits=waits, instrs=len(out))


VOPS = ["ar0", "ar1", "al", "tr0", "tr1", "tr2", "tr3", "ds0", "ds1", "ds2", "ds3", "qa", "kf", "sa", "sb", "soffa",
        "soffr", "flagv", "qo0", "qo1", "oo0", "oo1", "lo", "zero", "rq", "rl"]
SOPS = [("rsrc", "__amdgpu_buffer_rsrc_t"), ("fl", "int"), ("nscale", "float"), ("want", "int"), ("soffs", "int"),
        ("sumbase", "const void*"), ("m0a", "unsigned"), ("m0f", "unsigned"), ("m0q", "unsigned"), ("m0l", "unsigned"),
        ("qb", "const void*"), ("ob", "const void*"), ("lb", "const void*"), ("fb", "const void*")]


def operand_decl(kind, prof=False):
    masked = kind == "masked"
    outs = ['[lout] "=&s"(lout)', '[tmp] "=&s"(tmp)']
    if prof:
        outs += [f'[ts{i}] "=&s"(ts[{i}])' for i in range(5)]
    ins = []
    for n in VOPS:
        fld = f"{n[:-1]}[{n[-1]}]" if n[:-1] in ("tr", "ds", "qo", "oo") else n
        fld = {"ds": "dsa"}.get(fld.split("[")[0], fld.split("[")[0]) + (fld[fld.index("["):] if "[" in fld else "")
        ins.append(f'[{n}] "v"(f.{fld})')
    ins += [f'[{n}] "s"(s.{n})' for n, _ in SOPS]
    if masked:
        ins += [f'[mlo{i}] "v"(f.mlo[{i}])' for i in range(4)] + [f'[mhi{i}] "v"(f.mhi[{i}])' for i in range(4)]
    clob = ['"memory"', '"m0"', '"scc"'] + [f'"v{i}"' for i in range(VLO, 256)] + [f'"a{i}"' for i in range(256)]
    if masked:
        clob.append('"vcc"')
    return outs, ins, clob


def emit_function(name, kind, local, P):
    out = []
    for prof in (True, False):
        prog = build(kind, local, prof and kind != "empty", P)
        lines, st = finalize(prog)
        outs, ins, clob = operand_decl(kind, prof and kind != "empty")
        body = "\n".join(f'      "{l}\\n"' for l in lines)
        out.append(f"""// {name}: {st['instrs']} lines, {st['waits']} lgkmcnt waits, {st['nops']} hazard nops; returns whether the
// landing zone's 4 loads were issued (they are the youngest vector-memory operations then)
__attribute__((always_inline)) DEV int {name}(const F4Lane& f, const F4Scalar& s, unsigned long long (&ts)[5]) {{
  int lout, tmp;
  asm volatile(
{body}
      : {", ".join(outs)}
      : {", ".join(ins)}
      : {", ".join(clob)});
  return lout;
}}
""")
    s = ("#if OWLK_FUSED_PROF  // timing-only builds: s_memtime at the MFMA-block boundaries\n" + out[0] +
         "#else\n" + out[1] + "#endif\n")
    return s, st


def emit_run(local):
    """fused4_run_<local|wt>: n steps over FULL tiles with uniform conditions (the fp32 sum as the dQ store
    target, the ring DMA on, the predecessor check either on for every step (flags bit 3) or off) as ONE
    statement: per step the landing zone (vmcnt wait, or zeros without a predecessor), the step body of
    the tile's parity, the end-of-step wait, the barrier and the flag of tile t + 1, then every pointer
    moved back one tile -- no scalar work of the compiler's between steps.  Stops before a step whose
    predecessor's sum was not seen by the previous step's check (lout 0 with bit 3 set): the caller's
    loop then polls.  Returns the steps left; lout = the last step's check result."""
    bodies = {}
    for P in (0, 1):
        lines, st = finalize(build("full", local, False, P))
        bodies[P] = [l.replace("%=", f"%=q{P}") for l in lines]
    # (entry: the caller's last step left only its landing-zone loads, or none, in flight)
    t = ["s_waitcnt vmcnt(0)", "s_cmp_eq_u32 %[par], 0", "s_cbranch_scc0 .Lf4L1%="]
    for P in (0, 1):
        t += [f".Lf4L{P}%=:", "s_bitcmp1_b32 %[fl], 3", f"s_cbranch_scc0 .Lf4z{P}%=",
              "s_cmp_eq_u32 %[lout], 0", "s_cbranch_scc1 .Lf4x%=",
              "s_nop 0" if KNOB["xprep"] else ("s_waitcnt vmcnt(1)" if KNOB["flagall"] else "s_waitcnt vmcnt(0)"),
              f"s_branch .Lf4pd{P}%=", f".Lf4z{P}%=:"]
        t += [f"v_mov_b32 v{112 + i}, 0" for i in range(4)]
        t += [f"ds_write_b128 %[qa], v[112:115] offset:{1024 * e}" for e in range(4)]
        t += [f".Lf4pd{P}%=:"] + bodies[P]
        if KNOB["xend"]:
            t += ["s_waitcnt lgkmcnt(0)", "s_barrier"]
        else:
            t += ["s_cmp_eq_u32 %[lout], 0", f"s_cbranch_scc1 .Lf4v{P}%=", "s_waitcnt vmcnt(4)", f"s_branch .Lf4w{P}%=",
                  f".Lf4v{P}%=:", "s_waitcnt vmcnt(0)", f".Lf4w{P}%=:", "s_waitcnt lgkmcnt(0)", "s_barrier"]
        if KNOB["xbar"]:
            t[-1] = "s_nop 0"
        t += [
              # lane 0 of wave 0 raises the flag of tile t + 1 (every wave's dQ stores are done)
              ] + (["s_cmp_eq_u32 %[wid], 0", f"s_cbranch_scc0 .Lf4f{P}%="] if not KNOB["flagall"] else []) + [
              "s_mov_b64 s[78:79], exec", "s_mov_b64 exec, 1",
              "global_store_dword %[zero], %[fval], %[fb] offset:64 sc1", "s_mov_b64 exec, s[78:79]", f".Lf4f{P}%=:",
              ] + ([] if KNOB["xdmaconst"] else [
              "s_sub_u32 s64, s64, %[qstep]", "s_subb_u32 s65, s65, 0",
              "s_sub_u32 s66, s66, %[ostep]", "s_subb_u32 s67, s67, 0",
              "s_sub_u32 s68, s68, 256", "s_subb_u32 s69, s69, 0"]) + [
              "s_sub_u32 s70, s70, 64", "s_subb_u32 s71, s71, 0",
              "s_sub_u32 s72, s72, 0x4000", "s_subb_u32 s73, s73, 0",
              "s_sub_u32 s74, s74, 0x4000",
              "s_sub_u32 s75, s75, 1", "s_cmp_eq_u32 s75, 0", "s_cbranch_scc1 .Lf4x%="]
        if P == 1:
            t.append("s_branch .Lf4L0%=")
    t.append(".Lf4x%=:")
    outs = ['[lout] "+{s76}"(lout)', '[tmp] "=&s"(tmp)', '[n] "+{s75}"(n)', '[qb] "+{s[64:65]}"(qb)',
            '[ob] "+{s[66:67]}"(ob)', '[lb] "+{s[68:69]}"(lb)', '[fb] "+{s[70:71]}"(fb)', '[sumbase] "+{s[72:73]}"(sumbase)',
            '[soffs] "+{s74}"(soffs)']
    _, ins, clob = operand_decl("full")
    ins = [x for x in ins if not any(x.startswith(f"[{k}]") for k in ("qb", "ob", "lb", "fb", "sumbase", "soffs"))]
    ins += ['[par] "s"(par)', '[qstep] "s"(qstep)', '[ostep] "s"(ostep)', '[fval] "v"(fval)', '[wid] "s"(wid)']
    clob = clob + ['"s78"', '"s79"']
    body = "\n".join(f'      "{l}\\n"' for l in t)
    nm = f"fused4_run_{'local' if local else 'wt'}"
    return f"""// {nm}: {len(t)} lines
__attribute__((always_inline)) DEV int {nm}(int n, int par, int& lout, const F4Lane& f, const F4Scalar& s,
                                            unsigned qstep, unsigned ostep, unsigned fval, int wid) {{
  int tmp;
  const void *qb = s.qb, *ob = s.ob, *lb = s.lb, *fb = s.fb, *sumbase = s.sumbase;
  int soffs = s.soffs;
  asm volatile(
{body}
      : {", ".join(outs)}
      : {", ".join(ins)}
      : {", ".join(clob)});
  return n;
}}
"""


def emit_helpers():
    """fused4_agpr_init: dK^T / dV^T = 0 and the K' / V' fragments into their AGPRs (once per item);
    fused4_acc_read<I>: dK^T[I] and dV^T[I] (I = 4 ds + t4) back into VGPRs for the epilogue."""
    w = [f'"v_accvgpr_write_b32 a{i}, 0\\n"' for i in range(128)]
    ops = []
    for i in range(8):
        for e in range(4):
            w.append(f'"v_accvgpr_write_b32 a{KF(i) + e}, %[k{i}_{e}]\\n"')
            w.append(f'"v_accvgpr_write_b32 a{VF(i) + e}, %[v{i}_{e}]\\n"')
            ops.append(f'[k{i}_{e}] "v"(k[{i}][{e}])')
            ops.append(f'[v{i}_{e}] "v"(v[{i}][{e}])')
    w.append('"s_nop 3\\n"')
    clob = ['"memory"'] + [f'"a{i}"' for i in range(192)]
    s = ("// dK^T, dV^T = 0; K' / V' fragments (as 32-bit words) into a[128:191]\n"
         "__attribute__((always_inline)) DEV void fused4_agpr_init(const u32x4 (&k)[8], const u32x4 (&v)[8]) {\n"
         "  asm volatile(\n      " + "\n      ".join(w) + "\n      :\n      : " + ", ".join(ops) +
         "\n      : " + ", ".join(clob) + ");\n}\n")
    s += "// dK^T[I] -> o[0..3], dV^T[I] -> o[4..7] (the last MFMA that wrote them is >= 12 wait states back)\n"
    s += "template <int I>\n__attribute__((always_inline)) DEV void fused4_acc_read(float (&o)[8]);\n"
    for i in range(16):
        rd = [f'"v_accvgpr_read_b32 %{e}, a{DK(i) + e}\\n"' for e in range(4)] + \
             [f'"v_accvgpr_read_b32 %{4 + e}, a{DV(i) + e}\\n"' for e in range(4)]
        s += (f"template <>\n__attribute__((always_inline)) DEV void fused4_acc_read<{i}>(float (&o)[8]) {{\n"
              f"  asm volatile(" + " ".join(rd) + " : " + ", ".join(f'"=v"(o[{e}])' for e in range(8)) + ");\n}\n")
    return s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stats", action="store_true")
    args = ap.parse_args()
    parts = []
    for kind in ("full", "masked", "empty"):
        for local in (True, False):
            for P in (0, 1):
                name = f"fused4_step_{kind}_{'local' if local else 'wt'}_p{P}"
                s, st = emit_function(name, kind, local, P)
                print(f"{name}: {st}", file=sys.stderr)
                parts.append(s)
    disp = ["// the statement of a step: tile kind (TILE_FULL / TILE_PARTIAL / TILE_EMPTY), hand-off form, ring parity",
            "template <int KIND, bool LOCAL>",
            "__attribute__((always_inline)) DEV int fused4_step(int parity, const F4Lane& f, const F4Scalar& s,",
            "                                                 unsigned long long (&ts)[5]) {"]
    for kind, kv in (("full", "TILE_FULL"), ("masked", "TILE_PARTIAL"), ("empty", "TILE_EMPTY")):
        for local in (True, False):
            nm = f"fused4_step_{kind}_{'local' if local else 'wt'}"
            disp.append(f"  if constexpr (KIND == {kv} && {'LOCAL' if local else '!LOCAL'})")
            disp.append(f"    return parity ? {nm}_p1(f, s, ts) : {nm}_p0(f, s, ts);")
    disp += ["  return 0;", "}", ""]
    disp += ["#if !OWLK_FUSED_PROF", emit_run(True), emit_run(False), "#endif", ""]
    if args.stats:
        return
    hdr = ("// GENERATED by tools/gen_fused4_asm.py -- do not edit.  The hand-placed step of\n"
           "// attn_bwd_fused4_k (attn_bwd_fused4.hip): see the generator's docstring for the schedule.\n"
           "#pragma once\n\n"
           "// per-lane operands (VGPR; constant per item): LDS byte addresses of the Q / dO row reads (ks 0 / 1),\n"
           "// the lse2 / delta rows, the dO^T / Q^T reads, the -dS rows (slot / image 0: the other parity is an\n"
           "// immediate), the landing zone, the K^T and dS^T reads of dQ; dQ store offsets (fp32 sum / bf16 rows),\n"
           "// the polled flag; the ring DMA's source offsets (Q / dO rows h, lse2 or delta); a zero\n"
           "struct F4Lane {\n"
           "  unsigned ar0, ar1, al, tr[4], dsa[4], qa, kf, sa, sb, soffa, soffr, flagv, qo[2], oo[2], lo, zero, rq, rl;\n"
           "  int mlo[4], mhi[4];  // PARTIAL tiles: allowed query rows per key tile, relative to the tile, - 4 g\n"
           "};\n"
           "// wave-uniform operands (SGPR): the dQ store target (accumulator / dq rows / none) with flags bit 0 =\n"
           "// bf16 rows (the tile's last contributor), bit 1 = issue the ring's DMA, bit 2 = the lse2 / delta\n"
           "// piece; -scale; the check's want (INT_MAX: no check); the stores' soffset; the tile's sum in the\n"
           "// workspace; M0 bases (landing zone, flag area, ring rows of this wave, lse2 / delta row); DMA sources\n"
           "struct F4Scalar {\n"
           "  __amdgpu_buffer_rsrc_t rsrc;\n"
           "  int fl;\n"
           "  float nscale;\n"
           "  int want, soffs;\n"
           "  const void* sumbase;\n"
           "  unsigned m0a, m0f, m0q, m0l;\n"
           "  const void *qb, *ob, *lb, *fb;\n"
           "};\n\n")
    with open(OUT, "w") as f:
        f.write(hdr + emit_helpers() + "\n" + "\n".join(parts) + "\n" + "\n".join(disp))
    print("wrote", OUT, file=sys.stderr)


if __name__ == "__main__":
    main()
