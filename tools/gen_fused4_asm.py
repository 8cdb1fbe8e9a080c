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

Registers are fixed here, not by hipcc: the statement clobbers v[96:255] and a[192:255]; the
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

TILE_BYTES = 64 * 128
FQT = 64
MF = "v_mfma_f32_16x16x32_bf16"


class Ins:
    __slots__ = ("text", "kind", "reads", "writes", "lds", "cost", "mfma_c")

    def __init__(self, text, kind, reads=(), writes=(), lds=False, cost=4, mfma_c=()):
        self.text = text
        self.kind = kind  # mfma | valu | exp | ldsr | ldsw | cmp | nop | wait | salu
        self.reads = list(reads)  # physical registers ('v', n) / ('a', n)
        self.writes = list(writes)
        self.lds = lds
        self.cost = cost
        self.mfma_c = list(mfma_c)  # registers read as the accumulator input (chain)


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


def LR(h, qs):  # lse2 rows (the S chain's initial value)
    return 96 + 16 * h + 4 * qs


def DR(h, qs):  # delta rows
    return 96 + 16 * h + 8 + 4 * qs


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


def build(masked):
    """Program order of one step: list of Ins (operand names in %[...])."""
    pro = []  # before MFMA 0
    mf = []  # 128 MFMAs
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

    # ---- LDS reads
    def rd_group(g):  # Q row fragment (A of S) and dO row fragment (A of dP) of ring group g
        h, ks, qs = g // 4, (g // 2) & 1, g & 1
        row = 32 * h + 16 * qs
        slot = RING(g % 3)
        return [Ins(f"ds_read_b128 {rng('a', slot, 4)}, %[ar{ks}] offset:{128 * row}", "ldsr", writes=ar(slot, 4), lds=True),
                Ins(f"ds_read_b128 {rng('a', slot + 4, 4)}, %[ar{ks}] offset:{TILE_BYTES + 128 * row}", "ldsr",
                    writes=ar(slot + 4, 4), lds=True)]

    def rd_rows(h):
        out = []
        for qs in range(2):
            row = 32 * h + 16 * qs
            out.append(Ins(f"ds_read_b128 {rng('v', LR(h, qs), 4)}, %[al] offset:{2 * TILE_BYTES + 4 * row}", "ldsr",
                           writes=vr(LR(h, qs), 4), lds=True))
            out.append(Ins(f"ds_read_b128 {rng('v', DR(h, qs), 4)}, %[al] offset:{2 * TILE_BYTES + 4 * FQT + 4 * row}",
                           "ldsr", writes=vr(DR(h, qs), 4), lds=True))
        return out

    def rd_tr(h, ds):  # dO^T (A of dV^T) and Q^T (A of dK^T) of column group ds, permuted k order
        tq = TQ(h, ds)
        o = 4096 * h
        return [Ins(f"ds_read_b64_tr_b16 {rng('a', tq, 2)}, %[tr{ds}] offset:{TILE_BYTES + o}", "ldsr", writes=ar(tq, 2), lds=True),
                Ins(f"ds_read_b64_tr_b16 {rng('a', tq + 2, 2)}, %[tr{ds}] offset:{TILE_BYTES + o + 2048}", "ldsr",
                    writes=ar(tq + 2, 2), lds=True),
                Ins(f"ds_read_b64_tr_b16 {rng('a', tq + 4, 2)}, %[tr{ds}] offset:{o}", "ldsr", writes=ar(tq + 4, 2), lds=True),
                Ins(f"ds_read_b64_tr_b16 {rng('a', tq + 6, 2)}, %[tr{ds}] offset:{o + 2048}", "ldsr",
                    writes=ar(tq + 6, 2), lds=True)]

    # ---- softmax-gradient VALU of (h, t4), then its two -dS row writes
    def chunk(h, t4):
        out = []
        st0, dp0 = ST(h, t4, 0), DP(h, t4, 0)
        for i in range(8):  # P = exp2(-(lse2 - c s))
            out.append(Ins(f"v_exp_f32_e64 v{st0 + i}, -v{st0 + i}", "exp", reads=vr(st0 + i, 1), writes=vr(st0 + i, 1),
                           cost=8))
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
        out.append(Ins(f"ds_write_b64 %[ds{2 * h}], {rng('v', dp0, 2)} offset:{2048 * t4}", "ldsw", reads=vr(dp0, 2), lds=True,
                       cost=8))
        out.append(Ins(f"ds_write_b64 %[ds{2 * h + 1}], {rng('v', dp0 + 2, 2)} offset:{2048 * t4}", "ldsw",
                       reads=vr(dp0 + 2, 2), lds=True, cost=8))
        return out

    # ---- placement: fillers[i] = instructions issued right before MFMA i
    fill = [[] for _ in range(129)]
    # prologue: rows and ring groups 0, 1 of half 0
    pro += rd_rows(0)[0:2] + rd_group(0) + rd_rows(0)[2:4] + rd_group(1)
    # ring groups 2 .. 7, two groups ahead of their first MFMA (group g's MFMAs are 8 g .. 8 g + 7)
    for g in range(2, 8):
        fill[8 * (g - 2) + 1] += rd_group(g)
    # lse2 / delta rows of half 1 (for MFMA 32)
    fill[13] += rd_rows(1)
    # dO^T / Q^T of half 0 (first use MFMA 64) during M1_1; of half 1 (ring registers, free after
    # MFMA 63) during M2_0 (first use 96)
    for ds in range(4):
        fill[36 + 6 * ds] += rd_tr(0, ds)
        fill[66 + 6 * ds] += rd_tr(1, ds)
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
            fill[gap].append(x)
            k += 1
    prog = [Ins("s_waitcnt lgkmcnt(0)", "wait"), Ins("s_nop 3", "nop")] + pro
    for i in range(128):
        prog += fill[i]
        prog.append(mf[i])
    prog += fill[128]
    return prog


def finalize(prog):
    """Insert lgkmcnt waits and hazard nops; returns the instruction texts and statistics."""
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
                if r in ins.mfma_c and last_w.get(r, (-99, ""))[1] == "mfma":
                    continue  # accumulate chain
                w = last_w.get(r)
                if w and w[1] in ("valu", "exp"):
                    pad = max(pad, 2 - ws_since(w[0]))
                if w and w[1] == "mfma":
                    pad = max(pad, 10 - ws_since(w[0]))
            for r in ins.writes:
                w = last_w.get(r)
                if w and w[1] in ("valu", "exp"):
                    pad = max(pad, 2 - ws_since(w[0]))
        else:
            for r in ins.reads:
                w = last_w.get(r)
                if w and w[1] == "mfma":
                    pad = max(pad, 8 - ws_since(w[0]))
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
        # 3. issue
        out.append(ins.text)
        if ins.lds:
            idx = issued
            issued += 1
            if ins.kind == "ldsr":
                for r in ins.writes:
                    pending[r] = idx
        for r in ins.writes:
            last_w[r] = (pos, "mfma" if ins.kind == "mfma" else ("ld" if ins.kind == "ldsr" else "valu"))
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
    assert not pending, "LDS loads never waited for"
    return out, dict(nops=nops, waits=waits, instrs=len(out))


def operand_decl(masked):
    outs = []
    ins = ['[ar0] "v"(ar0)', '[ar1] "v"(ar1)', '[al] "v"(al)'] + [f'[tr{i}] "v"(tr[{i}])' for i in range(4)]
    ins += [f'[ds{i}] "v"(dsa[{i}])' for i in range(4)]
    if masked:
        ins += [f'[mlo{i}] "v"(mlo[{i}])' for i in range(4)] + [f'[mhi{i}] "v"(mhi[{i}])' for i in range(4)]
    clob = ['"memory"'] + [f'"v{i}"' for i in range(96, 256)] + [f'"a{i}"' for i in range(256)]
    if masked:
        clob.append('"vcc"')
    return outs, ins, clob


def emit_function(name, masked):
    prog = build(masked)
    lines, st = finalize(prog)
    outs, ins, clob = operand_decl(masked)
    mparams = ", const int (&mlo)[4], const int (&mhi)[4]" if masked else ""
    body = "\n".join(f'      "{l}\\n"' for l in lines)
    s = f"""// {name}: {st['instrs']} instructions, 128 MFMAs, {st['waits']} lgkmcnt waits, {st['nops']} hazard nops
__attribute__((always_inline)) DEV void {name}(unsigned ar0, unsigned ar1, unsigned al, const unsigned (&tr)[4],
    const unsigned (&dsa)[4]{mparams}) {{
  asm volatile(
{body}
      : {", ".join(outs)}
      : {", ".join(ins)}
      : {", ".join(clob)});
}}
"""
    return s, st


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
    for name, masked in (("fused4_main_full", False), ("fused4_main_masked", True)):
        s, st = emit_function(name, masked)
        print(f"{name}: {st}", file=sys.stderr)
        parts.append(s)
    if args.stats:
        return
    hdr = ("// GENERATED by tools/gen_fused4_asm.py -- do not edit.  The hand-placed main step of\n"
           "// attn_bwd_fused4_k (attn_bwd_fused4.hip): see the generator's docstring for the schedule.\n"
           "#pragma once\n\n")
    with open(OUT, "w") as f:
        f.write(hdr + emit_helpers() + "\n" + "\n".join(parts))
    print("wrote", OUT, file=sys.stderr)


if __name__ == "__main__":
    main()
