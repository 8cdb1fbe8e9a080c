#!/usr/bin/env python3
"""The one-wave-per-SIMD attention forward, 32x32x16 form (writes attn_fwd4_step.inc with FWD4_FORM 32).

    python tools/gen_fwd4w_asm.py [--stats]

Same work split, ring, run structure and schedule check as tools/gen_fwd4_asm.py (the 16x16x32 form,
bitwise equal to attn_fwd16_k), but the S^T and O^T products are v_mfma_f32_32x32x16_bf16: an MFMA
holds the SIMD's vector issue for 8 of its 32 cycles instead of 8 of 16 (MI355X_MICROARCH.md, vector
issue costs), which leaves room for the 64 exponentials + 32 packs per 32-key part beside the MFMAs.
Per part and wave (128 queries = 4 query tiles of 32):
  S^T[32 keys][32 q] = K q'^T: 4 k-steps of 16 d x 4 query tiles (16 MFMAs; K rows as A from LDS,
      q'^T as B from AGPRs); lane (q, h) holds keys 8 (j >> 2) + 4 h + (j & 3), j = 0..15;
  P = exp2(S^T), packed in place: step st = keys of j 8 st .. 8 st + 7 (the permuted key order of
      attn_common.hpp frag_tr);
  O^T[32 d][32 q] += V^T[32 d][16 keys] P (2 d tiles x 2 key steps x 4 query tiles = 16 MFMAs; V^T by
      frag_tr, two ds_read_b64_tr_b16);
  row sums: a 16x16x32 MFMA per query tile and key step with the packed P as its B operand and a
      selector A (rows 0-7 take lanes of query n, rows 8-15 those of query n + 16): lane (n, g) ends
      with the sum of query n (g < 2) or n + 16 (g >= 2) -- 8 MFMAs of 16 cycles, 4 registers per tile.
Registers: q'^T a[0:63], O^T a[64:191], row sums a[192:207], selector a[208:211], part-1 V^T fragments
a[212:227]; K fragments v[96:111], part-0 V^T v[112:127], S^T / P buffers v[128:191] (X), v[192:255] (Y).
"""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_fused4_asm import Ins as _Ins, vr, ar, rng, finalize  # noqa: E402

REPO = os.path.dirname(HERE)
OUT = os.path.join(REPO, "owl-audio-exps_amd", "csrc", "attn_fwd4_step.inc")
MF32 = "v_mfma_f32_32x32x16_bf16"
MF16 = "v_mfma_f32_16x16x32_bf16"
NQT = 4                # 32-query tiles per wave
SLOT = 16384
VOFF = 8192
NSLOT = 3
XNODMA = int(os.environ.get("W4F_XNODMA", "0"))
XEXP = int(os.environ.get("W4F_XEXP", "0"))


class Ins(_Ins):
    __slots__ = ("meta",)

    def __init__(self, *a, meta=None, **k):
        super().__init__(*a, **k)
        self.meta = meta


def QF(qt, ks):
    return 16 * qt + 4 * ks


def O(cb, qt):
    return 64 + 64 * cb + 16 * qt


def RS(qt):
    return 192 + 4 * qt


SEL = 208


def KF(ks):
    return 96 + 4 * ks


def VFR(cb, st, part):
    return ("v", 112 + 8 * cb + 4 * st) if part == 0 else ("a", 212 + 8 * cb + 4 * st)


BUF = {"X": 128, "Y": 192}


def ST(b, qt):
    return BUF[b] + 16 * qt


def PF(b, qt, st):
    return BUF[b] + 16 * qt + 4 * st


def regs(f, lo, n):
    return (vr if f == "v" else ar)(lo, n)


# ---------------------------------------------------------------- pieces
def s_mfmas(b, part):
    """S^T of one part (slot, kc) into buffer b: k-step ks outer; query tile qt completes at ks 3"""
    out = []
    for ks in range(4):
        for qt in range(NQT):
            d = ST(b, qt)
            c = "0" if ks == 0 else rng("v", d, 16)
            reads = vr(KF(ks), 4) + ar(QF(qt, ks), 4) + ([] if ks == 0 else vr(d, 16))
            out.append(Ins(f"{MF32} {rng('v', d, 16)}, {rng('v', KF(ks), 4)}, {rng('a', QF(qt, ks), 4)}, {c}", "mfma",
                           reads=reads, writes=vr(d, 16), mfma_c=[] if ks == 0 else vr(d, 16), passes=8,
                           meta=("S", b, ks, qt, part)))
    return out


def v_mfmas(b, part, tag):
    """O^T += V^T P (query tile outer, key step, d tile) and the row sums of the part in buffer b"""
    out = []
    for qt in range(NQT):
        for st in range(2):
            p = PF(b, qt, st)
            for cb in range(2):
                o = O(cb, qt)
                f, v = VFR(cb, st, part)
                out.append(Ins(f"{MF32} {rng('a', o, 16)}, {rng(f, v, 4)}, {rng('v', p, 4)}, {rng('a', o, 16)}", "mfma",
                               reads=regs(f, v, 4) + vr(p, 4) + ar(o, 16), writes=ar(o, 16), mfma_c=ar(o, 16),
                               passes=8, meta=("V", b, qt, st, cb, part, tag)))
            r = RS(qt)
            out.append(Ins(f"{MF16} {rng('a', r, 4)}, {rng('a', SEL, 4)}, {rng('v', p, 4)}, {rng('a', r, 4)}", "mfma",
                           reads=ar(SEL, 4) + vr(p, 4) + ar(r, 4), writes=ar(r, 4), mfma_c=ar(r, 4),
                           meta=("R", b, qt, st, tag)))
    return out


def e_valu(b, qts, tag, masked=False, kc=0):
    """exp2 of the S^T tiles of query tiles qts (in place), the mask (key 32 kc + 8 (j >> 2) + 4 h + (j & 3)
    allowed iff mlo[qt] <= 32 kc + 8 (j >> 2) + (j & 3) < mhi[qt], per lane), then P packed in place"""
    out = []
    for qt in qts:
        s0 = ST(b, qt)
        for j in range(16):
            txt = f"v_exp_f32_e32 v{s0 + j}, v{s0 + j}" if not XEXP else f"v_mov_b32 v{s0 + j}, v{s0 + j}"
            out.append(Ins(txt, "exp", reads=vr(s0 + j, 1), writes=vr(s0 + j, 1), cost=8, meta=("E", s0 + j, qt, tag)))
        if masked:
            for j in range(16):
                k = 32 * kc + 8 * (j >> 2) + (j & 3)
                out.append(Ins(f"v_cmp_ge_i32_e32 vcc, {k}, %[mlo{qt}]", "cmp"))
                out.append(Ins("s_nop 1", "nop", cost=8))
                out.append(Ins(f"v_cndmask_b32_e32 v{s0 + j}, 0, v{s0 + j}, vcc", "valu", reads=vr(s0 + j, 1),
                               writes=vr(s0 + j, 1)))
                out.append(Ins(f"v_cmp_lt_i32_e32 vcc, {k}, %[mhi{qt}]", "cmp"))
                out.append(Ins("s_nop 1", "nop", cost=8))
                out.append(Ins(f"v_cndmask_b32_e32 v{s0 + j}, 0, v{s0 + j}, vcc", "valu", reads=vr(s0 + j, 1),
                               writes=vr(s0 + j, 1)))
        for st in range(2):
            for w in range(4):
                d, x = s0 + 4 * st + w, s0 + 8 * st + 2 * w
                out.append(Ins(f"v_cvt_pk_bf16_f32 v{d}, v{x}, v{x + 1}", "valu", reads=vr(x, 2), writes=vr(d, 1),
                               meta=("C", d, x, x + 1, qt, tag)))
    return out


def rd_k(slot, kc):
    """K fragments of part kc: rows 32 kc + (lane & 31), d 16 ks + 8 h: one ds_read_b128 per k-step"""
    return [Ins(f"ds_read_b128 {rng('v', KF(ks), 4)}, %[kr{ks}] offset:{slot * SLOT + 32 * kc * 128}", "ldsr",
                writes=vr(KF(ks), 4), lds=True, meta=("LK", ks, (slot, kc))) for ks in range(4)]


def rd_v(slot, kc):
    """V^T fragments of part kc (frag_tr: key step st, d tile cb): two ds_read_b64_tr_b16 (rows
    16 st + 4 h + qq and + 8)"""
    out = []
    for st in range(2):
        for cb in range(2):
            f, v = VFR(cb, st, kc)
            base = slot * SLOT + VOFF + (32 * kc + 16 * st) * 128
            out.append(Ins(f"ds_read_b64_tr_b16 {rng(f, v, 2)}, %[vt{cb}] offset:{base}", "ldsr",
                           writes=regs(f, v, 2), lds=True, meta=("LV", cb, st, (slot, kc))))
            out.append(Ins(f"ds_read_b64_tr_b16 {rng(f, v + 2, 2)}, %[vt{cb}] offset:{base + 1024}", "ldsr",
                           writes=regs(f, v + 2, 2), lds=True, meta=("LV", cb, st, (slot, kc))))
    return out


def dma(slot, counted=False):
    out = []
    for i in range(4):
        if XNODMA:
            out.append(Ins("s_nop 0", "raw"))
            continue
        src, off = ("kb", f"ko{i % 2}") if i < 2 else ("vb", f"vo{i % 2}")
        dst = slot * SLOT + (VOFF if i >= 2 else 0) + 1024 * (i % 2)
        t = ["s_cmp_gt_i32 s69, 0" if counted else "s_bitcmp1_b32 %[fl], 0", f"s_cbranch_scc0 .Lw4d{i}%=",
             f"s_add_u32 m0, %[m0k], {dst}", "s_nop 0", f"global_load_lds_dwordx4 %[{off}], %[{src}]", f".Lw4d{i}%=:"]
        out.append(Ins("\n".join(t), "raw"))
    return out


def interleave(mfmas, fillers, lo=0, hi=None, first=None):
    n = len(mfmas)
    hi = n if hi is None else hi
    slots = [[] for _ in range(n + 1)]
    if first:
        for i, ins in first.items():
            slots[i] += ins
    m = len(fillers)
    for k, x in enumerate(fillers):
        slots[lo + (k * (hi - lo)) // max(m, 1)].append(x)
    prog = []
    for i in range(n):
        prog += slots[i]
        prog.append(mfmas[i])
    return prog + slots[n]


def half(first):
    return [0, 1] if first else [2, 3]


# ---------------------------------------------------------------- statements
def build_tile(slot, masked):
    nslot = (slot + 2) % NSLOT
    p0, p1 = (slot, 0), (slot, 1)
    k1 = rd_k(slot, 1)
    d = dma(nslot)
    v = rd_v(slot, 0) + rd_v(slot, 1)
    prog = [Ins("s_waitcnt lgkmcnt(0)", "wait"), Ins("s_nop 3", "nop")] + rd_k(slot, 0)
    # S0 (K fragment ks last read by MFMA 4 ks + 3), the V^T fragments of both parts, the DMA
    prog += interleave(s_mfmas("X", p0), [], first={1: v[0:4], 2: v[4:8], 3: v[8:12], 4: [k1[0]] + v[12:16],
                                                     8: [k1[1]], 12: [k1[2]], 16: [k1[3]], 5: [d[0]], 7: [d[1]],
                                                     9: [d[2]], 11: [d[3]]})
    prog += interleave(s_mfmas("Y", p1), e_valu("X", range(NQT), p0, masked, 0), 1, 16)
    prog += interleave(v_mfmas("X", 0, p0), e_valu("Y", range(NQT), p1, masked, 1), 0, 20)
    prog += v_mfmas("Y", 1, p1)
    return prog


def run_end(nxt):
    return ["s_waitcnt vmcnt(0)", "s_waitcnt lgkmcnt(0)", "s_barrier",
            "s_add_u32 s64, s64, %[kstep]", "s_addc_u32 s65, s65, 0",
            "s_add_u32 s66, s66, %[vstep]", "s_addc_u32 s67, s67, 0",
            "s_sub_u32 s68, s68, 1", "s_sub_u32 s69, s69, 1"] + nxt


def run_parts(slot0):
    pk1 = rd_k(slot0, 1)
    pro = [Ins("s_waitcnt lgkmcnt(0)", "wait"), Ins("s_nop 3", "nop")] + rd_k(slot0, 0)
    pro += interleave(s_mfmas("X", (slot0, 0)), [], first={4: [pk1[0]], 8: [pk1[1]], 12: [pk1[2]], 16: [pk1[3]],
                                                           1: rd_v(slot0, 0)})
    pro += e_valu("X", half(True), (slot0, 0))
    bodies, drains = {}, {}
    for s in range(NSLOT):
        s1, s2 = (s + 1) % NSLOT, (s + 2) % NSLOT
        d = dma(s2, counted=True)
        p = [Ins("s_nop 0", "nop")]
        # block 1 (16 S MFMAs of 32 cycles): S(t,1) | exp(t,0) 2nd half; DMA; V^T of (t,1)
        p += interleave(s_mfmas("Y", (s, 1)), e_valu("X", half(False), (s, 0)), 0, 16,
                        first={1: [d[0]], 3: [d[1]], 5: [d[2]], 7: [d[3]], 2: rd_v(s, 1)})
        # block 2 (16 + 8): V(t,0) | exp(t,1) 1st half; K fragments of (t+1, 0)
        p += interleave(v_mfmas("X", 0, (s, 0)), e_valu("Y", half(True), (s, 1)), 0, 22, first={1: rd_k(s1, 0)})
        # block 3: S(t+1,0) | exp(t,1) 2nd half; V^T of (t+1, 0)
        p += interleave(s_mfmas("X", (s1, 0)), e_valu("Y", half(False), (s, 1)), 0, 16, first={1: rd_v(s1, 0)})
        # block 4: V(t,1) | exp(t+1,0) 1st half; K fragments of (t+1,1)
        p += interleave(v_mfmas("Y", 1, (s, 1)), e_valu("X", half(True), (s1, 0)), 2, 24, first={1: rd_k(s1, 1)})
        bodies[s] = p
        p = [Ins("s_nop 0", "nop")]
        p += interleave(s_mfmas("Y", (s, 1)), e_valu("X", half(False), (s, 0)), 0, 16,
                        first={1: [d[0]], 3: [d[1]], 5: [d[2]], 7: [d[3]], 2: rd_v(s, 1)})
        p += interleave(v_mfmas("X", 0, (s, 0)), e_valu("Y", range(NQT), (s, 1)), 0, 24)
        p += v_mfmas("Y", 1, (s, 1))
        drains[s] = p
    return pro, bodies, drains


def build_run(slot0):
    pro, bodies, drains = run_parts(slot0)

    def emit(prog, tag):
        lines, _ = finalize(prog, allow_pending=True)
        return [x.replace("%=", f"%={tag}") for x in lines]

    t = emit(pro, "pr") + ["s_waitcnt lgkmcnt(0)", f"s_branch .Lw4L{slot0}%="]
    for s in range(NSLOT):
        s1 = (s + 1) % NSLOT
        t += [f".Lw4L{s}%=:"] + emit(bodies[s], f"b{s}")
        t += run_end(["s_cmp_eq_u32 s68, 1", f"s_cbranch_scc1 .Lw4D{s1}%=", f"s_branch .Lw4L{s1}%="])
    for s in range(NSLOT):
        t += [f".Lw4D{s}%=:"] + emit(drains[s], f"d{s}") + run_end(["s_branch .Lw4X%="])
    t.append(".Lw4X%=:")
    return t


# ---------------------------------------------------------------- schedule check
def check_program(prog, state=None):
    st = {} if state is None else state

    def need(rs, want, what):
        for r in rs:
            if st.get(r) != want:
                raise AssertionError(f"{what}: {r} holds {st.get(r)}, wants {want}")

    for ins in prog:
        m = getattr(ins, "meta", None)
        if not m:
            continue
        op = m[0]
        if op == "LK":
            for r in ins.writes:
                st[r] = ("K", m[1], m[2])
        elif op == "LV":
            for r in ins.writes:
                st[r] = ("V", m[1], m[2], m[3])
        elif op == "S":
            _, b, ks, qt, part = m
            need(vr(KF(ks), 4), ("K", ks, part), f"S {m}")
            d = vr(ST(b, qt), 16)
            if ks:
                need(d, ("S", ks - 1, qt, part), f"S chain {m}")
            for r in d:
                st[r] = ("S", ks, qt, part)
        elif op == "E":
            _, reg, qt, tag = m
            need([("v", reg)], ("S", 3, qt, tag), f"exp {m}")
            st[("v", reg)] = ("E", qt, tag)
        elif op == "C":
            _, d, x, y, qt, tag = m
            need([("v", x), ("v", y)], ("E", qt, tag), f"pack {m}")
            st[("v", d)] = ("P", qt, tag, d)
        elif op == "V":
            _, b, qt, s_, cb, part, tag = m
            f, v = VFR(cb, s_, part)
            need(regs(f, v, 4), ("V", cb, s_, tag), f"PV {m}")
            for r in range(4):
                need([("v", PF(b, qt, s_) + r)], ("P", qt, tag, PF(b, qt, s_) + r), f"PV P {m}")
        elif op == "R":
            _, b, qt, s_, tag = m
            for r in range(4):
                need([("v", PF(b, qt, s_) + r)], ("P", qt, tag, PF(b, qt, s_) + r), f"rowsum {m}")
    return st


def self_check():
    for masked in (False, True):
        for slot in range(NSLOT):
            check_program(build_tile(slot, masked))
    for slot0 in range(NSLOT):
        pro, bodies, drains = run_parts(slot0)
        for n in range(2, 8):
            st = check_program(pro)
            for i in range(n - 1):
                st = check_program(bodies[(slot0 + i) % NSLOT], st)
            check_program(drains[(slot0 + n - 1) % NSLOT], st)


# ---------------------------------------------------------------- emission
VOPS = ["kr0", "kr1", "kr2", "kr3", "vt0", "vt1", "ko0", "ko1", "vo0", "vo1"]
CLOB = ['"memory"', '"m0"', '"scc"'] + [f'"v{i}"' for i in range(96, 256)] + [f'"a{i}"' for i in range(256)]


def vop(n):
    return f'[{n}] "v"(f.{n[:-1]}[{n[-1]}])'


def emit_tile(slot, masked):
    lines, st = finalize(build_tile(slot, masked))
    body = "\n".join(f'      "{x}\\n"' for x in lines)
    ins = [vop(n) for n in VOPS] + ['[fl] "s"(fl)', '[m0k] "s"(s.m0k)', '[kb] "s"(s.kb)', '[vb] "s"(s.vb)']
    clob = list(CLOB)
    if masked:
        ins += [f'[mlo{i}] "v"(f.mlo[{i}])' for i in range(NQT)] + [f'[mhi{i}] "v"(f.mhi[{i}])' for i in range(NQT)]
        clob.append('"vcc"')
    nm = f"fwd4_tile_{'masked' if masked else 'full'}_s{slot}"
    return f"""// {nm}: {st['instrs']} lines, {st['waits']} lgkmcnt waits, {st['nops']} hazard nops
__attribute__((always_inline)) DEV void {nm}(const W4Lane& f, const W4Scalar& s, int fl) {{
  asm volatile(
{body}
      :
      : {", ".join(ins)}
      : {", ".join(clob)});
}}
"""


def emit_run(slot0):
    t = build_run(slot0)
    body = "\n".join(f'      "{x}\\n"' for x in t)
    ins = [vop(n) for n in VOPS] + ['[fl] "s"(fl)', '[m0k] "s"(s.m0k)', '[kstep] "s"(kstep)', '[vstep] "s"(vstep)']
    outs = ['[kb] "+{s[64:65]}"(kb)', '[vb] "+{s[66:67]}"(vb)', '[n] "+{s68}"(n)', '[dl] "+{s69}"(dl)']
    nm = f"fwd4_run_s{slot0}"
    return f"""// {nm}: {len(t)} lines
__attribute__((always_inline)) DEV void {nm}(int n, int dl, const W4Lane& f, const W4Scalar& s, int fl,
                                        unsigned kstep, unsigned vstep) {{
  const void *kb = s.kb, *vb = s.vb;
  asm volatile(
{body}
      : {", ".join(outs)}
      : {", ".join(ins)}
      : {", ".join(CLOB)});
}}
"""


def emit_helpers():
    w, ops = [], []
    for qt in range(NQT):
        for ks in range(4):
            for e in range(4):
                w.append(f'"v_accvgpr_write_b32 a{QF(qt, ks) + e}, %[q{qt}_{ks}_{e}]\\n"')
                ops.append(f'[q{qt}_{ks}_{e}] "v"(q[{qt}][{ks}][{e}])')
    w += [f'"v_accvgpr_write_b32 a{i}, 0\\n"' for i in range(64, 208)]
    w += [f'"v_accvgpr_write_b32 a{SEL + e}, %[sel]\\n"' for e in range(4)]
    ops.append('[sel] "v"(sel)')
    w.append('"s_nop 3\\n"')
    clob = ['"memory"'] + [f'"a{i}"' for i in range(256)]
    s = ("// q'^T fragments into a[0:63], O^T and the row sums = 0, the row-sum selector into a[208:211]\n"
         "__attribute__((always_inline)) DEV void fwd4_agpr_init(const unsigned (&q)[4][4][4], unsigned sel) {\n"
         "  asm volatile(\n      " + "\n      ".join(w) + "\n      :\n      : " + ", ".join(ops) +
         "\n      : " + ", ".join(clob) + ");\n}\n")
    s += ("// O^T[cb][qt] -> o[16 cb ..], the row-sum tile of qt -> o[32 ..] (the last MFMAs are >= 12 wait\n"
          "// states back)\ntemplate <int QT>\n__attribute__((always_inline)) DEV void fwd4_acc_read(float (&o)[36]);\n")
    for qt in range(NQT):
        rd = [f'"v_accvgpr_read_b32 %{16 * cb + e}, a{O(cb, qt) + e}\\n"' for cb in range(2) for e in range(16)]
        rd += [f'"v_accvgpr_read_b32 %{32 + e}, a{RS(qt) + e}\\n"' for e in range(4)]
        s += (f"template <>\n__attribute__((always_inline)) DEV void fwd4_acc_read<{qt}>(float (&o)[36]) {{\n"
              f"  asm volatile(" + " ".join(rd) + " : " + ", ".join(f'"=v"(o[{e}])' for e in range(36)) + ");\n}\n")
    return s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stats", action="store_true")
    args = ap.parse_args()
    self_check()
    parts = [emit_tile(slot, masked) for masked in (False, True) for slot in range(NSLOT)]
    parts += [emit_run(slot) for slot in range(NSLOT)]
    if args.stats:
        for p in parts:
            print(p.split("\n")[0], file=sys.stderr)
        return
    disp = ["template <bool MASKED>",
            "__attribute__((always_inline)) DEV void fwd4_tile(int slot, const W4Lane& f, const W4Scalar& s, int fl) {"]
    for masked in (False, True):
        nm = f"fwd4_tile_{'masked' if masked else 'full'}"
        disp += [f"  if constexpr ({'MASKED' if masked else '!MASKED'}) {{",
                 f"    if (slot == 0) {nm}_s0(f, s, fl); else if (slot == 1) {nm}_s1(f, s, fl); else {nm}_s2(f, s, fl);",
                 "  }"]
    disp += ["}", "",
             "__attribute__((always_inline)) DEV void fwd4_run(int slot, int n, int dl, const W4Lane& f, const W4Scalar& s,",
             "                                              int fl, unsigned kstep, unsigned vstep) {",
             "  if (slot == 0) fwd4_run_s0(n, dl, f, s, fl, kstep, vstep);",
             "  else if (slot == 1) fwd4_run_s1(n, dl, f, s, fl, kstep, vstep);",
             "  else fwd4_run_s2(n, dl, f, s, fl, kstep, vstep);", "}", ""]
    hdr = ("// GENERATED by tools/gen_fwd4w_asm.py -- do not edit.  The hand-placed statements of attn_fwd4_k\n"
           "// (attn_fwd4.hip), 32x32x16 form: see the generator's docstring.\n#pragma once\n#define FWD4_FORM 32\n\n"
           "// per-lane operands (VGPR): K fragment offsets (k-step ks), V^T fragment offsets (d tile cb), the\n"
           "// ring DMA's source offsets (K / V rows h); PARTIAL tiles: each query tile's allowed key range\n"
           "// relative to the tile and to the lane's 4 h rows\n"
           "struct W4Lane {\n  unsigned kr[4], vt[2], ko[2], vo[2];\n  int mlo[4], mhi[4];\n};\n"
           "struct W4Scalar {\n  unsigned m0k;\n  const void *kb, *vb;\n};\n\n")
    with open(OUT, "w") as f:
        f.write(hdr + emit_helpers() + "\n" + "\n".join(parts) + "\n" + "\n".join(disp))
    print("wrote", OUT, file=sys.stderr)


if __name__ == "__main__":
    main()
