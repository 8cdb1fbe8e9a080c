#!/usr/bin/env python3
"""Generate the hand-placed statements of the one-wave-per-SIMD attention forward (attn_fwd4.hip).

    python tools/gen_fwd4_asm.py            # writes owl-audio-exps_amd/csrc/attn_fwd4_step.inc
    python tools/gen_fwd4_asm.py --stats

A wave owns 128 queries (8 query tiles of 16) and sweeps 64-key tiles of K / V from a 3-slot LDS
ring, each as two 32-key parts.  Per part: S^T[16 keys][16 q] = K q'^T (32 v_mfma_f32_16x16x32_bf16,
K rows from LDS as A, q' = bf16(c q) from AGPRs as B), P = exp2(S^T) (bounded softmax: no running max,
attn_fwd.hip attn_fwd16_k), P packed to bf16 in the permuted key order, O^T[16 d][16 q] += V^T P
(32 MFMAs, V^T by ds_read_b64_tr_b16) and the row sums ones^T P (8 MFMAs).  The same products in the
same order as attn_fwd16_k (one 16x16x32 chain per output tile, key parts in sweep order), so O and
lse are bitwise those of attn_fwd16_k<64, true, 64, 8>-equivalent arithmetic.

Registers are fixed here: q' (a[0:63]), O^T (a[64:191]), the row sums (a[192:223]) and ones (a[224:227])
in AGPRs hipcc never touches (the translation unit is built with -amdgpu-mfma-vgpr-form
-amdgpu-spill-vgpr-to-agpr=0, as attn_bwd_fused4.hip); K fragments v[96:111], V^T fragments
v[112:127], two S^T / P buffers v[128:191] (X) and v[192:255] (Y).

Two statement forms:
* fwd4_tile_<full|masked>_s<slot>: one tile, parts in sequence (S0, S1 | exp 0, V0 | exp 1, V1),
  its 4 ring DMA pieces (tile t + 2) on flags bit 0 -- the tiles a run does not cover;
* fwd4_run_s<slot>: n >= 2 FULL tiles in one loop, software-pipelined across parts and tiles:
  iteration t = [S(t,1) | exp(t,0) 2nd half] [V(t,0) | exp(t,1) 1st half] [S(t+1,0) | exp(t,1) 2nd]
  [V(t,1) | exp(t+1,0) 1st], then vmcnt(0) + s_barrier (the ring: tiles t, t+1 resident, t+2 landing),
  unrolled by 3 for the ring slot; a prologue (S(t_a,0), exp) and a drain (last tile) around it.
"""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_fused4_asm import Ins as _Ins, vr, ar, rng, finalize  # noqa: E402


class Ins(_Ins):
    """an instruction with its meaning for the schedule check (check_program): meta = (op, ...)"""
    __slots__ = ("meta",)

    def __init__(self, *a, meta=None, **k):
        super().__init__(*a, **k)
        self.meta = meta

REPO = os.path.dirname(HERE)
OUT = os.path.join(REPO, "owl-audio-exps_amd", "csrc", "attn_fwd4_step.inc")
MF = "v_mfma_f32_16x16x32_bf16"
NQ = 8                 # 16-query tiles per wave
SLOT = 16384           # ring slot: K 64 x 128 B | V 64 x 128 B
VOFF = 8192
NSLOT = 3
# timing-only experiment builds (results wrong): W4F_XNODMA=1 no ring DMA, W4F_XEXP=1 v_exp -> v_mov
XNODMA = int(os.environ.get("W4F_XNODMA", "0"))
XEXP = int(os.environ.get("W4F_XEXP", "0"))


def QF(t4, kd):
    return 8 * t4 + 4 * kd


def O(ds, t4):
    return 64 + 32 * ds + 4 * t4


def LA(t4):
    return 192 + 4 * t4


ONES = 224


def KF(kk, kd):
    return 96 + 4 * (2 * kk + kd)


def VF(ds, part):  # V^T fragments: part 0 in v[112:127], part 1 in a[228:243] (both live across a block)
    return (112 if part == 0 else 228) + 4 * ds


def VFR(ds, part):
    return ("v" if part == 0 else "a"), VF(ds, part)


BUF = {"X": 128, "Y": 192}


def ST(b, kk, t4):
    return BUF[b] + 32 * kk + 4 * t4


def PF(b, t4):
    return BUF[b] + 4 * t4


# ---------------------------------------------------------------- pieces
def s_mfmas(b, part):
    """S^T of one part (slot, kc) into buffer b: (kk, kd, t4) order; tile (kk, t4) completes at its kd = 1 MFMA"""
    out = []
    for kk in range(2):
        for kd in range(2):
            for t4 in range(NQ):
                d = ST(b, kk, t4)
                c = "0" if kd == 0 else rng("v", d, 4)
                reads = vr(KF(kk, kd), 4) + ar(QF(t4, kd), 4) + ([] if kd == 0 else vr(d, 4))
                out.append(Ins(f"{MF} {rng('v', d, 4)}, {rng('v', KF(kk, kd), 4)}, {rng('a', QF(t4, kd), 4)}, {c}",
                               "mfma", reads=reads, writes=vr(d, 4), mfma_c=[] if kd == 0 else vr(d, 4),
                               meta=("S", b, kk, kd, t4, part)))
    return out


def v_mfmas(b, part, tag):
    """O^T += V^T P and the row sums for the part in buffer b: t4 outer (P of query tile t4 is due at
    MFMA 5 t4)"""
    out = []
    for t4 in range(NQ):
        p = PF(b, t4)
        for ds in range(4):
            o = O(ds, t4)
            f, v = VFR(ds, part)
            out.append(Ins(f"{MF} {rng('a', o, 4)}, {rng(f, v, 4)}, {rng('v', p, 4)}, {rng('a', o, 4)}", "mfma",
                           reads=(vr if f == "v" else ar)(v, 4) + vr(p, 4) + ar(o, 4), writes=ar(o, 4),
                           mfma_c=ar(o, 4), meta=("V", b, t4, ds, part, tag)))
        la = LA(t4)
        out.append(Ins(f"{MF} {rng('a', la, 4)}, {rng('a', ONES, 4)}, {rng('v', p, 4)}, {rng('a', la, 4)}", "mfma",
                       reads=ar(ONES, 4) + vr(p, 4) + ar(la, 4), writes=ar(la, 4), mfma_c=ar(la, 4),
                       meta=("R", b, t4, tag)))
    return out


def e_valu(b, t4s, tag, masked=False, kc=0):
    """exp2 of the S^T tiles of query tiles t4s in buffer b (in place), the mask (PARTIAL tiles: keys
    32 kc + 16 kk + 4 g + r of the tile allowed iff mlo[t4] <= 32 kc + 16 kk + r < mhi[t4], per lane),
    then P packed into PF(b, t4) (pack_perm order)"""
    out = []
    for t4 in t4s:
        for kk in range(2):
            s0 = ST(b, kk, t4)
            for r in range(4):
                out.append(Ins(f"v_exp_f32_e32 v{s0 + r}, v{s0 + r}" if not XEXP else f"v_mov_b32 v{s0 + r}, v{s0 + r}", "exp", reads=vr(s0 + r, 1), writes=vr(s0 + r, 1),
                               cost=8, meta=("E", s0 + r, kk, t4, tag)))
            if masked:
                for r in range(4):
                    k = 32 * kc + 16 * kk + r
                    out.append(Ins(f"v_cmp_ge_i32_e32 vcc, {k}, %[mlo{t4}]", "cmp"))
                    out.append(Ins("s_nop 1", "nop", cost=8))
                    out.append(Ins(f"v_cndmask_b32_e32 v{s0 + r}, 0, v{s0 + r}, vcc", "valu", reads=vr(s0 + r, 1),
                                   writes=vr(s0 + r, 1)))
                    out.append(Ins(f"v_cmp_lt_i32_e32 vcc, {k}, %[mhi{t4}]", "cmp"))
                    out.append(Ins("s_nop 1", "nop", cost=8))
                    out.append(Ins(f"v_cndmask_b32_e32 v{s0 + r}, 0, v{s0 + r}, vcc", "valu", reads=vr(s0 + r, 1),
                                   writes=vr(s0 + r, 1)))
        a, c = ST(b, 0, t4), ST(b, 1, t4)
        p = PF(b, t4)  # == a: words 0, 1 from kk 0 (in place), 2, 3 from kk 1
        for w, (x, y) in enumerate(((a, a + 1), (a + 2, a + 3), (c, c + 1), (c + 2, c + 3))):
            out.append(Ins(f"v_cvt_pk_bf16_f32 v{p + w}, v{x}, v{y}", "valu", reads=vr(x, 1) + vr(y, 1),
                           writes=vr(p + w, 1), meta=("C", p + w, x, y, t4, tag)))
    return out


def rd_k(slot, kc):
    """K fragments of part kc (rows 32 kc + 16 kk + (lane & 15), k-step kd): ds_read_b128"""
    return [Ins(f"ds_read_b128 {rng('v', KF(kk, kd), 4)}, %[kr{kd}] offset:{slot * SLOT + (32 * kc + 16 * kk) * 128}",
                "ldsr", writes=vr(KF(kk, kd), 4), lds=True, meta=("LK", kk, kd, (slot, kc)))
            for kk in range(2) for kd in range(2)]


def rd_v(slot, kc):
    """V^T fragments of part kc (into its register set), column group ds: two ds_read_b64_tr_b16 (rows
    4 g + .., + 16)"""
    out = []
    for ds in range(4):
        base = slot * SLOT + VOFF + 32 * kc * 128
        f, v = VFR(ds, kc)
        regs = vr if f == "v" else ar
        out.append(Ins(f"ds_read_b64_tr_b16 {rng(f, v, 2)}, %[vt{ds}] offset:{base}", "ldsr", writes=regs(v, 2),
                       lds=True, meta=("LV", f, v, ds, (slot, kc), 0)))
        out.append(Ins(f"ds_read_b64_tr_b16 {rng(f, v + 2, 2)}, %[vt{ds}] offset:{base + 16 * 128}", "ldsr",
                       writes=regs(v + 2, 2), lds=True, meta=("LV", f, v + 2, ds, (slot, kc), 1)))
    return out


def dma(slot, counted=False):
    """the ring DMA of tile t + 2 into `slot` (flags bit 0; in a run: while the DMA counter s69 > 0):
    K rows 16 w + 8 h, V rows, 1 KiB each"""
    out = []
    for i in range(4):
        src, off = ("kb", f"ko{i % 2}") if i < 2 else ("vb", f"vo{i % 2}")
        dst = slot * SLOT + (VOFF if i >= 2 else 0) + 1024 * (i % 2)
        if XNODMA:
            out.append(Ins("s_nop 0", "raw"))
            continue
        t = ["s_cmp_gt_i32 s69, 0" if counted else "s_bitcmp1_b32 %[fl], 0", f"s_cbranch_scc0 .Lw4d{i}%=",
             f"s_add_u32 m0, %[m0k], {dst}", "s_nop 0", f"global_load_lds_dwordx4 %[{off}], %[{src}]", f".Lw4d{i}%=:"]
        out.append(Ins("\n".join(t), "raw"))
    return out


def interleave(mfmas, fillers, lo=0, hi=None, first=None):
    """place the filler instructions (in order) evenly into the gaps before mfmas[lo:hi]; returns the
    program.  first: a list of filler groups that must go before specific MFMA indices {idx: [ins]}"""
    n = len(mfmas)
    hi = n if hi is None else hi
    slots = [[] for _ in range(n + 1)]
    if first:
        for i, ins in first.items():
            slots[i] += ins
    m = len(fillers)
    for k, x in enumerate(fillers):
        g = lo + (k * (hi - lo)) // max(m, 1)
        slots[g].append(x)
    prog = []
    for i in range(n):
        prog += slots[i]
        prog.append(mfmas[i])
    prog += slots[n]
    return prog


# ---------------------------------------------------------------- single-tile statement
def build_tile(slot, masked):
    nslot = (slot + 2) % NSLOT
    p0, p1 = (slot, 0), (slot, 1)
    S0, S1 = s_mfmas("X", p0), s_mfmas("Y", p1)
    V0, V1 = v_mfmas("X", 0, p0), v_mfmas("Y", 1, p1)
    E0 = e_valu("X", range(NQ), p0, masked, 0)
    E1 = e_valu("Y", range(NQ), p1, masked, 1)
    prog = [Ins("s_waitcnt lgkmcnt(0)", "wait"), Ins("s_nop 3", "nop")]
    prog += rd_k(slot, 0)
    # S0, with part 1's K fragments re-read as part 0's are consumed (fragment (kk, kd) last read by
    # MFMA 8 (2 kk + kd) + 7), both parts' V^T fragments and the ring DMA
    k1 = rd_k(slot, 1)
    d = dma(nslot)
    v = rd_v(slot, 0) + rd_v(slot, 1)
    prog += interleave(S0, [], first={1: v[0:4], 3: v[4:8], 5: v[8:12], 7: v[12:16], 8: [k1[0]], 16: [k1[1]],
                                       24: [k1[2]], 32: [k1[3]], 2: [d[0]], 6: [d[1]], 12: [d[2]], 20: [d[3]]})
    prog += interleave(S1, E0, 2, 32)   # S1 with part 0's exponentials
    prog += interleave(V0, E1, 0, 40)   # V0 with part 1's
    prog += V1
    return prog


# ---------------------------------------------------------------- pipelined run
def half(first):
    return list(range(0, 4)) if first else list(range(4, 8))


def run_end(nxt):
    """end of a run iteration: every wave's ring DMA landed, barrier; DMA sources one tile on; counters"""
    return ["s_waitcnt vmcnt(0)", "s_waitcnt lgkmcnt(0)", "s_barrier",
            "s_add_u32 s64, s64, %[kstep]", "s_addc_u32 s65, s65, 0",
            "s_add_u32 s66, s66, %[vstep]", "s_addc_u32 s67, s67, 0",
            "s_sub_u32 s68, s68, 1", "s_sub_u32 s69, s69, 1"] + nxt


def run_parts(slot0):
    """Ins programs of a run entered at ring slot slot0: prologue, the iteration of a tile in slot s,
    the drain of a last tile in slot s"""
    pk1 = rd_k(slot0, 1)
    pro = [Ins("s_waitcnt lgkmcnt(0)", "wait"), Ins("s_nop 3", "nop")] + rd_k(slot0, 0)
    # prologue: part 0 of t_a (S into X, the first half of its exponentials), the V^T fragments of
    # (t_a, 0), the K fragments of (t_a, 1) as part 0's are consumed; drained before the loop
    pro += interleave(s_mfmas("X", (slot0, 0)), [], first={8: [pk1[0]], 16: [pk1[1]], 24: [pk1[2]], 32: [pk1[3]],
                                                           2: rd_v(slot0, 0)})
    pro += e_valu("X", half(True), (slot0, 0))
    bodies, drains = {}, {}
    for s in range(NSLOT):  # iteration of tile t in slot s
        s1, s2 = (s + 1) % NSLOT, (s + 2) % NSLOT
        d = dma(s2, counted=True)
        p = [Ins("s_nop 0", "nop")]
        # block 1: S(t,1) | exp(t,0) 2nd half; the DMA of tile t + 2; V^T of (t,1) (its registers are
        # free since V(t-1,1))
        p += interleave(s_mfmas("Y", (s, 1)), e_valu("X", half(False), (s, 0)), 0, 32,
                        first={1: [d[0]], 5: [d[1]], 9: [d[2]], 13: [d[3]], 3: rd_v(s, 1)})
        # block 2: V(t,0) | exp(t,1) 1st half; K fragments of (t+1, 0) once S(t,1) is done with them
        p += interleave(v_mfmas("X", 0, (s, 0)), e_valu("Y", half(True), (s, 1)), 0, 36, first={1: rd_k(s1, 0)})
        # block 3: S(t+1,0) | exp(t,1) 2nd half; V^T of (t+1, 0) (free since V(t,0))
        p += interleave(s_mfmas("X", (s1, 0)), e_valu("Y", half(False), (s, 1)), 0, 32, first={2: rd_v(s1, 0)})
        # block 4: V(t,1) | exp(t+1,0) 1st half; K fragments of (t+1,1) once S(t+1,0) is done
        p += interleave(v_mfmas("Y", 1, (s, 1)), e_valu("X", half(True), (s1, 0)), 4, 40, first={1: rd_k(s1, 1)})
        bodies[s] = p
        # drain: the last tile: S(t_b,1) | exp 2nd half (X), V(t_b,0) | exp(t_b,1), V(t_b,1)
        p = [Ins("s_nop 0", "nop")]
        p += interleave(s_mfmas("Y", (s, 1)), e_valu("X", half(False), (s, 0)), 0, 32,
                        first={1: [d[0]], 5: [d[1]], 9: [d[2]], 13: [d[3]], 3: rd_v(s, 1)})
        p += interleave(v_mfmas("X", 0, (s, 0)), e_valu("Y", range(NQ), (s, 1)), 0, 40)
        p += v_mfmas("Y", 1, (s, 1))
        drains[s] = p
    return pro, bodies, drains


def build_run(slot0):
    """the loop statement entered with tile t_a in ring slot slot0 (n >= 2 tiles, s68 = n; s69 = the
    iterations that still issue the ring DMA of tile t + 2)"""
    pro, bodies, drains = run_parts(slot0)

    def emit(prog, tag):
        lines, st = finalize(prog, allow_pending=True)
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
    """Walk a program in issue order (every consumer of an LDS load gets its wait from finalize, so a
    register read sees the last write before it in program order) and check each instruction's
    operands hold what it means to consume: K fragments of the right part, complete S^T chains,
    exponentials and packed P of the right part, V^T fragments of the right part."""
    st = {} if state is None else state

    def need(regs, want, what):
        for r in regs:
            if st.get(r) != want:
                raise AssertionError(f"{what}: {r} holds {st.get(r)}, wants {want}")

    for ins in prog:
        m = getattr(ins, "meta", None)
        if not m:
            continue
        op = m[0]
        if op == "LK":
            _, kk, kd, tag = m
            for r in ins.writes:
                st[r] = ("K", kk, kd, tag)
        elif op == "LV":
            _, f, v, ds, tag, h = m
            for r in ins.writes:
                st[r] = ("V", ds, tag)
        elif op == "S":
            _, b, kk, kd, t4, part = m
            need(vr(KF(kk, kd), 4), ("K", kk, kd, part), f"S {m}")
            d = vr(ST(b, kk, t4), 4)
            if kd == 1:
                need(d, ("S0", kk, t4, part), f"S chain {m}")
            for r in d:
                st[r] = ("S0" if kd == 0 else "S1", kk, t4, part)
        elif op == "E":
            _, reg, kk, t4, tag = m
            need([("v", reg)], ("S1", kk, t4, tag), f"exp {m}")
            st[("v", reg)] = ("E", kk, t4, tag)
        elif op == "C":
            _, dst, x, y, t4, tag = m
            for r in (x, y):
                v = st.get(("v", r))
                if not (v and v[0] == "E" and v[2:] == (t4, tag)):
                    raise AssertionError(f"pack {m}: v{r} holds {v}")
            st[("v", dst)] = ("P", t4, tag, dst)
        elif op == "V":
            _, b, t4, ds, part, tag = m
            f, v = VFR(ds, part)
            need((vr if f == "v" else ar)(v, 4), ("V", ds, tag), f"PV {m}")
            for w in range(4):
                need([("v", PF(b, t4) + w)], ("P", t4, tag, PF(b, t4) + w), f"PV P {m}")
        elif op == "R":
            _, b, t4, tag = m
            for w in range(4):
                need([("v", PF(b, t4) + w)], ("P", t4, tag, PF(b, t4) + w), f"rowsum {m}")
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


VOPS = ["kr0", "kr1", "vt0", "vt1", "vt2", "vt3", "ko0", "ko1", "vo0", "vo1"]
CLOB = ['"memory"', '"m0"', '"scc"'] + [f'"v{i}"' for i in range(96, 256)] + [f'"a{i}"' for i in range(256)]


def emit_tile(slot, masked):
    prog = build_tile(slot, masked)
    lines, st = finalize(prog)
    body = "\n".join(f'      "{x}\\n"' for x in lines)
    ins = [f'[{n}] "v"(f.{n[:-1]}[{n[-1]}])' for n in VOPS]
    ins += ['[fl] "s"(fl)', '[m0k] "s"(s.m0k)', '[kb] "s"(s.kb)', '[vb] "s"(s.vb)']
    clob = list(CLOB)
    if masked:
        ins += [f'[mlo{i}] "v"(f.mlo[{i}])' for i in range(NQ)] + [f'[mhi{i}] "v"(f.mhi[{i}])' for i in range(NQ)]
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
    ins = [f'[{n}] "v"(f.{n[:-1]}[{n[-1]}])' for n in VOPS]
    ins += ['[fl] "s"(fl)', '[m0k] "s"(s.m0k)', '[kstep] "s"(kstep)', '[vstep] "s"(vstep)']
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
    w = []
    ops = []
    for t4 in range(NQ):
        for kd in range(2):
            for e in range(4):
                w.append(f'"v_accvgpr_write_b32 a{QF(t4, kd) + e}, %[q{t4}_{kd}_{e}]\\n"')
                ops.append(f'[q{t4}_{kd}_{e}] "v"(q[{t4}][{kd}][{e}])')
    w += [f'"v_accvgpr_write_b32 a{i}, 0\\n"' for i in range(64, 224)]
    w += [f'"v_accvgpr_write_b32 a{ONES + e}, %[one]\\n"' for e in range(4)]
    ops.append('[one] "v"(one)')
    w.append('"s_nop 3\\n"')
    clob = ['"memory"'] + [f'"a{i}"' for i in range(256)]
    s = ("// q' fragments into a[0:63], O^T and the row sums = 0, ones (bf16 pairs) into a[224:227]\n"
         "__attribute__((always_inline)) DEV void fwd4_agpr_init(const unsigned (&q)[8][2][4], unsigned one) {\n"
         "  asm volatile(\n      " + "\n      ".join(w) + "\n      :\n      : " + ", ".join(ops) +
         "\n      : " + ", ".join(clob) + ");\n}\n")
    s += "// O^T[ds][t4] -> o[4 ds ..], the row sums of t4 -> o[16] (the last MFMAs are >= 12 wait states back)\n"
    s += "template <int T4>\n__attribute__((always_inline)) DEV void fwd4_acc_read(float (&o)[17]);\n"
    for t4 in range(NQ):
        rd = [f'"v_accvgpr_read_b32 %{4 * ds + e}, a{O(ds, t4) + e}\\n"' for ds in range(4) for e in range(4)]
        rd.append(f'"v_accvgpr_read_b32 %16, a{LA(t4)}\\n"')
        s += (f"template <>\n__attribute__((always_inline)) DEV void fwd4_acc_read<{t4}>(float (&o)[17]) {{\n"
              f"  asm volatile(" + " ".join(rd) + " : " + ", ".join(f'"=v"(o[{e}])' for e in range(17)) + ");\n}\n")
    return s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stats", action="store_true")
    args = ap.parse_args()
    self_check()
    parts = []
    for masked in (False, True):
        for slot in range(NSLOT):
            parts.append(emit_tile(slot, masked))
    for slot in range(NSLOT):
        parts.append(emit_run(slot))
    if args.stats:
        for p in parts:
            print(p.split("\n")[0], file=sys.stderr)
        return
    disp = ["template <bool MASKED>",
            "__attribute__((always_inline)) DEV void fwd4_tile(int slot, const W4Lane& f, const W4Scalar& s, int fl) {"]
    for masked in (False, True):
        nm = f"fwd4_tile_{'masked' if masked else 'full'}"
        disp.append(f"  if constexpr ({'MASKED' if masked else '!MASKED'}) {{")
        disp.append(f"    if (slot == 0) {nm}_s0(f, s, fl); else if (slot == 1) {nm}_s1(f, s, fl); else {nm}_s2(f, s, fl);")
        disp.append("  }")
    disp += ["}", "",
             "__attribute__((always_inline)) DEV void fwd4_run(int slot, int n, int dl, const W4Lane& f, const W4Scalar& s,",
             "                                              int fl, unsigned kstep, unsigned vstep) {",
             "  if (slot == 0) fwd4_run_s0(n, dl, f, s, fl, kstep, vstep);",
             "  else if (slot == 1) fwd4_run_s1(n, dl, f, s, fl, kstep, vstep);",
             "  else fwd4_run_s2(n, dl, f, s, fl, kstep, vstep);", "}", ""]
    hdr = ("// GENERATED by tools/gen_fwd4_asm.py -- do not edit.  The hand-placed statements of attn_fwd4_k\n"
           "// (attn_fwd4.hip): see the generator's docstring for the schedule.\n#pragma once\n\n"
           "// per-lane operands (VGPR): K fragment row offsets (k-step 0 / 1), V^T fragment offsets (column\n"
           "// group ds), the ring DMA's source offsets (K / V rows h); PARTIAL tiles: the allowed key range of\n"
           "// each query tile relative to the tile and to the lane's 4 g rows\n"
           "struct W4Lane {\n  unsigned kr[2], vt[4], ko[2], vo[2];\n  int mlo[8], mhi[8];\n};\n"
           "// wave-uniform: M0 base of this wave's DMA rows, the DMA sources (K / V tile t + 2)\n"
           "struct W4Scalar {\n  unsigned m0k;\n  const void *kb, *vb;\n};\n\n")
    with open(OUT, "w") as f:
        f.write(hdr + emit_helpers() + "\n" + "\n".join(parts) + "\n" + "\n".join(disp))
    print("wrote", OUT, file=sys.stderr)


if __name__ == "__main__":
    main()
