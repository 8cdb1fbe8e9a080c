"""Host-side checks of the single-pass backward's work decomposition (csrc/attn_bwd_fused.hip):
the closed forms tile_jlo / tile_jhi (first / last key block that sweeps a query tile) against
their definitions over the blocks' sweep ranges, and that every allowed (query, key) pair of the
reference mask (attn.py:24-62, oracle frame_mask) lies inside its key block's sweep.  The kernel's
own hand-offs are checked against the same definitions on the GPU (counting mode,
tests/test_attn_fused_gpu.py)."""
import itertools

import pytest
import torch

from oracle import ref_ops as R
from tests.test_attn_fused_gpu import FQT, _jrange, _sweeps

FKB = 256


def _frame(i, tpf):
    return i // tpf


def tile_jlo(L, tpf, causal, window, i):  # attn_bwd_fused.hip tile_jlo
    if not window:
        return 0
    x = (_frame(i * FQT, tpf) - window + 1) * tpf
    return x // FKB if x > 0 else 0


def tile_jhi(L, tpf, causal, window, i):  # attn_bwd_fused.hip tile_jhi
    nkb = (L + FKB - 1) // FKB
    ql = min(i * FQT + FQT - 1, L - 1)
    f = _frame(ql, tpf)
    if not causal:
        if not window:
            return nkb - 1
        f += window - 1
    ke = min((f + 1) * tpf, L)
    return min((ke - 1) // FKB, nkb - 1)


CASES = list(itertools.product([1, 7, 64, 65, 100], [300, 1000, 4160, 4097], [True, False], [None, 1, 3, 16, 100]))


@pytest.mark.parametrize("tpf,L,causal,window", CASES)
def test_fused_tile_contributors_closed_forms(tpf, L, causal, window):
    lo, hi = _jrange(L, tpf, causal, window, FKB)
    for i in range(len(lo)):
        assert tile_jlo(L, tpf, causal, window, i) == lo[i].item(), i
        assert tile_jhi(L, tpf, causal, window, i) == hi[i].item(), i


@pytest.mark.parametrize("tpf,L,causal,window", [c for c in CASES if c[1] <= 1000])
def test_fused_sweeps_cover_the_mask(tpf, L, causal, window):
    m = R.frame_mask(L, L, tpf, window, None, causal=causal)[0]
    sw = _sweeps(L, tpf, causal, window, FKB)
    q, k = torch.nonzero(m, as_tuple=True)
    tiles, blocks = q // FQT, k // FKB
    lo = torch.tensor([a for a, _ in sw])[blocks]
    hi = torch.tensor([b for _, b in sw])[blocks]
    assert bool(((tiles >= lo) & (tiles <= hi)).all())


# ---- packed documents (causal; kv_lo / q_hi per frame, the runs form of kernels.frame_arrays)
def _doc_runs(nf, lens):
    doc = torch.zeros(1, nf, dtype=torch.int64)
    f = d = 0
    for n in lens:
        doc[0, f:f + n] = d
        f, d = f + n, d + 1
    doc[0, f:] = d
    return doc


def _sweeps_runs(L, tpf, q_hi):
    """attn_bwd_fused.hip with packed documents: block j sweeps from its first key's frame to the
    last query that sees its last key (q_hi_end_runs)"""
    out = []
    for j in range((L + FKB - 1) // FKB):
        f0, f1 = (j * FKB) // tpf, min(j * FKB + FKB - 1, L - 1) // tpf
        out.append(((f0 * tpf) // FQT, (min(L, (int(q_hi[f1]) + 1) * tpf) - 1) // FQT))
    return out


DOC_CASES = [(tpf, nf, lens, window) for tpf, nf, lens in
             [(64, 24, [5, 9, 3]), (65, 30, [10, 13]), (1, 300, [37, 100, 1, 62]), (7, 150, [1, 1, 40, 3, 60]),
              (64, 64, [16, 16, 16]), (100, 40, [39])]
             for window in (None, 4, 16)]


@pytest.mark.parametrize("tpf,nf,lens,window", DOC_CASES)
def test_fused_packed_documents_first_contributor(tpf, nf, lens, window):
    """fused_jlo_k's rule, tile i's first contributor = the block of key kv_lo[frame(i FQT)] tpf,
    against the definition over the sweeps; the last contributor keeps the causal closed form; and
    every allowed pair of the reference mask with the document predicate lies inside its block's
    sweep."""
    from owl_wms.kernels import frame_arrays
    L = nf * tpf
    doc = _doc_runs(nf, lens)
    a = frame_arrays(doc, nf, window)
    assert a["runs"]
    kv_lo, q_hi = a["kv_lo"][0], a["q_hi"][0]
    sw = _sweeps_runs(L, tpf, q_hi)
    for i in range((L + FQT - 1) // FQT):
        js = [j for j, (lo, hi) in enumerate(sw) if lo <= i <= hi]
        assert js == list(range(js[0], js[-1] + 1))
        assert (int(kv_lo[(i * FQT) // tpf]) * tpf) // FKB == js[0], i
        assert tile_jhi(L, tpf, True, None, i) == js[-1], i
    m = R.frame_mask(L, L, tpf, window, doc, causal=True)[0]
    q, k = torch.nonzero(m, as_tuple=True)
    tiles, blocks = q // FQT, k // FKB
    lo = torch.tensor([x for x, _ in sw])[blocks]
    hi = torch.tensor([y for _, y in sw])[blocks]
    assert bool(((tiles >= lo) & (tiles <= hi)).all())
    # each key's visible queries are the one range [fk tpf, (q_hi[fk] + 1) tpf) the kernel masks with
    fk = torch.arange(L) // tpf
    kf = fk[k]
    assert bool(((q >= kf * tpf) & (q < (q_hi[kf].long() + 1) * tpf)).all())
    assert int(m.sum()) == int(sum(min(L, (int(q_hi[f]) + 1) * tpf) - f * tpf for f in fk.tolist()))
