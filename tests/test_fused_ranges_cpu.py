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
