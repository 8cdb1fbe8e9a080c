"""The one-wave-per-SIMD attention forward (attn_fwd4.hip, head_dim 64, bounded softmax) against
attn_fwd16_k (OWLK_FWD4=0, the form every other forward test covers) and the CPU oracle.

Both kernels form every output element with the same products in the same order (q' = bf16(c q),
P = exp2(S) in bf16, one 16x16x32 chain per O^T / row-sum tile over the key parts in sweep order),
so O and lse must agree bit for bit; the oracle bounds both (rel 1e-2).  The cases
cover the pipelined run (long causal sweeps), the one-tile statement (diagonal, window edges),
ragged key tiles (tpf 65, Lkv % 64 != 0), query blocks past Lq, non-causal and token-causal masks.
"""
import pytest
import torch

from oracle import ref_ops as R

pytestmark = pytest.mark.gpu

DEV = "cuda"
D = 64


def K():
    from owl_wms import kernels
    return kernels


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.fixture(scope="module", autouse=True)
def _needs_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from owl_wms._lib import lib
    lib()


CASES = [  # (B, H, n_frames, tpf, window, causal)
    (1, 2, 16, 64, None, True),
    (2, 3, 20, 64, None, True),
    (1, 2, 7, 65, None, True),
    (1, 2, 40, 64, 64, True),
    (1, 2, 130, 65, 70, True),
    (1, 2, 24, 64, None, False),
    (1, 2, 150, 64, 70, False),
    (1, 1, 300, 1, None, True),
    (1, 2, 96, 64, None, True),
    (1, 1, 131, 64, 64, True),
]


def inputs(B, H, L, seed):
    g = torch.Generator().manual_seed(seed)
    unit = lambda t: (t.view(-1, H, D) * torch.rsqrt(t.view(-1, H, D).pow(2).mean(-1, keepdim=True))).view(B, L, H * D)
    q = unit(torch.randn(B, L, H * D, generator=g)).bfloat16()
    k = unit(torch.randn(B, L, H * D, generator=g)).bfloat16()
    v = torch.randn(B, L, H * D, generator=g).bfloat16()
    return q.to(DEV), k.to(DEV), v.to(DEV)


@pytest.mark.parametrize("case", CASES)
def test_fwd4_bitwise_vs_fwd16(case, monkeypatch):
    k = K()
    B, H, nf, tpf, window, causal = case
    L = nf * tpf
    q, kk, v = inputs(B, H, L, seed=nf * 7 + tpf)
    mask = k.FrameMask(tpf, window, causal)
    monkeypatch.setenv("OWLK_FWD4", "0")
    o0, lse0 = k.attn_fwd(q, kk, v, H, D, mask, score_bound=k.qk_norm_bound(D))
    monkeypatch.setenv("OWLK_FWD4", "1")
    o1, lse1 = k.attn_fwd(q, kk, v, H, D, mask, score_bound=k.qk_norm_bound(D))
    torch.cuda.synchronize()
    assert torch.isfinite(o1.float()).all()
    assert torch.equal(o0, o1), f"O differs: rel {rel(o1, o0):.3e}"
    assert torch.equal(lse0, lse1), f"lse differs: max {(lse1 - lse0).abs().max().item():.3e}"
    if L <= 2048:
        ref = R.attention(*(t.cpu().float().view(B, L, H, D).transpose(1, 2) for t in (q, kk, v)),
                          R.frame_mask(L, L, tpf, window, causal=causal))
        assert rel(o1.view(B, L, H, D).transpose(1, 2), ref) < 1e-2


def test_fwd4_deterministic(monkeypatch):
    k = K()
    B, H, nf, tpf = 1, 2, 48, 64
    L = nf * tpf
    q, kk, v = inputs(B, H, L, seed=5)
    mask = k.FrameMask(tpf, None, True)
    monkeypatch.setenv("OWLK_FWD4", "1")
    o1, lse1 = k.attn_fwd(q, kk, v, H, D, mask, score_bound=k.qk_norm_bound(D))
    o2, lse2 = k.attn_fwd(q, kk, v, H, D, mask, score_bound=k.qk_norm_bound(D))
    assert torch.equal(o1, o2) and torch.equal(lse1, lse2)
