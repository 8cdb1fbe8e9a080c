"""Decode attention (one 64-token frame per (batch, head), B = 2 for a CFG pair, 24 heads, D 64,
unmasked over [cache | frame]) per call, timed over HIP-graph replays.  OWLK_FWD_SPLIT=0 selects
the single-wave-per-block kernel for A/B.

    python tools/attn_decode_bench.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "owl-audio-exps_amd")]
import torch  # noqa: E402

from owl_wms import kernels as K  # noqa: E402
sys.path.insert(0, os.path.join(REPO, "tools"))
from decode_gemm_bench import timeit  # noqa: E402


def main():
    B, H, D, Lq = 2, 24, 64, 64
    torch.manual_seed(0)
    mask = K.FrameMask(1, None, False, 0, None)
    for frames in (4, 9, 16, 32, 61):
        Lkv = frames * 64
        q = torch.randn(B, Lq, H * D, device="cuda").bfloat16()
        k = torch.randn(B, Lkv, H * D, device="cuda").bfloat16()
        v = torch.randn(B, Lkv, H * D, device="cuda").bfloat16()
        qk = lambda t: (t.float().view(*t.shape[:2], H, D) * torch.rsqrt(t.float().view(*t.shape[:2], H, D)
                        .pow(2).mean(-1, keepdim=True))).bfloat16().view(t.shape)
        q, k = qk(q), qk(k)
        o = torch.empty_like(q)
        us = timeit(lambda: K.attn_fwd(q, k, v, H, D, mask, o=o, score_bound=K.qk_norm_bound(D)))
        print(f"Lkv {Lkv:5d} ({frames:2d} frames): {us:7.2f} us", flush=True)


if __name__ == "__main__":
    main()
