"""QK-RMSNorm + RoPE backward at the dit_v4 shape (98,304 tokens, 24 heads x 64): the plain pass +
a separate column sum of its q / k output (the qkv bias gradient's q / k part) against the fused
owlk_qk_rope_bwd_bias.

    python tools/rope_bwd_bench.py [--heads 24 --dim 64 --tokens 98304]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "owl-audio-exps_amd")]
import torch  # noqa: E402

from owl_wms import kernels as K  # noqa: E402
from gemm_bench import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--heads", type=int, default=24)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--tokens", type=int, default=98304)
    a = ap.parse_args()
    H, D, T = a.heads, a.dim, a.tokens
    pos = torch.arange(T, dtype=torch.float32)[:, None] / (1 + torch.arange(D // 2, dtype=torch.float32))[None]
    cos, sin = pos.cos().cuda(), pos.sin().cuda()
    qkv = torch.randn(T, 3 * H * D, device="cuda").bfloat16()
    _, rstd = K.qk_rope_fwd(qkv, H, D, cos, sin)
    dqk = torch.randn(T, 2 * H * D, device="cuda").bfloat16()
    dqkv = torch.empty(T, 3 * H * D, device="cuda", dtype=torch.bfloat16)
    db = torch.zeros(2 * H * D, device="cuda")
    t_plain = timeit(lambda: K.qk_rope_bwd(dqk, qkv, rstd, H, D, cos, sin, dqkv), iters=20)
    t_cs = timeit(lambda: K.colsum(dqkv[:, :2 * H * D], out=db), iters=20)
    t_fused = timeit(lambda: K.qk_rope_bwd(dqk, qkv, rstd, H, D, cos, sin, dqkv, dbias=db), iters=20)
    gb = T * (2 * H * D * 2 * 2 + 2 * H * D * 2 + 2 * H * 4) / 1e9  # dqk + qkv(q,k) in, dqkv(q,k) out, rstd
    print(f"plain rope bwd {t_plain * 1e3:8.1f} us ({gb / t_plain:5.2f} TB/s) + colsum {t_cs * 1e3:7.1f} us = "
          f"{(t_plain + t_cs) * 1e3:8.1f} us | fused {t_fused * 1e3:8.1f} us ({gb / t_fused:5.2f} TB/s)", flush=True)


if __name__ == "__main__":
    main()
