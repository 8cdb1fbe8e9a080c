"""HBM-bound fused passes at the dit_v4 shape (T = 98,304 tokens, d = 1536, 64 tokens per frame):
time per call (HIP-graph replay) and the rate of their algorithmic bytes.

    python tools/ew_bench.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "owl-audio-exps_amd"), os.path.join(REPO, "tools")]
import torch  # noqa: E402

from owl_wms import kernels as K  # noqa: E402
from decode_gemm_bench import timeit  # noqa: E402

T, d, tpf = 98304, 1536, 64
F_ = T // tpf
r = lambda *s: (torch.randn(*s, device="cuda") * 0.5).to(torch.bfloat16)
x, dy, dres, y = r(T, d), r(T, d), r(T, d), r(T, d)
mod = r(F_, 2 * d)
g = r(F_, d)
_, rstd = K.adaln_fwd(x, mod[:, :d], mod[:, d:], tpf)
cases = [
    ("adaln_fwd", 4 * d, lambda: K.adaln_fwd(x, mod[:, :d], mod[:, d:], tpf)),
    ("adaln_bwd", 8 * d, lambda: K.adaln_bwd(dy, x, rstd, mod[:, :d], tpf, dres=dres)),
    ("gate_bwd", 6 * d, lambda: K.gate_bwd(dy, y, g, tpf)),
]
for name, bpt, fn in cases:
    us = timeit(fn, iters=10, reps=5)
    print(f"{name:10s} {us:8.1f} us  {bpt * T / us / 1e6:5.2f} TB/s", flush=True)
