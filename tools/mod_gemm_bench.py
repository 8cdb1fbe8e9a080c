"""The per-block modulation GEMMs at dit_v4's per-frame shape (F = 1536 frames, d = 1536, 6d = 9216):
forward [F, d] x [6d, d]^T, dX [F, 6d] x [6d, d] (bf16 out vs fp32 split-K + cast), dW.

    python tools/mod_gemm_bench.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "owl-audio-exps_amd"), os.path.join(REPO, "tools")]
import torch  # noqa: E402

from owl_wms import kernels as K  # noqa: E402
from decode_gemm_bench import timeit  # noqa: E402

F_, d = 1536, 1536
r = lambda *s: (torch.randn(*s, device="cuda") * 0.5).to(torch.bfloat16)
x, W, dm = r(F_, d), r(6 * d, d), r(F_, 6 * d)
bias = torch.zeros(6 * d, device="cuda")
cases = [
    ("fwd [F x 6d x d]", lambda: K.gemm(x, W, bias=bias)),
    ("dX bf16 [F x d x 6d]", lambda: K.gemm(dm, W, b_trans=True)),
    ("dX f32 split + cast", lambda: K.gemm(dm, W, b_trans=True, out_f32=True).to(torch.bfloat16)),
    ("dW one [6d x d x F]", lambda: K.gemm_wgrad(dm, x)),
    ("dW four slices", lambda: [K.gemm_wgrad(dm[:, a:b], x) for a, b in ((0, 2 * d), (2 * d, 3 * d), (3 * d, 5 * d),
                                                                          (5 * d, 6 * d))]),
]
for name, fn in cases:
    print(f"{name:24s} {timeit(fn, iters=20, reps=5):8.1f} us", flush=True)
