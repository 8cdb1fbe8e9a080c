"""Column sums (bias gradients) at the dit_v4 shapes.

    python tools/colsum_bench.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "owl-audio-exps_amd")]
import torch  # noqa: E402

from owl_wms import kernels as K  # noqa: E402
from gemm_bench import timeit  # noqa: E402


def main():
    for R, N in ((98304, 4608), (98304, 6144), (98304, 1536), (1536, 3072)):
        x = torch.randn(R, N, device="cuda").to(torch.bfloat16)
        out = torch.zeros(N, device="cuda")
        t = timeit(lambda: K.colsum(x, out=out), iters=20)
        print(f"colsum [{R}x{N}] {t * 1e3:8.1f} us  {R * N * 2 / t / 1e9:6.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
