"""Is the GEMM epilogue bound per CU or chip-wide?  One round of 256^2 tiles at K = 1536 on 64,
128 and 256 CUs (tiles), plain store and SiLU (two outputs); compare with the OWLK_GEMM_EXP_NOEPI
build (tools/build_variant.sh) to get the epilogue's share.

    python tools/epi_probe.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "owl-audio-exps_amd"), os.path.join(REPO, "tools")]
import torch  # noqa: E402

from owl_wms import kernels as K  # noqa: E402
from decode_gemm_bench import timeit  # noqa: E402

Kd = 1536
r = lambda *s: (torch.randn(*s, device="cuda") * 0.5).to(torch.bfloat16)
for tiles_m, tiles_n in ((8, 8), (16, 8), (16, 16), (32, 16)):
    M, N = 256 * tiles_m, 256 * tiles_n
    A, B = r(M, Kd), r(N, Kd)
    aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    bias = torch.zeros(N, device="cuda")
    t0 = timeit(lambda: K.gemm(A, B), iters=20, reps=5)
    t1 = timeit(lambda: K.gemm(A, B, epi=K.EPI_SILU, bias=bias, aux=aux), iters=20, reps=5)
    print(f"{tiles_m * tiles_n:4d} tiles: store {t0:7.1f} us  silu {t1:7.1f} us", flush=True)
