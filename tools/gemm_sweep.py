"""Per-tile cost model of the 256^2 GEMM: time vs K at M = 98,304, N = 6,144 (t = c K + o per
tile-round), and the fused-epilogue variants at K = 1,536.

    python tools/gemm_sweep.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "owl-audio-exps_amd")]
import torch  # noqa: E402

from owl_wms import kernels as K  # noqa: E402
from gemm_bench import timeit  # noqa: E402


def main():
    M, N = 98304, 6144
    rounds = (M // 256) * (N // 256) / 256
    r = lambda *s: (torch.randn(*s, device="cuda") * 0.5).to(torch.bfloat16)
    for Kd in (64, 128, 256, 512, 1536, 3072):
        A, B = r(M, Kd), r(N, Kd)
        t = timeit(lambda: K.gemm(A, B), iters=10)
        print(f"K={Kd:5d}  {t:7.3f} ms  per tile-round {t / rounds * 1e3:7.2f} us  {2.0 * M * N * Kd / t / 1e9:7.1f} TF/s",
              flush=True)
    Kd = 1536
    A, B = r(M, Kd), r(N, Kd)
    bias = torch.randn(N, device="cuda") * 0.1
    aux, res, g = r(M, N), r(M, N), r(M // 64, N)
    cs = torch.zeros(N, device="cuda")
    cases = [("store", lambda: K.gemm(A, B)), ("store+bias", lambda: K.gemm(A, B, bias=bias)),
             ("silu", lambda: K.gemm(A, B, bias=bias, epi=K.EPI_SILU, aux=aux)),
             ("dsilu", lambda: K.gemm(A, B, epi=K.EPI_DSILU, aux=res)),
             ("dsilu+cs", lambda: K.gemm(A, B, epi=K.EPI_DSILU, aux=res, colsum=cs)),
             ("gate_resid", lambda: K.gemm(A, B, bias=bias, epi=K.EPI_GATE_RESID, aux=aux, gate=g, tpf=64, resid=res))]
    for nm, fn in cases:
        t = timeit(fn, iters=10)
        print(f"K=1536 {nm:11s} {t:7.3f} ms  per tile-round {t / rounds * 1e3:7.2f} us  {2.0 * M * N * Kd / t / 1e9:7.1f} TF/s",
              flush=True)


if __name__ == "__main__":
    main()
