"""Decode-shape GEMMs (M = 64 / 128 rows: one frame, or a CFG pair, against dit_v4's weights):
time per call and the weight-streaming rate.  OWLK_GEMM_DECODE=0 selects the older split-K +
reduce-kernel plan for A/B.

    python tools/decode_gemm_bench.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "owl-audio-exps_amd")]
import torch  # noqa: E402

from owl_wms import kernels as K  # noqa: E402


def timeit(fn, iters=50, reps=10):
    """GPU time per call: the calls are captured into a HIP graph and replayed (a Python loop of
    launches is CPU-bound at these sizes, ~14 us per call)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (iters * reps) * 1e3  # us


def main():
    d = 1536
    torch.manual_seed(0)
    r = lambda *s: (torch.randn(*s, device="cuda") * 0.5).to(torch.bfloat16)
    wq, wo, w1, w2 = r(3 * d, d), r(d, d), r(4 * d, d), r(d, 4 * d)
    b3, b1, b4 = (torch.zeros(n, device="cuda") for n in (3 * d, d, 4 * d))
    for M in (64, 128):
        x, h, res = r(M, d), r(M, 4 * d), r(M, d)
        gate = r(max(M // 64, 1), d)
        aux4, aux1 = torch.empty(M, 4 * d, device="cuda", dtype=torch.bfloat16), torch.empty_like(res)
        cases = [
            ("qkv+bias", wq, lambda: K.gemm(x, wq, bias=b3)),
            ("out gate", wo, lambda: K.gemm(x, wo, epi=K.EPI_GATE_RESID, bias=b1, aux=aux1, gate=gate, tpf=64,
                                            resid=res)),
            ("fc1 silu", w1, lambda: K.gemm(x, w1, epi=K.EPI_SILU, bias=b4, aux=aux4)),
            ("fc2 gate", w2, lambda: K.gemm(h, w2, epi=K.EPI_GATE_RESID, bias=b1, aux=aux1, gate=gate, tpf=64,
                                            resid=res)),
        ]
        tot = 0.0
        for name, w, fn in cases:
            us = timeit(fn)
            tot += us
            print(f"M {M:3d} {name:9s} {us:7.2f} us  weights {w.numel() * 2 / us / 1e6:6.3f} TB/s", flush=True)
        print(f"M {M:3d} block GEMMs {tot:7.2f} us", flush=True)


if __name__ == "__main__":
    main()
