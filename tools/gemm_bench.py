"""Time libowlk GEMMs at the dit_v4 shapes (M = 98,304 tokens) beside torch.matmul (hipBLASLt).

    python tools/gemm_bench.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "owl-audio-exps_amd")]
import torch  # noqa: E402

from owl_wms import kernels as K  # noqa: E402


def timeit(fn, iters=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--wgrad-only", action="store_true", help="only the split-K weight-gradient GEMMs, no hipBLASLt")
    args = ap.parse_args()
    T, d = 98304, 1536
    torch.manual_seed(0)
    r = lambda *s: (torch.randn(*s, device="cuda") * 0.5).to(torch.bfloat16)
    cases = [  # (name, A, B, a_trans, b_trans, M, N, K)
        ("qkv fwd", r(T, d), r(3 * d, d), False, False),
        ("fc1 fwd", r(T, d), r(4 * d, d), False, False),
        ("fc2 fwd", r(T, 4 * d), r(d, 4 * d), False, False),
        ("out fwd", r(T, d), r(d, d), False, False),
        ("fc2 dX", r(T, d), r(d, 4 * d), False, True),
        ("qkv dX", r(T, 3 * d), r(3 * d, d), False, True),
        ("fc1 dW", r(T, 4 * d), r(T, d), True, True),
        ("fc2 dW", r(T, d), r(T, 4 * d), True, True),
        ("qkv dW", r(T, 3 * d), r(T, d), True, True),
        ("out dW", r(T, d), r(T, d), True, True),
    ]
    for name, A, B, at, bt in cases:
        if args.wgrad_only and not at:
            continue
        M = A.shape[1] if at else A.shape[0]
        N = B.shape[1] if bt else B.shape[0]
        Kd = A.shape[0] if at else A.shape[1]
        fl = 2.0 * M * N * Kd
        if at:
            ours = timeit(lambda: K.gemm_wgrad(A, B))
        else:
            ours = timeit(lambda: K.gemm(A, B, b_trans=bt))
        if args.wgrad_only:
            print(f"{name:8s} [{M}x{N}x{Kd}]  owlk {ours:7.3f} ms {fl / ours / 1e9:7.1f} TF/s", flush=True)
            continue
        Am = A.T if at else A
        Bm = B if bt else B.T
        ref = timeit(lambda: torch.matmul(Am, Bm))
        print(f"{name:8s} [{M}x{N}x{Kd}]  owlk {ours:7.3f} ms {fl / ours / 1e9:7.1f} TF/s | "
              f"hipBLASLt {ref:7.3f} ms {fl / ref / 1e9:7.1f} TF/s", flush=True)
    if args.wgrad_only:
        return
    # fused epilogues at the block's shapes (fused.py): fc1 + SiLU, fc1 dX + dSiLU + bias-grad colsum,
    # out-proj / fc2 + gate + residual
    x, w1, w2, wo = r(T, d), r(4 * d, d), r(d, 4 * d), r(d, d)
    h, dy = r(T, 4 * d), r(T, d)
    aux4, aux1 = torch.empty_like(h), torch.empty_like(dy)
    b4, b1 = torch.zeros(4 * d, device="cuda"), torch.zeros(d, device="cuda")
    gate, cs = r(T // 64, d), torch.zeros(4 * d, device="cuda")
    epis = [
        ("fc1 silu", 2.0 * T * 4 * d * d, lambda: K.gemm(x, w1, epi=K.EPI_SILU, bias=b4, aux=aux4)),
        ("fc1 dsilu", 2.0 * T * 4 * d * d, lambda: K.gemm(dy, w2, b_trans=True, epi=K.EPI_DSILU, aux=h, colsum=cs)),
        ("fc2 gate", 2.0 * T * d * 4 * d, lambda: K.gemm(h, w2, epi=K.EPI_GATE_RESID, bias=b1, aux=aux1, gate=gate,
                                                        tpf=64, resid=dy)),
        ("out gate", 2.0 * T * d * d, lambda: K.gemm(x, wo, epi=K.EPI_GATE_RESID, bias=b1, aux=aux1, gate=gate,
                                                    tpf=64, resid=dy)),
    ]
    for name, fl, fn in epis:
        ours = timeit(fn)
        print(f"{name:9s} owlk {ours:7.3f} ms {fl / ours / 1e9:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
