"""Out-projection dX + attention delta at the dit_v4 shape (M 98,304, N = K = 1,536, 24 heads of 64):
the GEMM followed by owlk_attn_delta against owlk_gemm_attn_delta (one launch), HIP-event timed,
median of 20."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "owl-audio-exps_amd")]
import torch  # noqa: E402

from owl_wms import _lib  # noqa: E402
from owl_wms import kernels as K  # noqa: E402


def timed(fn, n=20):
    ts = []
    for _ in range(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[n // 2]


def main():
    M, H, D = 98304, 24, 64
    N = Kd = H * D
    g = torch.Generator(device="cuda").manual_seed(0)
    dy = torch.randn(M, Kd, device="cuda", generator=g).bfloat16()
    w = (torch.randn(Kd, N, device="cuda", generator=g) * 0.03).bfloat16()
    o = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    delta = torch.empty(1, H, M, device="cuda")

    def two():
        do = K.gemm(dy, w, b_trans=True)
        _lib.call("owlk_attn_delta", _lib.ptr(o), _lib.ptr(do), N, 1, M, H, D, _lib.ptr(delta), _lib.stream())

    def gemm_only():
        K.gemm(dy, w, b_trans=True)

    def one():
        K.gemm_attn_delta(dy, w, o, H, D, M)

    for f in (two, one, gemm_only):
        f()
    torch.cuda.synchronize()
    t2, t1, tg = timed(two), timed(one), timed(gemm_only)
    print(f"dX GEMM alone {tg:.3f} ms; GEMM + attn_delta {t2:.3f} ms; fused {t1:.3f} ms -> {t2 - t1:+.3f} ms per block",
          flush=True)


if __name__ == "__main__":
    main()
