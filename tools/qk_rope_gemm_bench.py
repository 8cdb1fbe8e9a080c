"""qkv projection + QK-RMSNorm / RoPE at the dit_v4 shape (M 98,304, K 1,536, N 4,608, 24 heads of 64):
the GEMM followed by owlk_qk_rope_fwd against owlk_gemm_qk_rope (one launch), HIP-event timed, median of 20."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "owl-audio-exps_amd")]
import torch  # noqa: E402

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
    M, H, D, Kd = 98304, 24, 64, 1536
    N = 3 * H * D
    g = torch.Generator(device="cuda").manual_seed(0)
    h = torch.randn(M, Kd, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, Kd, device="cuda", generator=g) * 0.03).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g)
    ang = torch.rand(M, D // 2, device="cuda", generator=g) * 6.28
    cos, sin = ang.cos(), ang.sin()

    def two():
        qkv = K.gemm(h, w, bias=bias)
        K.qk_rope_fwd(qkv, H, D, cos, sin, 0, M)

    def gemm_only():
        K.gemm(h, w, bias=bias)

    def one():
        K.gemm_qk_rope(h, w, bias, H, D, cos, sin, 0, M)

    for f in (two, one, gemm_only):
        f()
    torch.cuda.synchronize()
    t2, t1, tg = timed(two), timed(one), timed(gemm_only)
    print(f"qkv GEMM alone {tg:.3f} ms; GEMM + qk_rope_fwd {t2:.3f} ms; fused {t1:.3f} ms -> {t2 - t1:+.3f} ms per block",
          flush=True)


if __name__ == "__main__":
    main()
