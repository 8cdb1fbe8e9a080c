"""AdaLN backward + gate backward at the dit_v4 shape (T 98,304, d 1,536, 64 tokens per frame): the two
passes against owlk_adaln_gate_bwd (one pass), HIP-event timed, median of 20."""
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
    T, d, tpf = 98304, 1536, 64
    F = T // tpf
    g = torch.Generator(device="cuda").manual_seed(0)
    r = lambda *s: torch.randn(*s, device="cuda", generator=g).bfloat16()
    x, dh, dres, y = r(T, d), r(T, d), r(T, d), r(T, d)
    mod, gate = r(F, 2 * d) * 0.3, r(F, d)
    _, rstd = K.adaln_fwd(x, mod[:, :d], mod[:, d:], tpf)
    dm = torch.zeros(F, 3 * d, device="cuda", dtype=torch.bfloat16)

    def two():
        dx = K.adaln_bwd_into(dh, x, rstd, mod[:, :d], tpf, dm[:, d:], dres=dres)
        K.gate_bwd(dx, y, gate, tpf, dg_out=dm[:, :d])

    def adaln_only():
        K.adaln_bwd_into(dh, x, rstd, mod[:, :d], tpf, dm[:, d:], dres=dres)

    def one():
        K.adaln_gate_bwd_into(dh, x, rstd, mod[:, :d], tpf, dm[:, d:], dres, y, gate, dm[:, :d])

    for f in (two, one):
        f()
    torch.cuda.synchronize()
    t2, t1, ta = timed(two), timed(one), timed(adaln_only)
    gb = T * d * 2 / 1e9
    print(f"adaln_bwd alone {ta:.3f} ms ({4 * gb / ta:.2f} TB/s: dy, x, dres in, dx out)")
    print(f"adaln_bwd + gate_bwd {t2:.3f} ms ({8 * gb / t2:.2f} TB/s alg); fused {t1:.3f} ms "
          f"({6 * gb / t1:.2f} TB/s alg: dy, x, dres, y in, dx, dyg out)  -> {t2 - t1:+.3f} ms per block", flush=True)


if __name__ == "__main__":
    main()
