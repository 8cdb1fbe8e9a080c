"""The dit_v4 step's fused-epilogue GEMMs (M = 98,304 tokens, d = 1,536) on the library OWLK_LIB names:
per-launch time, and with --save the outputs of small cases of every epilogue, for a bit-exact
comparison between two builds (--compare a.pt b.pt).

    OWLK_LIB=.../libowlk_g1.so python tools/gemm_epi_bench.py [--save out.pt] [--iters 10]
    python tools/gemm_epi_bench.py --compare a.pt b.pt
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "owl-audio-exps_amd")]
import torch  # noqa: E402


def compare(a, b):
    A, B = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    bad = 0
    for k in sorted(A):
        same = torch.equal(A[k], B[k])
        bad += not same
        print(f"{k:28s} {'identical' if same else 'DIFFERENT'}")
    print("all identical" if not bad else f"{bad} outputs differ")
    return bad


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--save")
    ap.add_argument("--compare", nargs=2)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--d", type=int, default=1536, help="model width (dit_v4_5B: 2560)")
    args = ap.parse_args()
    if args.compare:
        sys.exit(1 if compare(*args.compare) else 0)
    from owl_wms import kernels as K
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s: (torch.randn(*s, device=dev, generator=g) * 0.5).to(torch.bfloat16)

    if args.save:  # every epilogue, ragged and frame-strided-free small shapes, saved for --compare
        out = {}
        for M, N, Kd in ((1024, 768, 512), (1000, 512, 256)):
            A, W = r(M, Kd), r(N, Kd) * 0.2
            bias = torch.randn(N, device=dev, generator=g) * 0.1
            aux = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            out[f"store_{M}"] = K.gemm(A, W, bias=bias)
            out[f"store_beta_{M}"] = K.gemm(A, W, out=r(M, N), beta=0.75, alpha=1.25)
            out[f"silu_{M}"] = K.gemm(A, W, bias=bias, epi=K.EPI_SILU, aux=aux)
            out[f"silu_aux_{M}"] = aux.clone()
            gate, res = r((M + 63) // 64, N), r(M, N)
            out[f"gate_{M}"] = K.gemm(A, W, bias=bias, epi=K.EPI_GATE_RESID, aux=aux, gate=gate, tpf=64, resid=res)
            out[f"gate_aux_{M}"] = aux.clone()
            x, act, cs = r(M, N), torch.empty(M, N, device=dev, dtype=torch.bfloat16), torch.zeros(N, device=dev)
            out[f"dsilu_{M}"] = K.gemm(A, W, epi=K.EPI_DSILU, aux=x, resid=act, colsum=cs)
            out[f"dsilu_act_{M}"] = act
            out[f"dsilu_colsum_{M}"] = cs
            Wt = r(Kd, N)
            out[f"dsilu_bt_{M}"] = K.gemm(A, Wt, b_trans=True, epi=K.EPI_DSILU, aux=x)
            sq = r(N, N)
            out[f"axpby_{M}"] = K.gemm(sq, sq, epi=K.EPI_AXPBY, alpha=2.0315, beta=-4.775, aux=sq)
            out[f"f32_{M}"] = K.gemm(A, W, out_f32=True)
        A2, W2 = r(512, 16384), r(768, 16384)  # split-K fp32 partials (the weight-gradient form)
        out["splitk_f32"] = K.gemm(A2, W2, out_f32=True)
        torch.save({k: v.cpu() for k, v in out.items()}, args.save)
        print(f"saved {len(out)} outputs to {args.save}")

    T, d = 98304, args.d
    x, h = r(T, d), r(T, 4 * d)
    w1, w2, wq, wo = r(4 * d, d) * 0.05, r(d, 4 * d) * 0.05, r(3 * d, d) * 0.05, r(d, d) * 0.05
    b1, b2 = torch.randn(4 * d, device=dev) * 0.1, torch.randn(d, device=dev) * 0.1
    aux4, out4, act4 = (torch.empty(T, 4 * d, device=dev, dtype=torch.bfloat16) for _ in range(3))
    gate, res, aux1 = r(T // 64, d), r(T, d), torch.empty(T, d, device=dev, dtype=torch.bfloat16)
    cs = torch.zeros(4 * d, device=dev)
    cases = [
        ("qkv fwd (store)", lambda: K.gemm(x, wq), 3 * d, d),
        ("fc1 fwd + SiLU", lambda: K.gemm(x, w1, bias=b1, epi=K.EPI_SILU, aux=aux4, out=out4), 4 * d, d),
        ("fc2 fwd + gate", lambda: K.gemm(h, w2, bias=b2, epi=K.EPI_GATE_RESID, aux=aux1, gate=gate, tpf=64,
                                           resid=res), d, 4 * d),
        ("out fwd + gate", lambda: K.gemm(x, wo, bias=b2, epi=K.EPI_GATE_RESID, aux=aux1, gate=gate, tpf=64,
                                           resid=res), d, d),
        ("fc2 dX dSiLU + colsum", lambda: K.gemm(x, w2, b_trans=True, epi=K.EPI_DSILU, aux=aux4, out=out4,
                                                  resid=act4, colsum=cs), 4 * d, d),
        ("fc2 dX plain", lambda: K.gemm(x, w2, b_trans=True, out=out4), 4 * d, d),
    ]
    # the per-frame modulation GEMM of every block (F = 1,536 frames x 6d outputs)
    cf, wm, bm = r(T // 64, d), r(6 * d, d) * 0.05, torch.randn(6 * d, device=dev) * 0.1
    modo = torch.empty(T // 64, 6 * d, device=dev, dtype=torch.bfloat16)
    cases.append(("modulation fwd", lambda: K.gemm(cf, wm, bias=bm, out=modo), 6 * d, d))
    # d cond += d mods [F x 6d] . Wmod [6d x d] (fp32 accumulate, beta 1)
    dmod, cg = r(T // 64, 6 * d), torch.zeros(T // 64, d, device=dev)
    cases.append(("cond grad", lambda: K.gemm(dmod, wm, b_trans=True, out=cg, out_f32=True, beta=1.0), d, 6 * d))
    # modulation weight gradients dW [2d | d x d] += dmods^T . s over the F frames (fp32, beta 1)
    s_ = r(T // 64, d)
    dw2, dw1 = torch.zeros(2 * d, d, device=dev), torch.zeros(d, d, device=dev)
    cases.append(("mod wgrad 2d", lambda: K.gemm(dmod[:, :2 * d], s_, a_trans=True, b_trans=True, out=dw2, out_f32=True,
                                                 beta=1.0), d, T // 64))
    cases.append(("mod wgrad d", lambda: K.gemm(dmod[:, :d], s_, a_trans=True, b_trans=True, out=dw1, out_f32=True,
                                                beta=1.0), d, T // 64))
    for name, fn, N, Kd in cases:
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.iters
        Mr = {"modulation fwd": T // 64, "cond grad": T // 64, "mod wgrad 2d": 2 * d, "mod wgrad d": d}.get(name, T)
        print(f"{name:24s} [{Mr}x{N}x{Kd}] {ms:7.3f} ms {2.0 * Mr * N * Kd / ms / 1e9:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
