"""Quick GPU check of the one-wave-per-SIMD single pass (variant bit 7) against the 8-wave kernel.

    python tools/fused4_check.py [--big] [--time]

Both kernels form every product in the same order (same MFMA chains, same dQ key order), so dQ,
dK and dV must agree bit for bit; prints the first mismatch otherwise.  --time also times both at
the dit_v4 shape (24 heads x 98,304 tokens; global, window 16, window 4).
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "owl-audio-exps_amd")]
import torch  # noqa: E402

from owl_wms import _lib  # noqa: E402
from owl_wms import kernels as K  # noqa: E402

CASES = [  # (B, H, n_frames, tpf, causal, window)
    (1, 2, 8, 64, True, None),
    (2, 3, 20, 64, True, None),
    (1, 2, 7, 65, True, None),
    (1, 1, 300, 1, True, None),
    (1, 2, 40, 64, False, None),
    (2, 8, 48, 64, True, None),
    (1, 2, 48, 64, True, 16),
    (1, 2, 30, 65, True, 4),
    (1, 2, 40, 64, False, 3),
    (1, 1, 600, 1, True, 100),
]


def run(B, H, nf, tpf, causal, window, variants, seed=0):
    D, L = 64, nf * tpf
    g = torch.Generator().manual_seed(seed)
    q, kk, v, do = (torch.randn(B, L, H * D, generator=g).to(torch.bfloat16).cuda() for _ in range(4))
    mask = K.FrameMask(tpf, window, causal)
    o, lse = K.attn_fwd(q, kk, v, H, D, mask)
    delta = torch.empty(B, H, L, device="cuda", dtype=torch.float32)
    _lib.call("owlk_attn_delta", _lib.ptr(o), _lib.ptr(do), o.stride(1), B, L, H, D, _lib.ptr(delta), _lib.stream())
    outs = []
    for var in variants:
        got = [torch.full_like(q, float("nan")) for _ in range(3)]
        ws = K.attn_bwd_fused(q, kk, v, do, lse, delta, H, D, mask, *got, D ** -0.5, var)
        torch.cuda.synchronize()
        err = ws[:256].view(torch.int32)[8].item()
        outs.append((got, err))
    return outs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--time", action="store_true")
    ap.add_argument("--only-time", action="store_true")
    ap.add_argument("--iters", type=int, default=3)
    args = ap.parse_args()
    ok = True
    if not args.only_time:
        for case in CASES:
            (ref, e0), (new, e1) = run(*case, variants=(1, 129))
            line = f"{case}: err words {e0} / {e1}"
            for name, a, b in zip(("dq", "dk", "dv"), ref, new):
                fin = torch.isfinite(b).all().item()
                eq = torch.equal(a, b)
                r = ((a.float() - b.float()).norm() / a.float().norm().clamp_min(1e-30)).item()
                line += f" | {name} eq={eq} finite={fin} rel={r:.2e}"
                ok &= eq and fin and e1 == 0
            print(line, flush=True)
        print("ALL BITWISE EQUAL" if ok else "MISMATCH", flush=True)
    if args.time or args.only_time:
        B, H, L, D = 1, 24, 1536 * 64, 64
        g = torch.Generator().manual_seed(0)
        qkv = torch.randn(1, L, 3 * H * D, generator=g).to(torch.bfloat16).cuda()
        qk = qkv[:, :, :2 * H * D].view(1, L, 2 * H, D)
        qk.copy_((qk.float() * torch.rsqrt(qk.float().pow(2).mean(-1, keepdim=True))).bfloat16())
        q, k, v = qkv[:, :, :H * D], qkv[:, :, H * D:2 * H * D], qkv[:, :, 2 * H * D:]
        do = torch.randn(1, L, H * D, generator=g).to(torch.bfloat16).cuda()
        dq, dk, dv = (torch.empty(1, L, H * D, device="cuda", dtype=torch.bfloat16) for _ in range(3))
        nb = _lib.lib().owlk_attn_bwd_fused_ws_bytes(1, H, L, D)
        ws = torch.empty(nb, device="cuda", dtype=torch.uint8)
        for window in (None, 16, 4):
            mask = K.FrameMask(64, window)
            pairs = K.mask_pairs(mask, L, L) * H
            o, lse = K.attn_fwd(q, k, v, H, D, mask)
            delta = torch.empty(1, H, L, device="cuda", dtype=torch.float32)
            _lib.call("owlk_attn_delta", _lib.ptr(o), _lib.ptr(do), o.stride(1), 1, L, H, D, _lib.ptr(delta),
                      _lib.stream())
            res = {}
            for _ in range(2):
                for var in (1, 129):
                    fn = lambda: K.attn_bwd_fused(q, k, v, do, lse, delta, H, D, mask, dq, dk, dv, D ** -0.5, var, ws)
                    fn()
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(args.iters):
                        fn()
                    e1.record()
                    torch.cuda.synchronize()
                    res.setdefault(var, []).append(e0.elapsed_time(e1) / args.iters)
            err = ws[:256].view(torch.int32)[8].item()
            for var, ts in res.items():
                t = min(ts)
                print(f"window={window} variant {var}: {t:8.3f} ms  {8 * D * pairs / t / 1e9:7.1f} TF/s alg  {ts} err {err}",
                      flush=True)


if __name__ == "__main__":
    main()
