"""Time the attention kernels at the dit_v4 shape (1 x 24 heads x 98,304 tokens, D 64).

    python tools/attn_bench.py [--frames 1536] [--iters 5] [--heads 20 --dim 128] [--bwd-only]
Reports ms per launch and algorithmic TF/s (allowed pairs only).
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "owl-audio-exps_amd")]
import torch  # noqa: E402

from owl_wms import _lib  # noqa: E402
from owl_wms import kernels as K  # noqa: E402


def timeit(fn, iters):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1536)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--heads", type=int, default=24)
    ap.add_argument("--dim", type=int, default=64, help="head_dim (dit_v4_5B: --heads 20 --dim 128)")
    ap.add_argument("--bwd-only", action="store_true")
    ap.add_argument("--fwd-only", action="store_true")
    ap.add_argument("--windows", default="none,16", help="comma list of frame windows ('none' = global)")
    ap.add_argument("--tpf", type=int, default=64, help="tokens per frame (mmdit_v2: 65)")
    args = ap.parse_args()
    H, D, tpf = args.heads, args.dim, args.tpf
    L = args.frames * tpf
    torch.manual_seed(0)
    qkv = torch.randn(1, L, 3 * H * D, device="cuda", dtype=torch.bfloat16)
    # q, k RMS-normalised per head as in the model (attn.py:84)
    qk = qkv[:, :, :2 * H * D].view(1, L, 2 * H, D)
    qk.copy_((qk.float() * torch.rsqrt(qk.float().pow(2).mean(-1, keepdim=True))).bfloat16())
    q, k, v = qkv[:, :, :H * D], qkv[:, :, H * D:2 * H * D], qkv[:, :, 2 * H * D:]
    do = torch.randn(1, L, H * D, device="cuda", dtype=torch.bfloat16)
    dq, dk, dv = (torch.empty(1, L, H * D, device="cuda", dtype=torch.bfloat16) for _ in range(3))
    for window in [None if w == "none" else int(w) for w in args.windows.split(",")]:
        mask = K.FrameMask(tpf, window)
        pairs = K.mask_pairs(mask, L, L) * H
        o, lse = K.attn_fwd(q, k, v, H, D, mask)
        delta = torch.empty(1, H, L, device="cuda", dtype=torch.float32)
        _lib.call("owlk_attn_delta", _lib.ptr(o), _lib.ptr(do), o.stride(1), 1, L, H, D, _lib.ptr(delta),
                  _lib.stream())
        args_b = (_lib.ptr(q), q.stride(1), q.stride(0), _lib.ptr(k), k.stride(1), k.stride(0), _lib.ptr(v),
                  v.stride(1), v.stride(0), _lib.ptr(do), do.stride(1), do.stride(0), _lib.ptr(lse),
                  _lib.ptr(delta), _lib.ptr(dq), dq.stride(1), dq.stride(0), _lib.ptr(dk), dk.stride(1),
                  dk.stride(0), _lib.ptr(dv), dv.stride(1), dv.stride(0), 1, H, L, L, D, D ** -0.5, tpf,
                  0 if window is None else window, 1, None, None, None, None, 0, _lib.stream())
        if args.bwd_only:
            t_f = t_f0 = float("nan")
        else:
            t_f = timeit(lambda: K.attn_fwd(q, k, v, H, D, mask, o=o, score_bound=K.qk_norm_bound(D)), args.iters)
            t_f0 = timeit(lambda: K.attn_fwd(q, k, v, H, D, mask, o=o), args.iters)
        if args.fwd_only:
            print(f"window={window}: pairs/head={pairs / H:.4e}")
            print(f"  fwd   {t_f:8.3f} ms  {4 * D * pairs / t_f / 1e9:7.1f} TF/s (4 D pairs; fixed-offset softmax)")
            print(f"  fwd0  {t_f0:8.3f} ms  {4 * D * pairs / t_f0 / 1e9:7.1f} TF/s (running-max softmax)", flush=True)
            continue
        t_kv = timeit(lambda: _lib.call("owlk_attn_bwd_dkdv", *args_b), args.iters)
        t_q = timeit(lambda: _lib.call("owlk_attn_bwd_dq", *args_b), args.iters)
        # dK/dV and dQ are independent given delta: the pair back to back on one stream against dQ
        # on a side stream (fork / join by events), same process, interleaved
        side = torch.cuda.Stream()
        args_s = args_b[:-1] + (side.cuda_stream,)

        def serial():
            _lib.call("owlk_attn_bwd_dkdv", *args_b)
            _lib.call("owlk_attn_bwd_dq", *args_b)

        def concurrent():
            side.wait_stream(torch.cuda.current_stream())
            _lib.call("owlk_attn_bwd_dkdv", *args_b)
            _lib.call("owlk_attn_bwd_dq", *args_s)
            torch.cuda.current_stream().wait_stream(side)

        t_ser, t_con = [], []
        for _ in range(2):
            t_ser.append(timeit(serial, args.iters))
            t_con.append(timeit(concurrent, args.iters))
        print(f"window={window}: pairs/head={pairs / H:.4e}")
        print(f"  bwd pair serial {min(t_ser):8.3f} ms, dQ on a side stream {min(t_con):8.3f} ms "
              f"({t_ser} / {t_con})")
        print(f"  fwd   {t_f:8.3f} ms  {4 * D * pairs / t_f / 1e9:7.1f} TF/s (4 D pairs; fixed-offset softmax)")
        print(f"  fwd0  {t_f0:8.3f} ms  {4 * D * pairs / t_f0 / 1e9:7.1f} TF/s (running-max softmax)")
        print(f"  dkdv  {t_kv:8.3f} ms  {6 * D * pairs / t_kv / 1e9:7.1f} TF/s alg (6 D pairs; 8 D executed: "
              f"{8 * D * pairs / t_kv / 1e9:.1f})")
        print(f"  dq    {t_q:8.3f} ms  {2 * D * pairs / t_q / 1e9:7.1f} TF/s alg (2 D pairs; 6 D executed: "
              f"{6 * D * pairs / t_q / 1e9:.1f})")
        print(f"  bwd   {t_kv + t_q:8.3f} ms  {8 * D * pairs / (t_kv + t_q) / 1e9:7.1f} TF/s alg", flush=True)
        if K.fused_bwd_variant(D, mask) is not None or (D == 64 and window is None):
            # single-pass backward (owlk_attn_bwd_fused): both hand-off forms, interleaved
            nb = _lib.lib().owlk_attn_bwd_fused_ws_bytes(1, H, L, D)
            ws = torch.empty(nb, device="cuda", dtype=torch.uint8)
            fvars = [int(x) for x in os.environ.get("FUSED_VARIANTS", "0,1").split(",")]
            t_fu = {v: [] for v in fvars}
            for _ in range(2):
                for var in fvars:
                    t_fu[var].append(timeit(lambda: K.attn_bwd_fused(q, k, v, do, lse, delta, H, D, mask, dq, dk, dv,
                                                                     D ** -0.5, var, ws), args.iters))
            hw = ws[:256].view(torch.int32).cpu()
            err = hw[8].item()
            pw = ws[128:256].view(torch.int64).cpu().tolist()
            if any(pw):  # OWLK_FUSED_PROF builds: cycles per phase, dQ waves | other waves
                names = ("dq", "main", "vmwait", "barrier", "dequeue", "prologue", "epilogue", "dq2")
                for nm, part in (("dQ waves", pw[:8]), ("other waves", pw[8:16])):
                    tot = sum(part) or 1
                    print(f"  fused phases, {nm} (s_memtime cycles, share of the workgroup time): " +
                          ", ".join(f"{n} {v / tot:.3f}" for n, v in zip(names, part)) +
                          f" | {tot:.3e} cycles", flush=True)
            if hw[11].item():  # OWLK_FUSED_STATS builds: the last call's (xcd-local) hand-offs
                print(f"  fused hand-offs (last call): {hw[10].item()} of {hw[11].item()} found the flag down at "
                      f"mid-step ({hw[10].item() / hw[11].item():.3f})", flush=True)
            for var in fvars:
                nm = ("xcd-local" if var & 1 else "write-through") + (f" group {(var >> 2) & 15}" if (var >> 2) & 15 else "") + \
                    (" 1 wave/SIMD" if var & 128 else "")
                t = min(t_fu[var])
                print(f"  fused {t:8.3f} ms  {8 * D * pairs / t / 1e9:7.1f} TF/s alg (8 D pairs; 10 D executed: "
                      f"{10 * D * pairs / t / 1e9:.1f}) [{nm}: {t_fu[var]}] timeout word {err}", flush=True)


if __name__ == "__main__":
    main()
