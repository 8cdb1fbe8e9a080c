"""Time one optimizer step (Muon + AdamW, libowlk Newton-Schulz) and one EMA update at dit_v4,
with random gradients in the reducer's flat buckets (N = 1).

    python tools/opt_bench.py [--config configs/dit_v4.yml] [--iters 5]
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "owl-audio-exps_amd")]
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="configs/dit_v4.yml")
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    from owl_wms import _lib
    from owl_wms.configs import Config
    from owl_wms.models import get_model_cls
    from owl_wms.muon import init_muon
    from owl_wms.utils.grad_reducer import EMA, GradReducer

    cfg = Config.from_yaml(os.path.join(REPO, args.config))
    torch.manual_seed(0)
    model = get_model_cls(cfg.model.model_id)(cfg.model).cuda().train()
    opt = init_muon(model, rank=0, world_size=1, **cfg.train.opt_kwargs)
    ema = EMA(model, beta=0.999)
    red = GradReducer(model.parameters(), world_size=1)
    for buf in red.flat:
        buf.normal_(0.0, 1e-3)

    def timed(fn, label):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        for _ in range(args.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / args.iters * 1e3
        print(f"{label:12s} {e0.elapsed_time(e1) / args.iters:8.2f} ms GPU span  {wall:8.2f} ms wall", flush=True)

    timed(opt.adamw.step, "adamw")
    timed(opt.muon.step, "muon")
    timed(ema.update, "ema")
    _lib.profile_begin()
    opt.muon.step()
    prof = _lib.profile_end()
    for k, (n, ms, fl) in sorted(prof.items(), key=lambda kv: -kv[1][1])[:12]:
        print(f"  {k:60s} n={n:3d} {ms:8.3f} ms  {fl / max(ms, 1e-9) / 1e9:7.1f} TF/s")


if __name__ == "__main__":
    main()
