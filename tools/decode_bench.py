"""Decode (AVCachingSamplerV2) wall time per generated frame, eager vs HIP-graph replay
(compile_on_decode), on a config's model with random-init weights (N = 1).

    python tools/decode_bench.py [--config configs/dit_v4.yml] [--ctx 8] [--frames 4] [--steps 16]
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
    ap.add_argument("--ctx", type=int, default=8)
    ap.add_argument("--frames", type=int, default=4)
    ap.add_argument("--steps", type=int, default=16)
    ap.add_argument("--cfg", type=float, default=1.3)
    args = ap.parse_args()
    from owl_wms.configs import Config
    from owl_wms.models import get_model_cls
    from owl_wms.sampling import get_sampler_cls
    cfg = Config.from_yaml(os.path.join(REPO, args.config))
    torch.manual_seed(0)
    model = get_model_cls(cfg.model.model_id)(cfg.model).cuda().eval()
    mc = cfg.model
    n = args.ctx + args.frames
    x = torch.randn(1, args.ctx, mc.channels, mc.sample_size, mc.sample_size, device="cuda").bfloat16()
    mouse = torch.randn(1, n, 2, device="cuda").bfloat16()
    btn = (torch.rand(1, n, mc.n_buttons, device="cuda") < 0.5).bfloat16()
    res = {}
    for graphed in (False, True, False, True):
        torch.manual_seed(1)
        s = get_sampler_cls("av_caching")(n_steps=args.steps, cfg_scale=args.cfg, num_frames=args.frames)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = s(model.core, x, mouse, btn, compile_on_decode=graphed)
        torch.cuda.synchronize()
        res[graphed] = ((time.perf_counter() - t0) * 1e3 / args.frames, out)
        print(f"{'graph' if graphed else 'eager'}: {res[graphed][0]:.1f} ms per generated frame "
              f"(ctx {args.ctx}, {args.frames} frames, {args.steps} steps, cfg {args.cfg})", flush=True)
    print("bit-identical:", torch.equal(res[False][1], res[True][1]),
          f"speedup {res[False][0] / res[True][0]:.2f}x")


if __name__ == "__main__":
    main()
