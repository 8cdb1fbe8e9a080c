"""Where a graphed decode frame's time goes: one eager forward (the cache update), capturing one
Euler step into a HIP graph, and one replay, at 8 context frames (dit_v4, CFG 1.3 as a B = 2 batch).

    python tools/decode_phases.py
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "owl-audio-exps_amd")]
import torch  # noqa: E402


def main():
    from owl_wms.configs import Config
    from owl_wms.models import get_model_cls
    from owl_wms.nn.kv_cache import KVCache
    cfg = Config.from_yaml(os.path.join(REPO, "configs/dit_v4.yml"))
    mc = cfg.model
    torch.manual_seed(0)
    model = get_model_cls(mc.model_id)(mc).cuda().eval().core
    ctx = 8
    B = 2
    x = torch.randn(B, ctx, mc.channels, mc.sample_size, mc.sample_size, device="cuda").bfloat16()
    t = torch.full((B, ctx), 0.2, device="cuda").bfloat16()
    mouse = torch.randn(B, ctx + 1, 2, device="cuda").bfloat16()
    btn = (torch.rand(B, ctx + 1, mc.n_buttons, device="cuda") < 0.5).bfloat16()
    with torch.no_grad():
        kv = KVCache(model.config)
        kv.reset(B)
        kv.enable_cache_updates()
        model(x, t, mouse[:, :ctx], btn[:, :ctx], kv_cache=kv)
        kv.disable_cache_updates()
        model.transformer.enable_decoding()
        xf, tf = torch.randn(B, 1, *x.shape[2:], device="cuda").bfloat16(), torch.ones(B, 1, device="cuda").bfloat16()
        mf, bf = mouse[:, ctx:ctx + 1], btn[:, ctx:ctx + 1]
        for _ in range(3):
            model(xf, tf, mf, bf, kv_cache=kv)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            model(xf, tf, mf, bf, kv_cache=kv)
        torch.cuda.synchronize()
        eager = (time.perf_counter() - t0) / 5 * 1e3
        t0 = time.perf_counter()
        for _ in range(5):
            model(xf, tf, mf, bf, kv_cache=kv)
        host = (time.perf_counter() - t0) / 5 * 1e3  # launch-only (no sync)
        torch.cuda.synchronize()
        sx = xf.clone()
        g = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(side):
            with torch.cuda.graph(g, stream=side):
                out = model(sx, tf, mf, bf, kv_cache=kv)
        torch.cuda.synchronize()
        cap = (time.perf_counter() - t0) * 1e3
        g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(16):
            g.replay()
        torch.cuda.synchronize()
        rep = (time.perf_counter() - t0) / 16 * 1e3
        model.transformer.disable_decoding()
    print(f"eager forward {eager:.2f} ms (host launch time {host:.2f} ms), capture {cap:.2f} ms, "
          f"replay {rep:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
