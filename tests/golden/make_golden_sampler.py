"""Golden fixtures for the KV-cache samplers from the REFERENCE on CPU.

Runs only where /root/reference exists.  Shims on top of make_golden's:
  * ``owl_wms.configs`` replaced by a stub exposing ``TransformerConfig`` (the real module needs
    omegaconf, absent) -- kv_cache.py only uses it as a type annotation;
  * ``SingleKVCache`` allocates on 'cpu' instead of its hard-coded 'cuda' (kv_cache.py:17);
  * ``owl_wms.sampling.schedulers.get_sd3_euler``: diffusers is absent, so the shifted-sigma
    schedule is taken from owl_wms.sampling.schedulers (restatement; PARITY-UNPINNED);
  * torch.randn / randn_like draws injected from seeded tensors in the reference's order.
Sampling runs under bf16 autocast, as the reference trainer's eval step does
(rft_trainer.py:214-215).

    python tests/golden/make_golden_sampler.py          # sampler_tiny.pt
    python tests/golden/make_golden_sampler.py d128     # sampler_d128.pt (head_dim 128, round 4)
"""
import os
import sys
import types

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as G  # noqa: E402

from oracle.params import det_init_, det_tensor  # noqa: E402

REPO = os.path.dirname(os.path.dirname(HERE))
_spec = G.importlib.util.spec_from_file_location(
    "owlk_schedulers", os.path.join(REPO, "owl-audio-exps_amd", "owl_wms", "sampling", "schedulers.py"))
_ours = G.importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(_ours)
get_sd3_euler = _ours.get_sd3_euler  # our restatement (torch/numpy only)

cfgmod = types.ModuleType("owl_wms.configs")
cfgmod.TransformerConfig = object
sys.modules["owl_wms.configs"] = cfgmod
samp = types.ModuleType("owl_wms.sampling")
samp.__path__ = [os.path.join(G.REF, "owl_wms", "sampling")]
sys.modules["owl_wms.sampling"] = samp
sched = types.ModuleType("owl_wms.sampling.schedulers")
sched.get_sd3_euler = get_sd3_euler
sys.modules["owl_wms.sampling.schedulers"] = sched

r_kv = G._load("owl_wms.nn.kv_cache", "owl_wms/nn/kv_cache.py")
_orig_init = r_kv.SingleKVCache.__init__


def _cpu_init(self, config):
    _orig_init(self, config)
    self.device = "cpu"


r_kv.SingleKVCache.__init__ = _cpu_init
r_av = G._load("owl_wms.sampling.av_caching_v2", "owl_wms/sampling/av_caching_v2.py")
r_au = G._load("owl_wms.sampling.audio_caching", "owl_wms/sampling/audio_caching.py")


def gen_av():
    cfg = G.tiny_video_cfg()
    model = det_init_(G.r_gamerft.GameRFT(cfg), base_seed=1000).eval()
    B, ctx, new, C, s = 1, 4, 3, cfg.channels, cfg.sample_size
    bf = G.bf16_exact
    x = bf(det_tensor((B, ctx, C, s, s), 8100))
    mouse = bf(det_tensor((B, ctx + new, 2), 8101))
    g = torch.Generator().manual_seed(8102)
    btn = (torch.rand((B, ctx + new, cfg.n_buttons), generator=g) < 0.5).float()
    like = [bf(det_tensor((B, ctx, C, s, s), 8110))]
    for f in range(new):
        like += [bf(det_tensor((B, 1, C, s, s), 8120 + 2 * f)), bf(det_tensor((B, 1, C, s, s), 8121 + 2 * f))]
    sampler = r_av.AVCachingSamplerV2(n_steps=2, cfg_scale=1.3, num_frames=new, noise_prev=0.2)
    with G.inject_rng(randn_like=like), torch.autocast("cpu", dtype=torch.bfloat16):
        out = sampler(model.core, x, mouse, btn)
    return {"av.in.x": x, "av.in.mouse": mouse, "av.in.btn": btn, "av.noise": like, "av.out": out.float(),
            "av.dt": get_sd3_euler(2)}


def gen_av_d128():
    """AVCachingSamplerV2 at head_dim 128 (configs/dit_v4_5B.yml's attention width): the tiny D = 128
    GameRFT of gamerft_d128.pt (d 256, 2 heads, base seed 1100), 4 context + 3 generated frames."""
    cfg = G.tiny_video_cfg(d_model=256, n_heads=2, gradient_checkpointing=True)
    model = det_init_(G.r_gamerft.GameRFT(cfg), base_seed=1100).eval()
    B, ctx, new, C, s = 1, 4, 3, cfg.channels, cfg.sample_size
    bf = G.bf16_exact
    x = bf(det_tensor((B, ctx, C, s, s), 8300))
    mouse = bf(det_tensor((B, ctx + new, 2), 8301))
    g = torch.Generator().manual_seed(8302)
    btn = (torch.rand((B, ctx + new, cfg.n_buttons), generator=g) < 0.5).float()
    like = [bf(det_tensor((B, ctx, C, s, s), 8310))]
    for f in range(new):
        like += [bf(det_tensor((B, 1, C, s, s), 8320 + 2 * f)), bf(det_tensor((B, 1, C, s, s), 8321 + 2 * f))]
    sampler = r_av.AVCachingSamplerV2(n_steps=2, cfg_scale=1.3, num_frames=new, noise_prev=0.2)
    with G.inject_rng(randn_like=like), torch.autocast("cpu", dtype=torch.bfloat16):
        out = sampler(model.core, x, mouse, btn)
    return {"av128.in.x": x, "av128.in.mouse": mouse, "av128.in.btn": btn, "av128.noise": like,
            "av128.out": out.float()}


def gen_audio():
    cfg = G.audio_cfg()
    model = det_init_(G.r_audiorft.AudioRFT(cfg), base_seed=3000).eval()
    B, ctx, new, C = 1, 8, 3, cfg.channels
    bf = G.bf16_exact
    x = bf(det_tensor((B, ctx, C), 8200))
    randn = [bf(det_tensor((B, 1, C), 8210 + t)) for t in range(new)]
    like = [bf(det_tensor((B, ctx, C), 8220))] + [bf(det_tensor((B, 1, C), 8230 + t)) for t in range(new)]
    sampler = r_au.AudioCachingSampler(n_steps=2, num_tokens=new, noise_prev=0.2)
    with G.inject_rng(randn=randn, randn_like=like), torch.autocast("cpu", dtype=torch.bfloat16):
        out = sampler(model.core, x)
    return {"audio.in.x": x, "audio.noise_randn": randn, "audio.noise_like": like, "audio.out": out.float()}


def main():
    if sys.argv[1:] == ["d128"]:
        out = gen_av_d128()
        path = os.path.join(HERE, "sampler_d128.pt")
        torch.save(out, path)
        print(path, os.path.getsize(path) // 1024, "KiB", tuple(out["av128.out"].shape))
        return
    out = gen_av()
    out.update(gen_audio())
    path = os.path.join(HERE, "sampler_tiny.pt")
    torch.save(out, path)
    print(path, os.path.getsize(path) // 1024, "KiB", tuple(out["av.out"].shape), tuple(out["audio.out"].shape))
    print("dt", out["av.dt"].tolist())


if __name__ == "__main__":
    main()
