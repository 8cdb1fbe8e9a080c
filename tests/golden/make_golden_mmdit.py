"""Golden fixtures for the MMDiT path (BASELINE configs[3], mmdit_v2) from the REFERENCE on CPU.

Runs only where /root/reference exists (the build container).  The reference cannot import
``mmattn.py`` as shipped (it imports a missing ``create_causal_block_mask``),
so the model is RECONSTRUCTED exactly as SURVEY.md §8(c) item 7 records, and these choices are
part of the fixture:
  * ``attn.create_causal_block_mask(n_tokens, tokens_per_frame, n_cached_tokens, window_len, device)``
    := ``get_block_mask(n_tokens, tokens_per_frame, window_len, None, n_cached_tokens, True, device)``;
  * ``has_audio = True`` (the 65-token frame RoPE layout; mmdit_v2.yml omits it);
  * ``torch.compile`` neutralised while ``GameRFTAudioCore`` is constructed (gamerft_audio.py:36)
    and mmattn's module-level compiled flex_attention replaced by the eager one.
OrthoRoPE needs rotary-embedding-torch's 'pixel' frequencies and ``get_axial_freqs``; the shim
below restates that library's published algorithm (not in this image, version unpinned), so the
RoPE tables are PARITY-UNPINNED: the fixture pins everything else given that restatement (the
host package's OrthoRoPE is the same restatement).

    python tests/golden/make_golden_mmdit.py
"""
import math
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as G  # noqa: E402  (installs the base shims, loads the reference modules)

from oracle.params import det_init_, det_tensor  # noqa: E402


class _RotaryPixel:
    """rotary-embedding-torch RotaryEmbedding subset: freqs_for='lang'|'pixel', get_axial_freqs."""

    def __init__(self, dim, freqs_for="lang", theta=10000, max_freq=10, **kw):
        self.freqs_for = freqs_for
        if freqs_for == "lang":
            self.freqs = 1.0 / (theta ** (torch.arange(0, dim, 2)[: dim // 2].float() / dim))
        elif freqs_for == "pixel":
            self.freqs = torch.linspace(1.0, max_freq / 2, dim // 2) * math.pi
        else:
            raise NotImplementedError(freqs_for)

    def get_axial_freqs(self, *dims, offsets=None):
        axes = []
        for i, n in enumerate(dims):
            pos = torch.linspace(-1, 1, steps=n) if self.freqs_for == "pixel" else torch.arange(n).float()
            pos = pos + (offsets[i] if offsets is not None else 0)
            f = (pos[:, None] * self.freqs[None]).repeat_interleave(2, dim=-1)
            shape = [1] * len(dims) + [f.shape[-1]]
            shape[i] = n
            axes.append(f.view(shape))
        return torch.cat(torch.broadcast_tensors(*axes), dim=-1)


sys.modules["rotary_embedding_torch"].RotaryEmbedding = _RotaryPixel
G.r_rope.RotaryEmbedding = _RotaryPixel


def _create_causal_block_mask(n_tokens, tokens_per_frame, n_cached_tokens, window_len, device):
    return G.r_attn.get_block_mask(n_tokens, tokens_per_frame, window_len, None, n_cached_tokens, True, device)


G.r_attn.create_causal_block_mask = _create_causal_block_mask
r_mmattn = G._load("owl_wms.nn.mmattn", "owl_wms/nn/mmattn.py")
r_mmattn.flex_attention = G._eager_flex
r_gra = G._load("owl_wms.models.gamerft_audio", "owl_wms/models/gamerft_audio.py")


def mmdit_cfg(**over):
    c = dict(model_id="game_rft_audio", sample_size=8, channels=32, audio_channels=16, n_layers=2, n_heads=2,
             d_model=128, tokens_per_frame=65, n_buttons=11, n_mouse_axes=2, cfg_prob=0.1, n_frames=6,
             causal=True, uncond=False, backbone="mmdit", local_window=2, global_window=4, has_audio=True)
    c.update(over)
    from types import SimpleNamespace
    return SimpleNamespace(**c)


def build(cfg):
    real = torch.compile
    torch.compile = lambda m, *a, **k: m
    try:
        return r_gra.GameRFTAudio(cfg)
    finally:
        torch.compile = real


def gen_mmdit():
    out = {}
    cfg = mmdit_cfg()
    model = det_init_(build(cfg), base_seed=5000).train()
    B, n, C, s, Ca = 2, cfg.n_frames, cfg.channels, cfg.sample_size, cfg.audio_channels
    bf = G.bf16_exact
    x = bf(det_tensor((B, n, C, s, s), 5100)).bfloat16()
    audio = bf(det_tensor((B, n, Ca), 5101)).bfloat16()
    mouse = bf(det_tensor((B, n, 2), 5102)).bfloat16()
    g = torch.Generator().manual_seed(5103)
    btn = (torch.rand((B, n, cfg.n_buttons), generator=g) < 0.5).bfloat16()
    rand_b = torch.tensor([0.05, 0.7])
    ts_raw = bf(det_tensor((B, n), 5104))
    zv = bf(det_tensor((B, n, C, s, s), 5105))
    za = bf(det_tensor((B, n, Ca), 5106))
    with G.inject_rng(rand=[rand_b], randn=[ts_raw], randn_like=[zv, za]), \
            torch.autocast("cpu", dtype=torch.bfloat16):
        d = model(x, audio, mouse, btn, return_dict=True)
        d["diffusion_loss"].backward()
    p = "mmdit.bf16."
    for k, v in dict(x=x, audio=audio, mouse=mouse, btn=btn, rand_b=rand_b, ts_raw=ts_raw, z_video=zv,
                     z_audio=za).items():
        out[p + "in." + k] = v
    for k in ("diffusion_loss", "video_loss", "audio_loss"):
        out[p + k] = d[k].detach().float()
    out[p + "pred_video"] = d["pred_video"].detach().float()
    out[p + "pred_audio"] = d["pred_audio"].detach().float()
    out[p + "cfg_mask"] = d["cfg_mask"]
    for i, (k, prm) in enumerate(sorted(model.named_parameters())):
        out[p + "gradstat." + k] = G.proj_stats(prm.grad, 11000 + i)
        if ".blocks.0." in k or "proj_out" in k or "proj_in" in k or "cond_proj" in k:
            out[p + "grad." + k] = prm.grad.clone()
    # the OrthoRoPE table the reconstruction used (restated rotary-embedding-torch; see header)
    rope = model.core.transformer.blocks[0].attn.rope
    out["mmdit.rope.cos"], out["mmdit.rope.sin"] = rope.cos.float().clone(), rope.sin.float().clone()
    out["mmdit.schema"] = [[k, list(v.shape)] for k, v in model.state_dict().items()]
    return out


def main():
    torch.manual_seed(0)
    out = gen_mmdit()
    path = os.path.join(HERE, "mmdit_tiny.pt")
    torch.save(out, path)
    print(path, os.path.getsize(path) // 1024, "KiB")
    print("losses", out["mmdit.bf16.diffusion_loss"].item(), out["mmdit.bf16.video_loss"].item(),
          out["mmdit.bf16.audio_loss"].item())


if __name__ == "__main__":
    main()
