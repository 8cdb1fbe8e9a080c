"""GameRFT / GameRFTCore (reference: owl_wms/models/gamerft.py:13-124) on libowlk.

Training runs token-major end to end: owlk_flow_noise draws x_t and the target straight into
the patchified layout ('b n c h w -> b (n h w) c', gamerft.py:52), the DiT runs on fused block
kernels, and the MSE + its gradient come from one kernel.  The reference API (``core(x5, t,
...)`` with [b, n, c, h, w] tensors, ``return_dict``) is kept.
"""
import torch
from torch import nn

from .. import kernels as K
from ..nn.attn import DiT, FinalLayer
from ..nn.cond import conditioning
from ..nn.embeddings import ControlEmbedding, TimestepEmbedding
from ..nn.fused import linear
from .flow import TorchNoise, flow_loss, handle_cfg, noised_tokens


class GameRFTCore(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.config = config
        assert config.backbone == "dit"
        self.transformer = DiT(config)
        if not config.uncond:
            self.control_embed = ControlEmbedding(config.n_buttons, config.d_model)
        self.t_embed = TimestepEmbedding(config.d_model)
        self.proj_in = nn.Linear(config.channels, config.d_model, bias=False)
        self.proj_out = FinalLayer(config.sample_size, config.d_model, config.channels)
        assert self.config.tokens_per_frame == self.config.sample_size ** 2
        self.uncond = config.uncond

    def cond(self, t, mouse, btn, has_controls=None):
        """gamerft.py:39-48: t_embed(t) + (has_controls ? control_embed(mouse, btn) : 0), bf16 [B, n, d]
        (one fused conditioning pass, nn/cond.py)."""
        return conditioning(self, t, mouse, btn, has_controls, want="cond")

    def forward_tokens(self, x_tok, t, mouse, btn, doc_id=None, has_controls=None, kv_cache=None,
                       local_block_mask=None, global_block_mask=None):
        """x_tok [B, n*h*w, C] -> velocity tokens [B, n*h*w, C] (bf16).  Every consumer of cond
        reads silu(cond), so the conditioning pass hands out s = silu(cond) directly."""
        s = conditioning(self, t, mouse, btn, has_controls, want="s")
        x = linear(x_tok, self.proj_in.weight)
        x = self.transformer(x, None, doc_id, kv_cache, local_block_mask, global_block_mask, scond=s)
        return self.proj_out(x, None, scond=s)

    def forward(self, x, t, mouse, btn, doc_id=None, has_controls=None, kv_cache=None, local_block_mask=None,
                global_block_mask=None):
        b, n, c, h, w = x.shape
        x_tok = x.permute(0, 1, 3, 4, 2).reshape(b, n * h * w, c)
        y = self.forward_tokens(x_tok, t, mouse, btn, doc_id, has_controls, kv_cache, local_block_mask,
                                global_block_mask)
        return K.unpatchify(y.reshape(-1, c).contiguous(), b, n, c, h, w)


class GameRFT(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.config = config
        self.core = GameRFTCore(config)
        self.noise_source = TorchNoise()

    def handle_cfg(self, has_controls=None, cfg_prob=None, frac_host=None):
        return handle_cfg(has_controls, self.config.cfg_prob if cfg_prob is None else cfg_prob, self.noise_source,
                          frac_host)

    def forward(self, x, mouse=None, btn=None, doc_id=None, return_dict=False, cfg_prob=None, has_controls=None):
        B, S, C, h, w = x.shape
        frac_host = None  # mean(has_controls) when built here: no device -> host sync in handle_cfg
        if has_controls is None:
            has_controls = torch.ones(B, device=x.device, dtype=torch.bool)
            frac_host = 1.0
        if mouse is None or btn is None:
            has_controls = torch.zeros_like(has_controls)
            frac_host = 0.0
        has_controls = self.handle_cfg(has_controls, cfg_prob, frac_host)
        with torch.no_grad():
            xt, tgt, ts, z = noised_tokens(x, self.noise_source)
        pred = self.core.forward_tokens(xt.view(B, S * h * w, C), ts, mouse, btn, doc_id, has_controls)
        loss = flow_loss(pred.reshape(-1, C), tgt)
        if not return_dict:
            return loss
        with torch.no_grad():
            un = lambda tk: K.unpatchify(tk.reshape(-1, C).contiguous(), B, S, C, h, w)
            return {"diffusion_loss": loss, "video_loss": loss, "lerpd_video": un(xt), "pred_video": un(pred.detach()),
                    "ts": ts, "z_video": z, "cfg_mask": has_controls}
