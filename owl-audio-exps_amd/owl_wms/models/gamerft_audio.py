"""GameRFTAudio / GameRFTAudioCore (reference: owl_wms/models/gamerft_audio.py:19-178) on libowlk.

Joint video + audio flow matching (BASELINE configs[3], mmdit_v2): one ts per frame shared by
both modalities, loss = MSE(video) + MSE(audio).  Backbones:
  * ``mmdit`` -- two-stream MMDiT (nn/mmattn.py), head proj_out(layer_norm(video), layer_norm(cond));
  * ``dit``   -- the audio token appended to each frame's video tokens (tpf = p*p + 1) through the
                 single-stream DiT, then split (gamerft_audio.py:68-76).
``torch.compile`` of the reference transformer (gamerft_audio.py:36) is not used: the block
kernels are hand-written, and state_dict keys carry no ``_orig_mod.`` prefix.
"""
import torch
from torch import nn

from .. import kernels as K
from ..nn.attn import DiT, FinalLayer
from ..nn.cond import conditioning
from ..nn.embeddings import ControlEmbedding, TimestepEmbedding
from ..nn.fused import linear
from ..nn.mmattn import MMDIT
from ..nn.normalization import layer_norm
from .flow import TorchNoise, flow_loss, handle_cfg, noised_av


class GameRFTAudioCore(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.config = config
        if not hasattr(config, "has_audio"):  # mmdit_v2.yml omits it; the 65-token frame needs it
            config.has_audio = True
        if config.backbone == "dit":
            backbone_cls = DiT
        elif config.backbone == "mmdit":
            backbone_cls = MMDIT
        else:
            raise ValueError(f"Invalid backbone: {config.backbone} (uvit is out of scope)")
        self.backbone = config.backbone
        self.transformer = backbone_cls(config)
        if not config.uncond:
            self.control_embed = ControlEmbedding(config.n_buttons, config.d_model)
        self.t_embed = TimestepEmbedding(config.d_model)
        self.proj_in = nn.Linear(config.channels, config.d_model, bias=False)
        self.proj_out = FinalLayer(config.sample_size, config.d_model, config.channels)
        self.audio_proj_in = nn.Linear(config.audio_channels, config.d_model, bias=False)
        self.audio_proj_out = FinalLayer(None, config.d_model, config.audio_channels)
        self.uncond = config.uncond

    def cond(self, t, mouse, btn, has_controls=None):
        """gamerft_audio.py: t_embed(t) + (has_controls ? control_embed(mouse, btn) : 0) (nn/cond.py)."""
        return conditioning(self, t, mouse, btn, has_controls, want="cond")

    def forward_tokens(self, xv, xa, t, mouse, btn, has_controls=None, kv_cache=None):
        """xv [B, n*h*w, C] video tokens, xa [B, n, Ca] -> (video [B, n*h*w, C], audio [B, n, Ca])."""
        cond = self.cond(t, mouse, btn, has_controls)
        B, n = xa.shape[:2]
        x = linear(xv, self.proj_in.weight)
        a = linear(xa, self.audio_proj_in.weight)
        if self.backbone == "mmdit":
            video, audio = self.transformer(x, a, cond, kv_cache)
        else:
            d = x.shape[-1]
            p2 = x.shape[1] // n
            joint = K.frame_interleave(x.reshape(-1, d), a.reshape(-1, d), p2, 1).view(B, n * (p2 + 1), d)
            joint = self.transformer(joint, cond, None, kv_cache)
            video, audio = K.frame_split(joint.reshape(-1, d).contiguous(), p2, 1)
            video, audio = video.view(B, n * p2, d), audio.view(B, n, d)
        video = self.proj_out(layer_norm(video), layer_norm(cond))
        audio = self.audio_proj_out(audio, cond)
        return video, audio

    def forward(self, x, audio, t, mouse, btn, has_controls=None, kv_cache=None):
        b, n, c, h, w = x.shape
        xv = x.permute(0, 1, 3, 4, 2).reshape(b, n * h * w, c)
        video, aud = self.forward_tokens(xv, audio, t, mouse, btn, has_controls, kv_cache)
        return K.unpatchify(video.reshape(-1, c).contiguous(), b, n, c, h, w), aud


class GameRFTAudio(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.config = config
        self.core = GameRFTAudioCore(config)
        self.cfg_prob = config.cfg_prob
        self.noise_source = TorchNoise()

    def handle_cfg(self, has_controls=None, cfg_prob=None, frac_host=None):
        return handle_cfg(has_controls, self.cfg_prob if cfg_prob is None else cfg_prob, self.noise_source, frac_host)

    def forward(self, x, audio, mouse, btn, return_dict=False, cfg_prob=None, has_controls=None):
        B, n, C, h, w = x.shape
        Ca = audio.shape[-1]
        frac_host = None
        if has_controls is None:
            has_controls = torch.ones(B, device=x.device, dtype=torch.bool)
            frac_host = 1.0
        has_controls = self.handle_cfg(has_controls, cfg_prob, frac_host)
        with torch.no_grad():
            xt, tgt, ts, zv, at, atgt, za = noised_av(x, audio, self.noise_source)
        pv, pa = self.core.forward_tokens(xt.view(B, n * h * w, C), at.view(B, n, Ca), ts, mouse, btn, has_controls)
        video_loss = flow_loss(pv.reshape(-1, C), tgt)
        audio_loss = flow_loss(pa.reshape(-1, Ca), atgt)
        diff_loss = video_loss + audio_loss
        if not return_dict:
            return diff_loss, video_loss, audio_loss
        with torch.no_grad():
            un = lambda tk: K.unpatchify(tk.reshape(-1, C).contiguous(), B, n, C, h, w)
            return {"diffusion_loss": diff_loss, "video_loss": video_loss, "audio_loss": audio_loss,
                    "lerpd_video": un(xt), "lerpd_audio": at.view(B, n, Ca), "pred_video": un(pv.detach()),
                    "pred_audio": pa.detach(), "ts": ts, "z_video": zv, "z_audio": za, "cfg_mask": has_controls}
