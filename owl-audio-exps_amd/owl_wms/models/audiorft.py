"""AudioRFT / AudioRFTCore (reference: owl_wms/models/audiorft.py:13-93) on libowlk."""
import torch
from torch import nn

from ..nn.attn import DiT, FinalLayer
from ..nn.cond import conditioning
from ..nn.embeddings import TimestepEmbedding
from ..nn.fused import linear
from .flow import TorchNoise, flow_loss, noised_tokens


class AudioRFTCore(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.config = config
        assert config.backbone == "dit"
        self.transformer = DiT(config)
        self.t_embed = TimestepEmbedding(config.d_model)
        self.proj_in = nn.Linear(config.channels, config.d_model, bias=False)
        self.proj_out = FinalLayer(1, config.d_model, config.channels)
        assert config.tokens_per_frame == 1

    def forward(self, x, t, doc_id=None, kv_cache=None, local_block_mask=None, global_block_mask=None):
        s = conditioning(self, t, want="s")  # silu(t_embed(t)) (unconditional: cond = t_embed(t))
        h = linear(x, self.proj_in.weight)
        h = self.transformer(h, None, doc_id, kv_cache, local_block_mask, global_block_mask, scond=s)
        return self.proj_out(h, None, scond=s)


class AudioRFT(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.config = config
        self.core = AudioRFTCore(config)
        self.noise_source = TorchNoise()

    def forward(self, x, doc_id=None, return_dict=False):
        B, n, C = x.shape
        with torch.no_grad():
            xt, tgt, ts, z = noised_tokens(x[:, :, :, None], self.noise_source)
        pred = self.core(xt.view(B, n, C), ts, doc_id)
        loss = flow_loss(pred.reshape(-1, C), tgt)
        if not return_dict:
            return loss
        return {"diffusion_loss": loss, "audio_loss": loss, "lerpd_audio": xt.view(B, n, C),
                "pred_audio": pred.detach(), "ts": ts, "z_audio": z.view(B, n, C)}
