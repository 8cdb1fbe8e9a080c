"""embeddings.py (reference: owl_wms/nn/embeddings.py:30-184) -- per-frame conditioning.

Tiny next to the DiT (<0.05 % of FLOPs): elementwise prep in torch, every Linear on libowlk.
"""
import math

import torch
from torch import nn

from .mlp import MLPCustom
from .fused import linear


class SinCosEmbed(nn.Module):
    """embeddings.py:30-72 (computed in the input dtype, bf16 during training)."""

    def __init__(self, dim, theta=300, mult=1000):
        super().__init__()
        self.dim, self.theta, self.mult = dim, theta, mult

    def _freqs(self, device, dtype):
        """exp(-i ln(theta) / (half - 1)), built on the CPU in fp32 as the reference does, then cached
        per (device, dtype): no host-to-device copy per call (the decode loop is graph-captured)."""
        key = (str(device), dtype)
        cache = self.__dict__.setdefault("_freq_cache", {})
        if key not in cache:
            half = self.dim // 2
            e = torch.log(torch.tensor(self.theta)) / (half - 1)
            cache[key] = torch.exp(torch.arange(half) * -e).to(device=device, dtype=dtype)
        return cache[key]

    def forward(self, x):
        if isinstance(x, float):
            x = torch.tensor([x])
        elif not isinstance(x, torch.Tensor):
            x = torch.tensor(x)
        if x.dim() == 0:
            x = x.unsqueeze(0)
        reshape_out = x.dim() == 2
        if reshape_out:
            b, n = x.shape
            x = x.reshape(b * n)
        x = x * self.mult
        e = self._freqs(x.device, x.dtype)
        e = x.unsqueeze(-1) * e.unsqueeze(0)
        e = torch.cat((torch.sin(e), torch.cos(e)), dim=-1)
        return e.reshape(b, n, -1) if reshape_out else e


class TimestepEmbedding(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.sincos = SinCosEmbed(512, theta=300, mult=1000)
        self.mlp = MLPCustom(512, dim * 4, dim)

    def forward(self, x):
        return self.mlp(self.sincos(x))


class MouseEmbedding(nn.Module):
    def __init__(self, dim_out, dim=512):
        super().__init__()
        self.angle_proj = nn.Linear(2, dim // 2, bias=False)
        self.magnitude_embed = SinCosEmbed(dim // 2)
        self.mlp = MLPCustom(dim, dim * 4, dim_out)

    def forward(self, x):
        with torch.no_grad():
            x = torch.sign(x) * torch.log1p(torch.abs(x))
            ang = torch.atan2(x[..., 1], x[..., 0])
            mag = torch.norm(x, dim=-1)
            ang_e = torch.stack([torch.cos(ang), torch.sin(ang)], dim=-1).to(x.dtype)
            mag_e = self.magnitude_embed(mag).to(x.dtype)
        ang_e = linear(ang_e, self.angle_proj.weight)
        return self.mlp(torch.cat([ang_e, mag_e.to(ang_e.dtype)], dim=-1))


class ButtonEmbeddding(nn.Module):  # (sic) reference spelling, embeddings.py:158
    def __init__(self, n_buttons, dim_out, dim=512):
        super().__init__()
        self.proj = MLPCustom(n_buttons, dim * 4, dim_out)

    def forward(self, x):
        return self.proj(x * 2 - 1)


class ControlEmbedding(nn.Module):
    def __init__(self, n_buttons, dim_out, dim=512):
        super().__init__()
        self.mouse = MouseEmbedding(dim_out, dim)
        self.button = ButtonEmbeddding(n_buttons, dim_out, dim)

    def forward(self, mouse, button, has_controls=None):
        return self.mouse(mouse) + self.button(button)
