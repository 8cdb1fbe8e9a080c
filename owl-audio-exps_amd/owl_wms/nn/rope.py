"""rope.py (reference: owl_wms/nn/rope.py).  Builds the fp32 cos/sin tables the QK-RoPE kernel
reads; ``forward`` keeps the reference ``rope(x, offset)`` signature for external callers.

MotionRoPE (rope.py:82-152) and Audio1DRoPE (:155-179) are pinned by golden vectors.  OrthoRoPE
(:57-79) depends on rotary-embedding-torch's 'pixel' frequencies + get_axial_freqs, which are
restated here from that library's published algorithm (version unpinned, absent offline):
PARITY UNPINNED.
"""
import math

import torch
from torch import nn


def get_rope_cls(cls_name):
    cls_name = cls_name.lower()
    if cls_name == "ortho":
        return OrthoRoPE
    if cls_name == "motion":
        return MotionRoPE
    if cls_name == "audio1d":
        return Audio1DRoPE
    raise ValueError(f"Invalid RoPE class: {cls_name}")


def lang_freqs(dim, theta=10000.0):
    return 1.0 / (theta ** (torch.arange(0, dim, 2)[: dim // 2].float() / dim))


class RoPE(nn.Module):
    def __init__(self, config):
        super().__init__()
        freqs = self.get_freqs(config)
        if not config.has_audio:  # rope.py:35-37: drop each frame's audio slot
            freqs = freqs.view(config.n_frames, -1, freqs.size(-1))[:, :-1].flatten(0, 1)
        self.register_buffer("cos", freqs.cos().float().contiguous(), persistent=False)
        self.register_buffer("sin", freqs.sin().float().contiguous(), persistent=False)

    def forward(self, x, offset: int = 0):
        """[..., n, d] -> rotated (fp32 math, [even || odd] layout, cast back) -- rope.py:43-51."""
        cos = self.cos[offset:offset + x.size(-2)]
        sin = self.sin[offset:offset + x.size(-2)]
        xf = x.float()
        x0, x1 = xf[..., 0::2], xf[..., 1::2]
        return torch.cat((x0 * cos - x1 * sin, x1 * cos + x0 * sin), dim=-1).type_as(x)

    def get_freqs(self, config):
        raise NotImplementedError


class MotionRoPE(RoPE):
    """rope.py:82-152 -- spatial coordinates drift linearly with time (ats_delta)."""

    def get_freqs(self, config):
        H = W = config.sample_size
        nf = config.n_frames
        d_head = config.d_model // config.n_heads
        dt = getattr(config, "rope_dim_t", d_head * 2 // 8)
        dx = getattr(config, "rope_dim_x", d_head * 3 // 8)
        dy = getattr(config, "rope_dim_y", d_head * 3 // 8)
        theta = getattr(config, "rope_base", 10000.0)
        delta = getattr(config, "rope_ats_delta", 2.0)
        base = lang_freqs(dt + dx + dy, theta)
        spatial, ft = base[: (dx + dy) // 2], base[(dx + dy) // 2:]
        fx, fy = spatial[0::2], spatial[1::2]
        t = torch.arange(nf, dtype=torch.float32) * delta
        hg = torch.arange(H, dtype=torch.float32) - (H - 1) / 2.0
        wg = torch.arange(W, dtype=torch.float32) - (W - 1) / 2.0
        tv = t[:, None, None].expand(nf, H, W)
        xv = (tv + wg[None, None, :]).reshape(nf, H * W)
        yv = (tv + hg[None, :, None]).reshape(nf, H * W)
        tv = tv.reshape(nf, H * W)
        xs = torch.cat([xv, t[:, None]], 1).reshape(-1)
        ys = torch.cat([yv, t[:, None] + (H - 1) / 2.0 + 1.0], 1).reshape(-1)
        ts = torch.cat([tv, t[:, None]], 1).reshape(-1)
        inter = torch.stack([xs[:, None] * fx[None], ys[:, None] * fy[None]], -1).reshape(xs.numel(), -1)
        return torch.cat([inter, ts[:, None] * ft[None]], -1)


class Audio1DRoPE(RoPE):
    """rope.py:155-179 -- 1-D temporal positions."""

    def get_freqs(self, config):
        d_head = config.d_model // config.n_heads
        return torch.arange(config.n_frames, dtype=torch.float32)[:, None] * lang_freqs(d_head)[None]


class OrthoRoPE(RoPE):
    """rope.py:57-79 (parity unpinned: rotary-embedding-torch 'pixel' axial freqs restated)."""

    def get_freqs(self, config):
        p = config.sample_size
        dim = (config.d_model // config.n_heads) // 4
        freqs = torch.linspace(1.0, 256 / 2, dim // 2) * math.pi  # freqs_for='pixel', max_freq=256
        dims, offsets = (config.n_frames, p + 1, p + 1, 1), (0, 0, 0, 1)
        axes = []
        for i, (n, off) in enumerate(zip(dims, offsets)):
            pos = torch.linspace(-1, 1, steps=n) + off
            f = (pos[:, None] * freqs[None]).repeat_interleave(2, dim=-1)  # [n, dim]
            shape = [1] * len(dims) + [f.shape[-1]]
            shape[i] = n
            axes.append(f.view(shape))
        full = torch.cat(torch.broadcast_tensors(*axes), dim=-1).view(config.n_frames, p + 1, p + 1, -1)
        vid = full[:, :p, :p].reshape(config.n_frames, p * p, -1)
        aud = full[:, -1, -1].unsqueeze(1)
        return torch.cat([vid, aud], dim=1).flatten(0, 1)[..., ::2]
