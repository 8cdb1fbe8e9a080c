"""Shared flow-matching objective pieces (gamerft.py:68-124, audiorft.py:59-93)."""
import numpy as np
import torch

from .. import kernels as K
from ..nn.fused import FlowLossFn


class TorchNoise:
    """Default noise source: the reference's draw order on the input's device
    (rand(b) for CFG dropout -> randn(B, S) for timesteps -> randn_like(x))."""

    def rand_b(self, b, device):
        return torch.rand(b, device=device)

    def ts_raw(self, B, S, device, dtype):
        return torch.randn(B, S, device=device, dtype=dtype)

    def z(self, x):
        return torch.randn_like(x)


class InjectedNoise:
    """Parity runs: replay pre-drawn tensors (a dict with rand_b / ts_raw / z)."""

    def __init__(self, d):
        self.d = d

    def rand_b(self, b, device):
        return self.d["rand_b"].to(device)

    def ts_raw(self, B, S, device, dtype):
        return self.d["ts_raw"].to(device=device, dtype=dtype)

    def z(self, x):
        z = self.d["z"]
        if isinstance(z, (list, tuple)):  # several randn_like draws in order (video, then audio)
            self._zi = getattr(self, "_zi", 0)
            z = z[self._zi]
            self._zi += 1
        return z.to(device=x.device, dtype=x.dtype)


def handle_cfg(has_controls, cfg_prob, noise, frac_host=None):
    """gamerft.py:68-90.  The Python-level comparison syncs the host, as in the reference, unless
    the caller knows mean(has_controls) on the host (frac_host: it built the mask itself); the
    fp32 arithmetic and the RNG draw order are the reference's either way."""
    if cfg_prob <= 0.0 or has_controls is None:
        return has_controls
    if frac_host is not None:
        f32 = np.float32
        frac = f32(frac_host)
        pct_without = f32(1.0) - frac
        if pct_without < f32(cfg_prob):
            needed_frac = float((f32(cfg_prob) - pct_without) / frac)
            b = has_controls.shape[0]
            mask = (noise.rand_b(b, has_controls.device) <= needed_frac) & has_controls
            has_controls = has_controls & (~mask)
        return has_controls
    frac = has_controls.float().mean()
    pct_without = 1.0 - frac
    if pct_without < cfg_prob:
        needed_frac = (cfg_prob - pct_without) / frac
        b = has_controls.shape[0]
        mask = (noise.rand_b(b, has_controls.device) <= needed_frac) & has_controls
        has_controls = has_controls & (~mask)
    return has_controls


def noised_tokens(x5, noise):
    """x5 [B, N, C, P...] -> (x_t tokens, target tokens, ts bf16 [B, N], z) via owlk_flow_noise."""
    B, N = x5.shape[:2]
    xb = x5.to(torch.bfloat16)
    ts_raw = noise.ts_raw(B, N, xb.device, torch.bfloat16)
    z = noise.z(xb)
    shp = xb.shape
    xt, tgt, ts = K.flow_noise(xb.reshape(B, N, shp[2], -1, 1), z.reshape(B, N, shp[2], -1, 1), ts_raw)
    return xt, tgt, ts, z


def flow_loss(pred_tok, tgt_tok):
    return FlowLossFn.apply(pred_tok, tgt_tok)


def noised_av(x5, a3, noise):
    """gamerft_audio.py:137-151: one ts for both modalities; draw order ts -> z_video -> z_audio.
    Returns token-major (xt, tgt, ts, z) for video and (at, atgt) for audio."""
    B, N = x5.shape[:2]
    xb, ab = x5.to(torch.bfloat16), a3.to(torch.bfloat16)
    ts_raw = noise.ts_raw(B, N, xb.device, torch.bfloat16)
    zv, za = noise.z(xb), noise.z(ab)
    shp = xb.shape
    xt, tgt, ts = K.flow_noise(xb.reshape(B, N, shp[2], -1, 1), zv.reshape(B, N, shp[2], -1, 1), ts_raw)
    at, atgt, _ = K.flow_noise(ab.reshape(B, N, ab.shape[2], 1, 1), za.reshape(B, N, ab.shape[2], 1, 1), ts_raw)
    return xt, tgt, ts, zv, at, atgt, za
