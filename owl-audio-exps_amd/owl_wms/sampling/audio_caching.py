"""AudioCachingSampler (reference: owl_wms/sampling/audio_caching.py:22-159) on libowlk.

One audio token per step of the outer loop (tpf = 1), unconditional, no CFG; same cache /
re-noise protocol as AVCachingSamplerV2.  Noise order: context zlerp, then per token randn
(x0) and zlerp.
"""
import torch

from ..nn.kv_cache import KVCache
from .schedulers import get_deltas, get_sd3_euler


class AudioCachingSampler:
    def __init__(self, n_steps: int = 16, num_tokens: int = 120, noise_prev: float = 0.2, custom_schedule=None,
                 max_window=None) -> None:
        self.n_steps = n_steps
        self.num_tokens = num_tokens
        self.noise_prev = noise_prev
        self.custom_schedule = custom_schedule
        self.max_window = max_window

    @staticmethod
    def zlerp(x, alpha):
        z = torch.randn_like(x)
        return x * (1.0 - alpha) + z * alpha

    @torch.no_grad()
    def __call__(self, model, x, decode_fn=None, vae_scale=1.0, compile_on_decode=False):
        """model: an AudioRFT core; x [b, init_len, c] -> [b, init_len + num_tokens, c] (+ waveforms)."""
        batch_size, init_len, latent_channels = x.shape
        if self.custom_schedule is None:
            dt = get_sd3_euler(self.n_steps).to(device=x.device, dtype=x.dtype)
        else:
            dt = get_deltas(self.custom_schedule)
        kv_cache = KVCache(model.config)
        kv_cache.reset(batch_size)
        latents = [x.clone()]
        prev_x_noisy = self.zlerp(x, self.noise_prev)
        prev_t = x.new_full((batch_size, x.size(1)), self.noise_prev)
        kv_cache.enable_cache_updates()
        model(prev_x_noisy, prev_t, doc_id=None, kv_cache=kv_cache)
        kv_cache.disable_cache_updates()
        model.transformer.enable_decoding()
        try:
            for _ in range(self.num_tokens):
                curr_x = torch.randn(batch_size, 1, latent_channels, device=x.device, dtype=x.dtype)
                curr_t = prev_t.new_ones(batch_size, 1)
                for t_idx in range(self.n_steps):
                    pred_v = model(curr_x, curr_t, doc_id=None, kv_cache=kv_cache).clone()
                    curr_x = curr_x - dt[t_idx] * pred_v
                    curr_t = curr_t - dt[t_idx]
                latents.append(curr_x.clone())
                curr_x_noisy = self.zlerp(curr_x, self.noise_prev)
                curr_t_noisy = torch.ones_like(curr_t) * self.noise_prev
                kv_cache.enable_cache_updates()
                model(curr_x_noisy, curr_t_noisy, kv_cache=kv_cache)
                kv_cache.disable_cache_updates()
                if self.max_window is not None and len(latents) > self.max_window:
                    kv_cache.truncate(1, front=False)
        finally:
            model.transformer.disable_decoding()
        full = torch.cat(latents, dim=1)
        if decode_fn is not None:
            return full, decode_fn(full * vae_scale)
        return full
