"""kv_cache.py (reference: owl_wms/nn/kv_cache.py:5-104).

Same interface; K/V are kept token-major ``[B, T, H*D]`` bf16 (the layout the attention kernel
reads directly) instead of ``[B, H, T, D]``.
"""
import torch


def KVCache(config):
    if config.backbone in ("dit", "mmdit"):
        return SingleKVCache(config)
    raise ValueError(f"Invalid backbone: {config.backbone}")


class SingleKVCache:
    def __init__(self, config):
        self.config = config
        self.cache = None
        self.device = "cuda"
        self.dtype = torch.bfloat16
        self.should_update = False
        self.noise_caches = 0.0
        self.offsets = [0] * config.n_layers

    def enable_cache_updates(self):
        self.should_update = True

    def disable_cache_updates(self):
        self.should_update = False

    def to(self, device="cuda", dtype=torch.bfloat16):
        self.device, self.dtype = device, dtype
        return self

    def reset(self, batch_size=1):
        d = self.config.d_model
        empty = torch.empty(batch_size, 0, d, device=self.device, dtype=self.dtype)
        self.cache = [(empty, empty) for _ in range(self.config.n_layers)]
        self.offsets = [0] * self.config.n_layers

    def get(self, layer_ind):
        assert self.cache is not None, "Must reset cache before using"
        k, v = self.cache[layer_ind]
        if self.noise_caches > 0.0:
            k = k + torch.randn_like(k) * self.noise_caches
            v = v + torch.randn_like(v) * self.noise_caches
        return k, v

    def update(self, new_k, new_v, layer_ind):
        assert self.cache is not None, "Must reset cache before using"
        self.offsets[layer_ind] += new_k.shape[1] - self.length_at(layer_ind)
        self.cache[layer_ind] = (new_k, new_v)

    def truncate(self, truncate_amt, front=False):
        """kv_cache.py:60-75: eject ``truncate_amt`` FRAMES; front=True drops the newest tokens,
        front=False the oldest (the reference's naming, kept as is); offsets are unchanged."""
        amt = truncate_amt * self.config.tokens_per_frame
        for i, (k, v) in enumerate(self.cache):
            self.cache[i] = (k[:, :-amt], v[:, :-amt]) if front else (k[:, amt:], v[:, amt:])

    def length_at(self, idx):
        return self.cache[idx][0].shape[1]

    def get_offset(self, idx=0):
        return self.offsets[idx]

    def __len__(self):
        assert self.cache is not None, "Must reset cache before using"
        return self.cache[0][0].shape[1]

    def n_frames(self):
        assert len(self) % self.config.tokens_per_frame == 0
        return len(self) // self.config.tokens_per_frame

    def clone(self):
        self.cache = [(k.clone(), v.clone()) for k, v in self.cache]
        return self

    def detach(self):
        self.cache = [(k.detach(), v.detach()) for k, v in self.cache]
        return self

    @property
    def shape(self):
        return self.cache[0][0].shape
