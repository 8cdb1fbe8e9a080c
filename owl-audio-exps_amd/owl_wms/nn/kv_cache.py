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
    """Per layer a preallocated token-major K/V buffer ``[B, cap, d]`` with a live window
    ``[start, start + len)``.  ``extend`` writes a new frame's K/V behind the window and returns
    views of ``[cache | new]``: the decode step reads the cache in place instead of re-copying it
    with ``torch.cat`` per layer and step, and the addresses stay fixed while a frame is denoised
    (the sampler's HIP-graph replay relies on that)."""

    def __init__(self, config):
        self.config = config
        self.bufs = None
        self.device = "cuda"
        self.dtype = torch.bfloat16
        self.should_update = False
        self.noise_caches = 0.0
        self.offsets = [0] * config.n_layers
        self.start = [0] * config.n_layers
        self.len = [0] * config.n_layers
        self.dev = None  # device state {start, cached tokens, rope offset} (enable_device_state)

    def enable_device_state(self, capacity):
        """Decode with the cache position on the device: every layer's buffer is reserved for
        `capacity` tokens (no reallocation or compaction while sampling: fixed addresses), and the
        decode kernels read {start, cached tokens, rope offset} from an int64 device vector, so a
        HIP graph captured once serves every frame while the cache grows.  All layers advance
        together in decode, so one vector describes them all."""
        for i in range(self.config.n_layers):
            kb = self.bufs[i]
            assert kb is not None, "enable_device_state after the context pass"
            if kb[0].shape[1] < capacity:
                n, s = self.len[i], self.start[i]
                new = tuple(torch.empty(kb[0].shape[0], capacity, kb[0].shape[2], device=kb[0].device,
                                        dtype=kb[0].dtype) for _ in range(2))
                if n:
                    for dst, src in zip(new, (kb[0][:, s:s + n], kb[1][:, s:s + n])):
                        dst[:, :n].copy_(src)
                self.bufs[i], self.start[i] = new, 0
        self.dev = torch.zeros(4, dtype=torch.int64, device=self.bufs[0][0].device)
        self.sync_device_state()

    def sync_device_state(self):
        """host position -> the device vector (outside graph capture: an H2D copy)"""
        if self.dev is None:
            return
        st = {(self.start[i], self.len[i], self.offsets[i]) for i in range(self.config.n_layers)}
        assert len(st) == 1, "device-state decode needs every layer at the same position"
        s, n, o = st.pop()
        assert s + n <= self.bufs[0][0].shape[1]
        self.dev.copy_(torch.tensor([s, n, o, 0], dtype=torch.int64))

    def commit_device(self, layer_ind, L):
        """host bookkeeping of a device-state decode step that wrote L new rows behind the window
        (the device vector is refreshed once per forward, sync_device_state)"""
        assert self.start[layer_ind] + self.len[layer_ind] + L <= self.bufs[layer_ind][0].shape[1], \
            "cache capacity exceeded (enable_device_state(capacity))"
        self.len[layer_ind] += L
        self.offsets[layer_ind] += L

    def enable_cache_updates(self):
        self.should_update = True

    def disable_cache_updates(self):
        self.should_update = False

    def to(self, device="cuda", dtype=torch.bfloat16):
        self.device, self.dtype = device, dtype
        return self

    def reset(self, batch_size=1):
        self.batch_size = batch_size
        self.dev = None
        self.bufs = [None] * self.config.n_layers
        self.offsets = [0] * self.config.n_layers
        self.start = [0] * self.config.n_layers
        self.len = [0] * self.config.n_layers

    def _views(self, i, n):
        kb, vb = self.bufs[i]
        s = self.start[i]
        return kb[:, s:s + n], vb[:, s:s + n]

    def _reserve(self, i, need, like):
        """Room for `need` tokens from `start`: compact to 0 or grow (x2), keeping the live window."""
        buf = self.bufs[i]
        if buf is not None and self.start[i] + need <= buf[0].shape[1]:
            return
        n = self.len[i]
        cap = buf[0].shape[1] if buf is not None else 0
        if buf is None or need > cap:
            cap = max(2 * need, need + 16 * self.config.tokens_per_frame)
        new = tuple(torch.empty(like.shape[0], cap, like.shape[2], device=like.device, dtype=like.dtype)
                    for _ in range(2))
        if buf is not None and n:
            for dst, src in zip(new, self._views(i, n)):
                dst[:, :n].copy_(src)
        self.bufs[i], self.start[i] = new, 0

    @property
    def cache(self):
        assert self.bufs is not None, "Must reset cache before using"
        return [self._views(i, self.len[i]) if self.bufs[i] is not None else (None, None)
                for i in range(self.config.n_layers)]

    def get(self, layer_ind):
        assert self.bufs is not None, "Must reset cache before using"
        k, v = self._views(layer_ind, self.len[layer_ind])
        if self.noise_caches > 0.0:
            k = k + torch.randn_like(k) * self.noise_caches
            v = v + torch.randn_like(v) * self.noise_caches
        return k, v

    def extend_slots(self, layer_ind, L, like):
        """Views of the [B, L, d] slots behind the layer's cached window where the new frame's K/V go
        (written there directly by the decode rope kernel); ``extended(layer_ind, L)`` then gives
        [cache | new]."""
        assert self.noise_caches == 0.0, "the slots are read as stored (noise_caches must be 0)"
        n = self.len[layer_ind]
        self._reserve(layer_ind, n + L, like)
        kb, vb = self.bufs[layer_ind]
        s = self.start[layer_ind]
        return kb[:, s + n:s + n + L], vb[:, s + n:s + n + L]

    def extended(self, layer_ind, L):
        return self._views(layer_ind, self.len[layer_ind] + L)

    def extend(self, layer_ind, new_k, new_v):
        """[cache | new] as views of the layer's buffer (new K/V written once behind the cache)."""
        assert self.noise_caches == 0.0, "extend reads the cache as stored (noise_caches must be 0)"
        n, L = self.len[layer_ind], new_k.shape[1]
        self._reserve(layer_ind, n + L, new_k)
        kb, vb = self.bufs[layer_ind]
        s = self.start[layer_ind]
        kb[:, s + n:s + n + L].copy_(new_k)
        vb[:, s + n:s + n + L].copy_(new_v)
        return self._views(layer_ind, n + L)

    def update(self, new_k, new_v, layer_ind):
        """kv_cache.py:47-58: the layer's cache becomes (new_k, new_v); a view returned by extend is
        committed in place."""
        assert self.bufs is not None, "Must reset cache before using"
        L = new_k.shape[1]
        self.offsets[layer_ind] += L - self.len[layer_ind]
        buf = self.bufs[layer_ind]
        if buf is not None and new_k.data_ptr() == buf[0][:, self.start[layer_ind]].data_ptr() \
                and new_k.stride() == buf[0].stride():
            self.len[layer_ind] = L
            return
        self.len[layer_ind] = 0
        self._reserve(layer_ind, L, new_k)
        kb, vb = self.bufs[layer_ind]
        kb[:, :L].copy_(new_k)
        vb[:, :L].copy_(new_v)
        self.start[layer_ind], self.len[layer_ind] = 0, L

    def truncate(self, truncate_amt, front=False):
        """kv_cache.py:60-75: eject ``truncate_amt`` FRAMES; front=True drops the newest tokens,
        front=False the oldest (the reference's naming, kept as is); offsets are unchanged."""
        amt = truncate_amt * self.config.tokens_per_frame
        for i in range(self.config.n_layers):
            amt_i = min(amt, self.len[i])
            if not front:
                self.start[i] += amt_i
            self.len[i] -= amt_i
        self.sync_device_state()

    def length_at(self, idx):
        return self.len[idx]

    def get_offset(self, idx=0):
        return self.offsets[idx]

    def __len__(self):
        assert self.bufs is not None, "Must reset cache before using"
        return self.len[0]

    def n_frames(self):
        assert len(self) % self.config.tokens_per_frame == 0
        return len(self) // self.config.tokens_per_frame

    def clone(self):
        for i in range(self.config.n_layers):
            if self.bufs[i] is not None:
                self.bufs[i] = tuple(b.clone() for b in self.bufs[i])
        return self

    def detach(self):
        return self

    @property
    def shape(self):
        return self.cache[0][0].shape
