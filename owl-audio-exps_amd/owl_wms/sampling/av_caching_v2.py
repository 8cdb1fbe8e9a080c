"""AVCachingSamplerV2 (reference: owl_wms/sampling/av_caching_v2.py:24-144) on libowlk.

Context frames are cached once at noise level ``noise_prev``; each new frame starts from
N(0, 1) at t = 1, takes ``n_steps`` Euler steps x -= dt_i v (optional CFG with null controls),
is re-noised (zlerp) and appended to the cache.  In decode mode the attention is unmasked over
[cache | new frame]; local layers keep the last local_window frames.  Noise is drawn with
torch.randn_like in the reference's order (context zlerp, then per frame: x0, then zlerp).

CFG (cfg_scale != 1): the reference runs the conditional and the null-control forward one after
the other over the same cache (av_caching_v2.py:98-118).  Here both run as ONE forward of batch
2B -- rows [cond | uncond] -- so each Euler step streams the weights once at twice the rows (a
decode step is weight-streaming bound).  The cache holds the context twice (both halves cached
from the conditioned passes, exactly what the reference's single cache holds), so every row sees
the keys the reference's forward sees.
"""
import torch

from .. import kernels as K
from ..nn.attn import check_rope_rows
from ..nn.kv_cache import KVCache
from .schedulers import get_deltas, get_sd3_euler


def _release_graph(g):
    """Destroy a step graph only after its queued replays have run: its exec (kernel arguments) and
    its private memory pool are released here, so no replay of it may still be queued then."""
    torch.cuda.current_stream().synchronize()
    g.reset()


class AVCachingSamplerV2:
    def __init__(self, n_steps: int = 16, cfg_scale: float = 1.3, num_frames: int = 60, noise_prev: float = 0.2,
                 max_window=None, custom_schedule=None) -> None:
        self.cfg_scale = cfg_scale
        self.n_steps = n_steps
        self.num_frames = num_frames
        self.noise_prev = noise_prev
        self.max_window = max_window
        self.custom_schedule = custom_schedule
        self._pool = None  # graph memory pool shared by the per-frame captures (compile_on_decode)
        self._graph_prev = None  # (graph, event) of the previous frame (compile_on_decode, host-position path)
        self._step_graph = None
        # keep the cache position on the device so one captured Euler step serves every frame
        # (False: the host-position path, one capture per frame with the cache length baked in)
        self.device_state = True

    @staticmethod
    def zlerp(x, alpha):
        z = torch.randn_like(x)
        return x * (1.0 - alpha) + z * alpha

    def _euler_step(self, model, kv_cache, x, t, mouse, btn, null_mouse, null_btn, dt):
        """av_caching_v2.py:96-110: one Euler step with optional CFG (cond | uncond as one 2B batch)."""
        if self.cfg_scale != 1.0:
            B = x.shape[0]
            pred = model(torch.cat([x, x]), torch.cat([t, t]), torch.cat([mouse, null_mouse]),
                         torch.cat([btn, null_btn]), kv_cache=kv_cache)
            pred_v, pred_u = pred[:B], pred[B:]
            pred_v = pred_u + self.cfg_scale * (pred_v - pred_u)
        else:
            pred_v = model(x, t, mouse, btn, kv_cache=kv_cache)
        return x - dt * pred_v, t - dt

    def _euler_graphed(self, model, kv_cache, x, t, mouse, btn, null_mouse, null_btn, dt, warm=True):
        """The frame's n_steps Euler steps replayed from one HIP graph.

        The cache is read-only and fixed in length while a frame is denoised, so every step launches
        the same kernels on the same buffers: one step is captured with x, t and dt in static device
        buffers and replayed -- same kernels and arithmetic as the eager loop (the reference's
        ``compile_on_decode`` switch).  With ``warm`` (the first frame) step 0
        runs eagerly first: it creates the per-weight bf16 copies and workspaces outside the graph's
        memory pool; later frames replay every step."""
        first = 0
        if warm:
            x, t = self._euler_step(model, kv_cache, x, t, mouse, btn, null_mouse, null_btn, dt[0])
            first = 1
            if self.n_steps == 1:
                return x, t
        sx, st, sdt = x.clone(), t.clone(), dt[first].clone()
        if self._pool is None:
            self._pool = torch.cuda.graph_pool_handle()
        g = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            with torch.cuda.graph(g, pool=self._pool, stream=side):
                nx, nt = self._euler_step(model, kv_cache, sx, st, mouse, btn, null_mouse, null_btn, sdt)
                sx.copy_(nx)
                st.copy_(nt)
        torch.cuda.current_stream().wait_stream(side)
        for t_idx in range(first, self.n_steps):
            sdt.copy_(dt[t_idx])
            g.replay()
        out = sx.clone(), st.clone()
        # keep this frame's graph until the next frame's replays are queued, then release the previous
        # one behind its own event (its replays ran long before): no full-stream sync per frame
        ev = torch.cuda.Event()
        ev.record()
        prev, self._graph_prev = self._graph_prev, (g, ev)
        if prev is not None:
            prev[1].synchronize()
            prev[0].reset()
        return out

    def _euler_replay(self, model, kv_cache, x, t, mouse, btn, null_mouse, null_btn, dt):
        """compile_on_decode with the cache position on the device (SingleKVCache.enable_device_state):
        ONE Euler step is captured on the first frame and replayed for every step of every frame
        (its inputs are copied into the graph's static buffers first; the decode kernels read the
        growing cache's position from the device).  The cache-update forward between frames stays
        eager: its launches overlap the replays still running on the GPU."""
        st = self._step_graph
        first = 0
        if st is None:
            # first frame: step 0 eagerly (bf16 weight copies, workspaces outside the graph pool)
            x, t = self._euler_step(model, kv_cache, x, t, mouse, btn, null_mouse, null_btn, dt[0])
            if self.n_steps == 1:
                return x, t
            bufs = {"x": x.clone(), "t": t.clone(), "dt": dt[1].clone(), "mouse": mouse.clone(), "btn": btn.clone(),
                    "nm": null_mouse.clone(), "nb": null_btn.clone()}
            if self._pool is None:
                self._pool = torch.cuda.graph_pool_handle()
            g = torch.cuda.CUDAGraph()
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                with torch.cuda.graph(g, pool=self._pool, stream=side):
                    nx, nt = self._euler_step(model, kv_cache, bufs["x"], bufs["t"], bufs["mouse"], bufs["btn"],
                                              bufs["nm"], bufs["nb"], bufs["dt"])
                    bufs["x"].copy_(nx)
                    bufs["t"].copy_(nt)
            torch.cuda.current_stream().wait_stream(side)
            self._step_graph = st = (g, bufs)
            first = 1
        else:
            g, bufs = st
            # the replayed step reads its positions from the device: check them here as the eager
            # step's Attn._attend does (the kernels would only poison the rows with NaN)
            rope = getattr(model.transformer, "rope", None)
            if rope is not None:
                check_rope_rows(rope, kv_cache.get_offset(0), model.config.tokens_per_frame)
            for k, v in (("x", x), ("t", t), ("mouse", mouse), ("btn", btn)):
                bufs[k].copy_(v)
        g, bufs = st
        for t_idx in range(first, self.n_steps):
            bufs["dt"].copy_(dt[t_idx])
            g.replay()
        return bufs["x"].clone(), bufs["t"].clone()

    @torch.no_grad()
    def __call__(self, model, x, mouse, btn, compile_on_decode=False):
        """model: a GameRFTCore ([b,n,c,h,w] latents, kv_cache API); returns [b, init+new, c, h, w]."""
        batch_size, init_len = x.size(0), x.size(1)
        if self.custom_schedule is None:
            dt = get_sd3_euler(self.n_steps).to(device=x.device, dtype=x.dtype)
        else:
            # Python floats in the reference: fp32 device scalars (same opmath; a captured graph
            # reads them from device memory)
            dt = torch.tensor(get_deltas(list(self.custom_schedule)), device=x.device, dtype=torch.float32)
        cfg = self.cfg_scale != 1.0
        rep = (lambda *ts: [torch.cat([a, a]) for a in ts]) if cfg else (lambda *ts: list(ts))
        kv_cache = KVCache(model.config)
        kv_cache.reset(2 * batch_size if cfg else batch_size)

        latents = [x.clone()]
        prev_x = x
        prev_mouse, prev_btn = mouse[:, :init_len], btn[:, :init_len]
        prev_x_noisy = self.zlerp(prev_x, self.noise_prev)
        prev_t = prev_x.new_full((batch_size, prev_x.size(1)), self.noise_prev)
        kv_cache.enable_cache_updates()
        model(*rep(prev_x_noisy, prev_t, prev_mouse, prev_btn), kv_cache=kv_cache)
        kv_cache.disable_cache_updates()

        num_frames = min(self.num_frames, mouse.size(1) - init_len)
        self._step_graph = None
        self._graph_prev = None
        # the cache position on the device (one captured step for every frame); the same kernels run
        # in eager mode too, so eager and graphed decode stay bit-identical
        cfgm = model.config
        dev_state = self.device_state and hasattr(kv_cache, "enable_device_state") and \
            K.decode_dev_supported(cfgm.d_model // cfgm.n_heads, cfgm.tokens_per_frame)
        if dev_state:  # room for every frame up front: fixed buffer addresses for the one graph
            kv_cache.enable_device_state((init_len + num_frames + 1) * model.config.tokens_per_frame)
        model.transformer.enable_decoding()
        try:
            for idx in range(num_frames):
                curr_x, curr_t = torch.randn_like(prev_x[:, :1]), prev_t.new_ones(batch_size, 1)
                start = init_len + idx
                curr_mouse, curr_btn = mouse[:, start:start + 1], btn[:, start:start + 1]
                null_mouse, null_btn = torch.zeros_like(curr_mouse), torch.zeros_like(curr_btn)
                if dev_state and compile_on_decode:
                    curr_x, curr_t = self._euler_replay(model, kv_cache, curr_x, curr_t, curr_mouse, curr_btn,
                                                        null_mouse, null_btn, dt)
                elif compile_on_decode:
                    curr_x, curr_t = self._euler_graphed(model, kv_cache, curr_x, curr_t, curr_mouse, curr_btn,
                                                         null_mouse, null_btn, dt, warm=idx == 0)
                else:
                    for t_idx in range(self.n_steps):
                        curr_x, curr_t = self._euler_step(model, kv_cache, curr_x, curr_t, curr_mouse, curr_btn,
                                                          null_mouse, null_btn, dt[t_idx])
                latents.append(curr_x.clone())
                curr_x_noisy = self.zlerp(curr_x, self.noise_prev)
                curr_t_noisy = torch.ones_like(curr_t) * self.noise_prev
                kv_cache.enable_cache_updates()
                model(*rep(curr_x_noisy, curr_t_noisy, curr_mouse, curr_btn), kv_cache=kv_cache)
                kv_cache.disable_cache_updates()
                if self.max_window is not None and len(latents) > self.max_window:
                    kv_cache.truncate(1, front=False)
        finally:
            model.transformer.disable_decoding()
            if self._step_graph is not None:
                _release_graph(self._step_graph[0])
            self._step_graph = None
            if self._graph_prev is not None:
                _release_graph(self._graph_prev[0])
            self._graph_prev = None
        return torch.cat(latents, dim=1)
