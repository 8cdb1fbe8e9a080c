"""mmattn.py (reference: owl_wms/nn/mmattn.py:28-152) -- two-stream MMDiT on libowlk.

Per layer (``MMDiTBlockFn``, one autograd Function for the whole block, both modalities):
    h_s   = cond_adaln(x_s, scale_s, bias_s)            adaln_fwd    (video tpf 64, audio tpf 1)
    qkv_s = h_s Wqkv_s^T + b                            GEMM
    joint = frame_interleave(qkv_v, qkv_a)              frame_mux: frame f = [64 video | 1 audio]
    q, k  = rope(rms(q)), rope(rms(k))                  qk_rope_fwd  (OrthoRoPE table, 65-token frames)
    o     = attn(q, k, v)                               attn_fwd     (frame mask, tpf 65, local/global window)
    o_s   = frame_split(o)                              frame_mux
    x_s  += gate_s * (o_s Wout_s^T + b)                 GEMM + gate/residual epilogue
    x_s  += gate2_s * MLP_s(cond_adaln(x_s, ...))       adaln_fwd + GEMM(SiLU) + GEMM(gate/residual)
and the mirrored backward.  The modulation is shared by every layer (DiT-Air, mmattn.py:126-130,
148): each block returns its [B, F, 6d] modulation gradient in the reference's chunk order
(attn scale, bias, gate, mlp scale, bias, gate) and autograd sums them across layers.

The reference module imports a missing ``create_causal_block_mask``; its
mask is reconstructed as get_block_mask(n, tpf, window, no docs, q_offset, causal) -- a
FrameMask here.

KV cache (mmattn.py:46-72, decode / sampling, no grad): the new joint frame(s) are rotated at
offset = the layer's cached length, [cache | new] K/V are read in place (SingleKVCache.extend),
the cache is committed when updates are enabled, and the attention keeps the frame mask with
q_offset = the cached length (the reference's create_causal_block_mask(n_cached_tokens=offset)).
"""
import torch
from torch import nn

from .. import kernels as K
from .fused import bf16_weight, cond_silu, grad_done, grad_sink, linear
from .mlp import MLP
from .rope import get_rope_cls

BF16 = torch.bfloat16


class MMGeometry:
    def __init__(self, n_heads, head_dim, n0, n1, mask, cos, sin):
        self.H, self.D, self.n0, self.n1, self.mask, self.cos, self.sin = n_heads, head_dim, n0, n1, mask, cos, sin


def _joint_views(j, n0, n1, cols):
    """The per-modality rows of a joint-sequence buffer j [F (n0 + n1), cols] as operands that
    libowlk reads / writes in place: the video rows as a frame-strided [F, n0, cols] view
    (kernels.frame_rows), the audio row of every frame as a plain strided [F, cols] view."""
    F_ = j.shape[0] // (n0 + n1)
    return K.frame_rows(j, n0, n1, 0, cols), j.view(F_, n0 + n1, cols)[:, n0, :]


def _in_place_ok(d, n0, n1, frames):
    """The joint layout is used in place (no frame_mux copies) where the video GEMMs tile by 256
    (owlk_gemm_frames): mmdit_v2 (d 1536, 8x8 latents + 1 audio token per frame), for more than
    four frames of video rows (fewer take the frame_mux path, as decode-sized GEMMs)."""
    return n0 == K.FRAME_ROWS and n1 == 1 and d % 256 == 0 and frames * n0 > 256


def _lane_ok(inplace, frames, n1):
    """The audio side stream only where its GEMMs (frames * n1 rows) stay off the decode plan, whose
    workspace counters are shared per device (kernels._decode_ws)."""
    return inplace and frames * n1 > 128


_AUDIO_STREAMS = {}


class _AudioLane:
    """The audio modality's per-block work (adaln, its 1,000-row GEMMs, gate / adaln backward) on a
    side HIP stream beside the video's: at mmdit_v2 the audio rows are 1/64 of the video's, so their
    GEMMs fill few CUs and run at a fifth of the video GEMMs' rate (3 % of the micro-step serially).
    fork(): the side stream waits for everything enqueued so far; join(): the caller's stream waits
    for the side stream.  Tensors the side stream allocates are marked for the caller's stream
    (record_stream), so the caching allocator never hands their blocks to later side-stream work while
    the caller's stream may still read them.  Serial (no side stream) for the frame_mux layout, while a
    profile window is open or a graph is being captured, or with OWLK_MMDIT_AUDIO_STREAM=0."""

    def __init__(self, device, enable):
        import os
        from .. import _lib
        self.main = torch.cuda.current_stream(device)
        self.side = None
        if enable and os.environ.get("OWLK_MMDIT_AUDIO_STREAM", "1") != "0" and not _lib.profiling() and \
                not torch.cuda.is_current_stream_capturing():
            self.side = _AUDIO_STREAMS.get(device)
            if self.side is None:
                self.side = _AUDIO_STREAMS[device] = torch.cuda.Stream(device=device)

    def fork(self):
        if self.side is not None:
            self.side.wait_stream(self.main)

    def join(self):
        if self.side is not None:
            self.main.wait_stream(self.side)

    def on(self, s):
        """context for modality s's work: the side stream for audio (s = 1)"""
        import contextlib
        return torch.cuda.stream(self.side) if (s == 1 and self.side is not None) else contextlib.nullcontext()

    def mark(self, ts):
        if self.side is not None:
            for t in ts:
                if isinstance(t, torch.Tensor):
                    t.record_stream(self.main)


class MMDiTBlockFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x0, x1, c0, c1, geo, *w):
        B, T0, d = x0.shape
        H, D, n0, n1 = geo.H, geo.D, geo.n0, geo.n1
        nf = B * (T0 // n0)
        T = (T0 // n0) * (n0 + n1)
        xs = (x0.reshape(-1, d), x1.reshape(-1, d))
        ms = (c0.reshape(nf, 6 * d), c1.reshape(nf, 6 * d))
        ns = (n0, n1)
        W = [w[0:2], w[2:4]], [w[4:6], w[6:8]], [w[8:12], w[12:16]]  # qkv, out, mlp (fc1 w/b, fc2 w/b)
        inplace = _in_place_ok(d, n0, n1, nf)
        lane = _AudioLane(x0.device, _lane_ok(inplace, nf, n1))
        h1, r1, qkv = [None, None], [None, None], [None, None]
        if inplace:  # each modality's qkv projection writes its rows of the joint frames directly
            qkvj = torch.empty(B * T, 3 * d, device=x0.device, dtype=BF16)
            qkv_dst = _joint_views(qkvj, n0, n1, 3 * d)
        wq = [bf16_weight(W[0][s][0]) for s in range(2)]
        lane.fork()
        for s in (1, 0):  # audio first: its launches go to the side stream, then the video's run beside
            with lane.on(s):
                h1[s], r1[s] = K.adaln_fwd(xs[s], ms[s][:, :d], ms[s][:, d:2 * d], ns[s])
                qkv[s] = K.gemm(h1[s], wq[s], bias=W[0][s][1], out=qkv_dst[s] if inplace else None)
        lane.mark(h1[1:] + r1[1:])
        lane.join()
        if not inplace:
            qkvj = K.frame_interleave(qkv[0], qkv[1], n0, n1)
        del qkv
        qkr, rq = K.qk_rope_fwd(qkvj, H, D, geo.cos, geo.sin, 0, T)
        q3, k3 = qkr.view(B, T, 2 * d)[:, :, :d], qkr.view(B, T, 2 * d)[:, :, d:]
        o, lse = K.attn_fwd(q3, k3, qkvj.view(B, T, 3 * d)[:, :, 2 * d:], H, D, geo.mask,
                            score_bound=K.qk_norm_bound(D))
        os_ = _joint_views(o.view(B * T, d), n0, n1, d) if inplace else K.frame_split(o.view(B * T, d), n0, n1)
        saved, outs = [None, None], [None, None]
        wts = [[bf16_weight(W[1][s][0]), bf16_weight(W[2][s][0]), bf16_weight(W[2][s][2])] for s in range(2)]
        lane.fork()
        for s in (1, 0):
            with lane.on(s):
                g1, g2 = ms[s][:, 2 * d:3 * d], ms[s][:, 5 * d:]
                M = xs[s].shape[0]
                y1 = torch.empty(M, d, device=x0.device, dtype=BF16)
                x1s = K.gemm(os_[s], wts[s][0], bias=W[1][s][1], epi=K.EPI_GATE_RESID, aux=y1, gate=g1, tpf=ns[s],
                             resid=xs[s])
                h2, r2 = K.adaln_fwd(x1s, ms[s][:, 3 * d:4 * d], ms[s][:, 4 * d:5 * d], ns[s])
                a_pre = torch.empty(M, W[2][s][0].shape[0], device=x0.device, dtype=BF16)
                a = K.gemm(h2, wts[s][1], bias=W[2][s][1], epi=K.EPI_SILU, aux=a_pre)
                y2 = torch.empty(M, d, device=x0.device, dtype=BF16)
                outs[s] = K.gemm(a, wts[s][2], bias=W[2][s][3], epi=K.EPI_GATE_RESID, aux=y2, gate=g2, tpf=ns[s],
                                 resid=x1s)
                saved[s] = [xs[s], ms[s], h1[s], r1[s], y1, x1s, h2, r2, a_pre, a, y2]
        lane.mark(saved[1][4:] + [outs[1]])
        lane.join()
        ctx.save_for_backward(qkvj, qkr, rq, o, lse, *saved[0], *saved[1], *w)
        ctx.geo, ctx.dims = geo, (B, T0, x1.shape[1], d, T, nf)
        ctx.params = w  # the Parameters themselves: their GradReducer bucket views are the gradient sinks
        return outs[0].view(B, T0, d), outs[1].view(B, x1.shape[1], d)

    @staticmethod
    def backward(ctx, dout0, dout1):
        qkvj, qkr, rq, o, lse = ctx.saved_tensors[:5]
        st = [ctx.saved_tensors[5:16], ctx.saved_tensors[16:27]]
        w = ctx.saved_tensors[27:]
        geo = ctx.geo
        B, T0, T1, d, T, nf = ctx.dims
        H, D, n0, n1 = geo.H, geo.D, geo.n0, geo.n1
        ns = (n0, n1)
        dW = [None] * 16
        prm = ctx.params
        done = []  # parameters whose bucket view is complete, reported to the reducer on the main stream

        def wgrad(i, dy, x):  # dW_i = dy^T x straight into the bucket view (beta 1) or returned
            sink = grad_sink(prm[i])
            if sink is None:
                dW[i] = K.gemm_wgrad(dy, x)
            else:
                K.gemm(dy, x, a_trans=True, b_trans=True, out=sink, out_f32=True, beta=1.0)
                done.append(prm[i])

        def bgrad(i, rows):  # db_i = column sums of rows (bf16 rows or fp32 per-frame partials)
            sink = grad_sink(prm[i])
            if sink is None:
                dW[i] = K.colsum(rows)
            else:
                K.colsum(rows, out=sink)
                done.append(prm[i])

        def report():  # after a lane join: every write above is ordered before the main stream's next work
            for q in done:
                grad_done(q)
            done.clear()

        dcs = [torch.empty(nf, 6 * d, device=dout0.device, dtype=BF16) for _ in range(2)]  # d mods, bf16
        douts = (dout0.reshape(-1, d).to(BF16).contiguous(), dout1.reshape(-1, d).to(BF16).contiguous())
        inplace = _in_place_ok(d, n0, n1, nf)
        lane = _AudioLane(o.device, _lane_ok(inplace, nf, n1))
        if inplace:  # per-modality views of the joint o, and the joint dO the two dX GEMMs write into
            os_ = _joint_views(o.view(B * T, d), n0, n1, d)
            do = torch.empty(B * T, d, device=o.device, dtype=BF16)
            do_dst = _joint_views(do, n0, n1, d)
        else:
            os_ = K.frame_split(o.view(B * T, d), n0, n1)
        dos, dx1s = [None, None], [None, None]
        wts = [[bf16_weight(w[10 + 4 * s]), bf16_weight(w[8 + 4 * s]), bf16_weight(w[4 + 2 * s])] for s in range(2)]
        lane.fork()
        for s in (1, 0):
            with lane.on(s):
                xs, ms, h1, r1, y1, x1s, h2, r2, a_pre, a, y2 = st[s]
                dm = dcs[s]
                # ---- MLP
                dy2, _, dbf2 = K.gate_bwd(douts[s], y2, ms[:, 5 * d:], ns[s], dg_out=dm[:, 5 * d:])
                bgrad(11 + 4 * s, dbf2)
                i_b1 = 9 + 4 * s
                sink_b1 = grad_sink(prm[i_b1])
                cs = sink_b1 if sink_b1 is not None else torch.zeros(a_pre.shape[1], device=a_pre.device,
                                                                     dtype=torch.float32)
                dapre = K.gemm(dy2, wts[s][0], b_trans=True, epi=K.EPI_DSILU, aux=a_pre, colsum=cs)
                if sink_b1 is not None:
                    done.append(prm[i_b1])
                else:
                    dW[i_b1] = cs
                wgrad(10 + 4 * s, dy2, a)
                wgrad(8 + 4 * s, dapre, h2)
                dh2 = K.gemm(dapre, wts[s][1], b_trans=True)
                del dapre, dy2
                if K.ADALN_GATE:  # + the attention output's gate backward on the dx rows (bit for bit)
                    dx1, dy1, dbf1 = K.adaln_gate_bwd_into(dh2, x1s, r2, ms[:, 3 * d:4 * d], ns[s], dm[:, 3 * d:5 * d],
                                                           douts[s], y1, ms[:, 2 * d:3 * d], dm[:, 2 * d:3 * d])
                else:
                    dx1 = K.adaln_bwd_into(dh2, x1s, r2, ms[:, 3 * d:4 * d], ns[s], dm[:, 3 * d:5 * d], dres=douts[s])
                    dy1, _, dbf1 = K.gate_bwd(dx1, y1, ms[:, 2 * d:3 * d], ns[s], dg_out=dm[:, 2 * d:3 * d])
                # ---- attention output projection
                bgrad(5 + 2 * s, dbf1)
                dos[s] = K.gemm(dy1, wts[s][2], b_trans=True, out=do_dst[s] if inplace else None)
                wgrad(4 + 2 * s, dy1, os_[s])
                dx1s[s] = dx1
        lane.mark([dW[i] for i in (6, 7, 12, 13, 14, 15)] + [dx1s[1]] + [dos[1]])  # audio's
        lane.join()
        report()
        del os_
        if not inplace:
            do = K.frame_interleave(dos[0], dos[1], n0, n1)
        del dos
        dqkvj = torch.empty(B * T, 3 * d, device=o.device, dtype=BF16)
        dqkr = torch.empty(B * T, 2 * d, device=o.device, dtype=BF16)
        q3, k3 = qkr.view(B, T, 2 * d)[:, :, :d], qkr.view(B, T, 2 * d)[:, :, d:]
        dq3, dk3 = dqkr.view(B, T, 2 * d)[:, :, :d], dqkr.view(B, T, 2 * d)[:, :, d:]
        K.attn_bwd(q3, k3, qkvj.view(B, T, 3 * d)[:, :, 2 * d:], o.view(B, T, d), do.view(B, T, d), lse, H, D,
                   geo.mask, dq3, dk3, dqkvj.view(B, T, 3 * d)[:, :, 2 * d:])
        del do
        K.qk_rope_bwd(dqkr, qkvj, rq, H, D, geo.cos, geo.sin, dqkvj, 0, T)
        del dqkr
        # the per-modality qkv gradients: views of the joint rows (in place) or split copies
        dqkv = _joint_views(dqkvj, n0, n1, 3 * d) if inplace else K.frame_split(dqkvj, n0, n1)
        dxs = [None, None]
        wq = [bf16_weight(w[2 * s]) for s in range(2)]
        lane.fork()
        for s in (1, 0):
            with lane.on(s):
                xs, ms, h1, r1 = st[s][:4]
                bgrad(1 + 2 * s, dqkv[s])
                wgrad(2 * s, dqkv[s], h1)
                dh1 = K.gemm(dqkv[s], wq[s], b_trans=True)
                dxs[s] = K.adaln_bwd_into(dh1, xs, r1, ms[:, :d], ns[s], dcs[s][:, :2 * d], dres=dx1s[s])
        lane.mark([dW[3], dW[2], dxs[1], dcs[1]])
        lane.join()
        report()
        return (dxs[0].view(B, T0, d), dxs[1].view(B, T1, d), dcs[0].view(B, nf // B, 6 * d),
                dcs[1].view(B, nf // B, 6 * d), None, *dW)


class MMAttn(nn.Module):
    """mmattn.py:28-86 -- parameters / keys of the reference; compute lives in MMDiTBlockFn."""

    def __init__(self, config, layer_idx, rope=None):
        super().__init__()
        self.config = config
        self.layer_idx = layer_idx
        self.n_heads = config.n_heads
        self.tok_per_frame_mod = [config.sample_size ** 2, 1]
        self.qkv_projs = nn.ModuleList([nn.Linear(config.d_model, 3 * config.d_model) for _ in range(2)])
        self.out_projs = nn.ModuleList([nn.Linear(config.d_model, config.d_model) for _ in range(2)])
        object.__setattr__(self, "rope", rope if rope is not None else
                           get_rope_cls(getattr(config, "rope_impl", "ortho"))(config))


class MMDiTBlock(nn.Module):
    def __init__(self, config, layer_idx, rope=None):
        super().__init__()
        self.config = config
        self.attn = MMAttn(config, layer_idx, rope)
        self.mlps = nn.ModuleList([MLP(config) for _ in range(2)])

    def forward(self, x0, x1, cond0, cond1, block_mask=None, kv_cache=None):
        if kv_cache is not None:
            with torch.no_grad():
                return self._forward_cached(x0, x1, cond0, cond1, block_mask, kv_cache)
        cfg, a = self.config, self.attn
        H = cfg.n_heads
        n0 = cfg.sample_size ** 2
        geo = MMGeometry(H, cfg.d_model // H, n0, 1, block_mask, a.rope.cos, a.rope.sin)
        ws = []
        for s in range(2):
            ws += [a.qkv_projs[s].weight, a.qkv_projs[s].bias]
        for s in range(2):
            ws += [a.out_projs[s].weight, a.out_projs[s].bias]
        for s in range(2):
            m = self.mlps[s]
            ws += [m.fc1.weight, m.fc1.bias, m.fc2.weight, m.fc2.bias]
        return MMDiTBlockFn.apply(x0.to(BF16).contiguous(), x1.to(BF16).contiguous(), cond0, cond1, geo, *ws)


    def _forward_cached(self, x0, x1, cond0, cond1, block_mask, kv_cache):
        """MMDiTBlock.forward (mmattn.py:98-114) with MMAttn's cache path (mmattn.py:46-72)."""
        cfg, a = self.config, self.attn
        d, H = cfg.d_model, cfg.n_heads
        D = d // H
        n0, n1 = cfg.sample_size ** 2, 1
        B, T0, _ = x0.shape
        nf = T0 // n0
        T = nf * (n0 + n1)
        ns = (n0, n1)
        xs = (x0.reshape(-1, d).to(BF16).contiguous(), x1.reshape(-1, d).to(BF16).contiguous())
        ms = (cond0.reshape(B * nf, 6 * d), cond1.reshape(B * nf, 6 * d))
        qkv = []
        for s in range(2):
            h, _ = K.adaln_fwd(xs[s], ms[s][:, :d], ms[s][:, d:2 * d], ns[s])
            qkv.append(K.gemm(h, bf16_weight(a.qkv_projs[s].weight), bias=a.qkv_projs[s].bias))
        qkvj = K.frame_interleave(qkv[0], qkv[1], n0, n1)
        del qkv
        li = a.layer_idx
        offset = kv_cache.length_at(li)
        qkr, _ = K.qk_rope_fwd(qkvj, H, D, a.rope.cos, a.rope.sin, offset, T)
        q = qkr.view(B, T, 2 * d)[:, :, :d]
        k = qkr.view(B, T, 2 * d)[:, :, d:]
        v = qkvj.view(B, T, 3 * d)[:, :, 2 * d:]
        if offset > 0:
            if kv_cache.noise_caches == 0.0 and hasattr(kv_cache, "extend"):
                k, v = kv_cache.extend(li, k, v)
            else:
                old_k, old_v = kv_cache.get(li)
                k, v = torch.cat([old_k, k], dim=1), torch.cat([old_v, v], dim=1)
        if kv_cache.should_update:
            kv_cache.update(k, v, li)
        mask = block_mask if block_mask is not None else K.FrameMask(1, None, False, 0, None)
        o, _ = K.attn_fwd(q, k, v, H, D, mask, score_bound=K.qk_norm_bound(D))
        os_ = K.frame_split(o.view(B * T, d), n0, n1)
        outs = []
        for s in range(2):
            x1s = K.gemm(os_[s], bf16_weight(a.out_projs[s].weight), bias=a.out_projs[s].bias, epi=K.EPI_GATE_RESID,
                         gate=ms[s][:, 2 * d:3 * d], tpf=ns[s], resid=xs[s])
            h2, _ = K.adaln_fwd(x1s, ms[s][:, 3 * d:4 * d], ms[s][:, 4 * d:5 * d], ns[s])
            m = self.mlps[s]
            a_pre = torch.empty(x1s.shape[0], m.fc1.weight.shape[0], device=x0.device, dtype=BF16)
            act = K.gemm(h2, bf16_weight(m.fc1.weight), bias=m.fc1.bias, epi=K.EPI_SILU, aux=a_pre)
            outs.append(K.gemm(act, bf16_weight(m.fc2.weight), bias=m.fc2.bias, epi=K.EPI_GATE_RESID,
                               gate=ms[s][:, 5 * d:], tpf=ns[s], resid=x1s))
        return outs[0].view(B, T0, d), outs[1].view(B, nf, d)


class MMDIT(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.config = config
        assert config.tokens_per_frame == config.sample_size ** 2 + 1, "MMDiT frames are [p*p video | 1 audio]"
        self.rope = get_rope_cls(getattr(config, "rope_impl", "ortho"))(config)
        self.local_layers = [(i % 4 != 0) for i in range(config.n_layers)]
        self.blocks = nn.ModuleList([MMDiTBlock(config, i, self.rope) for i in range(config.n_layers)])
        self.cond_proj = nn.Sequential(nn.SiLU(), nn.Linear(config.d_model, config.d_model * 2 * 2 * 3))

    def get_block_mask(self, x0, x1, kv_cache, window_len):
        """mmattn.py:132-143: causal frame mask over [cache | new] (q_offset = cached tokens)."""
        if not self.config.causal:
            return K.FrameMask(self.config.tokens_per_frame, None, False, 0, None)
        offset = kv_cache.length_at(0) if kv_cache is not None else 0
        return K.FrameMask(self.config.tokens_per_frame, window_len, True, offset, None)

    def forward(self, x0, x1, cond, kv_cache=None):
        local_mask = self.get_block_mask(x0, x1, kv_cache, self.config.local_window)
        global_mask = self.get_block_mask(x0, x1, kv_cache, getattr(self.config, "global_window", None))
        lin = self.cond_proj[1]
        c = linear(cond_silu(cond), lin.weight, lin.bias)
        cond0, cond1 = c.chunk(2, dim=-1)
        for i, block in enumerate(self.blocks):
            x0, x1 = block(x0, x1, cond0, cond1, local_mask if self.local_layers[i] else global_mask, kv_cache)
        return x0, x1
