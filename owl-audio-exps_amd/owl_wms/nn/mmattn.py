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
import torch.nn.functional as F
from torch import nn

from .. import kernels as K
from .fused import bf16_weight, linear
from .mlp import MLP
from .rope import get_rope_cls

BF16 = torch.bfloat16


class MMGeometry:
    def __init__(self, n_heads, head_dim, n0, n1, mask, cos, sin):
        self.H, self.D, self.n0, self.n1, self.mask, self.cos, self.sin = n_heads, head_dim, n0, n1, mask, cos, sin


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
        h1, r1, qkv = [], [], []
        for s in range(2):
            h, r = K.adaln_fwd(xs[s], ms[s][:, :d], ms[s][:, d:2 * d], ns[s])
            h1.append(h)
            r1.append(r)
            qkv.append(K.gemm(h, bf16_weight(W[0][s][0]), bias=W[0][s][1]))
        qkvj = K.frame_interleave(qkv[0], qkv[1], n0, n1)
        del qkv
        qkr, rq = K.qk_rope_fwd(qkvj, H, D, geo.cos, geo.sin, 0, T)
        q3, k3 = qkr.view(B, T, 2 * d)[:, :, :d], qkr.view(B, T, 2 * d)[:, :, d:]
        o, lse = K.attn_fwd(q3, k3, qkvj.view(B, T, 3 * d)[:, :, 2 * d:], H, D, geo.mask,
                            score_bound=K.qk_norm_bound(D))
        os_ = K.frame_split(o.view(B * T, d), n0, n1)
        saved, outs = [], []
        for s in range(2):
            g1, g2 = ms[s][:, 2 * d:3 * d], ms[s][:, 5 * d:]
            M = xs[s].shape[0]
            y1 = torch.empty(M, d, device=x0.device, dtype=BF16)
            x1s = K.gemm(os_[s], bf16_weight(W[1][s][0]), bias=W[1][s][1], epi=K.EPI_GATE_RESID, aux=y1, gate=g1,
                         tpf=ns[s], resid=xs[s])
            h2, r2 = K.adaln_fwd(x1s, ms[s][:, 3 * d:4 * d], ms[s][:, 4 * d:5 * d], ns[s])
            fc1w, fc1b, fc2w, fc2b = W[2][s]
            a_pre = torch.empty(M, fc1w.shape[0], device=x0.device, dtype=BF16)
            a = K.gemm(h2, bf16_weight(fc1w), bias=fc1b, epi=K.EPI_SILU, aux=a_pre)
            y2 = torch.empty(M, d, device=x0.device, dtype=BF16)
            outs.append(K.gemm(a, bf16_weight(fc2w), bias=fc2b, epi=K.EPI_GATE_RESID, aux=y2, gate=g2, tpf=ns[s],
                               resid=x1s))
            saved += [xs[s], ms[s], h1[s], r1[s], y1, x1s, h2, r2, a_pre, a, y2]
        ctx.save_for_backward(qkvj, qkr, rq, o, lse, *saved, *w)
        ctx.geo, ctx.dims = geo, (B, T0, x1.shape[1], d, T, nf)
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
        douts = (dout0.reshape(-1, d).to(BF16).contiguous(), dout1.reshape(-1, d).to(BF16).contiguous())
        os_ = K.frame_split(o.view(B * T, d), n0, n1)
        dos, dx1s, dmods = [], [], [[None] * 4, [None] * 4]
        for s in range(2):
            xs, ms, h1, r1, y1, x1s, h2, r2, a_pre, a, y2 = st[s]
            fc1w, fc2w, wout = w[8 + 4 * s], w[10 + 4 * s], w[4 + 2 * s]
            # ---- MLP
            dy2, dg2, dbf2 = K.gate_bwd(douts[s], y2, ms[:, 5 * d:], ns[s])
            dW[11 + 4 * s] = dbf2.sum(0)
            dW[9 + 4 * s] = torch.zeros(a_pre.shape[1], device=a_pre.device, dtype=torch.float32)
            dapre = K.gemm(dy2, bf16_weight(fc2w), b_trans=True, epi=K.EPI_DSILU, aux=a_pre, colsum=dW[9 + 4 * s])
            dW[10 + 4 * s] = K.gemm_wgrad(dy2, a)
            dW[8 + 4 * s] = K.gemm_wgrad(dapre, h2)
            dh2 = K.gemm(dapre, bf16_weight(fc1w), b_trans=True)
            del dapre, dy2
            dx1, dmod2 = K.adaln_bwd(dh2, x1s, r2, ms[:, 3 * d:4 * d], ns[s], dres=douts[s])
            # ---- attention output projection
            dy1, dg1, dbf1 = K.gate_bwd(dx1, y1, ms[:, 2 * d:3 * d], ns[s])
            dW[5 + 2 * s] = dbf1.sum(0)
            dos.append(K.gemm(dy1, bf16_weight(wout), b_trans=True))
            dW[4 + 2 * s] = K.gemm_wgrad(dy1, os_[s])
            dx1s.append(dx1)
            dmods[s][1], dmods[s][2], dmods[s][3] = dg1, dmod2, dg2
        del os_
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
        dqkv = K.frame_split(dqkvj, n0, n1)
        del dqkvj
        dxs, dcs = [], []
        for s in range(2):
            xs, ms, h1, r1 = st[s][:4]
            wq = w[2 * s]
            dW[1 + 2 * s] = K.colsum(dqkv[s])
            dW[2 * s] = K.gemm_wgrad(dqkv[s], h1)
            dh1 = K.gemm(dqkv[s], bf16_weight(wq), b_trans=True)
            dx, dmod1 = K.adaln_bwd(dh1, xs, r1, ms[:, :d], ns[s], dres=dx1s[s])
            dxs.append(dx)
            _, dg1, dmod2, dg2 = dmods[s]
            dcs.append(torch.cat([dmod1, dg1, dmod2, dg2], dim=1).view(B, nf // B, 6 * d))
        return (dxs[0].view(B, T0, d), dxs[1].view(B, T1, d), dcs[0], dcs[1], None, *dW)


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
        c = linear(F.silu(cond), lin.weight, lin.bias)
        cond0, cond1 = c.chunk(2, dim=-1)
        for i, block in enumerate(self.blocks):
            x0, x1 = block(x0, x1, cond0, cond1, local_mask if self.local_layers[i] else global_mask, kv_cache)
        return x0, x1
