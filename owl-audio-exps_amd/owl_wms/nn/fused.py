"""autograd Functions over libowlk: the training hot path of owl_wms on MI355X.

* ``linear``      nn.Linear under bf16 autocast (fp32 params, bf16 activations) -- every
                  Linear outside the block loop (embeddings, proj_in/out, modulation fcs).
* ``adaln``       AdaLN / cond_adaln modulate with optional fused SiLU (FinalLayer).
* ``DiTBlockFn``  one whole DiTBlock (attn.py:116-143) forward + backward:
                    h1 = AdaLN1(x)                      adaln_fwd
                    qkv = h1 Wqkv^T + b                 GEMM
                    q, k = rope(rms(q)), rope(rms(k))   qk_rope_fwd
                    o = attn(q, k, v)                   attn_fwd (frame mask, no mask tensor)
                    x1 = x + g1 * (o Wout^T + b)        GEMM + gate/residual epilogue
                    h2 = AdaLN2(x1)                     adaln_fwd
                    a = silu(h2 W1^T + b1)              GEMM + SiLU epilogue
                    x2 = x1 + g2 * (a W2^T + b2)        GEMM + gate/residual epilogue
                  and the mirrored backward (dX GEMMs with fused SiLU', dW GEMMs straight into
                  fp32, deterministic flash-attention backward).

Parameters stay fp32 (the reference trains fp32 master weights under autocast); their bf16
copies are cached on the parameter and refreshed only when its version counter moves (i.e.
after an optimizer step -- the fused optimizer passes bump it, kernels._written), not once per
micro-step.

Weight and bias gradients go straight into the parameter's gradient buffer when that buffer is a
GradReducer bucket view (zeroed once per optimizer step): the dW GEMMs run with beta = 1 onto it
and the bias column sums add onto it, the backward returns None for the parameter, and the
reducer is told the gradient is complete.  That replaces autograd's separate fp32
``p.grad += g`` pass per parameter per micro-step.  It needs each parameter used once per
forward, which holds for every module on this path.
"""
import os
import weakref

import torch
import torch.nn.functional as F

from .. import kernels as K

BF16 = torch.bfloat16


def bf16_weight(p, pad_k=0):
    """Cached bf16 (optionally K-padded) copy of an fp32 parameter."""
    ent = getattr(p, "_owl_bf16", None)
    ver = p._version
    if ent is None or ent[0] != ver or ent[1] != pad_k or ent[2].device != p.device:
        w = p.detach().to(BF16)
        if pad_k:
            w = F.pad(w, (0, pad_k))
        w = w.contiguous()
        p._owl_bf16 = (ver, pad_k, w)
        return w
    return ent[2]


def grad_sink(p):
    """p's GradReducer bucket view when the backward may accumulate into it directly, else None."""
    if p is None or not p.requires_grad:
        return None
    v = getattr(p, "_owl_grad_view", None)
    g = p.grad
    if v is None or g is None or g.data_ptr() != v.data_ptr():
        return None
    return v


def grad_done(p):
    """the direct write into p's bucket view is enqueued: tell the reducer (bucket readiness)."""
    r = getattr(p, "_owl_reducer", None)
    if r is not None:
        r.grad_ready(p)


def wgrad_into(p, dy, x):
    """weight gradient dW = dy^T x: accumulated into p's bucket view (returns None) or returned."""
    sink = grad_sink(p)
    if sink is None:
        return K.gemm_wgrad(dy, x)
    K.gemm(dy, x, a_trans=True, b_trans=True, out=sink, out_f32=True, beta=1.0)
    grad_done(p)
    return None


def bgrad_into(p, dy):
    """bias gradient sum_rows dy (bf16 or fp32 rows), accumulated into p's bucket view or returned."""
    sink = grad_sink(p)
    if sink is None:
        return K.colsum(dy)
    K.colsum(dy, out=sink)
    grad_done(p)
    return None


def _pad_k(K_):
    return (-K_) % 8


class LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        shp = x.shape
        Kd = shp[-1]
        pad = _pad_k(Kd)
        x2 = x.reshape(-1, Kd).to(BF16)
        if pad:
            x2 = F.pad(x2, (0, pad))
        x2 = x2.contiguous()
        wb = bf16_weight(w, pad)
        y = K.gemm(x2, wb, bias=b)
        ctx.save_for_backward(x2, w)
        ctx.pad, ctx.shp, ctx.has_b, ctx.xdtype = pad, shp, b is not None, x.dtype
        ctx.bias = b
        return y.view(*shp[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        N = w.shape[0]
        dy2 = dy.reshape(-1, N).to(BF16).contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            wb = bf16_weight(w, ctx.pad)
            dx = K.gemm(dy2, wb, b_trans=True)
            if ctx.pad:
                dx = dx[:, : ctx.shp[-1]]
            dx = dx.reshape(ctx.shp).to(ctx.xdtype)
        if ctx.needs_input_grad[1]:
            if ctx.pad:
                dw = K.gemm_wgrad(dy2, x2)[:, : ctx.shp[-1]].contiguous()
            else:
                dw = wgrad_into(w, dy2, x2)
        if ctx.has_b and ctx.needs_input_grad[2]:
            db = bgrad_into(ctx.bias, dy2)
        return dx, dw, db


def linear(x, w, b=None):
    """bf16-autocast nn.Linear on libowlk (x: [..., K] any float dtype -> [..., N] bf16)."""
    return LinearFn.apply(x, w, b)


class AdaLNFn(torch.autograd.Function):
    """y = bf16(rms(x)) * (1 + scale[frame]) + shift[frame]  (optionally -> silu(y))."""

    @staticmethod
    def forward(ctx, x, scale, shift, tpf, act):
        shp = x.shape
        d = shp[-1]
        x2 = x.reshape(-1, d).to(BF16).contiguous()
        sc2, sh2 = scale.reshape(-1, d), shift.reshape(-1, d)
        if sc2.stride(1) != 1 or sh2.stride(1) != 1 or sc2.stride(0) != sh2.stride(0):
            sc2, sh2 = sc2.contiguous(), sh2.contiguous()
        if act:
            y, rstd, ya = K.adaln_fwd(x2, sc2, sh2, tpf, act=True)
        else:
            (y, rstd), ya = K.adaln_fwd(x2, sc2, sh2, tpf), None
        ctx.save_for_backward(x2, rstd, sc2, y if act else None)
        ctx.tpf, ctx.shp, ctx.act, ctx.mshape = tpf, shp, act, scale.shape
        return (ya if act else y).view(shp)

    @staticmethod
    def backward(ctx, dy):
        x2, rstd, sc2, ypre = ctx.saved_tensors
        d = x2.shape[1]
        dy2 = dy.reshape(-1, d).to(BF16).contiguous()
        dx, dmod = K.adaln_bwd(dy2, x2, rstd, sc2, ctx.tpf, ypre=ypre if ctx.act else None)
        return dx.view(ctx.shp), dmod[:, :d].reshape(ctx.mshape), dmod[:, d:].reshape(ctx.mshape), None, None


def adaln(x, scale, shift, tpf, act=False):
    return AdaLNFn.apply(x, scale, shift, tpf, act)


class CondGrad:
    """The gradient of s = silu(cond), summed over every consumer of s in fp32.

    s feeds one GEMM per DiT block (the stacked modulation fc's) and the final layer's AdaLN fc.
    Under autograd each would hand back a bf16 [F, d] gradient and the engine would add them one
    by one (bf16 adds).  Instead each consumer's backward runs its dX GEMM with beta = 1 onto this
    accumulator and returns None for s; the producer of s (CondSiluFn / cond.CondFn) reads the sum
    in its own backward, which autograd runs after every consumer's.  Consumers find the
    accumulator on s (attribute ``_owl_cond_grad``, set by the producer's wrapper)."""

    __slots__ = ("ds",)

    def __init__(self):
        self.ds = None

    def take(self, g, shape):
        """the accumulated fp32 sum (+ g, a gradient some consumer returned through autograd) as
        [F, d] fp32, or None; the accumulator is emptied."""
        ds, self.ds = self.ds, None
        if g is not None:  # a consumer outside the fused path (reference-API callers)
            g = g.reshape(-1, shape[-1]).float()
            ds = g if ds is None else ds + g
        return ds


def cond_grad_of(s):
    return getattr(s, "_owl_cond_grad", None)


def cond_grad_add(cg, dm, w, shape):
    """consumer side of CondGrad: ds = dm w (dm [F, N] bf16 rows, any stride; w [N, d] bf16).  Added
    onto the accumulator (returns None) or, with none, returned as the bf16 gradient of s."""
    if cg is None:
        return K.gemm(dm, w, b_trans=True).view(shape)
    if cg.ds is None:
        cg.ds = K.gemm(dm, w, b_trans=True, out_f32=True)
    else:
        K.gemm(dm, w, b_trans=True, out=cg.ds, out_f32=True, beta=1.0)
    return None


class CondSiluFn(torch.autograd.Function):
    """s = silu(cond) (bf16, owlk_cond_silu_fwd) for callers that hold cond itself (DiT / FinalLayer /
    AdaLN called with the reference signature); its consumers accumulate into a CondGrad."""

    @staticmethod
    def forward(ctx, cond, cg):
        ctx.set_materialize_grads(False)
        shp = cond.shape
        c2 = cond.reshape(-1, shp[-1]).to(BF16).contiguous()
        _, s = K.cond_silu_fwd(c2)
        ctx.save_for_backward(c2)
        ctx.cg, ctx.shp, ctx.cdtype = cg, shp, cond.dtype
        return s.view(shp)

    @staticmethod
    def backward(ctx, g):
        (c2,) = ctx.saved_tensors
        ds = ctx.cg.take(g, ctx.shp)
        if ds is None:
            return None, None
        dc, _ = K.cond_silu_bwd(ds.contiguous(), c2)
        return dc.view(ctx.shp).to(ctx.cdtype), None


def cond_silu(cond):
    """silu(cond) as bf16 carrying a CondGrad (see CondGrad); a tensor that already is such an s
    (``_owl_cond_grad`` set) is returned as is."""
    if cond_grad_of(cond) is not None:
        return cond
    if not (torch.is_grad_enabled() and cond.requires_grad):
        return K.cond_silu_fwd(cond.reshape(-1, cond.shape[-1]).to(BF16).contiguous(),
                               keep_cond=False)[1].view(cond.shape)
    cg = CondGrad()
    s = CondSiluFn.apply(cond, cg)
    s._owl_cond_grad = cg
    return s


class AdaLNModFn(torch.autograd.Function):
    """AdaLN with its modulation Linear (modulation.py:7-25; FinalLayer attn.py:264-277):
    [scale | shift] = s W^T + b (one GEMM on s = silu(cond)), y = AdaLN(x) (optionally -> silu(y)).
    Backward: d[scale | shift] lands bf16 in one [F, 2d] matrix (owlk_adaln_bwd, mod_bf16), whose
    dX GEMM goes onto the CondGrad of s and whose dW / db go into the parameters' bucket views."""

    @staticmethod
    def forward(ctx, x, s, w, b, tpf, act):
        shp = x.shape
        d = shp[-1]
        s2 = s.reshape(-1, d).to(BF16).contiguous()
        wb = bf16_weight(w)
        ab = K.gemm(s2, wb, bias=b)
        x2 = x.reshape(-1, d).to(BF16).contiguous()
        if act:
            y, rstd, ya = K.adaln_fwd(x2, ab[:, :d], ab[:, d:], tpf, act=True)
        else:
            (y, rstd), ya = K.adaln_fwd(x2, ab[:, :d], ab[:, d:], tpf), None
        ctx.save_for_backward(x2, rstd, ab, y if act else None, s2, w)
        ctx.tpf, ctx.shp, ctx.act, ctx.sshape, ctx.b = tpf, shp, act, s.shape, b
        ctx.cg = cond_grad_of(s)
        return (ya if act else y).view(shp)

    @staticmethod
    def backward(ctx, dy):
        x2, rstd, ab, ypre, s2, w = ctx.saved_tensors
        d = x2.shape[1]
        dy2 = dy.reshape(-1, d).to(BF16).contiguous()
        dab = torch.empty_like(ab)
        dx = K.adaln_bwd_into(dy2, x2, rstd, ab[:, :d], ctx.tpf, dab, ypre=ypre if ctx.act else None)
        ds = dw = db = None
        if ctx.needs_input_grad[1]:
            ds = cond_grad_add(ctx.cg, dab, bf16_weight(w), ctx.sshape)
        if ctx.needs_input_grad[2]:
            dw = wgrad_into(w, dab, s2)
        if ctx.b is not None and ctx.needs_input_grad[3]:
            db = bgrad_into(ctx.b, dab)
        return dx.view(ctx.shp), ds, dw, db, None, None


def adaln_mod(x, s, w, b, tpf, act=False):
    """AdaLN(x) with [scale | shift] = s W^T + b; s = cond_silu(cond)."""
    return AdaLNModFn.apply(x, s, w, b, tpf, act)


class BlockGeometry:
    """Static per-forward data of a DiT block: heads, frame mask, RoPE tables; keep_attn = a key
    per block when the block runs under activation checkpointing (see _ATTN_KEEP)."""

    def __init__(self, n_heads, head_dim, tpf, mask, cos, sin, tab_off=0, keep_attn=None, lean=False):
        self.H, self.D, self.tpf, self.mask = n_heads, head_dim, tpf, mask
        self.cos, self.sin, self.tab_off = cos, sin, tab_off
        self.keep_attn = keep_attn
        self.lean = lean


# A checkpointed block (dit_v4_5B: gradient_checkpointing, attn.py:186) runs its forward again
# inside the backward.  Its attention output and lse are kept from the first pass (one entry per
# block, replaced by the block's next first pass) and handed to that re-run when it sees the very
# same input tensor, unmodified, and the same qkv weight version: the deterministic kernels would
# recompute them bit for bit.  The re-run skips the attention forward (≈ 9 % of a 5B micro-step)
# for ≈ 0.5 GB per block of HBM.
_ATTN_KEEP = {}


def _kept_attention(geo, x, wqkv):
    hit = _ATTN_KEEP.pop(geo.keep_attn, None) if geo.keep_attn is not None else None
    if hit is not None and hit[0]() is x and hit[1] == x._version and hit[2] is wqkv and hit[3] == wqkv._version:
        return hit[4], hit[5]
    return None


def _keep_attention(geo, x, wqkv, o, lse):
    if geo.keep_attn is not None:
        _ATTN_KEEP[geo.keep_attn] = (weakref.ref(x), x._version, wqkv, wqkv._version, o, lse)


class DiTBlockFn(torch.autograd.Function):
    """One DiTBlock with its modulation: mods = s Wmod^T + bmod ([F, 6d], s = silu(cond), the four
    modulation fc's stacked, see stacked_modulation_weights) as the block's first GEMM; the
    backward writes d mods bf16 straight into one [F, 6d] matrix (adaln / gate backward kernels),
    runs its dX GEMM onto the CondGrad of s and the four dW / db into the bucket views."""

    @staticmethod
    def forward(ctx, x, s, wmod, bmod, geo, wqkv, bqkv, wout, bout, w1, b1, w2, b2, *mparams):
        B, T, d = x.shape
        M = B * T
        H, D, tpf = geo.H, geo.D, geo.tpf
        xx = x.reshape(M, d)
        s2 = s.reshape(-1, d).to(BF16).contiguous()
        mods = K.gemm(s2, wmod, bias=bmod)
        a1, gg1, a2, gg2 = mods[:, :2 * d], mods[:, 2 * d:3 * d], mods[:, 3 * d:5 * d], mods[:, 5 * d:]

        h1, r1 = K.adaln_fwd(xx, a1[:, :d], a1[:, d:], tpf)
        # qkv and its QK-RMSNorm + RoPE rows in one launch (the GEMM epilogue)
        qkv, qkr, rq = K.gemm_qk_rope(h1, bf16_weight(wqkv), bqkv, H, D, geo.cos, geo.sin, geo.tab_off, T)
        q3, k3 = qkr.view(B, T, 2 * d)[:, :, :d], qkr.view(B, T, 2 * d)[:, :, d:]
        kept = _kept_attention(geo, x, wqkv)
        if kept is not None:
            o, lse = kept
        else:
            o, lse = K.attn_fwd(q3, k3, qkv.view(B, T, 3 * d)[:, :, 2 * d:], H, D, geo.mask,
                                score_bound=K.qk_norm_bound(D))
            _keep_attention(geo, x, wqkv, o, lse)
        o = o.view(M, d)
        y1 = torch.empty(M, d, device=x.device, dtype=BF16)
        x1 = K.gemm(o, bf16_weight(wout), bias=bout, epi=K.EPI_GATE_RESID, aux=y1, gate=gg1, tpf=tpf, resid=xx)
        h2, r2 = K.adaln_fwd(x1, a2[:, :d], a2[:, d:], tpf)
        a_pre = torch.empty(M, w1.shape[0], device=x.device, dtype=BF16)
        a = K.gemm(h2, bf16_weight(w1), bias=b1, epi=K.EPI_SILU, aux=a_pre)
        y2 = torch.empty(M, d, device=x.device, dtype=BF16)
        out = K.gemm(a, bf16_weight(w2), bias=b2, epi=K.EPI_GATE_RESID, aux=y2, gate=gg2, tpf=tpf, resid=x1)

        if geo.lean:
            # lean activations (memory-bound configs, e.g. dit_v4_5B with fewer checkpointed blocks):
            # h1, h2 (adaln of kept inputs), the roped q / k, a = silu(a_pre) and x1 = x + g1 y1 are
            # recomputed in the backward, bit for bit, from tensors kept anyway: 9 of 20 [T, d]
            # bf16 units per block
            h1 = qkr = h2 = a = x1 = None
        ctx.save_for_backward(xx, s2, wmod, mods, wqkv, wout, w1, w2, h1, r1, qkv, qkr, rq, o, lse, y1, x1, h2,
                              r2, a_pre, a, y2)
        ctx.geo, ctx.shape, ctx.sshape = geo, (B, T, d), s.shape
        ctx.params = (wqkv, bqkv, wout, bout, w1, b1, w2, b2) + tuple(mparams)
        ctx.cg = cond_grad_of(s)
        return out.view(B, T, d)

    @staticmethod
    def backward(ctx, dout):
        (xx, s2, wmod, mods, wqkv, wout, w1, w2, h1, r1, qkv, qkr, rq, o, lse, y1, x1, h2, r2, a_pre, a,
         y2) = ctx.saved_tensors
        geo = ctx.geo
        B, T, d = ctx.shape
        M = B * T
        H, D, tpf = geo.H, geo.D, geo.tpf
        a1, gg1, a2, gg2 = mods[:, :2 * d], mods[:, 2 * d:3 * d], mods[:, 3 * d:5 * d], mods[:, 5 * d:]
        dx2 = dout.reshape(M, d).to(BF16).contiguous()
        dm = torch.empty_like(mods)  # d mods, bf16 as the modulation Linears' output gradient
        if x1 is None:  # lean
            x1 = K.gate_resid(xx, y1, gg1, tpf)

        prm = ctx.params  # (wqkv, bqkv, wout, bout, w1, b1, w2, b2, 4 x (w, b) mod) Parameters: gradient sinks

        # ---- MLP branch
        dy2, _, dbf2 = K.gate_bwd(dx2, y2, gg2, tpf, dg_out=dm[:, 5 * d:])
        db2 = bgrad_into(prm[7], dbf2)  # per-frame partials [F, d] -> bias gradient
        sink_b1 = grad_sink(prm[5])
        db1 = sink_b1 if sink_b1 is not None else torch.zeros(a_pre.shape[1], device=a_pre.device,
                                                              dtype=torch.float32)
        if a is None:  # lean: the dSiLU epilogue also emits a = silu(a_pre)
            a = torch.empty_like(a_pre)
            dapre = K.gemm(dy2, bf16_weight(w2), b_trans=True, epi=K.EPI_DSILU, aux=a_pre, colsum=db1, resid=a)
        else:
            dapre = K.gemm(dy2, bf16_weight(w2), b_trans=True, epi=K.EPI_DSILU, aux=a_pre, colsum=db1)  # + colsum
        if sink_b1 is not None:
            grad_done(prm[5])
            db1 = None
        dw2 = wgrad_into(prm[6], dy2, a)
        del a
        if h2 is None:
            h2, _ = K.adaln_fwd(x1, a2[:, :d], a2[:, d:], tpf)
        dw1 = wgrad_into(prm[4], dapre, h2)
        del h2
        dh2 = K.gemm(dapre, bf16_weight(w1), b_trans=True)
        del dapre
        if K.ADALN_GATE:  # the attention branch's gate backward fused onto the dx rows (bit for bit)
            dx1, dy1, dbf1 = K.adaln_gate_bwd_into(dh2, x1, r2, a2[:, :d], tpf, dm[:, 3 * d:5 * d], dx2, y1, gg1,
                                                   dm[:, 2 * d:3 * d])
        else:
            dx1 = K.adaln_bwd_into(dh2, x1, r2, a2[:, :d], tpf, dm[:, 3 * d:5 * d], dres=dx2)
            dy1, _, dbf1 = K.gate_bwd(dx1, y1, gg1, tpf, dg_out=dm[:, 2 * d:3 * d])
        del dh2, x1

        # ---- attention branch
        dbout = bgrad_into(prm[3], dbf1)
        # dO and the attention backward's delta = rowsum(dO * O) in one launch (the GEMM epilogue)
        do, delta = K.gemm_attn_delta(dy1, bf16_weight(wout), o, H, D, T)
        dwout = wgrad_into(prm[2], dy1, o)
        del dy1
        if qkr is None:
            qkr, _ = K.qk_rope_fwd(qkv, H, D, geo.cos, geo.sin, geo.tab_off, T)
        dqkv = torch.empty(M, 3 * d, device=xx.device, dtype=BF16)
        dqkr = torch.empty(M, 2 * d, device=xx.device, dtype=BF16)
        q3, k3 = qkr.view(B, T, 2 * d)[:, :, :d], qkr.view(B, T, 2 * d)[:, :, d:]
        dq3, dk3 = dqkr.view(B, T, 2 * d)[:, :, :d], dqkr.view(B, T, 2 * d)[:, :, d:]
        K.attn_bwd(q3, k3, qkv.view(B, T, 3 * d)[:, :, 2 * d:], o.view(B, T, d), do.view(B, T, d), lse, H, D,
                   geo.mask, dq3, dk3, dqkv.view(B, T, 3 * d)[:, :, 2 * d:], delta=delta)
        del do, delta
        # qkv bias gradient: the q / k columns' sums fused into the rope backward, the v columns' by colsum
        sink_bqkv = grad_sink(prm[1])
        dbqkv = sink_bqkv if sink_bqkv is not None else torch.zeros(3 * d, device=xx.device, dtype=torch.float32)
        K.qk_rope_bwd(dqkr, qkv, rq, H, D, geo.cos, geo.sin, dqkv, geo.tab_off, T, dbias=dbqkv[:2 * d])
        del dqkr
        K.colsum(dqkv[:, 2 * d:], out=dbqkv[2 * d:])
        if sink_bqkv is not None:
            grad_done(prm[1])
            dbqkv = None
        del qkr, q3, k3
        if h1 is None:
            h1, _ = K.adaln_fwd(xx, a1[:, :d], a1[:, d:], tpf)
        dwqkv = wgrad_into(prm[0], dqkv, h1)
        del h1
        dh1 = K.gemm(dqkv, bf16_weight(wqkv), b_trans=True)
        del dqkv
        dx = K.adaln_bwd_into(dh1, xx, r1, a1[:, :d], tpf, dm[:, :2 * d], dres=dx1)
        del dh1

        # ---- modulation: one dX GEMM against the stack onto the CondGrad of s; dW / db per fc
        ds = cond_grad_add(ctx.cg, dm, wmod, ctx.sshape) if ctx.needs_input_grad[1] else None
        mgrads = []
        stacked = _stacked_mod_sink([prm[8 + 2 * i] for i in range(4)], d) \
            if all(ctx.needs_input_grad[13 + 2 * i] for i in range(4)) else None
        if stacked is not None:  # the four weights' gradient views are one [6d, d] stack: ONE GEMM
            K.gemm(dm, s2, a_trans=True, b_trans=True, out=stacked, out_f32=True, beta=1.0)
        for i, (lo, hi) in enumerate(_MOD_COLS(d)):
            w, bias = prm[8 + 2 * i], prm[9 + 2 * i]
            dmi = dm[:, lo:hi]
            if stacked is not None:
                grad_done(w)
                mgrads.append(None)
            else:
                mgrads.append(wgrad_into(w, dmi, s2) if ctx.needs_input_grad[13 + 2 * i] else None)
            mgrads.append(bgrad_into(bias, dmi) if ctx.needs_input_grad[14 + 2 * i] else None)
        return (dx.view(B, T, d), ds, None, None, None,
                dwqkv, dbqkv, dwout, dbout, dw1, db1, dw2, db2, *mgrads)


_MOD_STACK_GEMM = os.environ.get("OWL_MOD_STACK_GEMM", "1") != "0"  # 0: four weight-gradient GEMMs (A/B)


def _stacked_mod_sink(ws, d):
    """[6d, d] fp32 view over the four modulation weights' bucket views when GradReducer laid them
    out back to back in column order (DiTBlock tags them, utils/grad_reducer.py), else None."""
    if not _MOD_STACK_GEMM:
        return None
    sinks = [grad_sink(w) for w in ws]
    if any(v is None or not v.is_contiguous() for v in sinks):
        return None
    off = 0
    for v, (lo, hi) in zip(sinks, _MOD_COLS(d)):
        if v.shape != (hi - lo, d) or v.data_ptr() != sinks[0].data_ptr() + off * 4:
            return None
        off += v.numel()
    return torch.as_strided(sinks[0], (6 * d, d), (d, 1))


def _MOD_COLS(d):
    """column ranges of the stacked modulation output: adaln1 [2d] | gate1 [d] | adaln2 [2d] | gate2 [d]"""
    return ((0, 2 * d), (2 * d, 3 * d), (3 * d, 5 * d), (5 * d, 6 * d))


class ModFn(torch.autograd.Function):
    """DiTBlock.modulation: the fc's of adaln1, gate1, adaln2 and gate2 (modulation.py:13-40) all read
    the same silu(cond), so they run as ONE GEMM against the four weights stacked [6d, d] (bf16,
    with the biases stacked fp32).  The outputs are column views [2d | d | 2d | d] of that one
    result.  Backward: the four output gradients (bf16-rounded, as the Linears' own backward would)
    go into one [F, 6d] matrix; ONE dX GEMM against the stack replaces four GEMMs and autograd's
    three adds; the weight / bias gradients go into each parameter's bucket view as before."""

    @staticmethod
    def forward(ctx, s, wstack, bstack, *params):
        b, n, d = s.shape
        x2 = s.reshape(-1, d).to(BF16).contiguous()
        y = K.gemm(x2, wstack, bias=bstack).view(b, n, 6 * d)
        ctx.save_for_backward(x2, wstack)
        ctx.params, ctx.shp = params, (b, n, d)
        return y[..., :2 * d], y[..., 2 * d:3 * d], y[..., 3 * d:5 * d], y[..., 5 * d:]

    @staticmethod
    def backward(ctx, *gouts):
        x2, wstack = ctx.saved_tensors
        b, n, d = ctx.shp
        F_ = b * n
        cols = ((0, 2 * d), (2 * d, 3 * d), (3 * d, 5 * d), (5 * d, 6 * d))
        dm = torch.empty(F_, 6 * d, device=x2.device, dtype=BF16)
        for g, (lo, hi) in zip(gouts, cols):
            if g is None:
                dm[:, lo:hi].zero_()
            else:
                dm[:, lo:hi].copy_(g.reshape(F_, hi - lo))
        ds = None
        if ctx.needs_input_grad[0]:
            # K = 6d is long against a [F, d] output (36 256^2 tiles): the fp32 form takes the split-K
            # plan (partials + ordered reduce), ~4x faster than one pass of small tiles
            ds = K.gemm(dm, wstack, b_trans=True, out_f32=True).to(BF16).view(b, n, d)
        grads = []
        for i, (lo, hi) in enumerate(cols):
            w, bias = ctx.params[2 * i], ctx.params[2 * i + 1]
            dmi = dm[:, lo:hi]
            grads.append(wgrad_into(w, dmi, x2) if w.requires_grad else None)
            grads.append(bgrad_into(bias, dmi) if bias is not None and bias.requires_grad else None)
        return (ds, None, None, *grads)


def stacked_modulation_weights(owner, params):
    """bf16 [6d, d] stack of the four modulation weights and fp32 [6d] stack of their biases, cached
    on `owner` and rebuilt when a parameter's version (an optimizer step) or identity changes."""
    key = tuple((id(p), p._version, p.device) for p in params)
    ent = getattr(owner, "_owl_mod_stack", None)
    if ent is None or ent[0] != key:
        W = torch.cat([params[2 * i].detach().to(BF16) for i in range(4)]).contiguous()
        bvec = torch.cat([params[2 * i + 1].detach().float() for i in range(4)]).contiguous()
        ent = (key, W, bvec)
        object.__setattr__(owner, "_owl_mod_stack", ent)
    return ent[1], ent[2]


class LayerNormFn(torch.autograd.Function):
    """F.layer_norm(x, (d,)).type_as(x) (normalization.py:6-7): fp32 math, bf16 out, libowlk."""

    @staticmethod
    def forward(ctx, x):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1]).to(BF16).contiguous()
        y, mean, rstd = K.layernorm_fwd(x2)
        ctx.save_for_backward(x2, mean, rstd)
        ctx.shp, ctx.xdtype = shp, x.dtype
        return y.view(shp)

    @staticmethod
    def backward(ctx, dy):
        x2, mean, rstd = ctx.saved_tensors
        dx = K.layernorm_bwd(dy.reshape(x2.shape).to(BF16).contiguous(), x2, mean, rstd)
        return dx.view(ctx.shp).to(ctx.xdtype)


def layer_norm(x):
    return LayerNormFn.apply(x)


class FlowLossFn(torch.autograd.Function):
    """F.mse_loss(pred_tok, tgt_tok): the loss from one kernel pass (+ a fixed-order finish), the
    gradient in the backward from pred and tgt, scaled by the incoming loss gradient on the device
    (no host sync, no separate multiply)."""

    @staticmethod
    def forward(ctx, pred, tgt):
        pred, tgt = pred.contiguous(), tgt.contiguous()
        loss, _ = K.mse(pred, tgt, want_grad=False)
        ctx.save_for_backward(pred, tgt)
        return loss

    @staticmethod
    def backward(ctx, g):
        pred, tgt = ctx.saved_tensors
        return K.mse_grad(pred, tgt, g), None
