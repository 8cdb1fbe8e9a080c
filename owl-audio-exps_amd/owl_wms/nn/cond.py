"""Per-frame conditioning as ONE autograd Function on libowlk (reference: GameRFTCore.cond
gamerft.py:39-48, the embeddings embeddings.py:30-184, and the silu(cond) that every modulation
Linear applies first, modulation.py:13,32).

Forward (a handful of launches per micro-step, no ATen arithmetic):
    owlk_cond_embed     timestep sin/cos, mouse symlog -> polar (angle_proj + magnitude sin/cos),
                        button 2b - 1                                     one launch, R frame rows
    3 x MLP             fc1 GEMM with the SiLU epilogue, fc2 GEMM         (t, mouse, button)
    owlk_cond_silu_fwd  cond = t + (has_controls ? mouse + button : 0), s = silu(cond)
and hands out s (``want="s"``: the DiT path -- every consumer reads silu(cond)) or cond
(``want="cond"``: the MMDiT head, which also layer-norms cond).

Backward: the consumers of s sum their dX GEMMs into the fp32 accumulator carried by s
(fused.CondGrad) and return None; here owlk_cond_silu_bwd turns that sum into dcond (the
timestep MLP's output gradient) and dctrl = has_controls ? dcond : 0 (the mouse and button MLPs'),
and the MLP backwards write every weight / bias gradient into the GradReducer bucket views
(the K = 2 / 11 input layers, angle_proj and button fc1, by owlk_small_k_wgrad).
"""
import torch

from .. import kernels as K
from .fused import BF16, CondGrad, bf16_weight, bgrad_into, grad_done, grad_sink, wgrad_into

F32 = torch.float32


def _pad8(k):
    return (-k) % 8


def _mlp_fwd(x, mlp, pad=0):
    """MLPCustom (mlp.py:6-24) on libowlk: -> (y, a_pre, a)."""
    w1 = bf16_weight(mlp.fc1.weight, pad)
    a_pre = torch.empty(x.shape[0], w1.shape[0], device=x.device, dtype=BF16)
    a = K.gemm(x, w1, bias=mlp.fc1.bias, epi=K.EPI_SILU, aux=a_pre)
    return K.gemm(a, bf16_weight(mlp.fc2.weight), bias=mlp.fc2.bias), a_pre, a


def _wgrad_small_into(p, dy, x, k):
    """weight gradient of an input layer whose width k is not a multiple of 8 (x: its bf16 input rows,
    zero-padded to a multiple of 8): owlk_small_k_wgrad for k <= 16 (angle_proj, button fc1), else
    the padded input's split-K weight gradient cut to its first k columns."""
    sink = grad_sink(p)
    if k > 16:
        full = K.gemm_wgrad(dy, x)
        if sink is None:
            return full[:, :k].contiguous()
        sink += full[:, :k]
        grad_done(p)
        return None
    if sink is None:
        return K.small_k_wgrad(dy, x, k)
    K.small_k_wgrad(dy, x, k, out=sink, beta=1.0)
    grad_done(p)
    return None


def _mlp_bwd(dy, x, a_pre, a, mlp, need, pad=0, want_dx=False):
    """MLPCustom backward: dy [R, out] bf16 -> (dx or None, [dW1, db1, dW2, db2]) -- each gradient
    written into its bucket view (None returned) or returned; need: the four params' requires-grad."""
    w1, b1, w2, b2 = mlp.fc1.weight, mlp.fc1.bias, mlp.fc2.weight, mlp.fc2.bias
    g = [None] * 4
    if need[3]:
        g[3] = bgrad_into(b2, dy)
    if need[2]:
        g[2] = wgrad_into(w2, dy, a)
    if not (need[0] or need[1] or want_dx):
        return None, g
    sink_b1 = grad_sink(b1) if need[1] else None
    db1 = sink_b1 if sink_b1 is not None else (
        torch.zeros(a_pre.shape[1], device=dy.device, dtype=F32) if need[1] else None)
    da = K.gemm(dy, bf16_weight(w2), b_trans=True, epi=K.EPI_DSILU, aux=a_pre, colsum=db1)
    if sink_b1 is not None:
        grad_done(b1)
    elif need[1]:
        g[1] = db1
    if need[0]:
        g[0] = _wgrad_small_into(w1, da, x, w1.shape[1]) if pad else wgrad_into(w1, da, x)
    dx = K.gemm(da, bf16_weight(w1, pad), b_trans=True) if want_dx else None
    return dx, g


class MLPFn(torch.autograd.Function):
    """MLPCustom.forward (mlp.py:20-24) as one Function: fc1 GEMM with the SiLU epilogue, fc2 GEMM;
    backward with the SiLU' epilogue and the fc1 bias sums fused into the dX GEMM."""

    @staticmethod
    def forward(ctx, x, mlp, *params):
        shp = x.shape
        k = shp[-1]
        pad = _pad8(k)
        x2 = x.reshape(-1, k).to(BF16)
        if pad:
            x2 = torch.nn.functional.pad(x2, (0, pad))
        x2 = x2.contiguous()
        y, a_pre, a = _mlp_fwd(x2, mlp, pad)
        ctx.save_for_backward(x2, a_pre, a)
        ctx.mlp, ctx.pad, ctx.shp, ctx.xdtype = mlp, pad, shp, x.dtype
        return y.view(*shp[:-1], y.shape[1])

    @staticmethod
    def backward(ctx, dy):
        x2, a_pre, a = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1]).to(BF16).contiguous()
        want_dx = ctx.needs_input_grad[0]
        dx, g = _mlp_bwd(dy2, x2, a_pre, a, ctx.mlp, ctx.needs_input_grad[2:6], pad=ctx.pad, want_dx=want_dx)
        if dx is not None:
            dx = dx[:, :ctx.shp[-1]].reshape(ctx.shp).to(ctx.xdtype)
        return (dx, None, *g)


def mlp_custom(x, mlp):
    return MLPFn.apply(x, mlp, mlp.fc1.weight, mlp.fc1.bias, mlp.fc2.weight, mlp.fc2.bias)


class CondMeta:
    """Static description of a core's conditioning modules (frequency tables cached per device)."""

    def __init__(self, core):
        self.t = core.t_embed
        self.uncond = bool(getattr(core, "uncond", True)) or not hasattr(core, "control_embed")
        self.ctrl = None if self.uncond else core.control_embed
        self._freqs = {}

    def freqs(self, device):
        key = str(device)
        if key not in self._freqs:
            tf = self.t.sincos._freqs(device, F32)
            mf = self.ctrl.mouse.magnitude_embed._freqs(device, F32) if self.ctrl is not None else None
            self._freqs[key] = (tf, mf)
        return self._freqs[key]

    def params(self):
        t = self.t.mlp
        ps = [t.fc1.weight, t.fc1.bias, t.fc2.weight, t.fc2.bias]
        if self.ctrl is not None:
            m, b = self.ctrl.mouse, self.ctrl.button.proj
            ps += [m.angle_proj.weight, m.mlp.fc1.weight, m.mlp.fc1.bias, m.mlp.fc2.weight, m.mlp.fc2.bias,
                   b.fc1.weight, b.fc1.bias, b.fc2.weight, b.fc2.bias]
        return ps


_NIN = 7  # CondFn.forward's leading non-parameter inputs


class CondFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ts, mouse, btn, hc, meta, cg, want, *params):
        ctx.set_materialize_grads(False)
        B, n = ts.shape[:2]
        R = B * n
        dev = ts.device
        tf, mf = meta.freqs(dev)
        t_cfg = meta.t.sincos
        ctrl = meta.ctrl
        if ctrl is not None:
            mo = ctrl.mouse
            nb = btn.shape[-1]
            nbp = nb + _pad8(nb)
            ts_in, mouse_in, ang, btn_in = K.cond_embed(
                R, ts.reshape(R).contiguous(), tf, t_cfg.mult, mouse.reshape(R, 2), mf, mo.magnitude_embed.mult,
                mo.angle_proj.weight.detach().contiguous(), btn.reshape(R, nb), nbp)
        else:
            ts_in = K.cond_embed(R, ts.reshape(R).contiguous(), tf, t_cfg.mult)[0]
            mouse_in = ang = btn_in = None
        t_out, t_pre, t_a = _mlp_fwd(ts_in, meta.t.mlp)
        saved = [ts_in, t_pre, t_a]
        if ctrl is not None:
            m_out, m_pre, m_a = _mlp_fwd(mouse_in, ctrl.mouse.mlp)
            b_out, b_pre, b_a = _mlp_fwd(btn_in, ctrl.button.proj, nbp - nb)
            saved += [mouse_in, ang, m_pre, m_a, btn_in, b_pre, b_a]
            hc_ = hc.contiguous() if hc is not None else None
            cond, s = K.cond_silu_fwd(t_out, m_out, b_out, hc_, n, keep_cond=True)
        else:
            hc_ = None
            cond, s = K.cond_silu_fwd(t_out, keep_cond=True)
        d = cond.shape[1]
        ctx.save_for_backward(cond, hc_, *saved)
        ctx.meta, ctx.cg, ctx.want, ctx.shp, ctx.n = meta, cg, want, (B, n, d), n
        ctx.pad = (nbp - nb) if ctrl is not None else 0
        return (s if want == "s" else cond).view(B, n, d)

    @staticmethod
    def backward(ctx, g):
        cond, hc, *saved = ctx.saved_tensors
        meta, n = ctx.meta, ctx.n
        need = ctx.needs_input_grad[_NIN:]
        grads = [None] * len(need)
        if ctx.want == "s":
            ds = ctx.cg.take(g, ctx.shp)
            if ds is None:
                return (None,) * (_NIN + len(need))
            dcond, dctrl = K.cond_silu_bwd(ds.contiguous(), cond, hc, n, want_ctrl=meta.ctrl is not None)
        else:
            if g is None:
                return (None,) * (_NIN + len(need))
            g2 = g.reshape(-1, ctx.shp[2]).to(BF16).contiguous()
            dcond, dctrl = K.cond_silu_bwd(g2, None, hc, n, want_ctrl=meta.ctrl is not None)
        ts_in, t_pre, t_a = saved[:3]
        _, grads[0:4] = _mlp_bwd(dcond, ts_in, t_pre, t_a, meta.t.mlp, need[0:4])
        if meta.ctrl is not None:
            mouse_in, ang, m_pre, m_a, btn_in, b_pre, b_a = saved[3:]
            mo = meta.ctrl.mouse
            dmi, grads[5:9] = _mlp_bwd(dctrl, mouse_in, m_pre, m_a, mo.mlp, need[5:9], want_dx=need[4])
            if need[4]:
                h = mo.angle_proj.weight.shape[0]
                grads[4] = _wgrad_small_into(mo.angle_proj.weight, dmi[:, :h], ang, 2)
            _, grads[9:13] = _mlp_bwd(dctrl, btn_in, b_pre, b_a, meta.ctrl.button.proj, need[9:13], pad=ctx.pad)
        return (None,) * _NIN + tuple(grads)


def conditioning(core, t, mouse=None, btn=None, has_controls=None, want="s"):
    """GameRFTCore.cond on libowlk.  want="s": silu(cond) carrying a fused.CondGrad (what the DiT
    blocks and FinalLayer consume); want="cond": cond itself (bf16 [B, n, d])."""
    meta = core.__dict__.get("_owl_cond_meta")
    if meta is None:
        meta = CondMeta(core)
        core.__dict__["_owl_cond_meta"] = meta
    if not isinstance(t, torch.Tensor):
        t = torch.tensor(t, device=next(core.parameters()).device)
    if t.dim() == 1:
        t = t[:, None]
    if meta.ctrl is not None:
        assert mouse is not None and btn is not None, "conditioning: mouse / button inputs required"
        if mouse.dtype not in (BF16, F32):
            mouse = mouse.float()
        if btn.dtype not in (BF16, F32):
            btn = btn.float()
    if t.dtype not in (BF16, F32):
        t = t.float()
    if has_controls is not None and has_controls.dtype != torch.bool:
        has_controls = has_controls.bool()
    cg = CondGrad() if want == "s" else None
    out = CondFn.apply(t, mouse, btn, has_controls if meta.ctrl is not None else None, meta, cg, want,
                       *meta.params())
    if cg is not None:
        out._owl_cond_grad = cg
    return out
