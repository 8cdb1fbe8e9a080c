"""Parity of the fused conditioning path (nn/cond.py, csrc/cond.hip) against the CPU oracle.

The oracle's embedding modules (oracle/ref_model.py _TEmbed / _Control, restating
embeddings.py:30-184 and gamerft.py:39-48) run on the CPU under bf16 autocast -- the golden
fixtures' mode -- with the same weights.  Tolerances: elementwise kernels within 1 bf16 ulp-scale
error of the oracle on the same inputs (rel L2 <= 5e-3); outputs and gradients through bf16 GEMMs
rel L2 <= 2e-2.
"""
import pytest
import torch
import torch.nn.functional as F

from oracle import ref_model as RM
from oracle import ref_ops as R

pytestmark = pytest.mark.gpu

DEV = "cuda"
BF16 = torch.bfloat16


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.fixture(scope="module", autouse=True)
def _needs_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from owl_wms._lib import lib
    lib()


def _inputs(B, n, nb, dtype, seed=0):
    g = torch.Generator().manual_seed(seed)
    ts = torch.sigmoid(torch.randn(B, n, generator=g)).to(dtype)
    mouse = (torch.randn(B, n, 2, generator=g) * 3).to(dtype)
    mouse[0, 0] = 0.0  # atan2(0, 0), sign(0)
    mouse[0, 1, 0] = -2.5
    mouse[0, 1, 1] = 0.0
    btn = (torch.rand(B, n, nb, generator=g) < 0.5).to(dtype)
    return ts, mouse, btn


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_cond_embed_vs_oracle(dtype):
    """owlk_cond_embed: timestep sin/cos, mouse polar (angle_proj + magnitude sin/cos) and the button
    input, each op rounded in the input dtype (the reference runs them outside autocast's casts)."""
    from owl_wms import kernels as K
    from owl_wms.nn.embeddings import ControlEmbedding, TimestepEmbedding
    torch.manual_seed(1)
    B, n, nb, d = 2, 9, 11, 64
    te, ce = TimestepEmbedding(d), ControlEmbedding(nb, d)
    ts, mouse, btn = _inputs(B, n, nb, dtype)
    R_ = B * n
    tf = te.sincos._freqs(DEV, torch.float32)
    mf = ce.mouse.magnitude_embed._freqs(DEV, torch.float32)
    wang = ce.mouse.angle_proj.weight.detach().to(DEV).contiguous()
    ts_in, mouse_in, ang, btn_in = K.cond_embed(R_, ts.reshape(R_).to(DEV), tf, 1000.0, mouse.reshape(R_, 2).to(DEV),
                                                mf, 1000.0, wang, btn.reshape(R_, nb).to(DEV), 16)
    # oracle (CPU): the same ops in the input dtype, angle_proj under bf16 autocast
    ref_ts = R.sincos(ts.reshape(R_), 512).to(BF16)
    assert rel(ts_in, ref_ts) < 5e-3
    om = RM._Mouse(d)
    om.angle_proj.weight.data.copy_(ce.mouse.angle_proj.weight.data)
    x = mouse.reshape(R_, 2)
    x = torch.sign(x) * torch.log1p(x.abs())
    a = torch.atan2(x[..., 1], x[..., 0])
    mag = torch.norm(x, dim=-1)
    ae = torch.stack([torch.cos(a), torch.sin(a)], -1).to(x.dtype)
    me = R.sincos(mag, 256).to(x.dtype)
    with torch.autocast("cpu", dtype=BF16):
        ap = om.angle_proj(ae)
    ref_mouse = torch.cat([ap, me.to(ap.dtype)], -1)
    assert rel(mouse_in, ref_mouse) < 5e-3
    assert rel(ang, ae.to(BF16)) < 5e-3
    ref_btn = F.pad((btn.reshape(R_, nb) * 2 - 1).to(BF16), (0, 5))
    assert torch.equal(btn_in.cpu(), ref_btn)


def test_cond_silu_fwd_bwd_exact():
    """cond = t + (hc ? m + b : 0), s = silu(cond) and the backward: the reference's bf16 op chain."""
    from owl_wms import kernels as K
    g = torch.Generator().manual_seed(2)
    B, n, d = 3, 5, 256
    t, m, b = [torch.randn(B * n, d, generator=g).to(BF16) for _ in range(3)]
    hc = torch.tensor([True, False, True])
    cond, s = K.cond_silu_fwd(t.to(DEV), m.to(DEV), b.to(DEV), hc.to(DEV), n)
    ctrl = torch.where(hc.repeat_interleave(n)[:, None], m + b, torch.zeros_like(m))
    ref_c = t + ctrl
    assert torch.equal(cond.cpu(), ref_c)
    ref_s = F.silu(ref_c)
    assert rel(s, ref_s) < 2e-3
    ds = torch.randn(B * n, d, generator=g)
    dcond, dctrl = K.cond_silu_bwd(ds.to(DEV), cond, hc.to(DEV), n, want_ctrl=True)
    c = ref_c.float()
    sg = torch.sigmoid(c)
    ref_d = (ds.to(BF16).float() * sg * (1 + c * (1 - sg))).to(BF16)
    assert rel(dcond, ref_d) < 2e-3
    assert torch.equal(dctrl.cpu(), torch.where(hc.repeat_interleave(n)[:, None], dcond.cpu(), torch.zeros_like(ref_d)))
    # identity mode (the gradient of cond itself, bf16 in)
    g2 = ds.to(BF16).to(DEV)
    d2, c2 = K.cond_silu_bwd(g2, None, hc.to(DEV), n, want_ctrl=True)
    assert d2 is g2 and torch.equal(c2.cpu(), torch.where(hc.repeat_interleave(n)[:, None], ds.to(BF16),
                                                         torch.zeros_like(ref_d)))


@pytest.mark.parametrize("K_", [2, 11, 16])
def test_small_k_wgrad(K_):
    from owl_wms import kernels as K
    g = torch.Generator().manual_seed(3)
    Rr, N = 1000, 2048
    dy = torch.randn(Rr, N, generator=g).to(BF16)
    x = torch.randn(Rr, 16, generator=g).to(BF16)
    ref = dy.float().T @ x.float()[:, :K_]
    out = K.small_k_wgrad(dy.to(DEV), x.to(DEV), K_)
    assert rel(out, ref) < 1e-5
    K.small_k_wgrad(dy.to(DEV), x.to(DEV), K_, out=out, beta=1.0)
    assert rel(out, 2 * ref) < 1e-5


def test_mse_loss_and_grad():
    """owlk_mse's fixed-order loss and owlk_mse_grad's device-scaled gradient (the incoming loss
    gradient read on the device)."""
    from owl_wms import kernels as K
    g = torch.Generator().manual_seed(4)
    pred = torch.randn(4096, 24, generator=g).to(BF16)
    tgt = torch.randn(4096, 24, generator=g).to(BF16)
    loss, _ = K.mse(pred.to(DEV), tgt.to(DEV), want_grad=False)
    ref = F.mse_loss(pred.float(), tgt.float())
    assert loss.dim() == 0 and abs(loss.item() - ref.item()) < 1e-6 * ref.item()
    gout = torch.tensor(0.37, device=DEV)
    dp = K.mse_grad(pred.to(DEV), tgt.to(DEV), gout)
    ref_g = ((2.0 / pred.numel()) * (pred.float() - tgt.float()) * 0.37).to(BF16)
    assert rel(dp, ref_g) < 1e-3


class _Core(torch.nn.Module):
    def __init__(self, d, nb, uncond=False):
        super().__init__()
        from owl_wms.nn.embeddings import ControlEmbedding, TimestepEmbedding
        self.t_embed = TimestepEmbedding(d)
        self.uncond = uncond
        if not uncond:
            self.control_embed = ControlEmbedding(nb, d)


class _RefCore(torch.nn.Module):
    def __init__(self, d, nb, uncond=False):
        super().__init__()
        self.t_embed = RM._TEmbed(d)
        if not uncond:
            self.control_embed = RM._Control(nb, d)


@pytest.mark.parametrize("dtype,hc_mode,uncond", [(torch.bfloat16, "mixed", False), (torch.float32, "none", False),
                                                  (torch.bfloat16, "none", True)])
def test_conditioning_vs_oracle(dtype, hc_mode, uncond):
    """nn/cond.conditioning (want='s') feeding two AdaLN consumers that accumulate into the fp32
    CondGrad and one plain Linear whose gradient returns through autograd, against the oracle's
    modules under CPU bf16 autocast: the consumer outputs, every embedding weight / bias gradient and
    the consumers' weight gradients."""
    from owl_wms.nn.cond import conditioning
    from owl_wms.nn.fused import adaln_mod, linear
    torch.manual_seed(5)
    B, n, nb, d, tpf = 3, 4, 11, 128, 16
    core = _Core(d, nb, uncond).to(DEV)
    ref = _RefCore(d, nb, uncond)
    ref.load_state_dict({k: v.cpu() for k, v in core.state_dict().items()})
    ts, mouse, btn = _inputs(B, n, nb, dtype, seed=6)
    hc = torch.tensor([True, False, True]) if hc_mode == "mixed" else None
    g = torch.Generator().manual_seed(7)
    Ws = [(torch.randn(2 * d, d, generator=g) * d ** -0.5, torch.randn(2 * d, generator=g) * 0.1) for _ in range(2)]
    W3 = torch.randn(64, d, generator=g) * d ** -0.5
    xs = [torch.randn(B, n * tpf, d, generator=g).to(BF16) for _ in range(2)]
    rs = [torch.randn(B, n * tpf, d, generator=g) for _ in range(2)] + [torch.randn(B, n, 64, generator=g)]

    # ours
    cw = [(torch.nn.Parameter(w.to(DEV)), torch.nn.Parameter(b.to(DEV))) for w, b in Ws]
    cw3 = torch.nn.Parameter(W3.to(DEV))
    s = conditioning(core, ts.to(DEV), mouse.to(DEV), btn.to(DEV), hc.to(DEV) if hc is not None else None)
    outs = [adaln_mod(xs[i].to(DEV), s, cw[i][0], cw[i][1], tpf) for i in range(2)] + [linear(s, cw3)]
    loss = sum((o.float() * r.to(DEV)).sum() for o, r in zip(outs, rs))
    loss.backward()

    # oracle (CPU, bf16 autocast)
    rw = [(torch.nn.Parameter(w.clone()), torch.nn.Parameter(b.clone())) for w, b in Ws]
    rw3 = torch.nn.Parameter(W3.clone())
    with torch.autocast("cpu", dtype=BF16):
        cond = ref.t_embed(ts)
        if not uncond:
            ctrl = ref.control_embed(mouse, btn)
            if hc is not None:
                ctrl = torch.where(hc[:, None, None], ctrl, torch.zeros_like(ctrl))
            cond = cond + ctrl
        routs = [R.adaln(xs[i], cond, rw[i][0], rw[i][1]) for i in range(2)] + [F.linear(F.silu(cond), rw3)]
        rloss = sum((o.float() * r).sum() for o, r in zip(routs, rs))
    rloss.backward()

    for o, ro in zip(outs, routs):
        assert rel(o, ro) < 2e-2
    ours = dict(core.named_parameters())
    for k, p in ref.named_parameters():
        assert p.grad is not None and ours[k].grad is not None, k
        assert rel(ours[k].grad, p.grad) < 2e-2, k
    for (w, b), (rw_, rb_) in zip(cw, rw):
        assert rel(w.grad, rw_.grad) < 2e-2 and rel(b.grad, rb_.grad) < 2e-2
    assert rel(cw3.grad, rw3.grad) < 2e-2


def test_mlp_custom_vs_oracle():
    """MLPCustom.forward (cond.MLPFn: SiLU epilogue GEMM; K = 11 padded input) vs the oracle _MLP."""
    from owl_wms.nn.mlp import MLPCustom
    torch.manual_seed(8)
    m = MLPCustom(11, 256, 64).to(DEV)
    om = RM._MLP(11, 256, 64)
    om.load_state_dict({k: v.cpu() for k, v in m.state_dict().items()})
    x = torch.randn(40, 11).to(BF16)
    r = torch.randn(40, 64)
    xd = x.to(DEV).requires_grad_(True)
    y = m(xd)
    (y.float() * r.to(DEV)).sum().backward()
    xr = x.clone().requires_grad_(True)
    with torch.autocast("cpu", dtype=BF16):
        yr = om(xr)
    (yr.float() * r).sum().backward()
    assert rel(y, yr) < 2e-2 and rel(xd.grad, xr.grad) < 2e-2
    ours = dict(m.named_parameters())
    for k, p in om.named_parameters():
        assert rel(ours[k].grad, p.grad) < 2e-2, k
