"""The ping-pong GEMM's paired-rounding epilogues (gemm.hip epi_apply2, OWLK_GEMM_EPI2=1), bit for bit.

Shapes of >= 192 256^2 tiles take gemm_pp_kernel (M 8,232 is ragged: its last tile row is partial).
The fp32 accumulator comes from the same kernel with an fp32 STORE output (same main loop, same tile
order, alpha 1: v = acc exactly), and each epilogue's rounding chain is replayed on it in torch:
bias rounded to bf16, RNE conversions, the products in the order the kernel forms them.  alpha / beta
of the fused multiply-adds are powers of two (the FMA then rounds like the separate operations), so
STORE (bias, beta), AXPBY, SCALE2 and GATE_RESID must match exactly; SILU's aux output exactly and its
silu (hardware exp / rcp) within one bf16 ulp; DSILU within one ulp of the fp32 chain.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def K():
    from owl_wms import kernels
    return kernels


@pytest.fixture(scope="module", autouse=True)
def _needs_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from owl_wms._lib import lib
    lib()


M, N, KD = 8192 + 40, 2048, 512


def data(seed):
    g = torch.Generator().manual_seed(seed)
    A = (torch.randn(M, KD, generator=g) * 0.5).bfloat16().to(DEV)
    B = (torch.randn(N, KD, generator=g) * 0.05).bfloat16().to(DEV)
    bias = (torch.randn(N, generator=g) * 0.3).float().to(DEV)
    x = torch.randn(M, N, generator=g).bfloat16().to(DEV)
    return A, B, bias, x


def acc_of(k, A, B):
    return k.gemm(A, B, out_f32=True)


def bf(t):
    return t.to(torch.bfloat16)


def ulps(a, b):
    """bf16 ulp distance on the monotonic integer line (-0 == +0)"""
    def key(t):
        i = t.contiguous().view(torch.int16).int()
        return torch.where(i >= 0, i, -32768 - i)
    return (key(a) - key(b)).abs()


def test_store_bias_beta_exact():
    k = K()
    A, B, bias, x = data(1)
    acc = acc_of(k, A, B)
    c = x.clone()
    k.gemm(A, B, out=c, epi=k.EPI_STORE, alpha=1.0, beta=0.5, bias=bias)
    v = acc + bf(bias).float()
    v = v + 0.5 * x.float()
    assert torch.equal(c, bf(v))


def test_axpby_exact():
    k = K()
    A, B, bias, x = data(2)
    acc = acc_of(k, A, B)
    c = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    k.gemm(A, B, out=c, epi=k.EPI_AXPBY, alpha=0.75, beta=-1.25, aux=x)
    r = bf(acc).float()
    s1 = bf(0.75 * r).float()
    s2 = bf(-1.25 * x.float()).float()
    assert torch.equal(c, bf(s1 + s2))


def test_scale2_exact():
    k = K()
    A, B, bias, x = data(3)
    acc = acc_of(k, A, B)
    c = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    aux = torch.empty_like(c)
    k.gemm(A, B, out=c, epi=k.EPI_SCALE2, alpha=0.3, aux=aux)
    y = bf(acc)
    assert torch.equal(c, y)
    assert torch.equal(aux, bf(0.3 * y.float()))


@pytest.mark.parametrize("tpf", [1, 64])
def test_gate_resid_exact(tpf):
    k = K()
    A, B, bias, x = data(4)
    g = torch.Generator().manual_seed(40)
    F = (M + tpf - 1) // tpf
    gate = torch.randn(F, N, generator=g).bfloat16().to(DEV)
    acc = acc_of(k, A, B)
    c = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    aux = torch.empty_like(c)
    k.gemm(A, B, out=c, epi=k.EPI_GATE_RESID, bias=bias, aux=aux, gate=gate, tpf=tpf, resid=x)
    y = bf(acc + bf(bias).float())
    gm = gate.float()[torch.arange(M, device=DEV) // tpf]
    t = bf(gm * y.float())
    assert torch.equal(aux, y)
    assert torch.equal(c, bf(x.float() + t.float()))


def test_silu_aux_exact_out_one_ulp():
    k = K()
    A, B, bias, x = data(5)
    acc = acc_of(k, A, B)
    c = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    aux = torch.empty_like(c)
    k.gemm(A, B, out=c, epi=k.EPI_SILU, bias=bias, aux=aux)
    y = bf(acc + bf(bias).float())
    assert torch.equal(aux, y)
    ref = bf(torch.nn.functional.silu(y.float()))
    assert ulps(c, ref).max().item() <= 1


def test_dsilu_one_ulp():
    k = K()
    A, B, bias, x = data(6)
    acc = acc_of(k, A, B)
    c = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    act = torch.empty_like(c)
    k.gemm(A, B, out=c, epi=k.EPI_DSILU, aux=x, resid=act)
    xf = x.float()
    sg = torch.sigmoid(xf)
    ref = bf(bf(acc).float() * sg * (1.0 + xf * (1.0 - sg)))
    assert ulps(c, ref).max().item() <= 1
    assert ulps(act, bf(torch.nn.functional.silu(xf))).max().item() <= 1


@pytest.mark.parametrize("beta", [0.0, 1.0])
def test_split256_wgrad_plan_deterministic(beta):
    """The 256^2 split-K plan for the cond-gradient shape (K 9,216 >= 8,192, fewer than 128 256^2 tiles,
    fp32 out with the workspace, beta 0 and 1): deterministic bit for bit, and == fp32 torch."""
    k = K()
    g = torch.Generator().manual_seed(7)
    dy = torch.randn(9216, 1536, generator=g).bfloat16().to(DEV)
    x = torch.randn(9216, 1536, generator=g).bfloat16().to(DEV)
    c0 = torch.randn(1536, 1536, generator=g).float().to(DEV)
    outs = []
    for _ in range(2):
        out = c0.clone()
        k.gemm(dy, x, a_trans=True, b_trans=True, out=out, out_f32=True, beta=beta)
        outs.append(out)
    assert torch.equal(outs[0], outs[1])
    ref = dy.float().t() @ x.float() + (c0 if beta else 0.0)
    err = ((outs[0] - ref).norm() / ref.norm()).item()
    assert err < 1e-5, err


def test_modulation_shape_pingpong_bias():
    """[1,536 x 9,216 x 1,536] bf16 + bias: 216 256^2 tiles, above the ping-pong minimum of 192."""
    k = K()
    g = torch.Generator().manual_seed(8)
    A = torch.randn(1536, 1536, generator=g).bfloat16().to(DEV)
    B = (torch.randn(9216, 1536, generator=g) * 0.05).bfloat16().to(DEV)
    bias = torch.randn(9216, generator=g).float().to(DEV)
    c = k.gemm(A, B, bias=bias)
    acc = k.gemm(A, B, out_f32=True)
    assert torch.equal(c, bf(acc + bf(bias).float()))
    ref = A.float() @ B.float().t() + bf(bias).float()
    assert ((c.float() - ref).norm() / ref.norm()).item() < 1e-2


def test_split256_opt_plan_without_workspace():
    """The cond-gradient shape through the C ABI with no workspace: the opt split plan needs one, so the
    GEMM runs unsplit (deterministic: two runs equal) -- or the 128^2 split plan when a workspace for
    that one is given or atomics are asked for (gemm.hip)."""
    from owl_wms import _lib
    Mx, Nx, Kx = 1536, 1536, 9216
    g = torch.Generator().manual_seed(9)
    dy = torch.randn(Kx, Mx, generator=g).bfloat16().to(DEV)
    x = torch.randn(Kx, Nx, generator=g).bfloat16().to(DEV)
    ref = dy.float().t() @ x.float()
    for beta in (0.0, 1.0):
        outs = []
        for _ in range(2):
            out = torch.zeros(Mx, Nx, device=DEV) if beta == 0.0 else torch.ones(Mx, Nx, device=DEV)
            _lib.call("owlk_gemm", Mx, Nx, Kx, 1, _lib.ptr(dy), dy.stride(0), 0, 1, _lib.ptr(x), x.stride(0), 0, 1,
                      _lib.ptr(out), out.stride(0), 0, 1, 0, 1.0, beta, None, None, 0, 0, None, 0, 0, 1, None, 0, 0,
                      None, None, 0, _lib.stream())
            outs.append(out)
        assert torch.equal(outs[0], outs[1])
        err = ((outs[0] - (ref + beta)).norm() / (ref + beta).norm()).item()
        assert err < 1e-5, err


@pytest.mark.parametrize("Mx,L", [(8232, 4116), (8192, 8192), (512, 256)])
def test_gemm_attn_delta_equals_gemm_then_delta(Mx, L):
    """owlk_gemm_attn_delta (the out-projection dX with the attention backward's delta in the ping-pong
    epilogue, EPI_DELTA): dO bit for bit the plain GEMM and delta bit for bit owlk_attn_delta on that
    dO -- ragged M (8,232 = 2 samples of 4,116 tokens, 198 tiles), one sample, and a shape below the
    ping-pong minimum (512 x 1,536: the GEMM + attn_delta form)."""
    from owl_wms import _lib
    k = K()
    H, D, Kd = 24, 64, 1536
    g = torch.Generator().manual_seed(11)
    dy = torch.randn(Mx, Kd, generator=g).bfloat16().to(DEV)
    w = (torch.randn(Kd, H * D, generator=g) * 0.03).bfloat16().to(DEV)
    o = torch.randn(Mx, H * D, generator=g).bfloat16().to(DEV)
    do, delta = k.gemm_attn_delta(dy, w, o, H, D, L)
    ref_do = k.gemm(dy, w, b_trans=True)
    assert torch.equal(do, ref_do)
    ref = torch.empty(Mx // L, H, L, device=DEV, dtype=torch.float32)
    _lib.call("owlk_attn_delta", _lib.ptr(o), _lib.ptr(ref_do), H * D, Mx // L, L, H, D, _lib.ptr(ref), _lib.stream())
    assert torch.equal(delta, ref)
    exp = (do.float() * o.float()).view(Mx // L, L, H, D).sum(-1).transpose(1, 2)
    assert ((delta - exp).abs().max() <= 1e-3 * exp.abs().max()).item()


@pytest.mark.parametrize("Mx,tpos,off", [(8232, 4116, 0), (8192, 0, 3), (512, 256, 0)])
def test_gemm_qk_rope_equals_gemm_then_rope(Mx, tpos, off):
    """owlk_gemm_qk_rope (the qkv projection with QK-RMSNorm + RoPE in the ping-pong epilogue,
    EPI_QKROPE): qkv bit for bit the plain GEMM + bias, the rotated q | k rows and rstd bit for bit
    owlk_qk_rope_fwd on that qkv -- ragged M with per-sample positions, one sample with a table
    offset, and a shape below the ping-pong minimum (the GEMM + qk_rope_fwd form)."""
    k = K()
    from oracle import ref_ops as R
    H, D, Kd = 8, 64, 1536
    g = torch.Generator().manual_seed(12)
    h = torch.randn(Mx, Kd, generator=g).bfloat16().to(DEV)
    w = (torch.randn(3 * H * D, Kd, generator=g) * 0.03).bfloat16().to(DEV)
    bias = torch.randn(3 * H * D, generator=g).float().to(DEV)
    ang = R.motion_rope_angles(Mx // 64 + 8, 8, D)
    cos, sin = ang.cos().to(DEV).contiguous(), ang.sin().to(DEV).contiguous()
    qkv, out, rstd = k.gemm_qk_rope(h, w, bias, H, D, cos, sin, off, tpos)
    ref_qkv = k.gemm(h, w, bias=bias)
    assert torch.equal(qkv, ref_qkv)
    ref_out, ref_rstd = k.qk_rope_fwd(ref_qkv, H, D, cos, sin, off, tpos)
    assert torch.equal(out, ref_out) and torch.equal(rstd, ref_rstd)
