"""Per-kernel parity of libowlk (HIP, gfx950) against the CPU oracle / fp32 torch references.

Tolerances (bf16 I/O, fp32 accumulate): relative L2 <= 1e-2 for outputs and gradients
(SURVEY.md §8(c)); elementwise bf16 kernels that mimic the autocast rounding chain must be
within 1 bf16 ulp of the oracle evaluated on the same bf16 inputs.
"""
import pytest
import torch

from oracle import ref_ops as R

pytestmark = pytest.mark.gpu

DEV = "cuda"


def K():
    from owl_wms import kernels
    return kernels


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def rnd(*shape, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(torch.bfloat16).to(DEV)


@pytest.fixture(scope="module", autouse=True)
def _needs_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from owl_wms._lib import lib
    lib()


@pytest.mark.parametrize("M,N,K_", [(256, 256, 128), (300, 136, 72), (1536, 4608, 1536), (64, 64, 64), (2048, 128, 1536)])
@pytest.mark.parametrize("at,bt", [(False, False), (False, True), (True, True), (True, False)])
def test_gemm_layouts(M, N, K_, at, bt):
    if (at and M % 8) or (bt and N % 8) or (not at and K_ % 8) or (not bt and K_ % 8):
        pytest.skip("layout constraint")
    A = rnd(K_, M, seed=1) if at else rnd(M, K_, seed=1)
    B = rnd(K_, N, seed=2) if bt else rnd(N, K_, seed=2)
    Af = (A.float().T if at else A.float())
    Bf = (B.float() if bt else B.float().T)
    ref = Af @ Bf
    out = K().gemm(A, B, a_trans=at, b_trans=bt, out_f32=True)
    assert rel(out, ref) < 1e-5
    outb = K().gemm(A, B, a_trans=at, b_trans=bt)
    assert rel(outb, ref) < 5e-3


@pytest.mark.parametrize("K_", [64, 128, 192, 1536, 2560, 4096])
@pytest.mark.parametrize("at,bt", [(False, False), (False, True), (True, True), (True, False)])
def test_gemm256_pingpong(K_, at, bt):
    """>= 256 tiles of 256^2 route to the ping-pong LDS-DMA kernel: K-tile counts 1, 2, 3 (ring
    prologue / drain edge cases) and 24, every operand layout, rows clamped on a ragged M; K 2560 and
    4096 take the grouped tile order (groups of 4 tile rows, 17 rows on the ragged M: a last group
    of one)."""
    M, N = 4096 + (0 if at else 40), 4096
    A = rnd(K_, M, seed=11) if at else rnd(M, K_, seed=11)
    B = rnd(K_, N, seed=12) if bt else rnd(N, K_, seed=12)
    ref = (A.float().T if at else A.float()) @ (B.float() if bt else B.float().T)
    out = K().gemm(A, B, a_trans=at, b_trans=bt, out_f32=True)
    assert rel(out, ref) < 1e-5


@pytest.mark.parametrize("K_", [64, 192])
@pytest.mark.parametrize("at,bt", [(False, False), (False, True), (True, True), (True, False)])
def test_gemm256_many_tiles_bf16(K_, at, bt):
    """> 256 tiles of 256^2 with a bf16 output: 1 and 3 K-tiles, every layout, ragged M, bias and
    the SiLU epilogue (pre-activation and activation both stored)."""
    k = K()
    M, N = 16384 + (0 if at else 40), 1280
    A = rnd(K_, M, seed=17) if at else rnd(M, K_, seed=17)
    B = rnd(K_, N, scale=0.1, seed=18) if bt else rnd(N, K_, scale=0.1, seed=18)
    bias = (torch.randn(N) * 0.1).to(DEV)
    y = ((A.float().T if at else A.float()) @ (B.float() if bt else B.float().T) + bias.bfloat16().float())
    y = y.bfloat16().float()
    assert rel(k.gemm(A, B, a_trans=at, b_trans=bt, bias=bias), y) < 5e-3
    aux = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    s = k.gemm(A, B, a_trans=at, b_trans=bt, bias=bias, epi=k.EPI_SILU, aux=aux)
    assert rel(aux, y) < 5e-3 and rel(s, torch.nn.functional.silu(y)) < 5e-3


def test_gemm256_epilogues():
    """fused epilogues on the 256^2 ping-pong path (dit_v4-like widths)."""
    k = K()
    M, N, Kd, tpf = 8192, 2048, 512, 64
    A, W = rnd(M, Kd, seed=13), rnd(N, Kd, scale=0.1, seed=14)
    bias = (torch.randn(N) * 0.1).to(DEV)
    acc = A.float() @ W.float().T
    y = (acc + bias.bfloat16().float()).bfloat16().float()
    aux = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    s = k.gemm(A, W, bias=bias, epi=k.EPI_SILU, aux=aux)
    assert rel(aux, y) < 5e-3 and rel(s, torch.nn.functional.silu(y)) < 5e-3
    g, res = rnd(M // tpf, N, seed=15), rnd(M, N, seed=16)
    o = k.gemm(A, W, bias=bias, epi=k.EPI_GATE_RESID, aux=aux, gate=g, tpf=tpf, resid=res)
    assert rel(o, res.float() + g.float().repeat_interleave(tpf, 0) * y) < 5e-3 and rel(aux, y) < 5e-3
    x = res.float()
    sg = torch.sigmoid(x)
    d = k.gemm(A, W, epi=k.EPI_DSILU, aux=res)
    assert rel(d, acc * sg * (1 + x * (1 - sg))) < 5e-3


def test_gemm_epilogues():
    k = K()
    M, N, Kd, tpf = 512, 256, 192, 64
    A, W = rnd(M, Kd, seed=3), rnd(N, Kd, scale=0.1, seed=4)
    bias = (torch.randn(N) * 0.1).to(DEV)
    acc = A.float() @ W.float().T
    y = (acc + bias.bfloat16().float()).bfloat16().float()
    # store + bias, beta accumulate into fp32
    out = torch.ones(M, N, device=DEV)
    k.gemm(A, W, out=out, out_f32=True, beta=1.0)
    assert rel(out, acc + 1) < 1e-5
    assert rel(k.gemm(A, W, bias=bias), y) < 5e-3
    # silu
    aux = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    s = k.gemm(A, W, bias=bias, epi=k.EPI_SILU, aux=aux)
    assert rel(aux, y) < 5e-3 and rel(s, torch.nn.functional.silu(y)) < 5e-3
    # gate + residual
    g = rnd(M // tpf, N, seed=5)
    res = rnd(M, N, seed=6)
    o = k.gemm(A, W, bias=bias, epi=k.EPI_GATE_RESID, aux=aux, gate=g, tpf=tpf, resid=res)
    gref = g.float().repeat_interleave(tpf, 0)
    assert rel(o, res.float() + gref * y) < 5e-3 and rel(aux, y) < 5e-3
    # dsilu
    d = k.gemm(A, W, epi=k.EPI_DSILU, aux=res)
    x = res.float()
    sg = torch.sigmoid(x)
    assert rel(d, acc * sg * (1 + x * (1 - sg))) < 5e-3
    # axpby
    sq = rnd(N, N, seed=7)
    e = k.gemm(sq, sq, epi=k.EPI_AXPBY, alpha=2.0315, beta=-4.775, aux=sq)
    assert rel(e, -4.775 * sq.float() + 2.0315 * (sq.float() @ sq.float().T)) < 5e-3


@pytest.mark.parametrize("d,tpf,F", [(1536, 64, 6), (128, 64, 3), (128, 1, 40), (2560, 65, 2)])
def test_adaln_fwd_bwd(d, tpf, F):
    k = K()
    T = F * tpf
    x = rnd(T, d, seed=10)
    mod = rnd(F, 2 * d, scale=0.3, seed=11)
    y, rstd = k.adaln_fwd(x, mod[:, :d], mod[:, d:], tpf)
    xr = x.cpu().float().requires_grad_()
    a = mod[:, :d].cpu().float().requires_grad_()
    b_ = mod[:, d:].cpu().float().requires_grad_()
    yr = R.rms_norm(xr.bfloat16()).float() * (1 + R.frame_broadcast(a[None], tpf)[0]) + R.frame_broadcast(b_[None], tpf)[0]
    assert rel(y, yr) < 5e-3
    dy = rnd(T, d, seed=12)
    dres = rnd(T, d, seed=13)
    dx, dmod = k.adaln_bwd(dy, x, rstd, mod[:, :d], tpf, dres=dres)
    # fp32 reference gradient of the same function
    xr2 = x.cpu().float().requires_grad_()
    yr2 = R.rms_norm(xr2) * (1 + R.frame_broadcast(a[None], tpf)[0]) + R.frame_broadcast(b_[None], tpf)[0]
    yr2.backward(dy.cpu().float())
    assert rel(dx.float().cpu() - dres.float().cpu(), xr2.grad) < 1e-2
    assert rel(dmod[:, :d], a.grad) < 1e-2 and rel(dmod[:, d:], b_.grad) < 1e-2


def test_gate_bwd():
    k = K()
    d, tpf, F = 1536, 64, 4
    T = F * tpf
    dout, y, g = rnd(T, d, seed=20), rnd(T, d, seed=21), rnd(F, d, seed=22)
    dy, dg, dbf = k.gate_bwd(dout, y, g, tpf)
    gb = g.float().repeat_interleave(tpf, 0)
    assert rel(dy, dout.float() * gb) < 5e-3
    assert rel(dg, (dout.float() * y.float()).view(F, tpf, d).sum(1)) < 1e-4
    assert rel(dbf, (dout.float() * gb).bfloat16().float().view(F, tpf, d).sum(1)) < 1e-4


@pytest.mark.parametrize("D", [64, 128])
def test_qk_rope(D):
    """fused QK-RMSNorm + RoPE at dit_v4's head dim 64 and dit_v4_5B's 128 (MotionRoPE tables of
    that head dim, rope.py:88-152; the oracle's tables are pinned to the reference's at both)."""
    k = K()
    H, T = 3, 256
    ang = R.motion_rope_angles(4, 8, D)
    cos, sin = ang.cos().to(DEV), ang.sin().to(DEV)
    qkv = rnd(T, 3 * H * D, scale=2.0, seed=30)
    out, rstd = k.qk_rope_fwd(qkv, H, D, cos, sin)
    x = qkv.cpu().view(T, 3, H, D).permute(1, 2, 0, 3)  # [3, H, T, D]
    ref = torch.stack([R.rope_apply(R.rms_norm(x[i]), ang.cos(), ang.sin()) for i in range(2)])  # [2, H, T, D]
    got = out.cpu().view(T, 2, H, D).permute(1, 2, 0, 3)
    assert (got.float() - ref.float()).abs().max() <= 2 ** -7 * ref.float().abs().max()
    assert rel(got, ref) < 5e-3
    # backward vs autograd of the fp32 chain
    dqk = rnd(T, 2 * H * D, seed=31)
    dqkv = torch.zeros(T, 3 * H * D, device=DEV, dtype=torch.bfloat16)
    k.qk_rope_bwd(dqk, qkv, rstd, H, D, cos, sin, dqkv)
    xf = x[:2].float().clone().requires_grad_()
    yf = torch.stack([R.rope_apply(R.rms_norm(xf[i]), ang.cos(), ang.sin()) for i in range(2)])
    yf.backward(dqk.cpu().float().view(T, 2, H, D).permute(1, 2, 0, 3))
    g = dqkv.cpu().view(T, 3, H, D).permute(1, 2, 0, 3)[:2]
    assert rel(g, xf.grad) < 1e-2


@pytest.mark.parametrize("D,H,T", [(64, 4, 1000), (128, 2, 777), (64, 24, 300)])
def test_qk_rope_bwd_fused_bias(D, H, T):
    """owlk_qk_rope_bwd_bias: the same dq / dk rows as owlk_qk_rope_bwd, bit for bit, and dbias +=
    their column sums (the q / k part of the qkv bias gradient: sum over rows of the bf16 grads)."""
    k = K()
    ang = R.motion_rope_angles(4, 16, D)  # 1,024 positions >= T
    cos, sin = ang.cos().to(DEV), ang.sin().to(DEV)
    qkv = rnd(T, 3 * H * D, scale=2.0, seed=32)
    _, rstd = k.qk_rope_fwd(qkv, H, D, cos, sin)
    dqk = rnd(T, 2 * H * D, seed=33)
    ref = torch.zeros(T, 3 * H * D, device=DEV, dtype=torch.bfloat16)
    k.qk_rope_bwd(dqk, qkv, rstd, H, D, cos, sin, ref)
    got = torch.zeros_like(ref)
    dbias = torch.ones(2 * H * D, device=DEV, dtype=torch.float32)  # added onto
    k.qk_rope_bwd(dqk, qkv, rstd, H, D, cos, sin, got, dbias=dbias)
    assert torch.equal(got, ref)
    want = ref[:, :2 * H * D].double().sum(0) + 1.0
    assert ((dbias.double() - want).abs() <= 1e-5 * (want.abs() + 1.0)).all()


ATTN_CASES = [
    # (B, H, n_frames, tpf, window, docs)
    (1, 2, 8, 64, None, False),
    (1, 2, 8, 64, 2, False),
    (2, 2, 6, 64, None, True),
    (1, 1, 40, 1, 16, False),
    (1, 2, 5, 65, 2, False),
    (2, 1, 9, 4, 3, True),
    (1, 2, 24, 64, 16, True),
    (1, 2, 7, 65, None, False),  # unwindowed, ragged inside the second 64-row half of a 128-row dK/dV tile
    (2, 2, 8, 64, None, "split"),  # documents that recur (not one contiguous run): general doc path
    (1, 2, 12, 64, 4, "split"),
    (1, 2, 24, 64, None, False),  # unwindowed sweeps of 12 query tiles (dK/dV ping-pong ring wraps)
    (1, 1, 300, 1, None, False),  # token-causal: PARTIAL tiles on every diagonal, ragged end
    (1, 2, 80, 64, 64, False),  # window of 4096 tokens: the backward's 128-row tiles (attn_bwd.hip long_sweep)
    (2, 2, 70, 64, 64, "split"),  # the same long-sweep tile forms on PARTIAL tiles of the general document mask
    (1, 2, 72, 65, 64, False),  # mmdit_v2's joint 65-token frames with a cut long window (64 x 65 >= 4096 tokens)
]


def _docs(B, nf, docs):
    doc = torch.zeros(B, nf, dtype=torch.long)
    if docs == "split":
        doc[:] = (torch.arange(nf) // 2) % 2
    elif docs:
        doc[:, nf // 3:] = 1
        doc[-1, 2 * nf // 3:] = 2
    return doc


@pytest.mark.parametrize("case,D", [(c, 64) for c in ATTN_CASES] + [(ATTN_CASES[i], 128) for i in (0, 2, 4, 6, 12, 13)])
def test_attention_fwd_bwd(case, D):
    """dit_v4 / mmdit heads are 64 wide, dit_v4_5B heads 128 (d 2560 / 20 heads)."""
    k = K()
    B, H, nf, tpf, window, docs = case
    L = nf * tpf
    q, kk, v = rnd(B * L, H * D, seed=40), rnd(B * L, H * D, seed=41), rnd(B * L, H * D, seed=42)
    doc = _docs(B, nf, docs)
    arrays = k.frame_arrays(doc.to(DEV), nf, window) if docs else None
    if docs:
        assert arrays["runs"] == (docs is True)  # contiguous runs take the range form of the mask
    mask = k.FrameMask(tpf, window, True, 0, arrays)
    q, kk, v = (t.view(B, L, H * D) for t in (q, kk, v))
    o, lse = k.attn_fwd(q, kk, v, H, D, mask)
    qr = q.cpu().float().view(B, L, H, D).transpose(1, 2).requires_grad_()
    kr = kk.cpu().float().view(B, L, H, D).transpose(1, 2).requires_grad_()
    vr = v.cpu().float().view(B, L, H, D).transpose(1, 2).requires_grad_()
    m = R.frame_mask(L, L, tpf, window, doc if docs else None)
    oref = R.attention(qr, kr, vr, m)
    assert rel(o.view(B, L, H, D).transpose(1, 2), oref) < 1e-2
    # lse (internal fwd -> bwd contract) is base 2: lse2 = log2 sum exp(s / sqrt(D))
    sc = (qr.detach() @ kr.detach().transpose(-1, -2)) * D ** -0.5
    lref = torch.logsumexp(sc.masked_fill(~m[:, None], float("-inf")), -1) / torch.log(torch.tensor(2.0))
    assert (lse.cpu() - lref).abs().max().item() < 2e-2
    do = rnd(B * L, H * D, seed=43).view(B, L, H * D)
    oref.backward(do.cpu().float().view(B, L, H, D).transpose(1, 2))
    dq, dk, dv = (torch.empty_like(q) for _ in range(3))
    k.attn_bwd(q, kk, v, o, do, lse, H, D, mask, dq, dk, dv)
    for got, ref in ((dq, qr.grad), (dk, kr.grad), (dv, vr.grad)):
        assert rel(got.view(B, L, H, D).transpose(1, 2), ref) < 1e-2  # SURVEY §8(c) per-op


@pytest.mark.parametrize("D,window", [(128, None), (128, 16), (64, None), (64, 16)])
def test_attention_bwd_side_stream_equals_serial(D, window, monkeypatch):
    """dQ on a side stream beside dK/dV (the default for D 128 global layers) gives the same bits
    as the two kernels back to back on the caller's stream, and the caller's stream sees the
    results without a host sync."""
    k = K()
    B, H, nf, tpf = 1, 4, 48, 64
    L = nf * tpf
    q, kk, v, do = (rnd(B * L, H * D, seed=s).view(B, L, H * D) for s in (50, 51, 52, 53))
    mask = k.FrameMask(tpf, window)
    o, lse = k.attn_fwd(q, kk, v, H, D, mask)
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("OWLK_BWD_SIDE_STREAM", mode)
        assert (k._bwd_side_stream(q.device, D, mask) is not None) == (mode == "1")
        g = [torch.full_like(q, float("nan")) for _ in range(3)]
        k.attn_bwd(q, kk, v, o, do, lse, H, D, mask, *g)
        out[mode] = [t.clone() for t in g]  # on the caller's stream: ordered after the join
    for a, b in zip(out["0"], out["1"]):
        assert torch.equal(a, b)
    monkeypatch.delenv("OWLK_BWD_SIDE_STREAM")
    assert (k._bwd_side_stream(q.device, D, mask) is not None) == (D == 128 and window is None)


@pytest.mark.parametrize("case,D", [(ATTN_CASES[0], 64), (ATTN_CASES[2], 64), (ATTN_CASES[4], 64), (ATTN_CASES[6], 64),
                                    (ATTN_CASES[2], 128)])
def test_attention_fwd_score_bound(case, D):
    """Bounded softmax (score_bound: p = exp2(c s) with q prescaled by c in-kernel) on
    QK-RMSNorm'd inputs == oracle; its lse equals the running-max kernel's up to the one extra
    bf16 rounding of q' = q c (2^-9 relative per element -> measured <= 2.1e-3 in lse2)."""
    k = K()
    B, H, nf, tpf, window, docs = case
    L = nf * tpf
    unit = lambda t: (t.float().view(-1, H, D) * torch.rsqrt(t.float().view(-1, H, D).pow(2).mean(-1, keepdim=True))
                      ).bfloat16().view(B, L, H * D)
    q, kk = unit(rnd(B * L, H * D, seed=60)), unit(rnd(B * L, H * D, seed=61))
    v = rnd(B * L, H * D, seed=62).view(B, L, H * D)
    doc = torch.zeros(B, nf, dtype=torch.long)
    if docs:
        doc[:, nf // 3:] = 1
    mask = k.FrameMask(tpf, window, True, 0, k.frame_arrays(doc.to(DEV), nf, window) if docs else None)
    o, lse = k.attn_fwd(q, kk, v, H, D, mask, score_bound=k.qk_norm_bound(D))
    o0, lse0 = k.attn_fwd(q, kk, v, H, D, mask)
    ref = R.attention(*(t.cpu().float().view(B, L, H, D).transpose(1, 2) for t in (q, kk, v)),
                      R.frame_mask(L, L, tpf, window, doc if docs else None))
    assert rel(o.view(B, L, H, D).transpose(1, 2), ref) < 1e-2
    assert (lse - lse0).abs().max().item() < 4e-3
    assert rel(o, o0) < 5e-3


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("Lq,Lkv", [(64, 256), (64, 640), (37, 1000), (64, 4096), (1, 320)])
def test_attention_decode_split_keys(Lq, Lkv, D):
    """Decode attention (one frame of <= 64 queries, unmasked over [cache | frame], bounded
    softmax): the 4 waves of a workgroup split the key tiles and add their partial O / row sums.
    == oracle (rel 1e-2); lse within 4e-3 of the single-wave kernel (OWLK_FWD_SPLIT=0 path is the
    one every other test covers); deterministic.  D 128 (dit_v4_5B) sweeps 32-key tiles."""
    k = K()
    B, H = 2, 3
    unit = lambda t, L: (t.float().view(-1, H, D) * torch.rsqrt(t.float().view(-1, H, D).pow(2).mean(-1, keepdim=True))
                         ).bfloat16().view(B, L, H * D)
    q = unit(rnd(B * Lq, H * D, seed=70), Lq)
    kk = unit(rnd(B * Lkv, H * D, seed=71), Lkv)
    v = rnd(B * Lkv, H * D, seed=72).view(B, Lkv, H * D)
    mask = k.FrameMask(1, None, False, 0, None)
    o, lse = k.attn_fwd(q, kk, v, H, D, mask, score_bound=k.qk_norm_bound(D))
    ref = R.attention(q.cpu().float().view(B, Lq, H, D).transpose(1, 2), kk.cpu().float().view(B, Lkv, H, D).transpose(1, 2),
                      v.cpu().float().view(B, Lkv, H, D).transpose(1, 2))
    assert rel(o.view(B, Lq, H, D).transpose(1, 2), ref) < 1e-2
    o0, lse0 = k.attn_fwd(q, kk, v, H, D, mask)  # running-max kernel (no bound): another code path
    assert (lse - lse0).abs().max().item() < 4e-3
    assert rel(o, o0) < 5e-3
    o2, lse2 = k.attn_fwd(q, kk, v, H, D, mask, score_bound=k.qk_norm_bound(D))
    assert torch.equal(o, o2) and torch.equal(lse, lse2)


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("Lq,start,cached,window", [(64, 0, 576, 0), (64, 128, 960, 256), (50, 64, 200, 0),
                                                     (64, 0, 64, 128)])
def test_attention_decode_device_state(D, Lq, start, cached, window):
    """owlk_attn_decode_fwd (the cache position read from the device: {start, cached, offset}) over
    cache buffers with rows [start, start + cached + Lq) live == attn_fwd on the same keys as explicit
    views (the last `window` of them for a windowed layer), within the two kernels' summation order."""
    k = K()
    B, H, cap = 2, 2, 2048
    unit = lambda t: (t.float().view(*t.shape[:-1], H, D) * torch.rsqrt(
        t.float().view(*t.shape[:-1], H, D).pow(2).mean(-1, keepdim=True))).bfloat16().view(t.shape)
    q = unit(rnd(B, Lq, H * D, seed=80))
    kb = unit(rnd(B, cap, H * D, seed=81))
    vb = rnd(B, cap, H * D, seed=82)
    state = torch.tensor([start, cached, 0, 0], dtype=torch.int64, device=DEV)
    o, lse = k.attn_decode_fwd(q, kb, vb, H, D, state, Lq, window, score_bound=k.qk_norm_bound(D))
    total = cached + Lq
    first = total - window if 0 < window < total else 0
    ks, vs = kb[:, start + first:start + total], vb[:, start + first:start + total]
    o_ref, lse_ref = k.attn_fwd(q, ks, vs, H, D, k.FrameMask(1, None, False, 0, None), score_bound=k.qk_norm_bound(D))
    assert rel(o, o_ref) < 5e-3
    assert (lse - lse_ref).abs().max().item() < 4e-3


@pytest.mark.parametrize("D", [64, 128])
def test_decode_positions_are_bounded(D):
    """Every position a rope / decode kernel follows is bounded by the RoPE table rows and the cache
    capacity (round 4's illegal-address fault, profiles/r4ac_gemm_nowait_tests_fault.log, was a decode
    test running past the table: the rope kernels read 64 rows beyond it).  Host-given positions past
    the table raise (the reference's short cos slice fails, rope.py:46-49); a device state past them
    (a replayed graph) leaves the cache buffers untouched, reads nothing and poisons its outputs with
    NaN; in range, exactly rows start + cached .. + L are written, as the host-position form writes."""
    k = K()
    B, H, L, cap = 2, 2, 64, 256
    ang = R.motion_rope_angles(3, 8, D)  # 3 frames x 64 tokens = 192 table rows
    rows = ang.shape[0]
    cos, sin = ang.cos().to(DEV), ang.sin().to(DEV)
    qkv = rnd(B * L, 3 * H * D, seed=90)
    with pytest.raises(RuntimeError, match="rope table"):
        k.qk_rope_fwd(qkv, H, D, cos, sin, rows - L + 1, L)
    with pytest.raises(RuntimeError, match="rope table"):
        k.qk_rope_fwd(rnd(4 * L, 3 * H * D, seed=93), H, D, cos, sin, 0, 0)  # 256 rows from row 0, no wrap
    with pytest.raises(RuntimeError, match="rope table"):
        k.qk_rope_bwd(qkv[:, :2 * H * D].contiguous(), qkv, torch.ones(B * L, 2 * H, device=DEV), H, D, cos, sin,
                      torch.empty_like(qkv), rows - L + 1, L)
    kb, vb = rnd(B, cap, H * D, seed=91), rnd(B, cap, H * D, seed=92)
    qbuf = torch.empty(B, L, H * D, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="rope table"):
        k.qk_rope_fwd_kv(qkv, B, L, H, D, cos, sin, rows - L + 1, qbuf, kb[:, :L], vb[:, :L])
    k0, v0 = kb.clone(), vb.clone()
    for st in ([0, cap - L + 1, 0, 0], [cap, 0, 0, 0], [-64, 0, 0, 0], [0, 0, rows - L + 1, 0], [0, 0, -1, 0]):
        state = torch.tensor(st, dtype=torch.int64, device=DEV)
        q = torch.zeros(B, L, H * D, device=DEV, dtype=torch.bfloat16)
        k.qk_rope_fwd_kv_dev(qkv, B, L, H, D, cos, sin, state, q, kb, vb)
        torch.cuda.synchronize()
        assert torch.equal(kb, k0) and torch.equal(vb, v0), st
        assert torch.isnan(q.float()).all(), st
    # in range (last table rows, last cache rows): the host-position form's result, nothing else written
    start, cached = 16, cap - L - 16
    state = torch.tensor([start, cached, rows - L, 0], dtype=torch.int64, device=DEV)
    q = torch.empty(B, L, H * D, device=DEV, dtype=torch.bfloat16)
    k.qk_rope_fwd_kv_dev(qkv, B, L, H, D, cos, sin, state, q, kb, vb)
    qr, kr, vr = torch.empty_like(q), torch.empty_like(q), torch.empty_like(q)
    k.qk_rope_fwd_kv(qkv, B, L, H, D, cos, sin, rows - L, qr, kr, vr)
    r0 = start + cached
    assert torch.equal(q, qr) and torch.equal(kb[:, r0:], kr) and torch.equal(vb[:, r0:], vr)
    assert torch.equal(kb[:, :r0], k0[:, :r0]) and torch.equal(vb[:, :r0], v0[:, :r0])
    # decode attention over a window past the buffers: NaN rows, nothing read
    for st in ([0, cap, 0, 0], [cap - L, 1, 0, 0], [-1, 0, 0, 0]):
        state = torch.tensor(st, dtype=torch.int64, device=DEV)
        o, lse = k.attn_decode_fwd(qr, kb, vb, H, D, state, L, 0, score_bound=k.qk_norm_bound(D))
        torch.cuda.synchronize()
        assert torch.isnan(o.float()).all() and torch.isnan(lse).all(), st
    state = torch.tensor([start, cached, 0, 0], dtype=torch.int64, device=DEV)
    o, _ = k.attn_decode_fwd(qr, kb, vb, H, D, state, L, 0, score_bound=k.qk_norm_bound(D))
    assert torch.isfinite(o.float()).all()


@pytest.mark.parametrize("D,window", [(64, None), (64, 2), (128, None)])
def test_integration_binding_lse_contract(D, window):
    """The reference-side binding of INTEGRATION.md (owlk_bind.attn_fwd) run against the real
    libowlk.so: o == oracle attention, and lse2 is what include/owlk.h documents -- BASE 2,
    lse2 * ln 2 == torch.logsumexp(scale * q k^T) over the allowed keys (flex_attention's
    return_lse), on the frame mask of attn.py:24-62."""
    import math
    import os
    import re
    from conftest import REPO
    from owl_wms._lib import LIB_PATH, lib
    lib()  # torch's HIP runtime first, then the library (as the binding's comment says)
    text = open(os.path.join(REPO, "INTEGRATION.md")).read()
    block = [b for b in re.findall(r"```python\n(.*?)```", text, flags=re.S) if "ctypes.CDLL" in b][0]
    old = os.environ.get("OWLK_LIB")
    os.environ["OWLK_LIB"] = LIB_PATH
    try:
        ns = {}
        exec(compile(block, "INTEGRATION.md", "exec"), ns)
    finally:
        if old is None:
            os.environ.pop("OWLK_LIB")
        else:
            os.environ["OWLK_LIB"] = old
    B, H, nf, tpf = 2, 2, 6, 64
    L = nf * tpf
    q, kk, v = (rnd(B, L, H, D, seed=s) for s in (90, 91, 92))
    o, lse2 = ns["attn_fwd"](q, kk, v, tpf, window)
    torch.cuda.synchronize()
    qr, kr, vr = (t.cpu().float().transpose(1, 2) for t in (q, kk, v))
    m = R.frame_mask(L, L, tpf, window, None)
    assert rel(o.transpose(1, 2), R.attention(qr, kr, vr, m)) < 1e-2
    sc = (qr @ kr.transpose(-1, -2)) * D ** -0.5
    lse_nat = torch.logsumexp(sc.masked_fill(~m[:, None], float("-inf")), -1)
    assert (lse2.cpu() * math.log(2.0) - lse_nat).abs().max().item() < 2e-2


def test_attention_dit_v4_shape_smoke():
    """Full dit_v4 attention shape (24 heads x 98,304 tokens): finite, rows normalised."""
    k = K()
    B, H, nf, tpf, D = 1, 24, 1536, 64, 64
    L = nf * tpf
    torch.manual_seed(0)
    q = torch.randn(1, L, H * D, device=DEV, dtype=torch.bfloat16)
    kk = torch.randn(1, L, H * D, device=DEV, dtype=torch.bfloat16)
    v = torch.ones(1, L, H * D, device=DEV, dtype=torch.bfloat16)
    for window in (None, 16):
        o, lse = k.attn_fwd(q, kk, v, H, D, k.FrameMask(tpf, window))
        assert torch.isfinite(lse).all()
        assert (o.float() - 1).abs().max().item() < 1e-2  # softmax rows sum to one


def _sample_rows(L, tpf, n, seed):
    """edge rows (first / last token, frame and 128-row tile seams, the middle) plus random ones"""
    fixed = [0, 1, tpf - 1, tpf, 127, 128, 4095, 4096, L // 2, L // 2 + tpf - 1, L - tpf, L - 1]
    g = torch.Generator().manual_seed(seed)
    extra = torch.randint(0, L, (n - len(fixed),), generator=g).tolist()
    return torch.tensor(sorted(set(fixed + extra)), device=DEV)


@pytest.mark.parametrize("H,D", [(24, 64), (20, 128)])
@pytest.mark.parametrize("window", [None, 16])
def test_attention_bwd_dit_v4_shape_sampled_rows(window, H, D):
    """The production shape (B 1 x H 24 x 98,304 tokens, tpf 64, global and window-16 layers, the
    QK-RMSNorm'd inputs and score_bound of the model; attn.py:24-62, 106-109) through owlk_attn_fwd
    and the two backward kernels -- every block of the XCD-aware remap and the 128-row tile paths
    run as in the bench -- checked on sampled rows of four heads against fp32 torch: O and dQ of
    sampled query rows over all their allowed keys; dK and dV of sampled key rows over all their
    allowed queries (with fp32 lse and delta recomputed for every query of the head).  Tolerance:
    rel-L2 <= 1e-2 (SURVEY §8(c) per-op) over the sampled rows.  H 20 x D 128 is dit_v4_5B's shape
    (configs/dit_v4_5B.yml: d 2560 / 20 heads); its global layers run dQ on the side stream beside
    dK/dV (the default, kernels._bwd_side_stream)."""
    k = K()
    B, nf, tpf = 1, 1536, 64
    if D == 128 and window is None:
        assert k._bwd_side_stream(torch.device(DEV), D, k.FrameMask(tpf, window)) is not None
    L = nf * tpf
    gen = torch.Generator(device=DEV).manual_seed(11)

    def unit(t):  # QK-RMSNorm (attn.py:84): |q.k| <= D, what score_bound promises
        t = t.view(L, H, D)
        return (t * torch.rsqrt(t.pow(2).mean(-1, keepdim=True))).bfloat16().view(1, L, H * D)

    q = unit(torch.randn(L, H * D, device=DEV, generator=gen))
    kk = unit(torch.randn(L, H * D, device=DEV, generator=gen))
    v = torch.randn(1, L, H * D, device=DEV, generator=gen).bfloat16()
    do = torch.randn(1, L, H * D, device=DEV, generator=gen).bfloat16()
    mask = k.FrameMask(tpf, window)
    o, lse = k.attn_fwd(q, kk, v, H, D, mask, score_bound=k.qk_norm_bound(D))
    dq, dk, dv = (torch.empty_like(q) for _ in range(3))
    k.attn_bwd(q, kk, v, o, do, lse, H, D, mask, dq, dk, dv)
    torch.cuda.synchronize()
    scale = D ** -0.5
    fr = torch.arange(L, device=DEV) // tpf

    def allowed(qi, kj):  # frame mask predicate for index vectors
        ok = fr[kj][None, :] <= fr[qi][:, None]
        if window is not None:
            ok &= fr[qi][:, None] - fr[kj][None, :] < window
        return ok

    def key_range(c0, c1):
        lo = 0 if window is None else max(0, (c0 // tpf - window + 1) * tpf)
        return lo, ((c1 - 1) // tpf + 1) * tpf

    qrows, krows = _sample_rows(L, tpf, 16, 1), _sample_rows(L, tpf, 16, 2)
    got, ref = {n: [] for n in ("o", "dq", "dk", "dv")}, {n: [] for n in ("o", "dq", "dk", "dv")}
    for h in (0, 7, 13, H - 1):
        cs = slice(h * D, (h + 1) * D)
        qh, kh, vh, doh = (t[0, :, cs].float() for t in (q, kk, v, do))
        lse_r = torch.empty(L, device=DEV)
        o_r = torch.empty(L, D, device=DEV)
        CH = 4096
        for c0 in range(0, L, CH):
            c1 = min(L, c0 + CH)
            lo, hi = key_range(c0, c1)
            s = (qh[c0:c1] @ kh[lo:hi].T) * scale
            s.masked_fill_(~allowed(torch.arange(c0, c1, device=DEV), torch.arange(lo, hi, device=DEV)),
                           float("-inf"))
            lse_r[c0:c1] = torch.logsumexp(s, -1)
            o_r[c0:c1] = torch.exp(s - lse_r[c0:c1, None]) @ vh[lo:hi]
            del s
        delta_r = (doh * o_r).sum(-1)
        # lse is base 2 inside the kernels (lse2 = lse / ln 2)
        assert (lse[0, h, qrows] * torch.log(torch.tensor(2.0)) - lse_r[qrows]).abs().max().item() < 2e-2
        # sampled query rows: O, dQ over all allowed keys
        for i in qrows.tolist():
            lo, hi = key_range(i, i + 1)
            kj = torch.arange(lo, hi, device=DEV)
            ok = allowed(torch.tensor([i], device=DEV), kj)[0]
            s = (qh[i] @ kh[lo:hi].T) * scale
            p = torch.where(ok, torch.exp(s - lse_r[i]), torch.zeros_like(s))
            dp = doh[i] @ vh[lo:hi].T
            ref["o"].append(p @ vh[lo:hi])
            ref["dq"].append(scale * ((p * (dp - delta_r[i])) @ kh[lo:hi]))
            got["o"].append(o[0, i, cs].float())
            got["dq"].append(dq[0, i, cs].float())
        # sampled key rows: dK, dV over all allowed queries
        for j in krows.tolist():
            f = j // tpf
            q0, q1 = f * tpf, (L if window is None else min(L, (f + window) * tpf))
            qi = torch.arange(q0, q1, device=DEV)
            ok = allowed(qi, torch.tensor([j], device=DEV))[:, 0]
            s = (qh[q0:q1] @ kh[j]) * scale
            p = torch.where(ok, torch.exp(s - lse_r[q0:q1]), torch.zeros_like(s))
            dp = doh[q0:q1] @ vh[j]
            ref["dv"].append(p @ doh[q0:q1])
            ref["dk"].append(scale * ((p * (dp - delta_r[q0:q1])) @ qh[q0:q1]))
            got["dv"].append(dv[0, j, cs].float())
            got["dk"].append(dk[0, j, cs].float())
    for n in ("o", "dq", "dk", "dv"):
        assert rel(torch.stack(got[n]), torch.stack(ref[n])) < 1e-2, n


def test_flow_noise_mse():
    k = K()
    B, N, C, h = 2, 3, 32, 8
    x, z = rnd(B, N, C, h, h, seed=50), rnd(B, N, C, h, h, seed=51)
    ts_raw = rnd(B, N, seed=52).float()
    xt, tgt, ts = k.flow_noise(x, z, ts_raw)
    t = ts_raw.cpu().bfloat16().sigmoid()
    xr, tr = R.flow_noise(x.cpu(), t[:, :, None, None, None], z.cpu())
    tok = lambda a: a.permute(0, 1, 3, 4, 2).reshape(-1, C)
    assert torch.equal(ts.cpu(), t)
    assert torch.equal(xt.cpu(), tok(xr)) and torch.equal(tgt.cpu(), tok(tr))
    pred = rnd(B * N * h * h, C, seed=53)
    loss, dpred = k.mse(pred, tgt)
    ref = torch.nn.functional.mse_loss(pred.float(), tgt.float())
    assert abs(loss.item() - ref.item()) < 1e-5 * ref.item()
    assert rel(dpred, 2 * (pred.float() - tgt.float()) / pred.numel()) < 5e-3
    assert torch.equal(k.unpatchify(tgt, B, N, C, h, h).cpu(), tr)


@pytest.mark.parametrize("R,N", [(1000, 264), (98304, 1536), (7, 8), (20000, 4608)])
def test_colsum(R, N):
    """accumulates onto out; fp32 input too; ragged and narrow shapes."""
    k = K()
    x = rnd(R, N, seed=60)
    ref = x.float().sum(0)
    out = k.colsum(x)
    assert rel(out, ref) < 1e-5
    base = torch.randn(N, device=DEV)
    acc = base.clone()
    k.colsum(x, out=acc)
    assert rel(acc, base + ref) < 1e-5
    assert rel(k.colsum(x.float()), ref) < 1e-5


@pytest.mark.parametrize("shape", [(256, 768), (768, 256), (128, 128)])
def test_newton_schulz_matches_oracle(shape):
    """owlk_newton_schulz_bf16 (one C entry, reference rounding order: the A GEMM also emits
    bf16(c A), B = bf16(b A) + bf16(cA @ A)) against the reference's own output (ops.pt ns.*.y,
    generated by the reference's zeropower_via_newtonschulz5) and the oracle: within 2 bf16 ulp of
    1.0 (max-abs 2^-7).  What remains is the GEMMs' fp32 accumulation order (MFMA vs
    the CPU's), which flips single bf16 roundings that five chaotic iterations then amplify: rel-L2
    measured 1.0-1.5 % after 5 steps (2.7 % with the scalar applied after the product, round 1),
    and after 1-2 steps it stays at the rounding level (test_newton_schulz_steps_vs_oracle)."""
    from conftest import golden
    from owl_wms.muon import newton_schulz_bf16
    ops = golden("ops.pt")
    g = ops[f"ns.{shape[0]}x{shape[1]}.g"]
    y = newton_schulz_bf16(g.to(DEV)[None])[0].float().cpu()
    ref = ops[f"ns.{shape[0]}x{shape[1]}.y"].float()
    mine = R.newton_schulz5(g).float()
    for r in (ref, mine):
        assert (y - r).abs().max().item() <= 2 ** -7
        assert rel(y, r) < 2e-2


@pytest.mark.parametrize("steps,tol", [(1, 4e-3), (2, 6e-3)])
@pytest.mark.parametrize("shape", [(256, 768), (768, 256), (128, 128)])
def test_newton_schulz_steps_vs_oracle(shape, steps, tol):
    """Before the iteration's chaos amplifies it, the library NS equals the oracle (pinned exactly to
    the reference's eager body) at the bf16 rounding level: same rounding order, so only fp32
    accumulation order differs."""
    from conftest import golden
    g = golden("ops.pt")[f"ns.{shape[0]}x{shape[1]}.g"]
    y = K().newton_schulz(g.to(DEV)[None], steps)[0].float().cpu()
    r = R.newton_schulz5(g, steps).float()
    assert rel(y, r) < tol, rel(y, r)


@pytest.mark.parametrize("count,shape", [(3, (256, 768)), (2, (768, 256)), (16, (64, 128))])
def test_ns_iterate_equals_library_entry(count, shape):
    """Muon's in-step NS (normalise -> owlk_ns_iterate on a shape batch) and owlk_newton_schulz_bf16
    run the same kernels: bit-identical updates."""
    k = K()
    r, c = shape
    g = torch.randn(count, r, c, generator=torch.Generator().manual_seed(90)).to(DEV)
    whole = k.newton_schulz(g)
    tr = r > c
    x = k.ns_iterate(k.ns_normalize(g, tr), 5)
    x = x.transpose(1, 2) if tr else x
    assert torch.equal(x, whole)


@pytest.mark.parametrize("M,N,K_", [(128, 1536, 16384), (1536, 1536, 20480), (4608, 256, 12288),
                                     (1536, 2048, 24576)])
def test_gemm_splitk_weight_grad(M, N, K_):
    k = K()
    dy, x = rnd(K_, M, seed=70), rnd(K_, N, seed=71)
    ref = dy.float().T @ x.float()
    out = k.gemm_wgrad(dy, x)
    assert rel(out, ref) < 1e-5


@pytest.mark.parametrize("M,N,Kd", [(16384 + 40, 1024, 1536), (512, 256, 192)])
def test_gemm_dsilu_colsum(M, N, Kd):
    """colsum= on the DSILU epilogue: fused in the 256^2 kernel (first case, ragged M), separate pass
    otherwise (second case: too few tiles); equals the column sums of the stored bf16 output."""
    k = K()
    A, W = rnd(M, Kd, seed=80), rnd(N, Kd, scale=0.05, seed=81)
    res = rnd(M, N, seed=82)
    cs = torch.zeros(N, device=DEV)
    d = k.gemm(A, W, epi=k.EPI_DSILU, aux=res, colsum=cs)
    ref = k.gemm(A, W, epi=k.EPI_DSILU, aux=res)
    assert torch.equal(d, ref)
    assert rel(cs, ref.float().sum(0)) < 1e-5


def test_gemm_splitk_workspace_alpha_beta():
    """256^2 split-K (48 tiles x 12 splits): partials + reduce give alpha AB + beta C; beta 0 never
    reads C (NaN-filled here)."""
    k = K()
    M, N, K_ = 1536, 2048, 24576
    dy, x = rnd(K_, M, seed=72), rnd(K_, N, seed=73)
    ref = dy.float().T @ x.float()
    out = torch.full((M, N), float("nan"), device=DEV)
    k.gemm(dy, x, a_trans=True, b_trans=True, out=out, out_f32=True, beta=0.0)
    assert rel(out, ref) < 1e-5
    c0 = torch.randn(M, N, device=DEV)
    out = c0.clone()
    k.gemm(dy, x, a_trans=True, b_trans=True, out=out, out_f32=True, alpha=0.5, beta=1.0)
    assert rel(out, 0.5 * ref + c0) < 1e-5


def test_gemm_splitk_without_workspace():
    """owlk_gemm with no workspace on a split-K shape combines the splits by fp32 atomics: beta 0
    clears C first (NaN-filled here), beta 1 accumulates."""
    from owl_wms import _lib
    M, N, K_ = 1536, 2048, 24576
    dy, x = rnd(K_, M, seed=74), rnd(K_, N, seed=75)
    ref = dy.float().T @ x.float()
    assert _lib.lib().owlk_gemm_splitk_bytes(M, N, K_, 1, 1, 1, 1, 0, 0.0) > 0
    for beta in (0.0, 1.0):
        out = torch.full((M, N), float("nan"), device=DEV) if beta == 0.0 else torch.ones(M, N, device=DEV)
        _lib.call("owlk_gemm", M, N, K_, 1, _lib.ptr(dy), dy.stride(0), 0, 1, _lib.ptr(x), x.stride(0), 0, 1,
                  _lib.ptr(out), out.stride(0), 0, 1, 0, 1.0, beta, None, None, 0, 0, None, 0, 0, 1, None, 0, 0,
                  None, None, 0, _lib.stream())
        assert rel(out, ref + beta) < 1e-5


def test_frame_mux_roundtrip():
    """frame_interleave == per-frame torch.cat (mmattn.py:54-60); frame_split is its exact inverse."""
    k = K()
    F_, n0, n1, C = 7, 64, 1, 96
    a, b = rnd(F_ * n0, C, seed=70), rnd(F_ * n1, C, seed=71)
    j = k.frame_interleave(a, b, n0, n1)
    ref = torch.cat([a.view(F_, n0, C), b.view(F_, n1, C)], 1).reshape(-1, C)
    assert torch.equal(j, ref)
    a2, b2 = k.frame_split(j, n0, n1)
    assert torch.equal(a2, a) and torch.equal(b2, b)


@pytest.mark.parametrize("T,d", [(300, 128), (130, 1536), (65, 2560)])
def test_layernorm_fwd_bwd(T, d):
    """normalization.py:6-7 under autocast: fp32 layer_norm (eps 1e-5) of bf16 x, rounded to bf16."""
    k = K()
    x = rnd(T, d, scale=3.0, seed=72)
    y, mean, rstd = k.layernorm_fwd(x)
    xr = x.float().cpu().requires_grad_()
    yr = torch.nn.functional.layer_norm(xr, (d,))
    assert (y.float().cpu() - yr.detach().bfloat16().float()).abs().max() <= 2 ** -7 * yr.abs().max()
    dy = rnd(T, d, seed=73)
    yr.backward(dy.float().cpu())
    assert rel(k.layernorm_bwd(dy, x, mean, rstd), xr.grad) < 1e-2


@pytest.mark.parametrize("shape", [(256, 2), (3, 40), (12, 13)])
def test_newton_schulz_padded_shapes(shape):
    """Shapes whose dims are not multiples of 8 (mmdit_v2 puts control_embed.mouse.angle_proj
    [256, 2] under Muon) are zero-padded inside owlk_newton_schulz_bf16: same result as the oracle
    NS (reference rounding order)."""
    from owl_wms.muon import newton_schulz_bf16
    g = torch.randn(*shape, generator=torch.Generator().manual_seed(80))
    y = newton_schulz_bf16(g[None].to(DEV))[0]
    ref = R.newton_schulz5(g, 5)
    assert y.shape == shape and rel(y, ref) < 1e-2 and (y.float().cpu() - ref.float()).abs().max() <= 2 ** -7


def test_single_document_cache():
    """get_block_mask's one-document check on a device doc_id is cached per tensor object and
    version: an in-place edit or a new tensor (even at a recycled address) is re-evaluated."""
    from owl_wms.nn.attn import _single_document
    d = torch.zeros(2, 8, dtype=torch.long, device=DEV)
    assert _single_document(d, 8) and _single_document(d, 8)
    d[1, 4:] = 1
    assert not _single_document(d, 8)
    assert _single_document(d, 4)
    del d
    e = torch.zeros(2, 8, dtype=torch.long, device=DEV)
    e[0, 7] = 3
    assert not _single_document(e, 8)


# ------------------------------------------------------------ fused Muon passes (optim.hip)
def _torch_momentum(g, b, m, nesterov=True):
    """muon.py:67-73 with torch ops (the reference's own arithmetic)."""
    b = b.lerp(g, 1 - m)
    return (g.lerp(b, m) if nesterov else b), b


@pytest.mark.parametrize("count,shape,misalign", [(3, (96, 40), False), (20, (64, 24), False), (2, (33, 7), True),
                                                  (1, (4608, 1536), False)])
@pytest.mark.parametrize("nesterov", [True, False])
def test_muon_momentum_fused(count, shape, misalign, nesterov):
    """One pass = lerp + Nesterov lerp + stack + sum(bf16(g')^2), vs torch's lerp ops: fp32 within
    1 ulp-scale (2e-7 rel) -- FMA contraction may differ from ATen's lerp -- and the norm within 1e-5.
    misalign: grads at a 4-byte offset inside a flat bucket (the reducer's views), scalar path;
    count 20 > 16 spans two launches."""
    n = shape[0] * shape[1]
    gen = torch.Generator().manual_seed(7)
    flat = torch.randn(count * n + 1, generator=gen).to(DEV)
    off = 1 if misalign else 0
    grads = [flat[off + i * n: off + (i + 1) * n].view(shape) for i in range(count)]
    bufs = [torch.randn(shape, generator=gen).to(DEV) * 0.1 for _ in range(count)]
    exp = [_torch_momentum(g, b, 0.95, nesterov) for g, b in zip(grads, bufs)]
    out = torch.empty(count, n, device=DEV)
    sumsq = torch.full((count, K().NORM_PARTS), float("nan"), device=DEV)  # fully written by the pass
    g_before = [g.clone() for g in grads]
    K().muon_momentum(grads, bufs, 0.95, nesterov, out, sumsq)
    torch.cuda.synchronize()
    for i, (gp, b) in enumerate(exp):
        torch.testing.assert_close(bufs[i], b, rtol=2e-7, atol=1e-7)
        torch.testing.assert_close(out[i].view(shape), gp, rtol=2e-7, atol=1e-7)
        ss = gp.bfloat16().float().pow(2).sum()
        assert abs(sumsq[i].sum().item() / ss.item() - 1) < 1e-5
        assert torch.equal(grads[i], g_before[i])  # written to the stack, not into p.grad


@pytest.mark.parametrize("rows,cols,transpose,count", [(96, 40, False, 3), (40, 96, False, 2), (200, 72, True, 3),
                                                       (6144, 1536, True, 1), (64, 64, False, 18)])
def test_muon_apply_fused(rows, cols, transpose, count):
    """p = p*(1 - lr wd) - lr*s*u in one pass (muon.py:80-84) vs torch's mul_ + add_(alpha); u read
    from the NS iterate's transposed [cols, rows] layout when transpose."""
    gen = torch.Generator().manual_seed(9)
    ps = [torch.randn(rows, cols, generator=gen).to(DEV) for _ in range(count)]
    u = torch.randn(count, rows, cols, generator=gen).bfloat16().to(DEV)
    lr, wd = 1e-3, 0.01
    decay, alpha = 1 - lr * wd, lr * max(1, rows / cols) ** 0.5
    exp = [p.clone().mul_(decay).add_(u[i], alpha=-alpha) for i, p in enumerate(ps)]
    ua = u.transpose(1, 2).contiguous() if transpose else u
    K().muon_apply(ps, ua, rows, cols, transpose, decay, alpha)
    torch.cuda.synchronize()
    for p, e in zip(ps, exp):
        torch.testing.assert_close(p, e, rtol=2e-7, atol=1e-8)


def test_muon_step_fused_matches_unfused():
    """Muon.step on the fused passes against the same step spelled with torch ops + the
    library NS (newton_schulz_bf16), over a group mixing shapes: [96, 64] x3, [64, 96] x2 (transposed
    NS) and a zero-padded [256, 2]; two steps, so the momentum buffers carry over."""
    from owl_wms.muon import Muon, newton_schulz_bf16
    gen = torch.Generator().manual_seed(11)
    shapes = [(96, 64)] * 3 + [(64, 96)] * 2 + [(256, 2)]
    ps = [torch.nn.Parameter(torch.randn(s, generator=gen).to(DEV)) for s in shapes]
    qs = [p.detach().clone() for p in ps]
    bufs = [torch.zeros_like(q) for q in qs]
    opt = Muon(ps, lr=1e-2, momentum=0.95, rank=0, world_size=1)
    for step in range(2):
        grads = [torch.randn(s, generator=gen).to(DEV) for s in shapes]
        for p, g in zip(ps, grads):
            p.grad = g.clone()
        opt.step()
        for i, (q, g) in enumerate(zip(qs, grads)):
            gp, bufs[i] = _torch_momentum(g, bufs[i], 0.95)
            u = newton_schulz_bf16(gp[None])[0]
            r, c = q.shape
            q.mul_(1 - 1e-2 * 0.01).add_(u.float(), alpha=-1e-2 * max(1, r / c) ** 0.5)
    for p, q in zip(ps, qs):
        assert rel(p.detach(), q) < 1e-4


@pytest.mark.parametrize("eps,wd", [(1e-15, 1e-4), (1e-8, 0.01)])
def test_fused_adamw_matches_torch(eps, wd):
    """FusedAdamW (owlk_adamw) vs torch.optim.AdamW (foreach) over 3 steps on 20 tensors of mixed sizes
    (two launches of <= 16; a misaligned / odd-sized one takes the scalar path): params and both
    moments within 1e-6 relative; state_dict keys and 'step' identical."""
    from owl_wms.muon import FusedAdamW
    gen = torch.Generator().manual_seed(21)
    shapes = [(3072, 1536), (1536,), (7,), (128, 11)] + [(64, 64)] * 16
    ps = [torch.nn.Parameter(torch.randn(s, generator=gen).to(DEV)) for s in shapes]
    qs = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    kw = dict(lr=1e-3, betas=(0.9, 0.95), weight_decay=wd, eps=eps)
    fo, to = FusedAdamW(ps, **kw), torch.optim.AdamW(qs, foreach=True, **kw)
    for step in range(3):
        for p, q in zip(ps, qs):
            g = torch.randn(p.shape, generator=gen).to(DEV) * 1e-2
            p.grad, q.grad = g.clone(), g.clone()
        fo.step()
        to.step()
    torch.cuda.synchronize()
    for p, q in zip(ps, qs):
        torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-6, atol=1e-7)
        for k in ("exp_avg", "exp_avg_sq"):
            # lerp near zero cancels: compare at 1e-6 of the moment's magnitude (FMA contraction
            # in ATen's foreach kernels vs ours differs by an operand ulp)
            ref = to.state[q][k]
            torch.testing.assert_close(fo.state[p][k], ref, rtol=1e-6, atol=1e-6 * ref.abs().max().item())
        assert float(fo.state[p]["step"]) == float(to.state[q]["step"]) == 3.0
    assert fo.state_dict()["param_groups"][0].keys() == to.state_dict()["param_groups"][0].keys()


@pytest.mark.parametrize("M,N,Kd", [(64, 6144, 1536), (64, 1536, 6144), (128, 4608, 1536), (72, 256, 512),
                                    (1, 1536, 1536), (2, 3072, 128), (16, 256, 64), (40, 1536, 4608),
                                    (200, 1536, 1536), (128, 10240, 2560)])
def test_gemm_skinny_splitk_epilogues(M, N, Kd):
    """Skinny-M GEMMs (decode: one 64-token frame, a CFG pair, per-frame rows).  M <= 128 takes the
    one-launch decode plan (K chunks summed in order by each tile's last workgroup, arrival counters
    left zero), 128 < M <= 256 the split-K partials + reduce kernel.  Store + bias, SiLU + aux,
    gate + residual vs fp32 torch (bf16 output tolerance 5e-3), deterministic across runs."""
    k = K()
    from owl_wms._lib import lib
    if Kd >= 512 and M > 128:  # the split-K partials path is taken
        assert lib().owlk_gemm_splitk_bytes(M, N, Kd, 1, 0, 0, 0, k.EPI_SILU, 0.0) > 0
    tpf = 64 if M % 64 == 0 else M
    A, W = rnd(M, Kd, seed=13), rnd(N, Kd, scale=0.05, seed=14)
    bias = (torch.randn(N) * 0.1).to(DEV)
    acc = A.float() @ W.float().T
    y = (acc + bias.bfloat16().float()).bfloat16().float()
    o1 = k.gemm(A, W, bias=bias)
    assert rel(o1, y) < 5e-3
    assert torch.equal(o1, k.gemm(A, W, bias=bias))
    aux = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    s = k.gemm(A, W, bias=bias, epi=k.EPI_SILU, aux=aux)
    assert rel(aux, y) < 5e-3 and rel(s, torch.nn.functional.silu(y)) < 5e-3
    g = rnd((M + tpf - 1) // tpf, N, seed=15)
    res = rnd(M, N, seed=16)
    o = k.gemm(A, W, bias=bias, epi=k.EPI_GATE_RESID, gate=g, tpf=tpf, resid=res)
    gref = g.float().repeat_interleave(tpf, 0)[:M]
    assert rel(o, res.float() + gref * y) < 5e-3
    c0 = rnd(M, N, seed=17)
    c1 = k.gemm(A, W, out=c0.clone(), alpha=0.5, beta=1.0)  # STORE with beta: C read back
    assert rel(c1, 0.5 * acc + c0.float()) < 5e-3
    for ws in k._DECODE_WS.values():  # every launch left its arrival counters at zero
        assert int(ws[:4096].count_nonzero()) == 0


@pytest.mark.parametrize("case", [(2, 2, 12, 64, None), (1, 2, 24, 64, 16), (2, 1, 9, 4, 3), (1, 2, 7, 65, None),
                                  (1, 2, 10, 64, 4)])
@pytest.mark.parametrize("D", [64, 128])
def test_attention_packed_runs_match_general_doc_path(case, D):
    """Packed documents (contiguous runs, what the sequence-packing loader yields) through the
    range form of the mask (kv_lo / q_hi only) give the same O, lse, dQ, dK, dV as the general
    per-element document path, and match the oracle."""
    k = K()
    B, H, nf, tpf, window = case
    L = nf * tpf
    doc = torch.zeros(B, nf, dtype=torch.long)
    doc[0, 3:] = 1
    doc[0, nf - 2:] = 2
    if B > 1:
        doc[1, nf // 2:] = 7
    arrays = k.frame_arrays(doc.to(DEV), nf, window)
    assert arrays["runs"]
    q, kk, v = (rnd(B * L, H * D, seed=s).view(B, L, H * D) for s in (90, 91, 92))
    do = rnd(B * L, H * D, seed=93).view(B, L, H * D)
    res = []
    for runs in (True, False):
        mask = k.FrameMask(tpf, window, True, 0, dict(arrays, runs=runs))
        o, lse = k.attn_fwd(q, kk, v, H, D, mask)
        dq, dk, dv = (torch.empty_like(q) for _ in range(3))
        k.attn_bwd(q, kk, v, o, do, lse, H, D, mask, dq, dk, dv)
        res.append((o, lse, dq, dk, dv))
    # D = 64: the runs form's backward is the single pass (attn_bwd_fused.hip), whose dQ / dK / dV
    # differ from the two-kernel path's in fp32 summation order and the bf16 dS of the dQ product
    fused = k.fused_bwd_variant(D, k.FrameMask(tpf, window, True, 0, arrays)) is not None
    for i, (a, b) in enumerate(zip(*res)):
        assert rel(a, b) < (5e-3 if fused and i >= 2 else 1e-5)
    ref = R.attention(*(t.cpu().float().view(B, L, H, D).transpose(1, 2) for t in (q, kk, v)),
                      R.frame_mask(L, L, tpf, window, doc))
    assert rel(res[0][0].view(B, L, H, D).transpose(1, 2), ref) < 1e-2


def test_muon_multirank_path_on_gpu(monkeypatch):
    """The world_size > 1 branch of Muon.step (round-robin NS + one async all_gather per group,
    muon.py:86-115) on the HIP passes, in one process: the gather is emulated so that every slot gets
    this rank's updates, and the parameters this rank owns must equal a single-rank step of the same
    parameters."""
    import owl_wms.muon as mu
    gen = torch.Generator().manual_seed(31)
    shapes = [(96, 64), (96, 64), (96, 64)]
    p0 = [torch.randn(s, generator=gen).to(DEV) for s in shapes]
    gs = [torch.randn(s, generator=gen).to(DEV) for s in shapes]

    def run(ws, rank):
        ps = [torch.nn.Parameter(p.clone()) for p in p0]
        for p, g in zip(ps, gs):
            p.grad = g.clone()
        mu.Muon(ps, lr=1e-2, momentum=0.95, rank=rank, world_size=ws).step()
        return ps

    class Done:
        def wait(self):
            pass

    def fake_gather(out, inp):  # slot `rank` gets this rank's updates, the other slot a copy of them
        out.view(2, -1).copy_(inp.view(1, -1).expand(2, -1))
        return Done()

    monkeypatch.setattr(mu, "_all_gather_async", fake_gather)
    single = run(1, 0)
    multi = run(2, 0)  # rank 0 of 2 owns params 0 and 2 (chunks [0, 1], [2])
    for i in (0, 2):
        assert rel(multi[i].detach() - p0[i], single[i].detach() - p0[i]) < 1e-2


def test_ema_fused_matches_foreach_lerp():
    """EMA.update on owlk_ema (one multi-tensor pass) vs torch._foreach_lerp_ (the eager form of
    ema_pytorch's update): 20 tensors incl. odd sizes (scalar path) over 5 updates, within 1e-6 of
    each tensor's scale.  Schedule (ema_pytorch, update_after_step 0): update 0 copies; update 1
    copies again (sets initted) and lerps at decay 1 - 2^(-2/3) onto equal values; update t >= 2
    lerps at decay min(0.999, 1 - (1 + t)^(-2/3))."""
    from owl_wms.utils.grad_reducer import EMA
    gen = torch.Generator().manual_seed(41)
    shapes = [(3072, 1536), (1536,), (7,), (128, 11)] + [(64, 64)] * 16
    model = torch.nn.ParameterList([torch.nn.Parameter(torch.randn(s, generator=gen).to(DEV)) for s in shapes])
    ema = EMA(model, beta=0.999)
    ref = None
    for t in range(5):
        with torch.no_grad():
            for p in model:
                p.add_(torch.randn(p.shape, generator=gen).to(DEV) * 0.1)
        ema.update()
        if t <= 1:
            assert ema.initted == (t == 1)
            ref = [p.detach().clone() for p in model]
        else:
            decay = min(0.999, 1 - (1 + t) ** (-2 / 3))
            assert abs(ema.get_current_decay() - decay) < 1e-12
            torch._foreach_lerp_(ref, [p.detach() for p in model], 1.0 - decay)
    torch.cuda.synchronize()
    for a, b in zip(ema.shadow, ref):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-6 * b.abs().max().item())
    sd = ema.state_dict()
    assert int(sd["step"]) == 5 and bool(sd["initted"]) and all("ema_model." + k in sd for k, _ in
                                                                  model.named_parameters())


@pytest.mark.parametrize("F", [1, 2, 3, 4, 5])
def test_gemm_frames_few_frames(F):
    """owlk_gemm_frames on 1-5 frames (M = 64..320 frame-strided rows): such M would otherwise take
    the decode (M <= 128) or skinny split-K (M <= 256) plans, which read plain rows; the frame-strided
    form must stay on the 256^2 kernel.  A (frame rows of a joint [F x 65, 256] buffer) and C
    (frame rows of a joint output) against the dense product."""
    k = K()
    n0, n1, Kd, N = 64, 1, 256, 256
    joint = rnd(F * (n0 + n1), Kd, seed=300 + F)
    B = rnd(N, Kd, seed=310 + F)
    A = k.frame_rows(joint, n0, n1, 0, Kd)
    rows = A.reshape(F * n0, Kd)
    ref = rows.float() @ B.float().T
    got = k.gemm(A, B.T.contiguous(), b_trans=True)  # the layout the MMDiT dX GEMMs use (mask 1)
    assert rel(got, ref) < 1e-2
    out_joint = torch.zeros(F * (n0 + n1), N, device=DEV, dtype=torch.bfloat16)
    k.gemm(rows.contiguous(), B, out=k.frame_rows(out_joint, n0, n1, 0, N))
    assert rel(k.frame_rows(out_joint, n0, n1, 0, N).reshape(F * n0, N), ref) < 1e-2
    assert (out_joint.view(F, n0 + n1, N)[:, n0:] == 0).all()  # the audio rows are untouched


@pytest.mark.parametrize("k_in", [20, 37])
def test_mlp_custom_unaligned_wide_input(k_in):
    """MLPCustom (mlp.py:20-24) on an input width > 16 that is not a multiple of 8 (a ButtonEmbedding
    with more buttons than dit_v4's 11): the fc1 weight gradient takes the padded split-K path, not
    owlk_small_k_wgrad (K <= 16); fwd and all grads against fp32 torch."""
    from owl_wms.nn.mlp import MLPCustom
    torch.manual_seed(5)
    m = MLPCustom(k_in, 128, 64).cuda()
    x = torch.randn(192, k_in, device=DEV).bfloat16().requires_grad_()
    y = m(x)
    dy = torch.randn_like(y)
    y.backward(dy)
    w1, b1, w2, b2 = (t.detach().float().requires_grad_() for t in (m.fc1.weight, m.fc1.bias, m.fc2.weight, m.fc2.bias))
    xr = x.detach().float().requires_grad_()
    yr = torch.nn.functional.silu(xr @ w1.T + b1) @ w2.T + b2
    yr.backward(dy.float())
    assert rel(y, yr) < 1e-2
    for got, ref in ((x.grad, xr.grad), (m.fc1.weight.grad, w1.grad), (m.fc1.bias.grad, b1.grad),
                     (m.fc2.weight.grad, w2.grad), (m.fc2.bias.grad, b2.grad)):
        assert rel(got, ref) < 2e-2


@pytest.mark.parametrize("d,tpf,F,bias", [(1536, 64, 6, True), (128, 1, 40, False), (2560, 65, 2, True),
                                          (1536, 2, 9, True)])
def test_adaln_gate_bwd_fused_equals_two_passes(d, tpf, F, bias):
    """owlk_adaln_gate_bwd: the AdaLN backward and the gate backward on its dx in one pass, bit for bit
    the two separate kernels (dx, dscale | dshift, the gated dy, dg, the bias partials)."""
    k = K()
    T = F * tpf
    x = rnd(T, d, seed=40)
    mod = rnd(F, 2 * d, scale=0.3, seed=41)
    _, rstd = k.adaln_fwd(x, mod[:, :d], mod[:, d:], tpf)
    dh, dres, y = rnd(T, d, seed=42), rnd(T, d, seed=43), rnd(T, d, seed=44)
    g = rnd(F, d, seed=45)
    dm0 = torch.zeros(F, 3 * d, device=DEV, dtype=torch.bfloat16)
    dm1 = torch.zeros_like(dm0)
    dx0 = k.adaln_bwd_into(dh, x, rstd, mod[:, :d], tpf, dm0[:, d:], dres=dres)
    dy0, _, dbf0 = k.gate_bwd(dx0, y, g, tpf, want_bias=bias, dg_out=dm0[:, :d])
    dx1, dy1, dbf1 = k.adaln_gate_bwd_into(dh, x, rstd, mod[:, :d], tpf, dm1[:, d:], dres, y, g, dm1[:, :d],
                                           want_bias=bias)
    assert torch.equal(dx0, dx1) and torch.equal(dy0, dy1) and torch.equal(dm0, dm1)
    assert (dbf0 is None and dbf1 is None) or torch.equal(dbf0, dbf1)
