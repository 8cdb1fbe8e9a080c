"""Typed Python wrappers over libowlk (include/owlk.h).  Device tensors in, device tensors out.

Every function checks shapes/strides on the host before the launch (a kernel never sees an
operand its grid does not cover) and enqueues on torch's current HIP stream.
"""
import ctypes
import os

import torch
from torch.autograd.graph import increment_version

from . import _lib
from ._lib import call, lib, ptr, stream

BF16, F32 = torch.bfloat16, torch.float32

EPI_STORE, EPI_SILU, EPI_GATE_RESID, EPI_DSILU, EPI_AXPBY, EPI_SCALE2 = 0, 1, 2, 3, 4, 5


def _rowmajor(t, name):
    assert t.dim() == 2 and t.stride(1) == 1, f"{name} must be a row-major 2-D view (got {t.shape}/{t.stride()})"
    assert t.dtype == BF16, f"{name} must be bf16"
    return t


FRAME_ROWS = 64  # OWLK_FRAME_ROWS: rows per frame of a frame-strided operand


def frame_rows(joint, n0, n1, col0, cols):
    """The video rows of an MMDiT joint-sequence buffer (frame f = [n0 video | n1 audio] rows,
    mmattn.py:54-60) as a [F, n0, cols] view: row r of the video operand is joint row
    (r // n0) (n0 + n1) + r % n0.  libowlk's GEMM / column-sum entries read and write such frame-strided
    rows in place (owlk_gemm_frames), so no interleave / split copy of the joint buffer is made."""
    assert n0 == FRAME_ROWS and joint.dim() == 2 and joint.stride(1) == 1
    F_ = joint.shape[0] // (n0 + n1)
    return joint.view(F_, n0 + n1, joint.shape[1])[:, :n0, col0:col0 + cols]


def _operand(t, name):
    """2-D row-major view -> (rows, cols, ld, 0); 3-D frame_rows view [F, 64, cols] -> (F*64, cols,
    row stride, frame stride)."""
    if t.dim() == 3:
        assert t.shape[1] == FRAME_ROWS and t.stride(2) == 1 and t.dtype == BF16, f"{name}: frame rows view"
        return t.shape[0] * FRAME_ROWS, t.shape[2], t.stride(1), t.stride(0)
    _rowmajor(t, name)
    return t.shape[0], t.shape[1], t.stride(0), 0


def _gemm_frames(A, B, out, a_trans, b_trans, out_f32, epi, alpha, beta, bias, aux, gate, tpf, resid):
    """gemm() with frame-strided operand rows (3-D frame_rows views): owlk_gemm_frames."""
    ra, ca, lda, afs = _operand(A, "A")
    rb, cb, ldb, bfs = _operand(B, "B")
    M, K = (ca, ra) if a_trans else (ra, ca)
    N, Kb = (cb, rb) if b_trans else (rb, cb)
    assert K == Kb, f"gemm: K mismatch {K} vs {Kb}"
    if out is None:
        out = torch.empty(M, N, device=A.device, dtype=F32 if out_f32 else BF16)
    if out.dim() == 3:
        rc, cc, ldc, cfs = _operand(out, "out")
    else:
        assert out.dim() == 2 and out.stride(1) == 1
        rc, cc, ldc, cfs = out.shape[0], out.shape[1], out.stride(0), 0
    assert (rc, cc) == (M, N) and out.dtype == (F32 if out_f32 else BF16)
    if bias is not None:
        assert bias.dtype == F32 and bias.numel() == N and bias.is_contiguous()
    for t, nm in ((aux, "aux"), (resid, "resid")):
        if t is not None:
            assert t.shape == (M, N) and t.stride(1) == 1 and t.dtype == BF16, nm
    if gate is not None:
        assert gate.dim() == 2 and gate.shape[1] == N and gate.stride(1) == 1 and gate.shape[0] * tpf >= M
    ws_bytes = lib().owlk_gemm_ws_bytes(M, N, K, 1, int(a_trans), int(b_trans), int(out_f32), epi, float(beta), 0)
    ws = torch.empty(ws_bytes, device=out.device, dtype=torch.uint8) if ws_bytes > 0 else None
    call("owlk_gemm_frames", M, N, K, ptr(A), lda, afs, int(a_trans), ptr(B), ldb, bfs, int(b_trans),
         ptr(out), ldc, cfs, int(out_f32), epi, float(alpha), float(beta), ptr(bias),
         ptr(aux), aux.stride(0) if aux is not None else 0, ptr(gate), gate.stride(0) if gate is not None else 0,
         int(tpf), ptr(resid), resid.stride(0) if resid is not None else 0, ptr(ws), ws_bytes, stream(),
         key=f"gemm<256f,{int(a_trans)}{int(b_trans)},epi{epi},{'f32' if out_f32 else 'bf16'}>[{M}x{N}x{K}]",
         flops=lambda: 2.0 * M * N * K)
    return out


def gemm(A, B, *, a_trans=False, b_trans=False, out=None, out_f32=False, epi=EPI_STORE, alpha=1.0, beta=0.0,
         bias=None, aux=None, gate=None, tpf=1, resid=None, colsum=None):
    """C[m, n] = epi(sum_k A(m, k) B(n, k)) for 2-D views.

    A: [M, K] (a_trans False) or [K, M] (a_trans True); B: [N, K] or [K, N] (b_trans True).
    A, B or out may instead be 3-D frame_rows views (frame-strided rows, the MMDiT joint layout).
    colsum: optional fp32 [N], += column sums of the stored bf16 C (fused into the DSILU epilogue).
    With epi=EPI_DSILU a given resid is an OUTPUT: resid = bf16(silu(aux)).
    """
    if A.dim() == 3 or B.dim() == 3 or (out is not None and out.dim() == 3):
        assert colsum is None
        return _gemm_frames(A, B, out, a_trans, b_trans, out_f32, epi, alpha, beta, bias, aux, gate, tpf, resid)
    _rowmajor(A, "A")
    _rowmajor(B, "B")
    M, K = (A.shape[1], A.shape[0]) if a_trans else (A.shape[0], A.shape[1])
    N, Kb = (B.shape[1], B.shape[0]) if b_trans else (B.shape[0], B.shape[1])
    assert K == Kb, f"gemm: K mismatch {K} vs {Kb}"
    if out is None:
        out = torch.empty(M, N, device=A.device, dtype=F32 if out_f32 else BF16)
    assert out.shape == (M, N) and out.stride(1) == 1
    assert out.dtype == (F32 if out_f32 else BF16)
    if bias is not None:
        assert bias.dtype == F32 and bias.numel() == N and bias.is_contiguous()
    for t, nm in ((aux, "aux"), (resid, "resid")):
        if t is not None:
            assert t.shape == (M, N) and t.stride(1) == 1 and t.dtype == BF16, nm
    if gate is not None:
        assert gate.dim() == 2 and gate.shape[1] == N and gate.stride(1) == 1 and gate.shape[0] * tpf >= M
    if colsum is not None:
        assert colsum.dtype == F32 and colsum.numel() == N and colsum.is_contiguous() and not out_f32
    tile = 64 if ((M + 127) // 128) * ((N + 127) // 128) < 512 else 128
    # split-K partials (weight gradients, skinny-M decode) and column-sum partials: the workspace of
    # the deterministic form comes from torch's caching allocator (the library never allocates);
    # stream order keeps it alive for the launch
    ws, ws_bytes = None, 0
    if (out_f32 and K >= 8192) or (M <= 256 and not out_f32) or colsum is not None:
        ws_bytes = lib().owlk_gemm_ws_bytes(M, N, K, 1, int(a_trans), int(b_trans), int(out_f32), epi, float(beta),
                                            int(colsum is not None))
        if ws_bytes > 0:
            stateful = M <= 128 and not out_f32 and lib().owlk_gemm_ws_counter_bytes(
                M, N, K, 1, int(a_trans), int(b_trans), int(out_f32), epi, float(beta)) > 0
            ws = _decode_ws(A.device, ws_bytes) if stateful else \
                torch.empty(ws_bytes, device=A.device, dtype=torch.uint8)
    call("owlk_gemm", M, N, K, 1,
         ptr(A), A.stride(0), 0, int(a_trans),
         ptr(B), B.stride(0), 0, int(b_trans),
         ptr(out), out.stride(0), 0, int(out_f32),
         epi, float(alpha), float(beta), ptr(bias),
         ptr(aux), aux.stride(0) if aux is not None else 0, 0,
         ptr(gate), gate.stride(0) if gate is not None else 0, 0, int(tpf),
         ptr(resid), resid.stride(0) if resid is not None else 0, 0,
         ptr(colsum), ptr(ws), ws_bytes, stream(), key=f"gemm<{tile},{int(a_trans)}{int(b_trans)},epi{epi},{'f32' if out_f32 else 'bf16'}>[{M}x{N}x{K}]",
         flops=lambda: 2.0 * M * N * K)
    return out


_DECODE_WS = {}
_DECODE_WS_RETIRED = []  # replaced decode workspaces (zeroed counters), kept for captured graphs


def _decode_ws(device, nbytes):
    """The decode GEMM plan's workspace (M <= 128 rows): its first 4 KiB are per-tile arrival
    counters that must be zero on entry and that every launch leaves zero (owlk.h, owlk_gemm), so
    one zero-initialised buffer is kept per device and reused; it grows by reallocation.  Decode
    GEMMs therefore must not run concurrently on two streams of one device (the samplers issue them
    on one stream, eagerly or by graph replay).  Under graph capture a too-small buffer is replaced
    by a captured zero-fill of a fresh one."""
    key = torch.device(device)
    buf = _DECODE_WS.get(key)
    if buf is None or buf.numel() < nbytes:
        fresh = torch.zeros(max(nbytes, 1 << 20), device=device, dtype=torch.uint8)
        if torch.cuda.is_current_stream_capturing():
            return fresh
        if buf is not None:
            # a HIP graph captured earlier may still hold the old buffer's address (the samplers'
            # step graph outlives eager forwards between replays): keep it alive, never free it
            _DECODE_WS_RETIRED.append(buf)
        _DECODE_WS[key] = buf = fresh
    return buf


def gemm_wgrad(dy, x):
    """fp32 weight gradient dW[n, k] = sum_m dy[m, n] x[m, k] (split-K over the token dimension);
    dy / x may be frame_rows views."""
    out = torch.empty(dy.shape[-1], x.shape[-1], device=dy.device, dtype=F32)
    return gemm(dy, x, a_trans=True, b_trans=True, out=out, out_f32=True, beta=0.0)


def bgemm(A, B, out, *, a_trans=False, b_trans=False, epi=EPI_STORE, alpha=1.0, beta=0.0, aux=None):
    """Batched GEMM over dim 0 of 3-D row-major tensors (Newton-Schulz)."""
    bt = A.shape[0]
    M, K = (A.shape[2], A.shape[1]) if a_trans else (A.shape[1], A.shape[2])
    N, Kb = (B.shape[2], B.shape[1]) if b_trans else (B.shape[1], B.shape[2])
    assert K == Kb and out.shape == (bt, M, N)
    for t in (A, B, out) + ((aux,) if aux is not None else ()):
        assert t.dtype == BF16 and t.is_contiguous()
    call("owlk_gemm", M, N, K, bt,
         ptr(A), A.stride(1), A.stride(0), int(a_trans),
         ptr(B), B.stride(1), B.stride(0), int(b_trans),
         ptr(out), out.stride(1), out.stride(0), 0,
         epi, float(alpha), float(beta), None,
         ptr(aux), aux.stride(1) if aux is not None else 0, aux.stride(0) if aux is not None else 0,
         None, 0, 0, 1, None, 0, 0, None, None, 0, stream())
    return out


def adaln_fwd(x, scale, shift, tpf, act=False):
    """x [T, d] bf16; scale/shift [F, d] views (row stride ldm) -> y [T, d], rstd [T] (, silu(y))."""
    T, d = x.shape
    assert x.stride(1) == 1 and scale.stride(1) == 1 and shift.stride(1) == 1
    assert scale.stride(0) == shift.stride(0) and scale.shape[0] * tpf == T
    y = torch.empty(T, d, device=x.device, dtype=BF16)
    ya = torch.empty_like(y) if act else None
    rstd = torch.empty(T, device=x.device, dtype=F32)
    call("owlk_adaln_fwd", ptr(x), x.stride(0), ptr(scale), ptr(shift), scale.stride(0), tpf, T, d, ptr(y), d,
         ptr(rstd), ptr(ya), stream())
    return (y, rstd, ya) if act else (y, rstd)


def adaln_bwd(dy, x, rstd, scale, tpf, dres=None, ypre=None):
    """-> dx [T, d] bf16 (+ dres), dmod [F, 2d] fp32 (= [dscale | dshift])."""
    T, d = x.shape
    F_ = T // tpf
    dx = torch.empty(T, d, device=x.device, dtype=BF16)
    dmod = torch.empty(F_, 2 * d, device=x.device, dtype=F32)
    call("owlk_adaln_bwd", ptr(dy), dy.stride(0), ptr(x), x.stride(0), ptr(rstd), ptr(scale), scale.stride(0), tpf,
         T, d, ptr(dres), dres.stride(0) if dres is not None else 0, ptr(dx), d, ptr(dmod), ptr(dmod[:, d:]), 2 * d,
         ptr(ypre), 0, stream())
    return dx, dmod


def adaln_bwd_into(dy, x, rstd, scale, tpf, dmod, dres=None, ypre=None):
    """adaln_bwd writing [dscale | dshift] as bf16 straight into dmod (a [F, 2d] bf16 view of a
    modulation-gradient matrix, any row stride) -> dx [T, d] bf16."""
    T, d = x.shape
    assert dmod.dtype == BF16 and dmod.shape == (T // tpf, 2 * d) and dmod.stride(1) == 1
    dx = torch.empty(T, d, device=x.device, dtype=BF16)
    call("owlk_adaln_bwd", ptr(dy), dy.stride(0), ptr(x), x.stride(0), ptr(rstd), ptr(scale), scale.stride(0), tpf,
         T, d, ptr(dres), dres.stride(0) if dres is not None else 0, ptr(dx), d, ptr(dmod), ptr(dmod[:, d:]),
         dmod.stride(0), ptr(ypre), 1, stream())
    return dx


# the DiT / MMDiT blocks' MLP-branch AdaLN backward with the attention gate's backward in one pass
# (owlk_adaln_gate_bwd); OWLK_ADALN_GATE=0 runs the two passes (same bits), for A/B runs
ADALN_GATE = os.environ.get("OWLK_ADALN_GATE", "1") != "0"


def adaln_gate_bwd_into(dy, x, rstd, scale, tpf, dmod, dres, y, g, dg_out, want_bias=True):
    """adaln_bwd_into followed by gate_bwd on its dx, in one pass (dx is not read back): ->
    dx [T, d] bf16, the gate backward's dy [T, d] bf16, per-frame bias partials [F, d] fp32 (or None);
    dg lands bf16 in dg_out.  Bit for bit the two separate calls."""
    T, d = x.shape
    F_ = T // tpf
    assert dmod.dtype == BF16 and dmod.shape == (F_, 2 * d) and dmod.stride(1) == 1
    assert dg_out.dtype == BF16 and dg_out.shape == (F_, d) and dg_out.stride(1) == 1
    assert y.shape == (T, d) and y.stride(1) == 1 and g.shape == (F_, d) and g.stride(1) == 1
    dx = torch.empty(T, d, device=x.device, dtype=BF16)
    dyg = torch.empty(T, d, device=x.device, dtype=BF16)
    dbf = torch.empty(F_, d, device=x.device, dtype=F32) if want_bias else None
    call("owlk_adaln_gate_bwd", ptr(dy), dy.stride(0), ptr(x), x.stride(0), ptr(rstd), ptr(scale), scale.stride(0),
         tpf, T, d, ptr(dres), dres.stride(0) if dres is not None else 0, ptr(dx), d, ptr(dmod), ptr(dmod[:, d:]),
         dmod.stride(0), 1, ptr(y), y.stride(0), ptr(g), g.stride(0), ptr(dyg), d, ptr(dg_out), dg_out.stride(0), 1,
         ptr(dbf), d, stream())
    return dx, dyg, dbf


def gate_bwd(dout, y, g, tpf, want_bias=True, dg_out=None):
    """-> dy [T, d] bf16, dg [F, d] fp32 (or written as bf16 into dg_out, a [F, d] bf16 view of a
    modulation-gradient matrix), per-frame bias partials [F, d] fp32 (or None)."""
    T, d = y.shape
    F_ = T // tpf
    dy = torch.empty(T, d, device=y.device, dtype=BF16)
    if dg_out is None:
        dg = torch.empty(F_, d, device=y.device, dtype=F32)
    else:
        assert dg_out.dtype == BF16 and dg_out.shape == (F_, d) and dg_out.stride(1) == 1
        dg = dg_out
    dbf = torch.empty(F_, d, device=y.device, dtype=F32) if want_bias else None
    call("owlk_gate_bwd", ptr(dout), dout.stride(0), ptr(y), y.stride(0), ptr(g), g.stride(0), tpf, T, d, ptr(dy), d,
         ptr(dg), dg.stride(0), int(dg.dtype == BF16), ptr(dbf), d, stream())
    return dy, dg, dbf


def gate_resid(x, y, g, tpf):
    """bf16(x + bf16(g[t / tpf] * y)) for [T, d] row views (the GATE_RESID epilogue, recomputed)."""
    T, d = x.shape
    for t in (x, y, g):
        assert t.dtype == BF16 and t.stride(1) == 1
    assert y.shape == (T, d) and g.shape[1] == d and g.shape[0] * tpf == T
    out = torch.empty(T, d, device=x.device, dtype=BF16)
    call("owlk_gate_resid", ptr(x), x.stride(0), ptr(y), y.stride(0), ptr(g), g.stride(0), tpf, T, d, ptr(out), d,
         stream())
    return out


def qk_rope_fwd(qkv, H, D, cos, sin, tab_off=0, tpos_div=0):
    """qkv [T, 3 H D] -> out [T, 2 H D] (rotated q | k), rstd [T, 2H]."""
    T = qkv.shape[0]
    out = torch.empty(T, 2 * H * D, device=qkv.device, dtype=BF16)
    rstd = torch.empty(T, 2 * H, device=qkv.device, dtype=F32)
    call("owlk_qk_rope_fwd", ptr(qkv), qkv.stride(0), T, H, D, ptr(cos), ptr(sin), cos.stride(0), cos.shape[0],
         tab_off, tpos_div, ptr(out), out.stride(0), ptr(rstd), stream())
    return out, rstd


def gemm_qk_rope(h, w, bias, H, D, cos, sin, tab_off=0, tpos_div=0):
    """qkv = h @ w^T + bias [M, 3 H D] bf16 and qk_rope_fwd(qkv, ...) -> (qkv, out, rstd); one launch on
    the 256^2 ping-pong kernel's shapes (owlk_gemm_qk_rope), the same bits as the two calls."""
    M, K_ = h.shape
    N = w.shape[0]
    assert w.shape[1] == K_ and N == 3 * H * D and h.dtype == BF16 and w.dtype == BF16
    assert h.stride(1) == 1 and w.stride(1) == 1 and cos.stride(1) == 1 and sin.stride(0) == cos.stride(0)
    assert bias is None or (bias.dtype == F32 and bias.is_contiguous())
    qkv = torch.empty(M, N, device=h.device, dtype=BF16)
    out = torch.empty(M, 2 * H * D, device=h.device, dtype=BF16)
    rstd = torch.empty(M, 2 * H, device=h.device, dtype=F32)
    call("owlk_gemm_qk_rope", M, N, K_, ptr(h), h.stride(0), ptr(w), w.stride(0), ptr(bias), ptr(qkv), N, H, D,
         ptr(cos), ptr(sin), cos.stride(0), cos.shape[0], tab_off, tpos_div, ptr(out), out.stride(0), ptr(rstd),
         stream(), key="gemm_qk_rope", flops=2.0 * M * N * K_)
    return qkv, out, rstd


def qk_rope_fwd_kv(qkv, B, L, H, D, cos, sin, tab_off, q_out, k_out, v_out):
    """Decode form: qkv [B L, 3 H D] -> rotated q into q_out [B, L, H D], rotated k into k_out and
    v copied into v_out (views of the KV cache's slots; any row / batch strides)."""
    for t, nm in ((q_out, "q_out"), (k_out, "k_out"), (v_out, "v_out")):
        assert t.shape == (B, L, H * D) and t.stride(2) == 1 and t.dtype == BF16, nm
    call("owlk_qk_rope_fwd_kv", ptr(qkv), qkv.stride(0), B * L, L, H, D, ptr(cos), ptr(sin), cos.stride(0),
         cos.shape[0], tab_off, ptr(q_out), q_out.stride(1), q_out.stride(0), ptr(k_out), k_out.stride(1), k_out.stride(0),
         ptr(v_out), v_out.stride(1), v_out.stride(0), stream())


def qk_rope_fwd_kv_dev(qkv, B, L, H, D, cos, sin, state, q_out, kbuf, vbuf):
    """qk_rope_fwd_kv with the cache position on the device (state int64 {start, cached, offset}):
    k / v go to rows start + cached + t of the cache buffers kbuf / vbuf [B, cap, H D]."""
    assert state.dtype == torch.int64 and state.numel() >= 3 and state.is_cuda
    assert q_out.shape == (B, L, H * D) and q_out.stride(2) == 1
    for t in (kbuf, vbuf):
        assert t.dim() == 3 and t.shape[0] == B and t.shape[2] == H * D and t.stride(2) == 1 and t.dtype == BF16
    assert kbuf.shape[1] == vbuf.shape[1]
    call("owlk_qk_rope_fwd_kv_dev", ptr(qkv), qkv.stride(0), B * L, L, H, D, ptr(cos), ptr(sin), cos.stride(0),
         cos.shape[0], ptr(state), ptr(q_out), q_out.stride(1), q_out.stride(0), ptr(kbuf), kbuf.stride(1),
         kbuf.stride(0), ptr(vbuf), vbuf.stride(1), vbuf.stride(0), kbuf.shape[1], stream())


def decode_dev_supported(D, L):
    """owlk_attn_decode_fwd's shapes: head_dim 64 or 128, one frame of at most 64 query rows."""
    return D in (64, 128) and 0 < L <= 64


def attn_decode_fwd(q, kbuf, vbuf, H, D, state, Lnew, window_tokens=0, scale=None, score_bound=0.0):
    """Decode attention over the cache buffers with the cache position on the device (state, see
    qk_rope_fwd_kv_dev): q [B, Lq <= 64, H D] against [cache | Lnew new rows] (or its last
    window_tokens rows) -> o [B, Lq, H D], lse [B, H, Lq] (base 2)."""
    B, Lq, _ = q.shape
    assert decode_dev_supported(D, Lq), f"attn_decode_fwd: head_dim {D} / {Lq} query rows not supported"
    o = torch.empty_like(q)
    lse = torch.empty(B, H, Lq, device=q.device, dtype=F32)
    call("owlk_attn_decode_fwd", ptr(q), q.stride(1), q.stride(0), ptr(kbuf), kbuf.stride(1), kbuf.stride(0),
         ptr(vbuf), vbuf.stride(1), vbuf.stride(0), ptr(o), o.stride(1), o.stride(0), ptr(lse), B, H, Lq, D,
         float(scale if scale is not None else D ** -0.5), float(score_bound), ptr(state), Lnew, window_tokens,
         min(kbuf.shape[1], vbuf.shape[1]), stream())
    return o, lse


def qk_rope_bwd(dqk, qkv, rstd, H, D, cos, sin, dqkv, tab_off=0, tpos_div=0, dbias=None):
    """-> dqkv[:, :2HD]; with dbias (fp32 [2HD]) also dbias += column sums of those outputs (the q / k
    part of the qkv bias gradient), fused into the same pass where the shape allows."""
    T = qkv.shape[0]
    args = (ptr(dqk), dqk.stride(0), ptr(qkv), qkv.stride(0), T, H, D, ptr(cos), ptr(sin), cos.stride(0),
            cos.shape[0], tab_off, tpos_div, ptr(rstd), ptr(dqkv), dqkv.stride(0))
    nb = lib().owlk_qk_rope_bwd_ws_bytes(T, H, D) if dbias is not None else 0
    if nb > 0:
        assert dbias.dtype == F32 and dbias.is_contiguous() and dbias.numel() == 2 * H * D
        ws = torch.empty(nb, device=qkv.device, dtype=torch.uint8)
        call("owlk_qk_rope_bwd_bias", *args, ptr(dbias), ptr(ws), nb, stream())
        return
    call("owlk_qk_rope_bwd", *args, stream())
    if dbias is not None:
        colsum(dqkv[:, :2 * H * D], out=dbias)


class FrameMask:
    """Host-side description of the reference frame mask (attn.py:24-62) for the kernels."""

    def __init__(self, tpf, window=None, causal=True, q_offset=0, arrays=None):
        self.tpf, self.window, self.causal, self.q_offset = int(tpf), window, bool(causal), int(q_offset)
        self.arrays = arrays  # dict kv_lo, q_hi, run_start, doc: int32 [B, n_frames] or None

    def args(self):
        a = self.arrays
        w = 0 if self.window is None else int(self.window)
        if a is None:
            return (self.tpf, w, int(self.causal), None, None, None, None, 0)
        if a.get("runs") and self.causal:  # packed documents: kv_lo / q_hi alone describe the mask
            return (self.tpf, w, 1, ptr(a["kv_lo"]), ptr(a["q_hi"]), None, None, a["doc"].stride(0))
        return (self.tpf, w, int(self.causal), ptr(a["kv_lo"]), ptr(a["q_hi"]), ptr(a["run_start"]), ptr(a["doc"]),
                a["doc"].stride(0))


def frame_arrays(doc_id, n_frames, window, causal=True):
    """Per-frame helper arrays for a [B, n_frames] doc_id (any integer ids, runs or not)."""
    B = doc_id.shape[0]
    dev = doc_id.device
    doc = doc_id[:, :n_frames].to(torch.int64)
    idx = torch.arange(n_frames, device=dev).expand(B, n_frames)
    boundary = torch.ones_like(doc, dtype=torch.bool)
    boundary[:, 1:] = doc[:, 1:] != doc[:, :-1]
    run_start = torch.cummax(torch.where(boundary, idx, torch.zeros_like(idx)), dim=1).values
    # first / last occurrence of each frame's doc id (documents need not be contiguous)
    first = torch.empty_like(doc)
    last = torch.empty_like(doc)
    dense = torch.empty_like(doc)  # ids renumbered 0..k-1 per sample, so any int64 id fits int32
    for b in range(B):
        _, inv = torch.unique(doc[b], return_inverse=True)
        dense[b] = inv
        k = int(inv.max().item()) + 1
        fo = torch.full((k,), n_frames, device=dev, dtype=torch.int64).scatter_reduce(0, inv, idx[b], "amin")
        lo = torch.full((k,), -1, device=dev, dtype=torch.int64).scatter_reduce(0, inv, idx[b], "amax")
        first[b], last[b] = fo[inv], lo[inv]
    if window is None:
        kv_lo = first
        q_hi = last
    else:
        kv_lo = torch.maximum(first, idx - window + 1)
        q_hi = torch.minimum(last, idx + window - 1)
    if not causal:
        pass  # kernels widen the kv range symmetrically from the window themselves
    i32 = torch.int32
    # every document one contiguous run of frames (sequence packing always gives this): the
    # kernels then take the range form of the mask (attn_common.hpp runs_mode)
    runs = bool((first == run_start).all())
    return {"runs": runs, "kv_lo": kv_lo.to(i32).contiguous(), "q_hi": q_hi.to(i32).contiguous(),
            "run_start": run_start.to(i32).contiguous(), "doc": dense.to(i32).contiguous()}


def _v3(t, name):
    assert t.dim() == 3 and t.stride(2) == 1 and t.dtype == BF16, f"{name}: need a [B, L, cols] bf16 view"
    return t


# |q.k| bound for QK-RMSNorm'd q, k (attn.py:84): |q| = |k| = sqrt(D) up to bf16 rounding of the
# normalised, rotated values (<= 2^-8 relative each); 2 % margin.
def qk_norm_bound(D):
    return 0.0 if os.environ.get("OWLK_NO_SCORE_BOUND") else 1.02 * D


def attn_fwd(q, k, v, H, D, mask, scale=None, o=None, score_bound=0.0):
    """Frame-masked flash attention.  q [B, Lq, >=H*D], k/v [B, Lkv, >=H*D] token-major views
    (head h at columns h*D); returns o [B, Lq, H*D] bf16 and lse [B, H, Lq] fp32.
    score_bound > 0 promises |q.k| <= score_bound (see qk_norm_bound): fixed-offset softmax."""
    _v3(q, "q"), _v3(k, "k"), _v3(v, "v")
    B, Lq, Lkv = q.shape[0], q.shape[1], k.shape[1]
    assert k.shape[0] == B and v.shape[:2] == k.shape[:2]
    scale = D ** -0.5 if scale is None else scale
    if o is None:
        o = torch.empty(B, Lq, H * D, device=q.device, dtype=BF16)
    _v3(o, "o")
    lse = torch.empty(B, H, Lq, device=q.device, dtype=F32)
    call("owlk_attn_fwd", ptr(q), q.stride(1), q.stride(0), ptr(k), k.stride(1), k.stride(0),
         ptr(v), v.stride(1), v.stride(0), ptr(o), o.stride(1), o.stride(0), ptr(lse), B, H, Lq, Lkv, D,
         float(scale), float(score_bound), mask.tpf, 0 if mask.window is None else int(mask.window),
         int(mask.causal), mask.q_offset, *mask.args()[3:], stream(), key=f"attn_fwd[w{mask.window}]", flops=lambda: 4.0 * D * H * B * mask_pairs(mask, Lq, Lkv))
    return o, lse


_BWD_SIDE = {}


def _bwd_side_stream(device, D, mask):
    """A side stream for the dQ kernel, or None to run it after dK/dV on the caller's stream.
    The two kernels are independent given delta (different outputs, shared read-only inputs).
    Run side by side only where that measured faster (`tools/attn_bench.py --bwd-only`, same
    process, interleaved; profiles/r2s_attn_bwd_side_stream.log): D 128 global layers, 20 heads x
    98,304 tokens, 170.9 -> 161.8 ms (the one-wave-per-SIMD dK/dV leaves room for dQ workgroups).
    D 64 global layers went 86.2 -> 89.1 ms and D 128 windowed ones did not move. D 64 window-16
    layers gained in isolation (2.36 -> 2.33 ms) but the whole dit_v4 step lost 0.3 % with them
    side by side (bench.py, two interleaved pairs, profiles/r2t_bench_side_stream_ab.log), so
    everything but D 128 global stays serial. OWLK_BWD_SIDE_STREAM=0 / 1 forces serial /
    side-by-side. Serial while a profile window is open (its events time launches on the current
    stream) or a graph is being captured."""
    env = os.environ.get("OWLK_BWD_SIDE_STREAM")
    on = (D == 128 and mask.window is None) if env is None else env == "1"
    if not on or _lib.profiling() or torch.cuda.is_current_stream_capturing():
        return None
    s = _BWD_SIDE.get(device)
    if s is None:
        s = _BWD_SIDE[device] = torch.cuda.Stream(device=device)
    return s


FUSED_FAIL_TEST = False


def fused_bwd_variant(D, mask):
    """owlk_attn_bwd_fused variant for this layer, or None for the two-kernel backward.  The single
    pass serves head_dim 64 with a document-free mask, windowed or not (dit_v4's layers), and causal
    masks of packed documents (every document one run of frames: sequence packing; OWLK_BWD_FUSED_DOCS
    = 0 sends those to the two kernels);
    OWLK_BWD_FUSED = 0 turns it off, 1 takes the write-through hand-off, 2 (default) keeps each
    chain's dQ sums in one XCD's L2 (the library runs it write-through on a device without 8 XCCs;
    include/owlk.h)."""
    env = os.environ.get("OWLK_BWD_FUSED", "2")
    if env == "0" or D != 64 or mask.q_offset != 0:
        return None
    if mask.arrays is not None and not (mask.arrays.get("runs") and mask.causal
                                        and os.environ.get("OWLK_BWD_FUSED_DOCS", "1") != "0"):
        return None
    # windowed layers too, unless OWLK_BWD_FUSED_LOCAL = 0
    if mask.window is not None and os.environ.get("OWLK_BWD_FUSED_LOCAL", "1") == "0":
        return None
    # OWLK_BWD_FUSED_GROUP: chains of an XCD queue swept at a time (variant bits 2-5; 0 = all);
    # one at a time (default) gives each chain the XCD's 32 workgroups: -2 % time and -54 % HBM
    # traffic against all three of dit_v4's at once (profiles/r4j_ab.log)
    group = int(os.environ.get("OWLK_BWD_FUSED_GROUP", "1"))
    # OWLK_BWD_FUSED_W4 (variant bit 7): the one-wave-per-SIMD kernel with the hand-placed step
    # (attn_bwd_fused4.hip) -- "long" (default; "global" is the same): layers without a window or with
    # windows of >= 8,192 tokens (its per-item fixed cost loses on short sweeps: mmdit_v2-like tpf 65,
    # 24 heads x 1000 frames: window 256 frames 15.41 -> 14.90 ms, window 64 4.69 -> 4.77, window 16
    # 1.52 -> 1.88, profiles/r6ah_mmdit_w4.log), "1": every layer, "0": none
    w4env = os.environ.get("OWLK_BWD_FUSED_W4", "long")
    # packed documents stay on the 8-wave kernel (the W4 steady-run statement does not cover them)
    long_sweep = (mask.window is None or int(mask.window) * int(mask.tpf) >= 8192) and mask.arrays is None
    w4 = 128 if (w4env == "1" or (w4env in ("long", "global") and long_sweep)) else 0
    # FUSED_FAIL_TEST (tests only, set through monkeypatch; variant bit 6): chain 0's block-1 hand-off
    # waits time out, so the error path -- the error word and NaN dQ rows -- is exercised through
    # this entry.  A module attribute, not an environment variable: one left exported would turn
    # every training step's dQ into NaN
    fail = 64 if FUSED_FAIL_TEST else 0
    return (1 if env == "2" else 0) | (group & 15) << 2 | fail | w4


def attn_bwd_fused(q, k, v, do, lse, delta, H, D, mask, dq, dk, dv, scale, variant=0, ws=None):
    """One pass of owlk_attn_bwd_fused (the caller has delta); returns the workspace (its fp32 dQ
    sums and hand-off flags: tests read them in the counting variant)."""
    B, L = q.shape[:2]
    nb = lib().owlk_attn_bwd_fused_ws_bytes(B, H, L, D)
    assert nb > 0, "attn_bwd_fused: shape not supported"
    if ws is None:
        ws = torch.empty(nb, device=q.device, dtype=torch.uint8)
    call("owlk_attn_bwd_fused", ptr(q), q.stride(1), q.stride(0), ptr(k), k.stride(1), k.stride(0),
         ptr(v), v.stride(1), v.stride(0), ptr(do), do.stride(1), do.stride(0), ptr(lse), ptr(delta),
         ptr(dq), dq.stride(1), dq.stride(0), ptr(dk), dk.stride(1), dk.stride(0),
         ptr(dv), dv.stride(1), dv.stride(0), B, H, L, D, float(scale),
         *mask.args(), ptr(ws), ws.numel(), int(variant), stream(),
         key=f"attn_bwd_fused[w{mask.window}{'d' if mask.arrays is not None else ''}]", flops=lambda: 8.0 * D * H * B * mask_pairs(mask, L, L))
    return ws


def gemm_attn_delta(dy, w, o, H, D, L):
    """dO = dy @ w (w: the out-projection weight [out, in], bf16) and delta [M / L, H, L] fp32 =
    rowsum(dO * O) per head (the attention backward's softmax term) -> (dO [M, H D] bf16, delta);
    one launch on the 256^2 ping-pong kernel's shapes (owlk_gemm_attn_delta)."""
    M, K_ = dy.shape
    N = w.shape[1]
    assert w.shape[0] == K_ and N == H * D and M % L == 0 and o.shape == (M, N)
    for t in (dy, w, o):
        assert t.dtype == BF16 and t.stride(1) == 1
    do = torch.empty(M, N, device=dy.device, dtype=BF16)
    delta = torch.empty(M // L, H, L, device=dy.device, dtype=F32)
    call("owlk_gemm_attn_delta", M, N, K_, ptr(dy), dy.stride(0), ptr(w), w.stride(0), ptr(do), N, ptr(o), o.stride(0),
         L, H, D, ptr(delta), stream(), key="gemm_attn_delta", flops=2.0 * M * N * K_)
    return do, delta


def attn_bwd(q, k, v, o, do, lse, H, D, mask, dq, dk, dv, scale=None, delta=None):
    """Backward of attn_fwd (training shapes: Lq == Lkv, q_offset 0); all tensors [B, L, cols].
    delta: the softmax term rowsum(dO * O) [B, H, L] fp32 if the caller formed it (gemm_attn_delta)."""
    for t, n in ((q, "q"), (k, "k"), (v, "v"), (o, "o"), (do, "do"), (dq, "dq"), (dk, "dk"), (dv, "dv")):
        _v3(t, n)
    B, L = q.shape[:2]
    scale = D ** -0.5 if scale is None else scale
    if delta is None:
        delta = torch.empty(B, H, L, device=q.device, dtype=F32)
        assert o.is_contiguous() and do.is_contiguous() and o.shape == do.shape
        call("owlk_attn_delta", ptr(o), ptr(do), o.stride(1), B, L, H, D, ptr(delta), stream())
    else:
        assert delta.shape == (B, H, L) and delta.dtype == F32 and delta.is_contiguous()
    variant = fused_bwd_variant(D, mask)
    if variant is not None:
        # algorithmic FLOPs: the backward's 8 D per allowed pair (dV, dP, dK, dQ)
        attn_bwd_fused(q, k, v, do, lse, delta, H, D, mask, dq, dk, dv, scale, variant)
        return
    args = (ptr(q), q.stride(1), q.stride(0), ptr(k), k.stride(1), k.stride(0),
            ptr(v), v.stride(1), v.stride(0), ptr(do), do.stride(1), do.stride(0), ptr(lse), ptr(delta),
            ptr(dq), dq.stride(1), dq.stride(0), ptr(dk), dk.stride(1), dk.stride(0),
            ptr(dv), dv.stride(1), dv.stride(0), B, H, L, L, D, float(scale),
            mask.tpf, 0 if mask.window is None else int(mask.window), int(mask.causal), *mask.args()[3:], stream())
    # algorithmic FLOPs: dV, dP, dK belong to the key-owner sweep, dQ to the other;
    # the dq kernel's recomputed S and dP are not counted
    side = _bwd_side_stream(q.device, D, mask)
    if side is not None:
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)  # delta and every input are ready
    call("owlk_attn_bwd_dkdv", *args, key=f"attn_bwd_dkdv[w{mask.window}]",
         flops=lambda: 6.0 * D * H * B * mask_pairs(mask, L, L))
    if side is not None:
        call("owlk_attn_bwd_dq", *args[:-1], ctypes.c_void_p(side.cuda_stream))
        # joined before returning: later frees / reuses of these buffers on the caller's stream
        # are ordered after the side stream's reads and writes
        cur.wait_stream(side)
        return
    call("owlk_attn_bwd_dq", *args, key=f"attn_bwd_dq[w{mask.window}]",
         flops=lambda: 2.0 * D * H * B * mask_pairs(mask, L, L))


def mask_pairs(mask, Lq, Lkv):
    """Allowed (query, key) pairs per (batch, head), averaged over the batch (SURVEY §8(d) counts
    algorithmic FLOPs over allowed pairs only).  With document arrays the doc predicate is counted
    exactly on the device (frame x frame; profiling only); without them the mask is doc-free."""
    tpf, w = mask.tpf, mask.window
    nfq = (Lq + tpf - 1) // tpf
    off = mask.q_offset // tpf
    tot = 0
    if mask.arrays is not None and mask.causal:
        doc = mask.arrays["doc"]
        qf = torch.arange(off, off + nfq, device=doc.device)[:, None]
        kf = torch.arange(doc.shape[1], device=doc.device)[None, :]
        ok = kf <= qf
        if w is not None:
            ok &= kf > qf - w
        same = doc[:, off:off + nfq, None] == doc[:, None, :]
        return float((same & ok).sum().item()) / doc.shape[0] * tpf * tpf
    if not mask.causal:
        return float(Lq) * Lkv if w is None else float(Lq) * min(Lkv, (2 * w - 1) * tpf)
    for f in range(off, off + nfq):
        nk = (f + 1) if w is None else min(f + 1, w)
        tot += nk
    return float(tot) * tpf * tpf


def flow_noise(x, z, ts_raw):
    """x, z [B, N, C, h, w] bf16; ts_raw [B, N] -> xt_tok, tgt_tok [B*N*h*w, C] bf16, ts [B, N] bf16."""
    B, N, C, h, w = x.shape
    P = h * w
    xt = torch.empty(B * N * P, C, device=x.device, dtype=BF16)
    tgt = torch.empty_like(xt)
    ts = torch.empty(B, N, device=x.device, dtype=F32)
    call("owlk_flow_noise", ptr(x.contiguous()), ptr(z.contiguous()), ptr(ts_raw.float().contiguous()), C, P, B * N,
         ptr(xt), ptr(tgt), ptr(ts), stream())
    return xt, tgt, ts.to(BF16)


def unpatchify(tok, B, N, C, h, w):
    out = torch.empty(B, N, C, h, w, device=tok.device, dtype=BF16)
    call("owlk_unpatchify", ptr(tok), C, h * w, B * N, ptr(out), stream())
    return out


def mse(pred, tgt, want_grad=True, grad_scale=1.0):
    """F.mse_loss (fp32 math on bf16 inputs; fp32 0-dim loss) + d loss / d pred (bf16)."""
    n = pred.numel()
    nb = 1024
    partial = torch.empty(nb, device=pred.device, dtype=F32)
    loss = torch.empty((), device=pred.device, dtype=F32)
    dpred = torch.empty_like(pred) if want_grad else None
    call("owlk_mse", ptr(pred), ptr(tgt), n, float(2.0 * grad_scale / n), ptr(dpred), ptr(partial), nb, ptr(loss),
         stream())
    return loss, dpred


def mse_grad(pred, tgt, gout=None):
    """backward of F.mse_loss(pred, tgt): bf16((2 / n (pred - tgt)) gout), gout a device fp32 scalar."""
    assert pred.is_contiguous() and tgt.is_contiguous() and pred.dtype == tgt.dtype == BF16
    if gout is not None:
        gout = gout.to(F32).contiguous() if gout.dtype != F32 else gout.contiguous()
        assert gout.numel() == 1
    dpred = torch.empty_like(pred)
    n = pred.numel()
    call("owlk_mse_grad", ptr(pred), ptr(tgt), n, float(2.0 / n), ptr(gout), ptr(dpred), stream())
    return dpred


def colsum(x, out=None):
    """fp32 column sums of a 2-D row-major view (or a 3-D frame_rows view), added onto out
    (deterministic: row-split partials in a workspace, summed in order)."""
    if x.dim() == 3:
        R, N, ld, fs = _operand(x, "x")
    else:
        (R, N), ld, fs = x.shape, x.stride(0), 0
    if out is None:
        out = torch.zeros(N, device=x.device, dtype=F32)
    nb = lib().owlk_colsum_ws_bytes(R, N)
    ws = torch.empty(nb, device=x.device, dtype=torch.uint8)
    call("owlk_colsum_frames", ptr(x), int(x.dtype == F32), R, N, ld, fs, ptr(out), ptr(ws), nb, stream(),
         key="owlk_colsum")
    return out


NORM_PARTS = 256  # OWLK_NORM_PARTS: per-matrix partial sums of the Frobenius norm (fixed-order reduce)


def ns_normalize(g, transpose, work=None):
    """g [b, r, c] (fp32 or bf16) -> X bf16 [b, r, c] or [b, c, r] (transpose) / (||X||_F + 1e-7)."""
    b, r, c = g.shape
    x = torch.empty(b, c, r, device=g.device, dtype=BF16) if transpose else torch.empty(b, r, c, device=g.device,
                                                                                        dtype=BF16)
    work = torch.empty(b, NORM_PARTS, device=g.device, dtype=F32) if work is None else work
    assert work.dtype == F32 and work.numel() >= b * NORM_PARTS
    g = g.contiguous()
    call("owlk_ns_normalize", ptr(g), int(g.dtype == F32), r, c, b, int(transpose), ptr(x), ptr(work), stream())
    return x


def ns_scale(g, transpose, sumsq, out=None):
    """owlk_ns_normalize's scale pass given sumsq [b, NORM_PARTS], the partial sums of sum(bf16(g)^2)
    that muon_momentum writes."""
    b, r, c = g.shape
    assert g.is_contiguous() and sumsq.dtype == F32 and sumsq.shape == (b, NORM_PARTS) and sumsq.is_contiguous()
    x = torch.empty((b, c, r) if transpose else (b, r, c), device=g.device, dtype=BF16) if out is None else out
    assert x.shape == ((b, c, r) if transpose else (b, r, c)) and x.is_contiguous() and x.dtype == BF16
    call("owlk_ns_scale", ptr(g), int(g.dtype == F32), r, c, b, int(transpose), ptr(x), ptr(sumsq), stream())
    return x


NS_COEFFS = (3.4445, -4.7750, 2.0315)  # muon.py:23


def ns_iterate(x, steps, coeffs=NS_COEFFS):
    """owlk_ns_iterate: the quintic iterations in place on a normalised bf16 X [b, m, k] (m <= k)."""
    b, m, k = x.shape
    assert x.dtype == BF16 and x.is_contiguous() and m <= k
    nb = lib().owlk_ns_iterate_ws_bytes(b, m, k)
    ws = torch.empty(nb, device=x.device, dtype=torch.uint8)
    call("owlk_ns_iterate", ptr(x), b, m, k, int(steps), *(float(v) for v in coeffs), ptr(ws), nb, stream(),
         key=f"ns_iterate[{b}x{m}x{k}]", flops=lambda: steps * b * (4.0 * m * m * k + 2.0 * m ** 3))
    return x


def newton_schulz(g, steps=5, coeffs=NS_COEFFS):
    """owlk_newton_schulz_bf16: g [b, r, c] fp32 / bf16 -> bf16 [b, r, c] (muon.py:11-38 in one entry)."""
    b, r, c = g.shape
    g = g.contiguous()
    assert g.dtype in (F32, BF16)
    out = torch.empty(b, r, c, device=g.device, dtype=BF16)
    nb = lib().owlk_newton_schulz_ws_bytes(b, r, c)
    ws = torch.empty(nb, device=g.device, dtype=torch.uint8)
    call("owlk_newton_schulz_bf16", ptr(g), int(g.dtype == F32), b, r, c, int(steps), *(float(v) for v in coeffs),
         ptr(out), ptr(ws), nb, stream())
    return out


def _written(ts):
    """In-place writes made through raw pointers are invisible to autograd's version counters:
    bump them, so that every version-keyed cache (the bf16 weight copies of nn/fused.py) and
    saved-tensor check sees the new values."""
    increment_version(list(ts))


def _ptr_array(ts):
    import ctypes
    return (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])


def muon_momentum(grads, bufs, momentum, nesterov, stack, sumsq):
    """Fused buf.lerp_(g, 1-m); g' = lerp(g, buf, m) (or buf); stack[i] = g'; sumsq[i] = the NORM_PARTS
    partial sums of |bf16 g'|^2 (their sum is the squared norm).  grads / bufs: same-numel fp32
    contiguous tensors; stack fp32 [len, numel]; sumsq fp32 [len, NORM_PARTS] (fully written)."""
    n = grads[0].numel()
    for t in list(grads) + list(bufs):
        assert t.dtype == F32 and t.is_contiguous() and t.numel() == n and t.is_cuda
    assert stack.dtype == F32 and stack.is_contiguous() and stack.shape == (len(grads), n)
    assert sumsq.dtype == F32 and sumsq.shape == (len(grads), NORM_PARTS) and sumsq.is_contiguous()
    call("owlk_muon_momentum", len(grads), _ptr_array(grads), _ptr_array(bufs), n, float(momentum),
         int(bool(nesterov)), ptr(stack), ptr(sumsq), stream())
    _written(bufs)


def muon_apply(params, u, rows, cols, transpose, decay, alpha):
    """params[i] (fp32 [rows, cols] contiguous) = params[i] * decay - alpha * u[i]; u bf16 contiguous
    [len, rows, cols], or [len, cols, rows] with transpose."""
    for t in params:
        assert t.dtype == F32 and t.is_contiguous() and t.numel() == rows * cols and t.is_cuda
    assert u.dtype == BF16 and u.is_contiguous() and u.numel() == len(params) * rows * cols
    call("owlk_muon_apply", len(params), _ptr_array(params), ptr(u), rows, cols, int(bool(transpose)), float(decay),
         float(alpha), stream())
    _written(params)


def adamw(params, grads, exp_avgs, exp_avg_sqs, lr, beta1, beta2, weight_decay, eps, step):
    """One torch.optim.AdamW step (same order and state) over fp32 contiguous tensors, fused."""
    import ctypes
    for ts in (params, grads, exp_avgs, exp_avg_sqs):
        assert len(ts) == len(params)
        for t in ts:
            assert t.dtype == F32 and t.is_contiguous() and t.is_cuda
    ns = [t.numel() for t in params]
    assert [t.numel() for t in grads] == ns == [t.numel() for t in exp_avgs] == [t.numel() for t in exp_avg_sqs]
    step_size = -lr / (1 - beta1 ** step)
    bc2s = (1 - beta2 ** step) ** 0.5
    call("owlk_adamw", len(params), _ptr_array(params), _ptr_array(grads), _ptr_array(exp_avgs),
         _ptr_array(exp_avg_sqs), (ctypes.c_long * len(ns))(*ns), float(lr), float(beta1), float(beta2),
         float(weight_decay), float(eps), float(step_size), float(bc2s), stream())
    _written(list(params) + list(exp_avgs) + list(exp_avg_sqs))


def ema_lerp(shadow, params, weight):
    """shadow[i] = lerp(shadow[i], params[i], weight) in one multi-tensor pass (owlk_ema)."""
    import ctypes
    assert len(shadow) == len(params)
    for a, b in zip(shadow, params):
        assert a.dtype == F32 and b.dtype == F32 and a.is_contiguous() and b.is_contiguous() and a.is_cuda
        assert a.numel() == b.numel()
    ns = [t.numel() for t in shadow]
    call("owlk_ema", len(shadow), _ptr_array(shadow), _ptr_array(params), (ctypes.c_long * len(ns))(*ns),
         float(weight), stream())
    _written(shadow)


# ---------------------------------------------------------------- MMDiT plumbing (frames.hip)
def frame_interleave(a, b, n0, n1, out=None):
    """a [F*n0, C], b [F*n1, C] token-major -> joint [F*(n0+n1), C] (frame f = a-rows | b-rows)."""
    C = a.shape[1]
    F_ = a.shape[0] // n0
    assert a.shape[0] == F_ * n0 and b.shape[0] == F_ * n1 and b.shape[1] == C
    if out is None:
        out = torch.empty(F_ * (n0 + n1), C, device=a.device, dtype=BF16)
    call("owlk_frame_mux", 0, F_, n0, n1, C, ptr(a), a.stride(0), ptr(b), b.stride(0), ptr(out), out.stride(0),
         stream(), key="frame_mux")
    return out


def frame_split(j, n0, n1, a=None, b=None):
    """inverse of frame_interleave: joint [F*(n0+n1), C] -> (a [F*n0, C], b [F*n1, C])."""
    C = j.shape[1]
    F_ = j.shape[0] // (n0 + n1)
    assert j.shape[0] == F_ * (n0 + n1)
    if a is None:
        a = torch.empty(F_ * n0, C, device=j.device, dtype=BF16)
    if b is None:
        b = torch.empty(F_ * n1, C, device=j.device, dtype=BF16)
    call("owlk_frame_mux", 1, F_, n0, n1, C, ptr(a), a.stride(0), ptr(b), b.stride(0), ptr(j), j.stride(0),
         stream(), key="frame_mux")
    return a, b


def layernorm_fwd(x):
    """F.layer_norm(x, (d,)) (no affine, eps 1e-5) -> (y bf16, mean, rstd)."""
    T, d = x.shape
    y = torch.empty(T, d, device=x.device, dtype=BF16)
    mean = torch.empty(T, device=x.device, dtype=F32)
    rstd = torch.empty(T, device=x.device, dtype=F32)
    call("owlk_layernorm_fwd", ptr(x), x.stride(0), T, d, ptr(y), y.stride(0), ptr(mean), ptr(rstd), stream(),
         key="layernorm_fwd")
    return y, mean, rstd


def layernorm_bwd(dy, x, mean, rstd):
    T, d = x.shape
    dx = torch.empty(T, d, device=x.device, dtype=BF16)
    call("owlk_layernorm_bwd", ptr(dy), dy.stride(0), ptr(x), x.stride(0), ptr(mean), ptr(rstd), T, d, ptr(dx),
         dx.stride(0), stream(), key="layernorm_bwd")
    return dx


def _in_dtype_flag(t, name):
    assert t.dtype in (BF16, F32), f"{name}: bf16 or fp32 input expected (got {t.dtype})"
    return int(t.dtype == F32)


def cond_embed(R, ts=None, tfreq=None, tmult=1000.0, mouse=None, mfreq=None, mmult=1000.0, wang=None, btn=None,
               nbp=0):
    """owlk_cond_embed over R frame rows -> (ts_in [R, 2 ht], mouse_in [R, 4 hm], ang [R, 2], btn_in [R, nbp]),
    bf16 (None where the input is None).  ts [R], mouse [R, 2] (any row stride), btn [R, nb] (row stride),
    bf16 or fp32; tfreq / mfreq fp32 [ht] / [hm]; wang the angle_proj weight fp32 [2 hm, 2]."""
    dev = (ts if ts is not None else mouse if mouse is not None else btn).device
    ts_in = mouse_in = ang = btn_in = None
    ht = hm = nb = 0
    ldm = ldb = 0
    if ts is not None:
        assert ts.numel() == R and ts.is_contiguous() and tfreq.dtype == F32 and tfreq.is_contiguous()
        ht = tfreq.numel()
        ts_in = torch.empty(R, 2 * ht, device=dev, dtype=BF16)
    if mouse is not None:
        assert mouse.dim() == 2 and mouse.shape == (R, 2) and mouse.stride(1) == 1
        assert mfreq.dtype == F32 and mfreq.is_contiguous() and wang.dtype == F32 and wang.is_contiguous()
        hm = mfreq.numel()
        assert wang.shape == (2 * hm, 2)
        ldm = mouse.stride(0)
        mouse_in = torch.empty(R, 4 * hm, device=dev, dtype=BF16)
        ang = torch.empty(R, 2, device=dev, dtype=BF16)
    if btn is not None:
        assert btn.dim() == 2 and btn.shape[0] == R and btn.stride(1) == 1
        nb, ldb = btn.shape[1], btn.stride(0)
        assert nbp >= nb
        btn_in = torch.empty(R, nbp, device=dev, dtype=BF16)
    call("owlk_cond_embed", ptr(ts), _in_dtype_flag(ts, "ts") if ts is not None else 0, ptr(tfreq), ht,
         float(tmult), ptr(ts_in), 2 * ht, ptr(mouse), _in_dtype_flag(mouse, "mouse") if mouse is not None else 0,
         ldm, ptr(mfreq), hm, float(mmult), ptr(wang), ptr(mouse_in), 4 * hm, ptr(ang), ptr(btn),
         _in_dtype_flag(btn, "btn") if btn is not None else 0, ldb, nb, nbp, ptr(btn_in), nbp, R, stream())
    return ts_in, mouse_in, ang, btn_in


def cond_silu_fwd(t, m=None, b=None, hc=None, rows_per=1, keep_cond=True):
    """cond = t + (hc ? m + b : 0) (bf16 adds), s = silu(cond): -> (cond or None, s), [R, d] bf16.
    hc: bool [R / rows_per] (has_controls per sample) or None."""
    R, d = t.shape
    for x in (t, m, b):
        assert x is None or (x.shape == (R, d) and x.is_contiguous() and x.dtype == BF16)
    if hc is not None:
        assert hc.dtype == torch.bool and hc.is_contiguous() and hc.numel() * rows_per == R
    cond = torch.empty_like(t) if keep_cond and m is not None else (t if keep_cond else None)
    s = torch.empty_like(t)
    call("owlk_cond_silu_fwd", ptr(t), ptr(m), ptr(b), ptr(hc), rows_per, R, d,
         ptr(cond) if cond is not t else None, ptr(s), stream())
    return cond, s


def cond_silu_bwd(ds, cond=None, hc=None, rows_per=1, want_cond=True, want_ctrl=False):
    """ds [R, d] (fp32, or bf16) -> (dcond, dctrl) bf16: dcond = bf16(ds) silu'(cond), or ds itself
    when cond is None (then dcond is only returned, not written); dctrl = hc ? dcond : 0.  Either
    is None when not wanted."""
    R, d = ds.shape
    assert ds.dtype in (F32, BF16) and ds.is_contiguous()
    assert cond is None or (cond.shape == (R, d) and cond.is_contiguous() and cond.dtype == BF16)
    if hc is not None:
        assert hc.dtype == torch.bool and hc.is_contiguous() and hc.numel() * rows_per == R
    if cond is None:
        assert ds.dtype == BF16
        dcond = ds if want_cond else None
    else:
        dcond = torch.empty(R, d, device=ds.device, dtype=BF16) if want_cond else None
    dctrl = torch.empty(R, d, device=ds.device, dtype=BF16) if want_ctrl else None
    call("owlk_cond_silu_bwd", ptr(ds), int(ds.dtype == BF16), ptr(cond), ptr(hc), rows_per, R, d,
         ptr(dcond) if cond is not None else None, ptr(dctrl), stream())
    return dcond, dctrl


def small_k_wgrad(dy, x, K_, out=None, beta=0.0):
    """fp32 dW[n, k] = beta dW + sum_r dy[r, n] x[r, k] for k < K_ <= 16 (x may be wider: its first K_
    columns are used); out: [N, K_] fp32 (row stride any)."""
    R, N = dy.shape
    assert dy.stride(1) == 1 and x.stride(1) == 1 and x.shape[0] == R and x.shape[1] >= K_
    assert dy.dtype == BF16 and x.dtype == BF16
    if out is None:
        out = torch.empty(N, K_, device=dy.device, dtype=F32)
        beta = 0.0
    assert out.shape == (N, K_) and out.dtype == F32 and out.stride(1) == 1
    call("owlk_small_k_wgrad", ptr(dy), dy.stride(0), ptr(x), x.stride(0), R, N, K_, ptr(out), out.stride(0),
         float(beta), stream())
    return out
