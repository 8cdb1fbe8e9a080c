"""CPU restatement of the owl_wms hot-path operators (fp32 / eager PyTorch on CPU).

TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py.  Each function cites the reference
file:line whose arithmetic it restates; tests/test_oracle_golden.py pins them against the
reference-generated golden vectors.
"""
import math

import torch
import torch.nn.functional as F

RMS_EPS = torch.finfo(torch.float32).eps  # F.rms_norm default eps (normalization.py:10-11)


def rms_norm(x):
    """normalization.py:10-11 -- F.rms_norm without weight; fp32 internal math, output in x.dtype."""
    xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + RMS_EPS)
    return y.to(x.dtype)


def layer_norm(x):
    """normalization.py:6-7 (MMDiT head)."""
    return F.layer_norm(x, (x.size(-1),)).type_as(x)


def frame_broadcast(t, m):
    """[b, n, c] -> [b, n*m, c] (modulation.py:17-20)."""
    b, n, c = t.shape
    return t[:, :, None, :].expand(b, n, m, c).reshape(b, n * m, c)


def adaln(x, cond, w, bias):
    """modulation.py:7-26: y = rms_norm(x) * (1 + a) + b with [a|b] = fc(silu(cond)) per frame."""
    m = x.shape[1] // cond.shape[1]
    ab = F.linear(F.silu(cond), w, bias)
    a, b_ = frame_broadcast(ab, m).chunk(2, dim=-1)
    return rms_norm(x) * (1 + a) + b_


def gate(x, cond, w, bias):
    """modulation.py:28-43: y = fc_c(silu(cond)) (per frame, broadcast) * x."""
    m = x.shape[1] // cond.shape[1]
    return frame_broadcast(F.linear(F.silu(cond), w, bias), m) * x


def cond_adaln(x, scale, bias):
    """modulation.py:46-55 (MMDiT)."""
    m = x.shape[1] // scale.shape[1]
    return rms_norm(x) * (1 + frame_broadcast(scale, m)) + frame_broadcast(bias, m)


def cond_gate(x, g):
    """modulation.py:57-63 (MMDiT)."""
    return frame_broadcast(g, x.shape[1] // g.shape[1]) * x


# ----------------------------------------------------------------------------- RoPE
def lang_freqs(dim, theta=10000.0):
    """rotary-embedding-torch 'lang' freqs as read by rope.py:104,164-174."""
    return 1.0 / (theta ** (torch.arange(0, dim, 2)[: dim // 2].float() / dim))


def motion_rope_angles(n_frames, sample_size, d_head, ats_delta=2.0, theta=10000.0, has_audio=False):
    """rope.py:88-152 (MotionRoPE.get_freqs) + rope.py:35-37 (audio slot drop).

    Returns fp32 angles [n_frames * tpf, d_head // 2]; tpf = sample_size**2 (+1 with audio).
    """
    H = W = sample_size
    dt, dx, dy = d_head * 2 // 8, d_head * 3 // 8, d_head * 3 // 8
    base = lang_freqs(dt + dx + dy, theta)
    spatial, ft = base[: (dx + dy) // 2], base[(dx + dy) // 2:]
    fx, fy = spatial[0::2], spatial[1::2]
    t = torch.arange(n_frames, dtype=torch.float32) * ats_delta
    h = torch.arange(H, dtype=torch.float32) - (H - 1) / 2.0
    w = torch.arange(W, dtype=torch.float32) - (W - 1) / 2.0
    # video tokens, frame-major then h then w
    tv = t[:, None, None].expand(n_frames, H, W)
    xv = tv + w[None, None, :]
    yv = tv + h[None, :, None]
    xv, yv, tv = xv.reshape(n_frames, H * W), yv.reshape(n_frames, H * W), tv.reshape(n_frames, H * W)
    # the per-frame audio slot
    xa, ya, ta = t[:, None], t[:, None] + (H - 1) / 2.0 + 1.0, t[:, None]
    xs = torch.cat([xv, xa], 1).reshape(-1)
    ys = torch.cat([yv, ya], 1).reshape(-1)
    ts = torch.cat([tv, ta], 1).reshape(-1)
    ang_x = xs[:, None] * fx[None]
    ang_y = ys[:, None] * fy[None]
    ang_t = ts[:, None] * ft[None]
    inter = torch.stack([ang_x, ang_y], -1).reshape(xs.numel(), -1)
    ang = torch.cat([inter, ang_t], -1)
    if not has_audio:
        ang = ang.view(n_frames, H * W + 1, -1)[:, :-1].reshape(-1, ang.shape[-1])
    return ang


def audio1d_rope_angles(n_latents, d_head):
    """rope.py:159-179 (Audio1DRoPE)."""
    return torch.arange(n_latents, dtype=torch.float32)[:, None] * lang_freqs(d_head)[None]


def ortho_rope_angles(n_frames, sample_size, d_head, max_freq=256.0):
    """rope.py:57-79 OrthoRoPE.  PARITY-UNPINNED: restates rotary-embedding-torch (absent, version
    unpinned) 'pixel' freqs = linspace(1, max_freq/2, dim//2) * pi and get_axial_freqs (positions
    linspace(-1, 1, n) + offset per axis, each freq repeated x2, axes broadcast and concatenated).
    Returns [n_frames * (p*p + 1), d_head/2] (video tokens of a frame, then its audio token)."""
    p = sample_size
    dim = d_head // 4
    freqs = torch.linspace(1.0, max_freq / 2, dim // 2) * math.pi
    dims, offsets = (n_frames, p + 1, p + 1, 1), (0, 0, 0, 1)
    axes = []
    for i, (n, off) in enumerate(zip(dims, offsets)):
        pos = torch.linspace(-1, 1, steps=n) + off
        f = (pos[:, None] * freqs[None]).repeat_interleave(2, dim=-1)
        shape = [1] * len(dims) + [f.shape[-1]]
        shape[i] = n
        axes.append(f.view(shape))
    full = torch.cat(torch.broadcast_tensors(*axes), dim=-1).view(n_frames, p + 1, p + 1, -1)
    vid = full[:, :p, :p].reshape(n_frames, p * p, -1)
    aud = full[:, -1, -1].unsqueeze(1)
    return torch.cat([vid, aud], dim=1).flatten(0, 1)[..., ::2]


def rope_apply(x, cos, sin, offset=0):
    """rope.py:43-51: fp32 pairwise rotation, output laid out [rot_even || rot_odd], cast back."""
    L = x.shape[-2]
    c, s = cos[offset:offset + L], sin[offset:offset + L]
    xf = x.float()
    x0, x1 = xf[..., 0::2], xf[..., 1::2]
    return torch.cat([x0 * c - x1 * s, x1 * c + x0 * s], -1).type_as(x)


# ----------------------------------------------------------------------------- attention
def frame_mask(n_q, n_kv, tpf, window=None, doc_id=None, q_offset=0, causal=True):
    """attn.py:24-62 mask_mod evaluated densely: [B or 1, n_q, n_kv] bool."""
    fq = (torch.arange(n_q) + q_offset) // tpf
    fk = torch.arange(n_kv) // tpf
    n_frames = n_kv // tpf
    w = n_frames if window is None else window
    m = (fq[:, None] - fk[None, :]).abs() < w
    if causal:
        m = m & (fk[None, :] <= fq[:, None])
    m = m[None]
    if doc_id is not None:
        dq = doc_id[:, fq]
        dk = doc_id[:, fk]
        m = m & (dq[:, :, None] == dk[:, None, :])
    return m


def attention(q, k, v, mask=None, scale=None):
    """flex_attention semantics (attn.py:106-109): softmax(q k^T * D^-0.5) v over allowed keys.

    q,k,v: [B, H, L, D]; mask: [B or 1, Lq, Lkv] bool.  Rows with no allowed key return 0.
    """
    D = q.shape[-1]
    scale = D ** -0.5 if scale is None else scale
    s = (q.float() @ k.float().transpose(-1, -2)) * scale
    if mask is not None:
        s = s.masked_fill(~mask[:, None], float("-inf"))
    p = torch.softmax(s, -1)
    p = torch.nan_to_num(p, nan=0.0)
    return (p @ v.float()).to(q.dtype)


# ----------------------------------------------------------------------------- embeddings
def sincos(x, dim, theta=300.0, mult=1000.0):
    """embeddings.py:30-72 (computed in x.dtype)."""
    shp = x.shape
    x = x.reshape(-1) * mult
    half = dim // 2
    e = torch.log(torch.tensor(theta)) / (half - 1)
    e = torch.exp(torch.arange(half) * -e).to(dtype=x.dtype)
    e = x[:, None] * e[None]
    return torch.cat([torch.sin(e), torch.cos(e)], -1).reshape(*shp, dim)


# ----------------------------------------------------------------------------- Muon
NS_COEF = (3.4445, -4.7750, 2.0315)


def newton_schulz5(G, steps=5):
    """muon.py:11-38: quintic Newton-Schulz in bf16, in the eager reference's rounding order:
    A = X X^T; B = bf16(b*A) + bf16(bf16(c*A) @ A) (`c * A @ A` is `(c*A) @ A`); X = bf16(a*X) +
    bf16(B @ X).  (bf16 NS is chaotic in its rounding order: another valid order, e.g. c applied
    after the product, differs by ~2.7% rel-L2 after 5 steps.)"""
    a, b, c = NS_COEF
    X = G.bfloat16()
    tr = G.size(-2) > G.size(-1)
    if tr:
        X = X.mT
    X = X / (X.norm(dim=(-2, -1), keepdim=True) + 1e-7)
    for _ in range(steps):
        A = X @ X.mT
        B = b * A + c * A @ A
        X = a * X + B @ X
    if tr:
        X = X.mT
    return X


def flow_noise(x, ts, z):
    """gamerft.py:92-95."""
    return x * (1 - ts) + z * ts, z - x
