"""CPU restatement of the owl_wms models (GameRFT, AudioRFT, MMDiT) and the Muon/AdamW step.

TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py.  Module attribute names reproduce the
reference state_dict schema so the deterministic parameter recipe
(oracle/params.py) gives the reference, this oracle and the HIP path identical weights.
Noise is injected explicitly (``noise=`` dicts) instead of drawn from a global RNG.
"""
import torch
import torch.nn.functional as F
from torch import nn

from . import ref_ops as R


class _MLP(nn.Module):  # mlp.py:6-37
    def __init__(self, din, dmid, dout):
        super().__init__()
        self.fc1, self.fc2 = nn.Linear(din, dmid), nn.Linear(dmid, dout)

    def forward(self, x):
        return self.fc2(F.silu(self.fc1(x)))


class _AdaLN(nn.Module):  # modulation.py:7-26
    def __init__(self, d):
        super().__init__()
        self.fc = nn.Linear(d, 2 * d)

    def forward(self, x, cond):
        return R.adaln(x, cond, self.fc.weight, self.fc.bias)


class _Gate(nn.Module):  # modulation.py:28-43
    def __init__(self, d):
        super().__init__()
        self.fc_c = nn.Linear(d, d)

    def forward(self, x, cond):
        return R.gate(x, cond, self.fc_c.weight, self.fc_c.bias)


def rope_tables(cfg):
    """rope.py:11-20,30-41 -> fp32 cos/sin [n_tokens_total, D/2]."""
    D = cfg.d_model // cfg.n_heads
    impl = getattr(cfg, "rope_impl", "ortho").lower()
    if impl == "motion":
        ang = R.motion_rope_angles(cfg.n_frames, cfg.sample_size, D, getattr(cfg, "rope_ats_delta", 2.0),
                                   getattr(cfg, "rope_base", 10000.0), has_audio=cfg.has_audio)
    elif impl == "audio1d":
        ang = R.audio1d_rope_angles(cfg.n_frames, D)
    else:  # OrthoRoPE: parity-unpinned restatement of rotary-embedding-torch (ref_ops)
        ang = R.ortho_rope_angles(cfg.n_frames, cfg.sample_size, D)
        if not cfg.has_audio:
            ang = ang.view(cfg.n_frames, -1, ang.shape[-1])[:, :-1].flatten(0, 1)
    return ang.cos().contiguous(), ang.sin().contiguous()


class _Attn(nn.Module):  # attn.py:65-113
    def __init__(self, cfg, local):
        super().__init__()
        d = cfg.d_model
        self.h = cfg.n_heads
        self.qkv, self.out = nn.Linear(d, 3 * d), nn.Linear(d, d)
        self.local = local
        self.local_offset = cfg.local_window * cfg.tokens_per_frame

    def forward(self, x, mask, cos, sin, cache=None, layer=0):
        B, L, d = x.shape
        qkv = self.qkv(x).view(B, L, 3, self.h, d // self.h).permute(2, 0, 3, 1, 4)
        q, k, v = qkv[0], qkv[1], qkv[2]
        q, k = R.rms_norm(q), R.rms_norm(k)
        off = cache.offset(layer) if cache is not None else 0
        q, k = R.rope_apply(q, cos, sin, off), R.rope_apply(k, cos, sin, off)
        if off > 0:
            ok, ov = cache.get(layer)
            k, v = torch.cat([ok, k], 2), torch.cat([ov, v], 2)
        if cache is not None and cache.should_update:
            cache.update(layer, k, v)
        if self.local and mask is None:
            k, v = k[:, :, -self.local_offset:], v[:, :, -self.local_offset:]
        o = R.attention(q, k, v, mask)
        return self.out(o.permute(0, 2, 1, 3).reshape(B, L, d))


class _Block(nn.Module):  # attn.py:116-143
    def __init__(self, cfg, local):
        super().__init__()
        d = cfg.d_model
        self.attn = _Attn(cfg, local)
        self.mlp = _MLP(d, 4 * d, d)
        self.adaln1, self.gate1, self.adaln2, self.gate2 = _AdaLN(d), _Gate(d), _AdaLN(d), _Gate(d)

    def forward(self, x, cond, mask, cos, sin, cache=None, layer=0):
        x = x + self.gate1(self.attn(self.adaln1(x, cond), mask, cos, sin, cache, layer), cond)
        x = x + self.gate2(self.mlp(self.adaln2(x, cond)), cond)
        return x


class DiT(nn.Module):  # attn.py:146-191
    def __init__(self, cfg):
        super().__init__()
        self.cfg = cfg
        self.local_layers = [(i % 4 != 0) for i in range(cfg.n_layers)]
        self.blocks = nn.ModuleList([_Block(cfg, loc) for loc in self.local_layers])
        cos, sin = rope_tables(cfg)
        self.register_buffer("cos", cos, persistent=False)
        self.register_buffer("sin", sin, persistent=False)
        self.decoding = False

    def forward(self, x, cond, doc_id=None, cache=None):
        L = x.shape[1]
        off = cache.length() if cache is not None else 0
        if self.decoding:
            lm = gm = None
        else:
            n = L + off
            lm = R.frame_mask(L, n, self.cfg.tokens_per_frame, self.cfg.local_window, doc_id, off, self.cfg.causal)
            gm = R.frame_mask(L, n, self.cfg.tokens_per_frame, getattr(self.cfg, "global_window", None), doc_id,
                              off, self.cfg.causal)
        for i, blk in enumerate(self.blocks):
            x = blk(x, cond, lm if self.local_layers[i] else gm, self.cos, self.sin, cache, i)
        return x


class _Final(nn.Module):  # attn.py:264-277
    def __init__(self, d, c):
        super().__init__()
        self.norm = _AdaLN(d)
        self.proj = nn.Linear(d, c)

    def forward(self, x, cond):
        return self.proj(F.silu(self.norm(x, cond)))


class _Mouse(nn.Module):  # embeddings.py:119-156
    def __init__(self, dout, dim=512):
        super().__init__()
        self.angle_proj = nn.Linear(2, dim // 2, bias=False)
        self.mlp = _MLP(dim, dim * 4, dout)
        self.dim = dim

    def forward(self, x):
        with torch.no_grad():
            x = torch.sign(x) * torch.log1p(x.abs())
            ang = torch.atan2(x[..., 1], x[..., 0])
            mag = torch.norm(x, dim=-1)
            ae = torch.stack([torch.cos(ang), torch.sin(ang)], -1).to(x.dtype)
            me = R.sincos(mag, self.dim // 2).to(x.dtype)
        return self.mlp(torch.cat([self.angle_proj(ae), me], -1))


class _Button(nn.Module):  # embeddings.py:158-168
    def __init__(self, nb, dout, dim=512):
        super().__init__()
        self.proj = _MLP(nb, dim * 4, dout)

    def forward(self, x):
        return self.proj(x * 2 - 1)


class _Control(nn.Module):  # embeddings.py:170-184
    def __init__(self, nb, dout):
        super().__init__()
        self.mouse, self.button = _Mouse(dout), _Button(nb, dout)

    def forward(self, mouse, btn):
        return self.mouse(mouse) + self.button(btn)


class _TEmbed(nn.Module):  # embeddings.py:74-84
    def __init__(self, d):
        super().__init__()
        self.mlp = _MLP(512, 4 * d, d)

    def forward(self, t):
        return self.mlp(R.sincos(t, 512))


class GameRFTCore(nn.Module):  # gamerft.py:13-59
    def __init__(self, cfg):
        super().__init__()
        self.cfg = cfg
        self.transformer = DiT(cfg)
        if not cfg.uncond:
            self.control_embed = _Control(cfg.n_buttons, cfg.d_model)
        self.t_embed = _TEmbed(cfg.d_model)
        self.proj_in = nn.Linear(cfg.channels, cfg.d_model, bias=False)
        self.proj_out = _Final(cfg.d_model, cfg.channels)

    def forward(self, x, t, mouse, btn, doc_id=None, has_controls=None, cache=None):
        b, n, c, h, w = x.shape
        cond = self.t_embed(t)
        if not self.cfg.uncond:
            ctrl = self.control_embed(mouse, btn)
            if has_controls is not None:
                ctrl = torch.where(has_controls[:, None, None], ctrl, torch.zeros_like(ctrl))
            cond = cond + ctrl
        x = x.permute(0, 1, 3, 4, 2).reshape(b, n * h * w, c)
        x = self.transformer(self.proj_in(x), cond, doc_id, cache)
        x = self.proj_out(x, cond)
        return x.reshape(b, n, h, w, c).permute(0, 1, 4, 2, 3)


class GameRFT(nn.Module):  # gamerft.py:62-124
    def __init__(self, cfg):
        super().__init__()
        self.config = cfg
        self.core = GameRFTCore(cfg)

    @staticmethod
    def handle_cfg(has_controls, cfg_prob, rand_b):
        """gamerft.py:68-90 with the rand(b) draw injected."""
        if cfg_prob <= 0.0 or has_controls is None:
            return has_controls
        frac = has_controls.float().mean()
        pct_without = 1.0 - frac
        if pct_without < cfg_prob:
            needed_frac = (cfg_prob - pct_without) / frac
            mask = (rand_b <= needed_frac) & has_controls
            has_controls = has_controls & ~mask
        return has_controls

    def forward(self, x, mouse, btn, doc_id, noise, cfg_prob=None):
        B, S = x.shape[:2]
        hc = torch.ones(B, dtype=torch.bool)
        hc = self.handle_cfg(hc, self.config.cfg_prob if cfg_prob is None else cfg_prob, noise["rand_b"])
        with torch.no_grad():
            ts = noise["ts_raw"].to(x.dtype).sigmoid()
            xt, target = R.flow_noise(x, ts[:, :, None, None, None], noise["z"].to(x.dtype))
        pred = self.core(xt, ts, mouse, btn, doc_id, hc)
        return F.mse_loss(pred, target), pred, hc


class AudioRFT(nn.Module):  # audiorft.py:13-93
    def __init__(self, cfg):
        super().__init__()
        self.config = cfg
        core = nn.Module()
        core.transformer = DiT(cfg)
        core.t_embed = _TEmbed(cfg.d_model)
        core.proj_in = nn.Linear(cfg.channels, cfg.d_model, bias=False)
        core.proj_out = _Final(cfg.d_model, cfg.channels)
        self.core = core

    def forward(self, x, noise, doc_id=None):
        with torch.no_grad():
            ts = noise["ts_raw"].to(x.dtype).sigmoid()
            xt, target = R.flow_noise(x, ts[:, :, None], noise["z"].to(x.dtype))
        c = self.core
        cond = c.t_embed(ts)
        h = c.transformer(c.proj_in(xt), cond, doc_id)
        pred = c.proj_out(h, cond)
        return F.mse_loss(pred, target), pred


# ----------------------------------------------------------------------------- MMDiT
class _MMAttn(nn.Module):  # mmattn.py:28-86
    def __init__(self, cfg):
        super().__init__()
        d = cfg.d_model
        self.h = cfg.n_heads
        self.n = [cfg.sample_size ** 2, 1]
        self.qkv_projs = nn.ModuleList([nn.Linear(d, 3 * d) for _ in range(2)])
        self.out_projs = nn.ModuleList([nn.Linear(d, d) for _ in range(2)])

    def forward(self, x0, x1, mask, cos, sin):
        B, d = x0.shape[0], x0.shape[-1]
        # per-modality qkv, concatenated per frame: frame f = [n0 video | n1 audio] (mmattn.py:54-60)
        parts = [self.qkv_projs[i](x).view(B, -1, self.n[i], 3 * d) for i, x in enumerate((x0, x1))]
        qkv = torch.cat(parts, 2).reshape(B, -1, 3 * d)
        L = qkv.shape[1]
        q, k, v = qkv.view(B, L, 3, self.h, d // self.h).permute(2, 0, 3, 1, 4)
        q, k = R.rms_norm(q), R.rms_norm(k)
        q, k = R.rope_apply(q, cos, sin, 0), R.rope_apply(k, cos, sin, 0)
        o = R.attention(q, k, v, mask).permute(0, 2, 1, 3).reshape(B, -1, self.n[0] + self.n[1], d)
        o0, o1 = o[:, :, :self.n[0]].reshape(B, -1, d), o[:, :, self.n[0]:].reshape(B, -1, d)
        return self.out_projs[0](o0), self.out_projs[1](o1)


class _MMBlock(nn.Module):  # mmattn.py:89-114
    def __init__(self, cfg):
        super().__init__()
        d = cfg.d_model
        self.attn = _MMAttn(cfg)
        self.mlps = nn.ModuleList([_MLP(d, 4 * d, d) for _ in range(2)])

    def forward(self, x0, x1, c0, c1, mask, cos, sin):
        m0, m1 = c0.chunk(6, dim=-1), c1.chunk(6, dim=-1)
        h0, h1 = self.attn(R.cond_adaln(x0, m0[0], m0[1]), R.cond_adaln(x1, m1[0], m1[1]), mask, cos, sin)
        x0, x1 = x0 + R.cond_gate(h0, m0[2]), x1 + R.cond_gate(h1, m1[2])
        h0 = self.mlps[0](R.cond_adaln(x0, m0[3], m0[4]))
        h1 = self.mlps[1](R.cond_adaln(x1, m1[3], m1[4]))
        return x0 + R.cond_gate(h0, m0[5]), x1 + R.cond_gate(h1, m1[5])


class MMDIT(nn.Module):  # mmattn.py:117-152 (modulation shared by all layers, DiT-Air)
    def __init__(self, cfg):
        super().__init__()
        self.cfg = cfg
        d = cfg.d_model
        self.local_layers = [(i % 4 != 0) for i in range(cfg.n_layers)]
        self.blocks = nn.ModuleList([_MMBlock(cfg) for _ in range(cfg.n_layers)])
        self.cond_proj = nn.Sequential(nn.SiLU(), nn.Linear(d, d * 2 * 2 * 3))
        cos, sin = rope_tables(cfg)
        self.register_buffer("cos", cos, persistent=False)
        self.register_buffer("sin", sin, persistent=False)

    def forward(self, x0, x1, cond):
        L = x0.shape[1] + x1.shape[1]
        tpf = self.cfg.tokens_per_frame
        lm = gm = None
        if self.cfg.causal:  # create_causal_block_mask, reconstructed
            lm = R.frame_mask(L, L, tpf, self.cfg.local_window)
            gm = R.frame_mask(L, L, tpf, self.cfg.global_window)
        c0, c1 = self.cond_proj(cond).chunk(2, dim=-1)
        for i, blk in enumerate(self.blocks):
            x0, x1 = blk(x0, x1, c0, c1, lm if self.local_layers[i] else gm, self.cos, self.sin)
        return x0, x1


class GameRFTAudioCore(nn.Module):  # gamerft_audio.py:19-97 (mmdit backbone)
    def __init__(self, cfg):
        super().__init__()
        self.cfg = cfg
        d = cfg.d_model
        self.transformer = MMDIT(cfg)
        if not cfg.uncond:
            self.control_embed = _Control(cfg.n_buttons, d)
        self.t_embed = _TEmbed(d)
        self.proj_in = nn.Linear(cfg.channels, d, bias=False)
        self.proj_out = _Final(d, cfg.channels)
        self.audio_proj_in = nn.Linear(cfg.audio_channels, d, bias=False)
        self.audio_proj_out = _Final(d, cfg.audio_channels)

    def forward(self, x, audio, t, mouse, btn, has_controls=None):
        cond = self.t_embed(t)
        if not self.cfg.uncond:
            ctrl = self.control_embed(mouse, btn)
            if has_controls is not None:
                ctrl = torch.where(has_controls[:, None, None], ctrl, torch.zeros_like(ctrl))
            cond = cond + ctrl
        b, n, c, h, w = x.shape
        x = self.proj_in(x.permute(0, 1, 3, 4, 2).reshape(b, n * h * w, c))
        video, aud = self.transformer(x, self.audio_proj_in(audio), cond)
        video = self.proj_out(R.layer_norm(video), R.layer_norm(cond))
        video = video.reshape(b, n, h, w, c).permute(0, 1, 4, 2, 3)
        return video, self.audio_proj_out(aud, cond)


class GameRFTAudio(nn.Module):  # gamerft_audio.py:99-178
    def __init__(self, cfg):
        super().__init__()
        self.config = cfg
        self.core = GameRFTAudioCore(cfg)

    def forward(self, x, audio, mouse, btn, noise, cfg_prob=None):
        B = x.shape[0]
        hc = GameRFT.handle_cfg(torch.ones(B, dtype=torch.bool), self.config.cfg_prob if cfg_prob is None
                                else cfg_prob, noise["rand_b"])
        with torch.no_grad():
            ts = noise["ts_raw"].to(x.dtype).sigmoid()
            xt, tv = R.flow_noise(x, ts[:, :, None, None, None], noise["z_video"].to(x.dtype))
            at, ta = R.flow_noise(audio, ts[:, :, None], noise["z_audio"].to(audio.dtype))
        pv, pa = self.core(xt, at, ts, mouse, btn, hc)
        lv, la = F.mse_loss(pv, tv), F.mse_loss(pa, ta)
        return lv + la, lv, la, pv, pa, hc


# ----------------------------------------------------------------------------- optimizer
def muon_partition(model, adamw_keys):
    """muon.py:124-127: AdamW for names containing an adamw_key or ndim < 2; Muon for the rest."""
    named = {n.replace("._orig_mod", ""): p for n, p in model.named_parameters()}
    adamw = [p for n, p in named.items() if any(k in n for k in adamw_keys) or p.ndim < 2]
    muon = [p for n, p in named.items() if not any(k in n for k in adamw_keys) and p.ndim >= 2]
    return adamw, muon


@torch.no_grad()
def muon_step_1rank(params, state, lr, momentum=0.95, weight_decay=0.01, ns_steps=5):
    """muon.py:66-84 (world_size == 1 branch)."""
    for p in params:
        g = p.grad
        if g is None:
            continue
        buf = state.setdefault(id(p), torch.zeros_like(g))
        buf.lerp_(g, 1 - momentum)
        g = g.lerp_(buf, momentum)
        u = R.newton_schulz5(g, ns_steps).view_as(p)
        p.mul_(1 - lr * weight_decay)
        p.add_(u, alpha=-lr * max(1, p.size(-2) / p.size(-1)) ** 0.5)
