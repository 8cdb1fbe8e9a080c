"""Generate the golden fixtures in tests/golden/ by importing the REFERENCE on CPU.

Runs only where /root/reference exists (the build container), never on the GPU box.
Recipe: SURVEY.md §8(c).  Shims supplied here (all our own code, no reference text):
  * ``rotary_embedding_torch``: only ``RotaryEmbedding(...).freqs`` for freqs_for='lang'
    (1/theta^(arange(0,dim,2)[:dim//2]/dim)), which is all MotionRoPE/Audio1DRoPE read.
  * bare package modules ``owl_wms``, ``owl_wms.nn``, ``owl_wms.models`` pointing into
    /root/reference so ``owl_wms/__init__.py`` (omegaconf/diffusers/owl-vaes) is not executed.
  * ``attn.flex_attention`` replaced by the eager flex_attention (compiled one fails on CPU).
  * Muon's ``device="cuda"`` update buffer redirected to CPU during construction.
  * the training RNG (rand(b) -> randn(B,S) -> randn_like(x)) injected from seeded CPU tensors.

Outputs are small .pt dicts (tensors / ints / floats / strings) loaded with weights_only=True.
Parameters are NOT stored: they come from oracle/params.py's deterministic recipe.

    python tests/golden/make_golden.py          # every fixture below
    python tests/golden/make_golden.py d128     # gamerft_d128.pt only
"""
import importlib.util
import os
import sys
import types
from types import SimpleNamespace

import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.dont_write_bytecode = True

from oracle.params import det_init_, det_tensor  # noqa: E402


# ----------------------------------------------------------------------------- shims
def _install_shims():
    rot = types.ModuleType("rotary_embedding_torch")

    class RotaryEmbedding:
        def __init__(self, dim, freqs_for="lang", theta=10000, max_freq=10, **kw):
            if freqs_for == "lang":
                self.freqs = 1.0 / (theta ** (torch.arange(0, dim, 2)[: dim // 2].float() / dim))
            else:
                raise NotImplementedError("only 'lang' freqs are needed for the pinned paths")

    rot.RotaryEmbedding = RotaryEmbedding
    rot.apply_rotary_emb = None
    sys.modules["rotary_embedding_torch"] = rot

    for name, sub in [("owl_wms", ""), ("owl_wms.nn", "nn"), ("owl_wms.models", "models")]:
        m = types.ModuleType(name)
        m.__path__ = [os.path.join(REF, "owl_wms", sub) if sub else os.path.join(REF, "owl_wms")]
        sys.modules[name] = m


def _load(modname, relpath):
    spec = importlib.util.spec_from_file_location(modname, os.path.join(REF, relpath))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[modname] = mod
    spec.loader.exec_module(mod)
    return mod


_install_shims()
from torch.nn.attention.flex_attention import flex_attention as _eager_flex  # noqa: E402

r_norm = _load("owl_wms.nn.normalization", "owl_wms/nn/normalization.py")
r_mlp = _load("owl_wms.nn.mlp", "owl_wms/nn/mlp.py")
r_mod = _load("owl_wms.nn.modulation", "owl_wms/nn/modulation.py")
r_rope = _load("owl_wms.nn.rope", "owl_wms/nn/rope.py")
r_emb = _load("owl_wms.nn.embeddings", "owl_wms/nn/embeddings.py")
r_attn = _load("owl_wms.nn.attn", "owl_wms/nn/attn.py")
r_attn.flex_attention = _eager_flex
r_gamerft = _load("owl_wms.models.gamerft", "owl_wms/models/gamerft.py")
r_audiorft = _load("owl_wms.models.audiorft", "owl_wms/models/audiorft.py")
r_muon = _load("owl_wms.muon", "owl_wms/muon.py")


class inject_rng:
    """Replace torch.rand / torch.randn / torch.randn_like by queues of given tensors."""

    def __init__(self, rand=(), randn=(), randn_like=()):
        self.q = {"rand": list(rand), "randn": list(randn), "randn_like": list(randn_like)}

    def __enter__(self):
        self.saved = (torch.rand, torch.randn, torch.randn_like)

        def mk(kind):
            def f(*a, **kw):
                t = self.q[kind].pop(0)
                dt = kw.get("dtype", None)
                if kind == "randn_like":
                    dt = a[0].dtype
                return t.to(dt) if dt is not None else t.clone()
            return f

        torch.rand, torch.randn, torch.randn_like = mk("rand"), mk("randn"), mk("randn_like")
        return self

    def __exit__(self, *exc):
        torch.rand, torch.randn, torch.randn_like = self.saved
        for k, v in self.q.items():
            assert not v, f"unconsumed injected {k}"


def proj_stats(t, seed):
    """Size-independent fingerprints of a tensor: 3 seeded random projections + L2 norm."""
    f = t.detach().double().flatten()
    g = torch.Generator().manual_seed(seed)
    r = torch.randn(3, f.numel(), generator=g, dtype=torch.float64)
    return torch.cat([r @ f, f.norm().view(1)])


def bf16_exact(t):
    return t.to(torch.bfloat16).float()


# ----------------------------------------------------------------------------- configs
def tiny_video_cfg(**over):
    c = dict(model_id="game_rft", sample_size=8, channels=32, n_layers=2, n_heads=2, d_model=128,
             tokens_per_frame=64, n_buttons=11, n_mouse_axes=2, cfg_prob=0.1, n_frames=8,
             causal=True, uncond=False, backbone="dit", has_audio=False, rope_impl="motion",
             rope_ats_delta=2.0, local_window=2, global_window=None)
    c.update(over)
    return SimpleNamespace(**c)


def audio_cfg(**over):
    c = dict(model_id="audio_rft", sample_size=120, channels=64, n_layers=2, n_heads=2, d_model=128,
             tokens_per_frame=1, n_frames=10000, cfg_prob=0.0, causal=True, uncond=True,
             backbone="dit", has_audio=True, rope_impl="audio1d", local_window=16,
             global_window=None, gradient_checkpointing=False)
    c.update(over)
    return SimpleNamespace(**c)


# ----------------------------------------------------------------------------- op fixtures
def gen_ops():
    out = {}
    # rms_norm
    x = det_tensor((4, 64), 100)
    out["rms.x"], out["rms.y"] = x, r_norm.rms_norm(x)
    xb = bf16_exact(det_tensor((4, 64), 101, 3.0)).to(torch.bfloat16)
    out["rms.xb"], out["rms.yb"] = xb, r_norm.rms_norm(xb)

    # AdaLN / Gate fwd + bwd (n=3 frames, m=8 tokens/frame, d=32)
    for name, cls in [("adaln", r_mod.AdaLN), ("gate", r_mod.Gate)]:
        mod = det_init_(cls(32), base_seed=200)
        x = det_tensor((1, 24, 32), 201).requires_grad_()
        c = det_tensor((1, 3, 32), 202).requires_grad_()
        y = mod(x, c)
        dy = det_tensor(y.shape, 203)
        y.backward(dy)
        out[f"{name}.x"], out[f"{name}.cond"], out[f"{name}.dy"] = x.detach(), c.detach(), dy
        out[f"{name}.y"], out[f"{name}.dx"], out[f"{name}.dcond"] = y.detach(), x.grad, c.grad
        for k, p in mod.named_parameters():
            out[f"{name}.grad.{k}"] = p.grad.clone()

    # MotionRoPE tables: tiny config full, dit_v4 config slices
    cfg = tiny_video_cfg(n_frames=4)
    rope = r_rope.MotionRoPE(cfg)
    out["mrope.tiny.cos"], out["mrope.tiny.sin"] = rope.cos, rope.sin
    big = tiny_video_cfg(n_frames=1536, d_model=1536, n_heads=24)
    rb = r_rope.MotionRoPE(big)
    out["mrope.v4.cos.head"], out["mrope.v4.sin.head"] = rb.cos[:128].clone(), rb.sin[:128].clone()
    out["mrope.v4.cos.tail"], out["mrope.v4.sin.tail"] = rb.cos[-128:].clone(), rb.sin[-128:].clone()
    out["mrope.v4.shape"] = list(rb.cos.shape)
    # rotation on a [1, 2, 256, 64] input (fp32 and bf16)
    xq = det_tensor((1, 2, 256, 64), 300)
    out["rope.x"], out["rope.y"] = xq, rope(xq)
    out["rope.y.off64"] = rope(xq[:, :, :192], offset=64)
    xqb = xq.to(torch.bfloat16)
    out["rope.xb"], out["rope.yb"] = xqb, rope(xqb)
    # Audio1D tables
    ar = r_rope.Audio1DRoPE(audio_cfg())
    out["arope.cos.head"], out["arope.sin.head"] = ar.cos[:256].clone(), ar.sin[:256].clone()

    # masked attention fwd + bwd through the reference block mask + eager flex_attention
    for tpf, nf, tag in [(4, 8, "t4"), (64, 6, "t64"), (1, 40, "t1")]:
        L = tpf * nf
        doc = torch.zeros(1, nf, dtype=torch.long)
        doc[:, nf // 2 + 1:] = 1
        for window, wtag in [(2, "w2"), (None, "wN")]:
            q = det_tensor((1, 2, L, 64), 400 + L).requires_grad_()
            k = det_tensor((1, 2, L, 64), 401 + L).requires_grad_()
            v = det_tensor((1, 2, L, 64), 402 + L).requires_grad_()
            bm = r_attn.get_block_mask(L, tpf, window, doc, 0, True, "cpu")
            o = _eager_flex(q, k, v, block_mask=bm)
            do = det_tensor(o.shape, 403 + L)
            o.backward(do)
            p = f"attn.{tag}.{wtag}"
            out[p + ".q"], out[p + ".k"], out[p + ".v"], out[p + ".do"] = q.detach(), k.detach(), v.detach(), do
            out[p + ".o"], out[p + ".dq"], out[p + ".dk"], out[p + ".dv"] = o.detach(), q.grad, k.grad, v.grad
            out[p + ".doc"], out[p + ".window"], out[p + ".tpf"] = doc, (-1 if window is None else window), tpf

    # Newton-Schulz (eager body of the compiled function), bf16
    ns = getattr(r_muon.zeropower_via_newtonschulz5, "_torchdynamo_orig_callable",
                 r_muon.zeropower_via_newtonschulz5)
    for shape in [(256, 768), (768, 256), (128, 128)]:
        g = det_tensor(shape, 500 + shape[0])
        out[f"ns.{shape[0]}x{shape[1]}.g"] = g
        out[f"ns.{shape[0]}x{shape[1]}.y"] = ns(g, 5)
    return out


# ----------------------------------------------------------------------------- model fixtures
def video_inputs(cfg, B, dtype, seed=600):
    n, C, s = cfg.n_frames, cfg.channels, cfg.sample_size
    x = bf16_exact(det_tensor((B, n, C, s, s), seed)).to(dtype)
    mouse = bf16_exact(det_tensor((B, n, 2), seed + 1)).to(dtype)
    g = torch.Generator().manual_seed(seed + 2)
    btn = (torch.rand((B, n, cfg.n_buttons), generator=g) < 0.5).to(dtype)
    doc = torch.zeros(B, n, dtype=torch.long)
    doc[1:, n // 2:] = 1  # second sample holds two packed documents
    rand_b = torch.tensor([0.05, 0.7])[:B]
    ts_raw = bf16_exact(det_tensor((B, n), seed + 3))
    z = bf16_exact(det_tensor((B, n, C, s, s), seed + 4))
    return dict(x=x, mouse=mouse, btn=btn, doc_id=doc, rand_b=rand_b, ts_raw=ts_raw, z=z)


def gen_gamerft():
    out = {}
    cfg = tiny_video_cfg()
    for mode in ["fp32", "bf16"]:
        model = det_init_(r_gamerft.GameRFT(cfg), base_seed=1000).train()
        dtype = torch.float32 if mode == "fp32" else torch.bfloat16
        inp = video_inputs(cfg, 2, dtype)
        ctx = torch.autocast("cpu", dtype=torch.bfloat16, enabled=(mode == "bf16"))
        with inject_rng(rand=[inp["rand_b"]], randn=[inp["ts_raw"]], randn_like=[inp["z"]]), ctx:
            d = model(inp["x"], inp["mouse"], inp["btn"], inp["doc_id"], return_dict=True)
            d["diffusion_loss"].backward()
        p = f"gamerft.{mode}."
        for k, v in inp.items():
            out[p + "in." + k] = v
        out[p + "loss"] = d["diffusion_loss"].detach().float()
        out[p + "pred"] = d["pred_video"].detach().float()
        out[p + "cfg_mask"] = d["cfg_mask"]
        for i, (k, prm) in enumerate(sorted(model.named_parameters())):
            out[p + "gradstat." + k] = proj_stats(prm.grad, 7000 + i)
            if ".blocks.0." in k or "proj_out" in k or "proj_in" in k:
                out[p + "grad." + k] = prm.grad.clone()
        if mode == "fp32":
            # one CombinedOptimizer (AdamW + Muon) step with the dit_v4 opt_kwargs
            real_empty = torch.empty

            def cpu_empty(*a, **kw):
                kw["device"] = "cpu"
                return real_empty(*a, **kw)

            torch.empty = cpu_empty
            try:
                opt = r_muon.init_muon(model, rank=0, world_size=1, lr=1e-3, momentum=0.95, adamw_lr=1e-4,
                                       adamw_wd=1e-4, adamw_eps=1e-15, adamw_betas=[0.9, 0.95],
                                       adamw_keys=["core.proj_in", "core.proj_out.proj", "core.t_embed",
                                                   "core.control_embed", "gate", "adaln"])
            finally:
                torch.empty = real_empty
            ns_eager = getattr(r_muon.zeropower_via_newtonschulz5, "_torchdynamo_orig_callable", None)
            if ns_eager is not None:
                r_muon.zeropower_via_newtonschulz5 = ns_eager
            out["muon.muon_params"] = [n for n, prm in sorted(model.named_parameters())
                                       if any(prm is q for g in opt.muon.param_groups for q in g["params"])]
            opt.step()
            for i, (k, prm) in enumerate(sorted(model.named_parameters())):
                out["muon.after." + k] = proj_stats(prm.detach(), 9000 + i)
                if ".blocks.0.attn.qkv.weight" in k or ".blocks.0.adaln1" in k:
                    out["muon.after.full." + k] = prm.detach().clone()
    return out


def gen_d128():
    """Head dim 128 (configs/dit_v4_5B.yml: d 2560 / 20 heads): MotionRoPE tables of the 5B config
    (head / tail rows), the rotation at D = 128, and a tiny D = 128 GameRFT (d 256, 2 heads,
    gradient_checkpointing as the 5B config) trained one fwd+bwd under bf16 autocast."""
    out = {}
    big = tiny_video_cfg(n_frames=1536, d_model=2560, n_heads=20)
    rb = r_rope.MotionRoPE(big)
    out["mrope.5b.cos.head"], out["mrope.5b.sin.head"] = rb.cos[:128].clone(), rb.sin[:128].clone()
    out["mrope.5b.cos.tail"], out["mrope.5b.sin.tail"] = rb.cos[-128:].clone(), rb.sin[-128:].clone()
    out["mrope.5b.shape"] = list(rb.cos.shape)
    cfg = tiny_video_cfg(d_model=256, n_heads=2, gradient_checkpointing=True)
    rope = r_rope.MotionRoPE(cfg)
    xq = det_tensor((1, 2, 256, 128), 310)
    out["rope128.x"], out["rope128.y"] = xq, rope(xq)
    out["rope128.xb"], out["rope128.yb"] = xq.to(torch.bfloat16), rope(xq.to(torch.bfloat16))
    model = det_init_(r_gamerft.GameRFT(cfg), base_seed=1100).train()
    inp = video_inputs(cfg, 2, torch.bfloat16, seed=620)
    with inject_rng(rand=[inp["rand_b"]], randn=[inp["ts_raw"]], randn_like=[inp["z"]]), \
            torch.autocast("cpu", dtype=torch.bfloat16):
        d = model(inp["x"], inp["mouse"], inp["btn"], inp["doc_id"], return_dict=True)
        d["diffusion_loss"].backward()
    p = "d128.bf16."
    for k, v in inp.items():
        out[p + "in." + k] = v
    out[p + "loss"] = d["diffusion_loss"].detach().float()
    out[p + "pred"] = d["pred_video"].detach().float()
    out[p + "cfg_mask"] = d["cfg_mask"]
    for i, (k, prm) in enumerate(sorted(model.named_parameters())):
        out[p + "gradstat." + k] = proj_stats(prm.grad, 7500 + i)
        if ".blocks.0.attn." in k or ".blocks.1.attn.qkv" in k or ".blocks.0.adaln1" in k or \
                "proj_out.proj" in k or "proj_in" in k:
            out[p + "grad." + k] = prm.grad.clone()
    out["d128.schema"] = [[k, list(v.shape)] for k, v in model.state_dict().items()]
    return out


def gen_audio_traj():
    out = {}
    cfg = audio_cfg()
    model = det_init_(r_audiorft.AudioRFT(cfg), base_seed=3000).train()
    opt = torch.optim.AdamW(model.parameters(), lr=1e-4, betas=(0.9, 0.999), weight_decay=0.01, eps=1e-8)
    losses = []
    for step in range(10):
        x = det_tensor((1, 120, 64), 3100 + step)
        ts_raw = det_tensor((1, 120), 3200 + step)
        z = det_tensor((1, 120, 64), 3300 + step)
        with inject_rng(randn=[ts_raw], randn_like=[z]):
            loss = model(x)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=10.0)
        opt.step()
        opt.zero_grad(set_to_none=True)
        losses.append(loss.item())
    out["audio.losses"] = torch.tensor(losses, dtype=torch.float64)
    return out


def gen_schema():
    """state_dict key -> shape of the reference models (checkpoint compatibility)."""
    out = {}
    for tag, cfg in [("tiny", tiny_video_cfg()),
                     ("dit_v4", tiny_video_cfg(channels=128, n_layers=16, n_heads=24, d_model=1536, n_frames=1536,
                                               local_window=16))]:
        m = r_gamerft.GameRFT(cfg)
        out[tag] = [[k, list(v.shape)] for k, v in m.state_dict().items()]
        del m
    m = r_audiorft.AudioRFT(audio_cfg())
    out["audio_tiny"] = [[k, list(v.shape)] for k, v in m.state_dict().items()]
    return out


def main():
    torch.manual_seed(0)
    if sys.argv[1:] == ["d128"]:  # only the head-dim-128 fixture (added in round 2)
        d = gen_d128()
        torch.save(d, os.path.join(HERE, "gamerft_d128.pt"))
        print("gamerft_d128.pt", os.path.getsize(os.path.join(HERE, "gamerft_d128.pt")) // 1024, "KiB",
              "loss", d["d128.bf16.loss"].item())
        return
    import json
    with open(os.path.join(HERE, "schema.json"), "w") as f:
        json.dump(gen_schema(), f)
    ops = gen_ops()
    torch.save(ops, os.path.join(HERE, "ops.pt"))
    gr = gen_gamerft()
    torch.save(gr, os.path.join(HERE, "gamerft_tiny.pt"))
    au = gen_audio_traj()
    torch.save(au, os.path.join(HERE, "audio_traj.pt"))
    for f in ["ops.pt", "gamerft_tiny.pt", "audio_traj.pt"]:
        print(f, os.path.getsize(os.path.join(HERE, f)) // 1024, "KiB")
    print("audio losses", au["audio.losses"].tolist())
    print("gamerft loss fp32/bf16", gr["gamerft.fp32.loss"].item(), gr["gamerft.bf16.loss"].item())


if __name__ == "__main__":
    main()
