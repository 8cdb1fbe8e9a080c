"""Pin the CPU oracle against the reference-generated golden vectors (CPU only)."""
from types import SimpleNamespace

import pytest
import torch

from conftest import golden
from oracle import ref_model as M
from oracle import ref_ops as R
from oracle.params import det_init_, det_tensor

OPS = golden("ops.pt")
GR = golden("gamerft_tiny.pt")


def close(a, b, atol=1e-5, rtol=1e-5):
    torch.testing.assert_close(a.float(), b.float(), atol=atol, rtol=rtol)


def tiny_cfg(**over):
    c = dict(model_id="game_rft", sample_size=8, channels=32, n_layers=2, n_heads=2, d_model=128,
             tokens_per_frame=64, n_buttons=11, cfg_prob=0.1, n_frames=8, causal=True, uncond=False,
             backbone="dit", has_audio=False, rope_impl="motion", rope_ats_delta=2.0, local_window=2,
             global_window=None)
    c.update(over)
    return SimpleNamespace(**c)


def test_rms_norm():
    close(R.rms_norm(OPS["rms.x"]), OPS["rms.y"], 1e-6, 1e-6)
    assert R.rms_norm(OPS["rms.xb"]).dtype == torch.bfloat16
    assert torch.equal(R.rms_norm(OPS["rms.xb"]), OPS["rms.yb"])


@pytest.mark.parametrize("name", ["adaln", "gate"])
def test_modulation_fwd_bwd(name):
    mod = det_init_(M._AdaLN(32) if name == "adaln" else M._Gate(32), base_seed=200)
    x = OPS[f"{name}.x"].clone().requires_grad_()
    c = OPS[f"{name}.cond"].clone().requires_grad_()
    y = mod(x, c)
    y.backward(OPS[f"{name}.dy"])
    close(y, OPS[f"{name}.y"], 1e-6, 1e-5)
    close(x.grad, OPS[f"{name}.dx"])
    close(c.grad, OPS[f"{name}.dcond"])
    for k, p in mod.named_parameters():
        close(p.grad, OPS[f"{name}.grad.{k}"])


def test_motion_rope_tables():
    a = R.motion_rope_angles(4, 8, 64)
    close(a.cos(), OPS["mrope.tiny.cos"], 0, 0)
    close(a.sin(), OPS["mrope.tiny.sin"], 0, 0)
    big = R.motion_rope_angles(1536, 8, 64)
    assert list(big.shape) == OPS["mrope.v4.shape"]
    close(big[:128].cos(), OPS["mrope.v4.cos.head"], 0, 0)
    close(big[-128:].sin(), OPS["mrope.v4.sin.tail"], 0, 0)
    ar = R.audio1d_rope_angles(10000, 64)
    close(ar[:256].cos(), OPS["arope.cos.head"], 0, 0)


def test_rope_apply():
    a = R.motion_rope_angles(4, 8, 64)
    c, s = a.cos(), a.sin()
    close(R.rope_apply(OPS["rope.x"], c, s), OPS["rope.y"], 0, 0)
    close(R.rope_apply(OPS["rope.x"][:, :, :192], c, s, 64), OPS["rope.y.off64"], 0, 0)
    assert torch.equal(R.rope_apply(OPS["rope.xb"], c, s), OPS["rope.yb"])


@pytest.mark.parametrize("tag", ["t4", "t64", "t1"])
@pytest.mark.parametrize("wtag", ["w2", "wN"])
def test_masked_attention(tag, wtag):
    p = f"attn.{tag}.{wtag}."
    q, k, v = (OPS[p + n].clone().requires_grad_() for n in "qkv")
    w = OPS[p + "window"]
    m = R.frame_mask(q.shape[2], k.shape[2], OPS[p + "tpf"], None if w < 0 else w, OPS[p + "doc"])
    o = R.attention(q, k, v, m)
    o.backward(OPS[p + "do"])
    close(o, OPS[p + "o"], 2e-6, 1e-5)
    for n in "qkv":
        close(getattr(locals()[n], "grad"), OPS[p + "d" + n], 2e-6, 1e-5)


@pytest.mark.parametrize("shape", ["256x768", "768x256", "128x128"])
def test_newton_schulz(shape):
    y = R.newton_schulz5(OPS[f"ns.{shape}.g"])
    # eager bf16 restatement vs the reference's eager body: same op order -> identical
    assert (y.float() - OPS[f"ns.{shape}.y"].float()).abs().max().item() <= 0.0079


def _tiny_model():
    return det_init_(M.GameRFT(tiny_cfg()), base_seed=1000).train()


def _noise(p):
    return {"rand_b": GR[p + "in.rand_b"], "ts_raw": GR[p + "in.ts_raw"], "z": GR[p + "in.z"]}


def test_gamerft_fp32_loss_pred_grads():
    p = "gamerft.fp32."
    model = _tiny_model()
    loss, pred, hc = model(GR[p + "in.x"], GR[p + "in.mouse"], GR[p + "in.btn"], GR[p + "in.doc_id"], _noise(p))
    loss.backward()
    assert torch.equal(hc, GR[p + "cfg_mask"])
    close(pred, GR[p + "pred"], 2e-5, 1e-4)
    assert abs(loss.item() - GR[p + "loss"].item()) < 1e-5
    for i, (k, prm) in enumerate(sorted(model.named_parameters())):
        if p + "grad." + k in GR:
            close(prm.grad, GR[p + "grad." + k], 1e-6, 2e-4)
        st = GR[p + "gradstat." + k]
        assert abs(prm.grad.double().norm().item() - st[3].item()) <= 1e-4 * st[3].item() + 1e-9, k


def test_gamerft_bf16_autocast_loss():
    p = "gamerft.bf16."
    model = _tiny_model()
    with torch.autocast("cpu", dtype=torch.bfloat16):
        loss, pred, _ = model(GR[p + "in.x"], GR[p + "in.mouse"], GR[p + "in.btn"], GR[p + "in.doc_id"], _noise(p))
    rel = (pred.float() - GR[p + "pred"]).norm() / GR[p + "pred"].norm()
    assert rel < 2e-2
    assert abs(loss.item() - GR[p + "loss"].item()) / GR[p + "loss"].item() < 5e-3


def test_combined_optimizer_step():
    p = "gamerft.fp32."
    model = _tiny_model()
    loss, _, _ = model(GR[p + "in.x"], GR[p + "in.mouse"], GR[p + "in.btn"], GR[p + "in.doc_id"], _noise(p))
    loss.backward()
    keys = ["core.proj_in", "core.proj_out.proj", "core.t_embed", "core.control_embed", "gate", "adaln"]
    adamw_p, muon_p = M.muon_partition(model, keys)
    names = {id(prm): n for n, prm in model.named_parameters()}
    assert sorted(names[id(q)] for q in muon_p) == sorted(GR["muon.muon_params"])
    adamw = torch.optim.AdamW(adamw_p, lr=1e-4, betas=(0.9, 0.95), weight_decay=1e-4, eps=1e-15)
    adamw.step()
    M.muon_step_1rank(muon_p, {}, lr=1e-3, momentum=0.95)
    before = dict(_tiny_model().named_parameters())
    for i, (k, prm) in enumerate(sorted(model.named_parameters())):
        st = GR["muon.after." + k]
        f = prm.detach().double().flatten()
        assert abs(f.norm().item() - st[3].item()) <= 1e-5 * st[3].item() + 1e-9, k
        if "muon.after.full." + k in GR:
            # bf16 Newton-Schulz flips ulps on 1e-7 input differences: compare the update by rel-L2
            upd = prm.detach() - before[k].detach()
            ref_upd = GR["muon.after.full." + k] - before[k].detach()
            assert (upd - ref_upd).norm() / ref_upd.norm() < 5e-2, k


def test_muon_step_on_reference_grads():
    """Muon (muon.py:66-84) fed the reference's own grads reproduces its update to 1e-5."""
    k = "core.transformer.blocks.0.attn.qkv.weight"
    p = dict(_tiny_model().named_parameters())[k]
    p0 = p.detach().clone()
    p.grad = GR["gamerft.fp32.grad." + k].clone()
    M.muon_step_1rank([p], {}, lr=1e-3, momentum=0.95)
    ref = GR["muon.after.full." + k]
    assert ((p.detach() - p0) - (ref - p0)).norm() / (ref - p0).norm() < 1e-5


def test_audio_trajectory():
    ref = golden("audio_traj.pt")["audio.losses"]
    cfg = SimpleNamespace(model_id="audio_rft", sample_size=120, channels=64, n_layers=2, n_heads=2, d_model=128,
                          tokens_per_frame=1, n_frames=10000, cfg_prob=0.0, causal=True, uncond=True,
                          backbone="dit", has_audio=True, rope_impl="audio1d", local_window=16,
                          global_window=None)
    model = det_init_(M.AudioRFT(cfg), base_seed=3000).train()
    opt = torch.optim.AdamW(model.parameters(), lr=1e-4, betas=(0.9, 0.999), weight_decay=0.01, eps=1e-8)
    for step in range(10):
        noise = {"ts_raw": det_tensor((1, 120), 3200 + step), "z": det_tensor((1, 120, 64), 3300 + step)}
        loss, _ = model(det_tensor((1, 120, 64), 3100 + step), noise)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=10.0)
        opt.step()
        opt.zero_grad(set_to_none=True)
        assert abs(loss.item() - ref[step].item()) < 2e-5, (step, loss.item(), ref[step].item())


# ----------------------------------------------------------------------------- MMDiT (configs[3])
MM = golden("mmdit_tiny.pt")


def mmdit_cfg(**over):
    c = dict(model_id="game_rft_audio", sample_size=8, channels=32, audio_channels=16, n_layers=2, n_heads=2,
             d_model=128, tokens_per_frame=65, n_buttons=11, n_mouse_axes=2, cfg_prob=0.1, n_frames=6,
             causal=True, uncond=False, backbone="mmdit", local_window=2, global_window=4, has_audio=True)
    c.update(over)
    return SimpleNamespace(**c)


def test_mmdit_schema_and_ortho_rope():
    """Reconstructed reference MMDiT: same state_dict schema; the OrthoRoPE
    restatement (parity-unpinned: rotary-embedding-torch is absent) matches the table the
    reconstruction used."""
    m = M.GameRFTAudio(mmdit_cfg())
    assert [[k, list(v.shape)] for k, v in m.state_dict().items()] == MM["mmdit.schema"]
    close(m.core.transformer.cos, MM["mmdit.rope.cos"], 0, 0)
    close(m.core.transformer.sin, MM["mmdit.rope.sin"], 0, 0)


def test_mmdit_bf16_autocast_loss_pred_grads():
    p = "mmdit.bf16."
    m = det_init_(M.GameRFTAudio(mmdit_cfg()), base_seed=5000).train()
    noise = {k: MM[p + "in." + k] for k in ("rand_b", "ts_raw", "z_video", "z_audio")}
    with torch.autocast("cpu", dtype=torch.bfloat16):
        loss, lv, la, pv, pa, hc = m(MM[p + "in.x"], MM[p + "in.audio"], MM[p + "in.mouse"], MM[p + "in.btn"],
                                     noise)
    loss.backward()
    assert torch.equal(hc, MM[p + "cfg_mask"])
    for got, k in ((loss, "diffusion_loss"), (lv, "video_loss"), (la, "audio_loss")):
        assert abs(got.item() - MM[p + k].item()) <= 1e-4 * MM[p + k].item(), k
    close(pv, MM[p + "pred_video"], 2e-2, 2e-2)
    close(pa, MM[p + "pred_audio"], 2e-2, 2e-2)
    n = 0
    for k, prm in m.named_parameters():
        if p + "grad." + k in MM:
            ref = MM[p + "grad." + k]
            assert ((prm.grad.double() - ref.double()).norm() / ref.double().norm()).item() < 1e-2, k
            n += 1
    assert n >= 10


# ----------------------------------------------------------------------------- head dim 128 (configs[4])
D128 = golden("gamerft_d128.pt")


def test_motion_rope_tables_d128():
    """MotionRoPE at head_dim 128 (dit_v4_5B: d 2560 / 20 heads, rope.py:88-152): exact."""
    big = R.motion_rope_angles(1536, 8, 128)
    assert list(big.shape) == D128["mrope.5b.shape"]
    for part, sl in (("head", slice(0, 128)), ("tail", slice(-128, None))):
        close(big[sl].cos(), D128[f"mrope.5b.cos.{part}"], 0, 0)
        close(big[sl].sin(), D128[f"mrope.5b.sin.{part}"], 0, 0)
    a = R.motion_rope_angles(8, 8, 128)
    close(R.rope_apply(D128["rope128.x"], a.cos(), a.sin()), D128["rope128.y"], 0, 0)
    assert torch.equal(R.rope_apply(D128["rope128.xb"], a.cos(), a.sin()), D128["rope128.yb"])


def test_gamerft_d128_bf16_autocast_loss_pred_grads():
    """Tiny D = 128 GameRFT (d 256, 2 heads, gradient checkpointing) under bf16 autocast: the oracle
    reproduces the reference's loss, prediction and gradients."""
    p = "d128.bf16."
    model = det_init_(M.GameRFT(tiny_cfg(d_model=256, n_heads=2)), base_seed=1100).train()
    assert [[k, list(v.shape)] for k, v in model.state_dict().items()] == D128["d128.schema"]
    noise = {"rand_b": D128[p + "in.rand_b"], "ts_raw": D128[p + "in.ts_raw"], "z": D128[p + "in.z"]}
    with torch.autocast("cpu", dtype=torch.bfloat16):
        loss, pred, hc = model(D128[p + "in.x"], D128[p + "in.mouse"], D128[p + "in.btn"], D128[p + "in.doc_id"],
                               noise)
    loss.backward()
    assert torch.equal(hc, D128[p + "cfg_mask"])
    assert abs(loss.item() - D128[p + "loss"].item()) <= 1e-4 * D128[p + "loss"].item()
    close(pred, D128[p + "pred"], 2e-2, 2e-2)
    n = 0
    for k, prm in model.named_parameters():
        if p + "grad." + k in D128:
            ref = D128[p + "grad." + k]
            assert ((prm.grad.double() - ref.double()).norm() / ref.double().norm()).item() < 1e-2, k
            n += 1
    assert n >= 6
