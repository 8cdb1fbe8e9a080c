"""Host-side logic, CPU only: checkpoint schema, configs, the C ABI's exported symbols, frame-mask
helper arrays, and the N>1 data-parallel paths on gloo (world_size 2)."""
import ctypes
import json
import os
import re
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO
from oracle import ref_ops as R


def _schema():
    return json.load(open(os.path.join(REPO, "tests", "golden", "schema.json")))


@pytest.mark.parametrize("tag,cfgfile", [("dit_v4", "configs/dit_v4.yml")])
def test_state_dict_schema_matches_reference(tag, cfgfile):
    from owl_wms.configs import Config
    from owl_wms.models import get_model_cls
    cfg = Config.from_yaml(os.path.join(REPO, cfgfile))
    m = get_model_cls(cfg.model.model_id)(cfg.model)
    ours = [[k, list(v.shape)] for k, v in m.state_dict().items()]
    assert sorted(ours) == sorted(_schema()[tag])
    assert sum(p.numel() for p in m.parameters()) == 704_921_728


def test_tiny_and_audio_schema():
    from owl_wms.configs import model_config
    from owl_wms.models.audiorft import AudioRFT
    from owl_wms.models.gamerft import GameRFT
    tiny = model_config(model_id="game_rft", sample_size=8, channels=32, n_layers=2, n_heads=2, d_model=128,
                        tokens_per_frame=64, n_buttons=11, cfg_prob=0.1, n_frames=8, causal=True, uncond=False,
                        backbone="dit", has_audio=False, rope_impl="motion", local_window=2, global_window=None)
    assert sorted([k, list(v.shape)] for k, v in GameRFT(tiny).state_dict().items()) == sorted(_schema()["tiny"])
    au = model_config(model_id="audio_rft", sample_size=120, channels=64, n_layers=2, n_heads=2, d_model=128,
                      tokens_per_frame=1, n_frames=10000, cfg_prob=0.0, causal=True, uncond=True, backbone="dit",
                      has_audio=True, rope_impl="audio1d", local_window=16, global_window=None)
    assert sorted([k, list(v.shape)] for k, v in AudioRFT(au).state_dict().items()) == sorted(
        _schema()["audio_tiny"])


def test_rope_tables_match_oracle():
    from owl_wms.configs import model_config
    from owl_wms.nn.rope import Audio1DRoPE, MotionRoPE
    c = model_config(sample_size=8, n_frames=1536, d_model=1536, n_heads=24, has_audio=False)
    r = MotionRoPE(c)
    a = R.motion_rope_angles(1536, 8, 64)
    assert torch.equal(r.cos, a.cos()) and torch.equal(r.sin, a.sin())
    ra = Audio1DRoPE(model_config(n_frames=10000, d_model=128, n_heads=2, has_audio=True))
    assert torch.equal(ra.cos, R.audio1d_rope_angles(10000, 64).cos())


def test_configs_load():
    from owl_wms.configs import Config
    for f in ["dit_v4.yml", "dit_v4_5B.yml", "audio.yml", "audio_tiny.yml", "mmdit_v2.yml"]:
        c = Config.from_yaml(os.path.join(REPO, "configs", f))
        assert c.model.model_id and c.train.trainer_id
        assert getattr(c.model, "backbone") in ("dit", "mmdit")
        assert getattr(c.model, "nonexistent_key", "dflt") == "dflt"


def test_library_exports_every_header_symbol():
    from owl_wms._lib import LIB_PATH, exported_symbols
    if not os.path.exists(LIB_PATH):
        pytest.skip("libowlk.so not built (run __graft_entry__.build())")
    hdr = open(os.path.join(REPO, "include", "owlk.h")).read()
    declared = set(re.findall(r"\b(owlk_\w+)\s*\(", hdr))
    h = ctypes.CDLL(LIB_PATH)
    for s in declared:
        assert hasattr(h, s), s
    assert declared == set(exported_symbols())


def _header_protos():
    """include/owlk.h prototypes -> {name: [kind per argument]}, kinds P (pointer), L, I, F."""
    hdr = re.sub(r"/\*.*?\*/", " ", open(os.path.join(REPO, "include", "owlk.h")).read(), flags=re.S)
    protos = {}
    for m in re.finditer(r"\b(?:const\s+)?(?:char|int|long|void)\s*\*?\s*(owlk_\w+)\s*\(([^)]*)\)\s*;", hdr):
        kinds = []
        for a in [x.strip() for x in m.group(2).split(",")]:
            if a in ("", "void"):
                continue
            if "*" in a:
                kinds.append("P")
            else:
                t = re.match(r"(?:const\s+)?(long|int|float)\b", a)
                assert t, f"{m.group(1)}: unparsed argument {a!r}"
                kinds.append({"long": "L", "int": "I", "float": "F"}[t.group(1)])
        protos[m.group(1)] = kinds
    return protos


_KIND = {ctypes.c_void_p: "P", ctypes.c_long: "L", ctypes.c_int: "I", ctypes.c_float: "F"}


def test_ctypes_signatures_match_header():
    """Every _SIGS entry (the package's ctypes binding) equals its owlk.h prototype argument by
    argument; every header prototype is bound."""
    from owl_wms._lib import _SIGS
    protos = _header_protos()
    assert set(protos) - {"owlk_last_error", "owlk_version", "owlk_device_ok"} == set(_SIGS)
    for name, args in _SIGS.items():
        assert [_KIND[a] for a in args] == protos[name], name


def test_integration_binding_matches_header(monkeypatch):
    """The reference-side binding in INTEGRATION.md (owl_wms/nn/owlk_bind.py): its argtypes equal
    the owlk.h prototypes, and its attn_fwd / newton_schulz5 pass exactly the header's arguments
    (count and kind) -- run against a stand-in library, no GPU."""
    protos = _header_protos()
    text = open(os.path.join(REPO, "INTEGRATION.md")).read()
    block = [b for b in re.findall(r"```python\n(.*?)```", text, flags=re.S) if "ctypes.CDLL" in b]
    assert len(block) == 1
    calls = []

    class Fn:
        def __init__(self, name):
            self.name, self.argtypes, self.restype = name, None, None

        def __call__(self, *args):
            kinds = protos[self.name]
            assert len(args) == len(kinds), (self.name, len(args), len(kinds))
            for a, k in zip(args, kinds):
                if k == "P":
                    assert a is None or isinstance(a, (ctypes.c_void_p, int)), (self.name, a)
                elif k == "F":
                    assert isinstance(a, (float, int)) and not isinstance(a, bool), (self.name, a)
                else:
                    assert isinstance(a, int) and not isinstance(a, bool), (self.name, a)
            calls.append(self.name)
            return 256 if self.name.endswith("_bytes") else 0

    class Lib:
        def __init__(self, *a, **k):
            self.fns = {}

        def __getattr__(self, name):
            return self.fns.setdefault(name, Fn(name))

    monkeypatch.setattr(ctypes, "CDLL", Lib)

    class S:
        cuda_stream = 0

    monkeypatch.setattr(torch.cuda, "current_stream", lambda *a, **k: S())
    ns = {}
    exec(compile(block[0], "INTEGRATION.md", "exec"), ns)
    lib = ns["_L"]
    for name, fn in lib.fns.items():
        if fn.argtypes is not None:
            assert [_KIND[a] for a in fn.argtypes] == protos[name], name
    q = torch.zeros(1, 4, 2, 8, dtype=torch.bfloat16)
    ns["attn_fwd"](q, q, q, tpf=2, window=None)
    ns["attn_fwd"](q, q, q, tpf=2, window=3, score_bound=1.02 * 8)
    ns["newton_schulz5"](torch.zeros(3, 16, 24), steps=5)
    assert calls == ["owlk_attn_fwd", "owlk_attn_fwd", "owlk_newton_schulz_ws_bytes", "owlk_newton_schulz_bf16"]


def _brute_arrays(doc, window):
    nf = doc.numel()
    kv_lo, q_hi = [], []
    for f in range(nf):
        ok = [g for g in range(nf) if g <= f and (window is None or f - g < window) and doc[g] == doc[f]]
        kv_lo.append(min(ok))
        okq = [g for g in range(nf) if g >= f and (window is None or g - f < window) and doc[g] == doc[f]]
        q_hi.append(max(okq))
    return kv_lo, q_hi


@pytest.mark.parametrize("window", [None, 3])
def test_frame_arrays_bruteforce(window):
    from owl_wms.kernels import frame_arrays
    g = torch.Generator().manual_seed(0)
    for _ in range(5):
        doc = torch.randint(0, 3, (2, 17), generator=g)
        a = frame_arrays(doc, 17, window)
        for b in range(2):
            lo, hi = _brute_arrays(doc[b], window)
            # kv_lo / q_hi bound every allowed frame (conservative envelope of the exact mask)
            assert all(a["kv_lo"][b, f].item() <= lo[f] for f in range(17))
            assert all(a["q_hi"][b, f].item() >= hi[f] for f in range(17))
            rs = a["run_start"][b].tolist()
            for f in range(17):
                assert all(doc[b, g] == doc[b, f] for g in range(rs[f], f + 1))
                assert rs[f] == 0 or doc[b, rs[f] - 1] != doc[b, f]


def test_grad_reducer_cu_reserve_brackets_the_sync_micro_step(monkeypatch):
    """The CU reserve for RCCL (owlk_set_cu_reserve) is asked for at the first bucket launch of the
    synchronising micro-step and dropped in finish(); never on gloo, never on earlier micro-steps."""
    import owl_wms.utils.grad_reducer as gr

    class _Work:
        def wait(self):
            pass

    monkeypatch.setattr(gr.dist, "all_reduce", lambda *a, **k: _Work())
    model = torch.nn.Sequential(torch.nn.Linear(4, 8), torch.nn.Linear(8, 2))
    red = gr.GradReducer(model.parameters(), bucket_mb=0.0001, world_size=2)
    assert red.reserve_cus == 0  # no RCCL process group here
    red.reserve_cus = 32
    calls = []
    monkeypatch.setattr(red, "_reserve", lambda cus: (calls.append(cus), setattr(red, "_reserved", cus > 0)))
    for micro in range(3):
        red.begin(sync=micro == 2)
        model(torch.randn(3, 4)).sum().backward()
        if micro < 2:
            assert calls == []
        red.finish()
    assert len(red.buckets) > 1 and calls == [32, 0]


# ------------------------------------------------------------------ world_size 2 on gloo
# one numel (96) in three shapes: the group mixes transposed (r > c) and plain NS layouts, and 5
# params over 2 ranks leave the last chunk short
MUON_SHAPES = [(8, 12), (8, 12), (12, 8), (12, 8), (8, 12)]


def _worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from owl_wms.utils.grad_reducer import GradReducer
        torch.manual_seed(0)
        model = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.SiLU(), torch.nn.Linear(32, 8))
        red = GradReducer(model.parameters(), bucket_mb=0.001, world_size=ws)  # several tiny buckets
        g = torch.Generator().manual_seed(100 + rank)
        accum = 3
        for micro in range(accum):
            red.begin(sync=micro == accum - 1)
            x = torch.randn(4, 16, generator=g)
            (model(x).pow(2).mean() / accum).backward()
            red.finish()
        q.put((rank, [p.grad.numpy().copy() for p in model.parameters()], len(red.buckets)))

        # distributed Muon: round-robin NS + one async all_gather per group, NS from the CPU oracle
        import owl_wms.muon as mu

        # torch restatements of the fused HIP passes (muon.py:67-84) stand in for them on the CPU
        def _mom(grads, bufs, m, nesterov, out, sumsq):
            for i, (g, b) in enumerate(zip(grads, bufs)):
                b.lerp_(g, 1 - m)
                out[i] = (g.lerp(b, m) if nesterov else b).flatten()

        def _ns(G, sumsq, steps, out=None):
            tr = G.shape[1] > G.shape[2]
            U = torch.stack([R.newton_schulz5(x, steps) for x in G])
            U = U.transpose(1, 2).contiguous() if tr else U  # the iterate's layout before its transpose back
            if out is not None:
                out.copy_(U)
                U = out
            return U, tr

        def _app(params, u, r, c, tr, decay, alpha):
            for i, p in enumerate(params):
                ui = u.reshape(len(params), c, r)[i].T if tr else u.reshape(len(params), r, c)[i]
                p.mul_(decay).add_(ui.float(), alpha=-alpha)

        mu.momentum_update, mu.ns_orthogonalize, mu.apply_update = _mom, _ns, _app
        ps = [torch.nn.Parameter(torch.randn(*MUON_SHAPES[i], generator=torch.Generator().manual_seed(i)))
              for i in range(len(MUON_SHAPES))]
        for i, p in enumerate(ps):
            p.grad = torch.randn(*MUON_SHAPES[i], generator=torch.Generator().manual_seed(50 + i))
        opt = mu.Muon(ps, lr=0.1, momentum=0.95, rank=rank, world_size=ws)
        opt.step()
        q.put((rank, "muon", [p.detach().numpy().copy() for p in ps]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("ws", [2, 8])
def test_reducer_and_muon_world_size(ws):
    """ws 8 = the bench's largest node: 5 Muon matrices over 8 ranks leave ranks that own none."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as sk:  # a free port (a fixed one can still be held by an earlier run)
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = [ctx.Process(target=_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(2 * ws)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    grads = {r: [torch.from_numpy(a) for a in g] for r, g, *_ in [x for x in res if x[1] != "muon"]}
    nb = [x[2] for x in res if x[1] != "muon"][0]
    assert nb > 1
    # expected: mean over ranks of each rank's accumulated grads (single-process recompute)
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.SiLU(), torch.nn.Linear(32, 8))
    for rank in range(ws):
        g = torch.Generator().manual_seed(100 + rank)
        for micro in range(3):
            x = torch.randn(4, 16, generator=g)
            (model(x).pow(2).mean() / 3 / ws).backward()
    for r in range(ws):
        for a, b in zip(grads[r], [p.grad for p in model.parameters()]):
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    muon = [[torch.from_numpy(a) for a in x[2]] for x in res if x[1] == "muon"]
    for other in muon[1:]:
        for a, b in zip(muon[0], other):
            assert torch.equal(a, b)  # replicas bit-identical after the gathered updates
    # and equal to the single-rank update
    ps = [torch.randn(*s, generator=torch.Generator().manual_seed(i)) for i, s in enumerate(MUON_SHAPES)]
    for i, p in enumerate(ps):
        g = torch.randn(*MUON_SHAPES[i], generator=torch.Generator().manual_seed(50 + i))
        g2 = g.lerp(torch.zeros_like(g).lerp(g, 0.05), 0.95)
        u = R.newton_schulz5(g2).float()
        exp = p * (1 - 0.1 * 0.01) - 0.1 * max(1, p.shape[0] / p.shape[1]) ** 0.5 * u
        torch.testing.assert_close(muon[0][i], exp, rtol=1e-5, atol=1e-6)


def test_mmdit_schema_matches_reconstructed_reference():
    """GameRFTAudio (mmdit backbone) keys/shapes == the reconstructed reference's (mmdit_tiny.pt)."""
    from conftest import golden
    from owl_wms.configs import model_config
    from owl_wms.models.gamerft_audio import GameRFTAudio
    MM = golden("mmdit_tiny.pt")
    cfg = model_config(model_id="game_rft_audio", sample_size=8, channels=32, audio_channels=16, n_layers=2,
                       n_heads=2, d_model=128, tokens_per_frame=65, n_buttons=11, n_mouse_axes=2, cfg_prob=0.1,
                       n_frames=6, causal=True, uncond=False, backbone="mmdit", local_window=2, global_window=4,
                       has_audio=True)
    m = GameRFTAudio(cfg)
    assert [[k, list(v.shape)] for k, v in m.state_dict().items()] == MM["mmdit.schema"]
    torch.testing.assert_close(m.core.transformer.rope.cos, MM["mmdit.rope.cos"], atol=0, rtol=0)


def test_sd3_euler_schedule():
    """schedulers.py:5-13 restated (diffusers absent: parity-unpinned beyond this formula check):
    sigma' = 3 s / (1 + 2 s), s = (N - i) / N, dt_i = sigma'_i - sigma'_{i+1}, sigma'_N = 0."""
    from conftest import golden
    from owl_wms.sampling.schedulers import get_deltas, get_sd3_euler
    dt = get_sd3_euler(16)
    assert dt.shape == (16,) and abs(dt.sum().item() - 1.0) < 1e-6
    assert abs(dt[0].item() - (1 - 2.8125 / 2.875)) < 1e-6 and abs(dt[-1].item() - 0.1875 / 1.125) < 1e-6
    torch.testing.assert_close(get_sd3_euler(2), golden("sampler_tiny.pt")["av.dt"], atol=0, rtol=0)
    assert get_deltas([1.0, 0.5]) == [0.5, 0.5]


@pytest.mark.parametrize("n_ctrl,b", [(8, 8), (7, 8), (1, 8), (0, 8), (3, 4)])
def test_handle_cfg_host_fraction_matches_device_path(n_ctrl, b):
    """handle_cfg with the mask's mean known on the host (frac_host, no device -> host sync) draws
    the same rand(b) under the same condition and returns the same mask as the reference-order
    tensor path (gamerft.py:68-90), for every has_controls fraction around cfg_prob."""
    from owl_wms.models.flow import handle_cfg

    class Rec:
        def __init__(self, r):
            self.r, self.calls = r, 0

        def rand_b(self, n, device):
            self.calls += 1
            return self.r[:n]

    r = torch.rand(b, generator=torch.Generator().manual_seed(n_ctrl))
    hc = torch.zeros(b, dtype=torch.bool)
    hc[:n_ctrl] = True
    for cfg_prob in (0.1, 0.3, 0.9):
        a, bb = Rec(r), Rec(r)
        ref = handle_cfg(hc.clone(), cfg_prob, a)
        got = handle_cfg(hc.clone(), cfg_prob, bb, frac_host=n_ctrl / b)
        assert a.calls == bb.calls
        assert torch.equal(ref, got)


def test_gemm_splitk_workspace_query():
    """owlk_gemm_splitk_bytes (host-only arithmetic): the split-K workspace a weight-gradient GEMM
    needs; 0 where owlk_gemm does not split (short K, bf16 output, too many tiles)."""
    from owl_wms._lib import LIB_PATH, lib
    if not os.path.exists(LIB_PATH):
        pytest.skip("libowlk.so not built (run __graft_entry__.build())")
    q = lib().owlk_gemm_splitk_bytes
    # fc1 dW at dit_v4: 24 x 6 = 144 tiles of 256^2, K = 98,304 -> 7 splits (1,008 workgroups,
    # 3.94 rounds of 256 CUs)
    assert q(6144, 1536, 98304, 1, 1, 1, 1, 0, 0.0) == 7 * 6144 * 1536 * 4
    assert q(6144, 1536, 98304, 1, 1, 1, 1, 0, 1.0) == 7 * 6144 * 1536 * 4
    assert q(6144, 1536, 1536, 1, 1, 1, 1, 0, 0.0) == 0        # short K
    assert q(6144, 1536, 98304, 1, 1, 1, 0, 0, 0.0) == 0       # bf16 output
    assert q(98304, 6144, 98304, 1, 1, 1, 1, 0, 0.0) == 0      # enough tiles, no split
    assert q(6144, 1536, 98304, 1, 1, 1, 1, 0, 0.5) == 0       # beta other than 0 / 1


def _gemm_args(M=64, N=64, K=64, batch=1, A=4096, C=8192, c_f32=0, epi=0, colsum=None):
    return (M, N, K, batch, A, K, 0, 0, 4096, K, 0, 1, C, N, 0, c_f32, epi, 1.0, 0.0, None, None, 0, 0, None, 0, 0,
            0, None, 0, 0, colsum, None, 0, None)


def _attn_fwd_args(Lq=128, Lkv=128, D=64, doc=None, run_start=None):
    # q, k, v, o at 16-byte-aligned stand-in addresses; nothing is dereferenced (the checks fail first)
    return (4096, 3 * D, 0, 4096, 3 * D, 0, 4096, 3 * D, 0, 8192, D, 0, None, 1, 1, Lq, Lkv, D, D ** -0.5, 0.0, 64,
            0, 1, 0, None, None, run_start, doc, 0, None)


def _attn_bwd_args(Lq=128, Lkv=128, D=64):
    p = (4096, D, 0)
    return (p + p + p + p + (None, None) + p + p + p + (1, 1, Lq, Lkv, D, D ** -0.5, 64, 0, 1)
            + (None, None, None, None, 0, None))


@pytest.mark.parametrize("name,args,msg", [
    ("owlk_gemm", _gemm_args(M=0), "gemm: bad sizes M=0"),
    ("owlk_gemm", _gemm_args(N=12), "N=12 must be a multiple of 8"),
    ("owlk_gemm", _gemm_args(A=4104), "16-byte aligned"),
    ("owlk_gemm", _gemm_args(c_f32=1, epi=1), "fp32 output only with EPI_STORE"),
    ("owlk_gemm", _gemm_args(batch=2, colsum=4096), "colsum needs batch 1"),
    ("owlk_attn_fwd", _attn_fwd_args(D=96), "head_dim 96 not built"),
    ("owlk_attn_fwd", _attn_fwd_args(Lq=0), "attn_fwd: bad sizes"),
    ("owlk_attn_fwd", _attn_fwd_args(doc=4096), "doc mask needs run_start"),
    ("owlk_attn_bwd", _attn_bwd_args(Lkv=256), "training shapes only"),
    ("owlk_attn_bwd_dq", _attn_bwd_args(D=32), "head_dim 32 not built"),
    ("owlk_adaln_fwd", (4096, 12, 4096, 4096, 12, 64, 128, 12, 8192, 12, None, None, None), "adaln_fwd: bad d=12"),
    ("owlk_adaln_fwd", (4096, 64, 4096, 4096, 64, 64, 100, 64, 8192, 64, None, None, None), "T=100"),
])
def test_c_abi_rejects_bad_arguments(name, args, msg):
    """The C ABI's error behaviour (owlk.h: every entry returns 0 or an error code with a message in
    owlk_last_error()): shapes, layouts and alignments a kernel cannot take are refused on the host
    before any HIP call, so this runs without a GPU; through the package binding they raise
    RuntimeError (the reference's ops raise on unsupported shapes too, e.g. flex_attention)."""
    from owl_wms import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libowlk.so not built (run __graft_entry__.build())")
    assert getattr(_lib.lib(), name)(*args) != 0
    assert msg in _lib.lib().owlk_last_error().decode()
    with pytest.raises(RuntimeError, match=re.escape(msg)):
        _lib.call(name, *args)


@pytest.mark.parametrize("window", [None, 3])
def test_mask_pairs_counts_documents(window):
    """The algorithmic FLOP count (allowed pairs only) with document arrays equals a
    brute-force count of the reference predicate (attn.py:24-62) and, for one document, the
    analytic doc-free count."""
    from owl_wms import kernels as K
    tpf, nf = 4, 12
    doc = torch.tensor([[0] * 5 + [1] * 4 + [2] * 3, [7] * 12])
    m = K.FrameMask(tpf, window, arrays=K.frame_arrays(doc, nf, window))
    brute = 0
    for b in range(2):
        for qf in range(nf):
            for kf in range(nf):
                ok = kf <= qf and (window is None or qf - kf < window) and bool(doc[b, qf] == doc[b, kf])
                brute += ok * tpf * tpf
    assert K.mask_pairs(m, nf * tpf, nf * tpf) == brute / 2
    one = K.FrameMask(tpf, window, arrays=K.frame_arrays(doc[1:], nf, window))
    assert K.mask_pairs(one, nf * tpf, nf * tpf) == K.mask_pairs(K.FrameMask(tpf, window), nf * tpf, nf * tpf)


@pytest.mark.parametrize("window", [None, 1, 3])
def test_frame_arrays_runs_form_is_exact(window):
    """Packed (contiguous-run) documents: frame_arrays flags them and the range form the kernels
    then use -- allowed(q, k) <=> kv_lo[q] <= k <= q <=> k <= q <= q_hi[k] -- equals the reference
    predicate (attn.py:24-62) exactly; recurring documents are not flagged."""
    from owl_wms.kernels import frame_arrays
    g = torch.Generator().manual_seed(3)
    nf = 23
    for _ in range(6):
        cuts = sorted(torch.randperm(nf - 1, generator=g)[:4].add(1).tolist())
        doc = torch.zeros(1, nf, dtype=torch.long)
        for i, c in enumerate(cuts):
            doc[0, c:] = 10 * (i + 1)
        a = frame_arrays(doc, nf, window)
        assert a["runs"]
        lo, hi = a["kv_lo"][0].tolist(), a["q_hi"][0].tolist()
        for fq in range(nf):
            for fk in range(nf):
                ref = fk <= fq and (window is None or fq - fk < window) and bool(doc[0, fq] == doc[0, fk])
                assert ref == (lo[fq] <= fk <= fq) == (fk <= fq <= hi[fk])
    rec = torch.tensor([[0, 0, 1, 1, 0, 0]])
    assert not frame_arrays(rec, 6, window)["runs"]


def test_kv_cache_extend_matches_cat_model():
    """The preallocated KV cache (kv_cache.py:5-104 API): extend == torch.cat([cache, new]) with the
    cache unchanged until update commits it; update / truncate (both ends) / get / offsets behave as
    the reference's list-of-tensors cache, across buffer growth and compaction."""
    from types import SimpleNamespace
    from owl_wms.nn.kv_cache import SingleKVCache
    cfg = SimpleNamespace(n_layers=2, tokens_per_frame=4)
    c = SingleKVCache(cfg)
    c.reset(2)
    g = torch.Generator().manual_seed(0)
    new = lambda n: torch.randn(2, n, 8, generator=g)
    ref = []
    for i in range(2):
        k, v = new(12), new(12)
        c.update(k[:, :], v, i)
        ref.append((k.clone(), v.clone()))
    off = [12, 12]
    for step in range(30):
        for i in range(2):
            kn, vn = new(4), new(4)
            K_, V_ = c.extend(i, kn, vn)
            RK, RV = torch.cat([ref[i][0], kn], 1), torch.cat([ref[i][1], vn], 1)
            assert torch.equal(K_, RK) and torch.equal(V_, RV)
            if step % 3 == 0:
                c.update(K_, V_, i)
                ref[i] = (RK, RV)
                off[i] += 4
        if step % 7 == 6:
            c.truncate(1, front=False)
            ref = [(a[:, 4:], b[:, 4:]) for a, b in ref]
        if step % 11 == 10:
            c.truncate(1, front=True)
            ref = [(a[:, :-4], b[:, :-4]) for a, b in ref]
        for i in range(2):
            k, v = c.get(i)
            assert torch.equal(k, ref[i][0]) and torch.equal(v, ref[i][1])
            assert c.length_at(i) == ref[i][0].shape[1]
    assert c.offsets == off


def test_log_helper_semantics():
    """utils/logging.py:33-64: per-key sums of value / world_size over the logged micro-steps
    (the caller divides by accum); pop() clears.  Device tensors are summed without host syncs."""
    from owl_wms.utils.logging import LogHelper
    m = LogHelper()
    for v in (torch.tensor(0.5), torch.tensor(0.25), 0.125):
        m.log("diffusion_loss", v)
    m.log_dict({"x": 2.0})
    out = m.pop()
    assert out == {"diffusion_loss": 0.875, "x": 2.0}
    assert m.pop() == {}


def test_strip_prefixes_model_and_ema_keys():
    """rft_trainer.py:86-89: compiled / DDP prefixes stripped from model AND EMA keys."""
    from owl_wms.utils import strip_prefixes
    sd = {"_orig_mod.module.core.proj_in.weight": 1, "module.core.x": 2, "core.y": 3,
          "ema_model._orig_mod.module.core.proj_in.weight": 4, "ema_model.module.core.z": 5, "initted": 6, "step": 7}
    assert strip_prefixes(sd) == {"core.proj_in.weight": 1, "core.x": 2, "core.y": 3,
                                  "ema_model.core.proj_in.weight": 4, "ema_model.core.z": 5, "initted": 6, "step": 7}


def test_scheduler_registry():
    """schedulers.py: the reference's factory is an empty stub; names resolve to torch LR schedulers,
    anything else fails loudly at construction."""
    from owl_wms.schedulers import get_scheduler_cls
    assert get_scheduler_cls("LinearLR") is torch.optim.lr_scheduler.LinearLR
    with pytest.raises(NotImplementedError):
        get_scheduler_cls("warmup_cosine_custom")


def test_muon_group_order_matches_reference():
    """muon.py:52 iterates a set of numels: the param groups come out in that order (dit_v4: qkv,
    out, fc), so a reference Muon state_dict loads onto the same parameters."""
    from owl_wms.muon import Muon
    numels = [(4608, 1536), (1536, 1536), (6144, 1536), (1536, 6144)] * 2 + [(3072, 1536)]
    ps = [torch.nn.Parameter(torch.empty(s, device="meta")) for s in numels]
    opt = Muon(ps, lr=1e-3, rank=0, world_size=1)
    ref_order = list({p.numel() for p in ps})
    assert [g["params"][0].numel() for g in opt.param_groups] == ref_order
    assert ref_order[:3] == [7077888, 2359296, 9437184]  # the order the survey recorded for dit_v4


def test_batch_permute_to_length():
    """utils/__init__.py:69-118: controls doubled by batch permutation until long enough."""
    from owl_wms.utils import batch_permute_to_length
    m, b = torch.randn(4, 5, 2), torch.randn(4, 5, 11)
    m2, b2 = batch_permute_to_length(m, b, 17)
    assert m2.shape == (4, 17, 2) and b2.shape == (4, 17, 11)
    assert torch.equal(m2[:, :5], m) and torch.equal(b2[:, :5], b)


def test_grad_reducer_stacks_tagged_params_back_to_back():
    """Parameters tagged _owl_grad_stack (the DiT block's four modulation weights) get adjacent bucket
    views in index order, whatever the bucket size, so the block's backward can form their gradients
    as one [6d, d] GEMM (nn/fused.py _stacked_mod_sink)."""
    from owl_wms.configs import model_config
    from owl_wms.models.gamerft import GameRFT
    from owl_wms.nn.fused import _stacked_mod_sink
    from owl_wms.utils.grad_reducer import GradReducer
    cfg = model_config(model_id="game_rft", sample_size=8, channels=32, n_layers=2, n_heads=2, d_model=128,
                       tokens_per_frame=64, n_buttons=11, cfg_prob=0.1, n_frames=8, causal=True, uncond=False,
                       backbone="dit", has_audio=False, rope_impl="motion", local_window=2, global_window=None)
    m = GameRFT(cfg)
    for mb in (256, 0.05):  # one bucket; buckets smaller than a stack (the stack stays whole)
        red = GradReducer(m.parameters(), bucket_mb=mb, world_size=1)
        blocks = [b for b in m.modules() if hasattr(b, "mod_params") and hasattr(b, "gate2")]
        assert blocks
        for b in blocks:
            ws = b.mod_params()[0]
            assert len({red.bucket_of[w] for w in ws}) == 1
            st = _stacked_mod_sink(ws, 128)
            assert st is not None and st.shape == (6 * 128, 128)
            st.fill_(0)
            st[:256].fill_(1)
            assert (ws[0].grad == 1).all() and (ws[1].grad == 0).all()
        for h in red.hooks:
            h.remove()
