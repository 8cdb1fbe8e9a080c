"""The single-pass attention backward (owlk_attn_bwd_fused, csrc/attn_bwd_fused.hip) against the
fp32 oracle and the two-kernel backward, and its ordered dQ hand-off checked word by word.

Reference: the one compiled flex_attention backward of attn.py:13-16, 106-109 (dQ, dK, dV from one
pass); mask attn.py:24-62 without window / documents (dit_v4's global layers).  Tolerances: rel-L2
<= 1e-2 against the fp32 oracle (SURVEY §8(c) per-op); the fused and the two-kernel bf16 results
differ only in fp32 summation order and in the bf16 rounding of dS in the dQ product (<= 5e-3).
"""
import pytest
import torch

from oracle import ref_ops as R

pytestmark = pytest.mark.gpu

DEV = "cuda"
FQT = 64  # query rows per swept tile (attn_bwd_fused.hip); keys per work item: workspace int32 word 9


def K():
    from owl_wms import kernels
    return kernels


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def rnd(*shape, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g).to(torch.bfloat16).to(DEV)


@pytest.fixture(scope="module", autouse=True)
def _needs_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from owl_wms._lib import lib
    lib()


def _inputs(B, H, L, D, seed):
    q, kk, v, do = (rnd(B, L, H * D, seed=seed + i) for i in range(4))
    return q, kk, v, do


def _delta(o, do, H, D):
    from owl_wms import _lib
    B, L = o.shape[:2]
    delta = torch.empty(B, H, L, device=DEV, dtype=torch.float32)
    _lib.call("owlk_attn_delta", _lib.ptr(o), _lib.ptr(do), o.stride(1), B, L, H, D, _lib.ptr(delta), _lib.stream())
    return delta


def _hdr(ws):
    return ws[:256].view(torch.int32).cpu()


def _sweeps(L, tpf, causal, window, FKB):
    """query tiles each key block sweeps (attn_bwd_fused.hip sweep_lo / sweep_hi): from the first
    query tile that sees its first key's frame to the last that sees its last key's frame"""
    out = []
    for j in range((L + FKB - 1) // FKB):
        f0, f1 = (j * FKB) // tpf, min(j * FKB + FKB - 1, L - 1) // tpf
        qlo = f0 if causal else (max(0, f0 - window + 1) if window else 0)
        qend = min(L, (f1 + window) * tpf) if window else L
        out.append(((qlo * tpf) // FQT, (qend - 1) // FQT))
    return out


def _jrange(L, tpf, causal, window, FKB):
    """the key blocks that sweep each query tile, by the definition (min / max over the sweeps),
    independent of the kernel's closed forms tile_jlo / tile_jhi"""
    sw = _sweeps(L, tpf, causal, window, FKB)
    lo, hi = [], []
    for i in range((L + FQT - 1) // FQT):
        js = [j for j, (a, b) in enumerate(sw) if a <= i <= b]
        assert js == list(range(js[0], js[-1] + 1)), "sweep ranges must give contiguous contributors"
        lo.append(js[0])
        hi.append(js[-1])
    return torch.tensor(lo), torch.tensor(hi)


FUSED_CASES = [
    # (B, H, n_frames, tpf, causal, window)
    (1, 2, 8, 64, True, None),  # 2 key blocks, 8 query tiles
    (2, 3, 20, 64, True, None),  # 6 chains (< 8 XCD queues), 5 key blocks
    (1, 2, 7, 65, True, None),  # ragged end, frames across tile seams (455 tokens)
    (1, 1, 300, 1, True, None),  # token-causal: PARTIAL diagonal tiles, ragged last key block
    (1, 2, 40, 64, False, None),  # unmasked (every block sweeps every tile)
    (2, 8, 48, 64, True, None),  # 16 chains x 12 key blocks
    (1, 2, 48, 64, True, 16),  # dit_v4's local layers: a tile's first contributor is not block 0
    (1, 2, 30, 65, True, 4),  # window of 4 frames across tile seams
    (1, 2, 40, 64, False, 3),  # windowed, not causal (keys see queries on both sides)
    (1, 1, 600, 1, True, 100),  # token-causal window: PARTIAL tiles on both edges
    (2, 3, 30, 65, True, 4),  # batch 2 x 3 heads, windowed (mmdit_v2's 65-token frames)
]


# write-through, XCD-local, XCD-local one chain at a time; bit 7: one wave per SIMD (attn_bwd_fused4.hip,
# the hand-placed main step)
@pytest.mark.parametrize("variant", [0, 1, 5, 128, 129])
@pytest.mark.parametrize("case", FUSED_CASES)
def test_attention_bwd_fused_vs_oracle_and_split(case, variant, monkeypatch):
    k = K()
    B, H, nf, tpf, causal, window = case
    D, L = 64, nf * tpf
    q, kk, v, do = _inputs(B, H, L, D, 100)
    mask = k.FrameMask(tpf, window, causal)
    o, lse = k.attn_fwd(q, kk, v, H, D, mask)
    delta = _delta(o, do, H, D)
    got = [torch.full_like(q, float("nan")) for _ in range(3)]
    ws = k.attn_bwd_fused(q, kk, v, do, lse, delta, H, D, mask, *got, D ** -0.5, variant)
    torch.cuda.synchronize()
    assert _hdr(ws)[8].item() == 0, "hand-off wait timed out"
    monkeypatch.setenv("OWLK_BWD_FUSED", "0")
    split = [torch.empty_like(q) for _ in range(3)]
    k.attn_bwd(q, kk, v, o, do, lse, H, D, mask, *split)
    # fp32 oracle
    qr, kr, vr = (t.cpu().float().view(B, L, H, D).transpose(1, 2).requires_grad_() for t in (q, kk, v))
    m = R.frame_mask(L, L, tpf, window, None, causal=causal)
    oref = R.attention(qr, kr, vr, m)
    oref.backward(do.cpu().float().view(B, L, H, D).transpose(1, 2))
    for name, g, s, ref in zip(("dq", "dk", "dv"), got, split, (qr.grad, kr.grad, vr.grad)):
        assert torch.isfinite(g).all(), name
        assert rel(g.view(B, L, H, D).transpose(1, 2), ref) < 1e-2, name
        assert rel(g, s) < 5e-3, name


@pytest.mark.parametrize("variant_env", ["1", "2"])  # write-through, XCD-local
def test_attention_bwd_fused_timeout_poisons_dq(variant_env, monkeypatch):
    """A hand-off wait that times out cannot pass unnoticed: forced in test mode (variant bit 6: chain
    0's key block 1 waits for a flag no block stores), kernels.attn_bwd -- the production entry --
    returns NaN dQ rows (the tiles that block sweeps, and every tile whose wait gave up after it),
    sets the error word, and leaves dK / dV (formed without the hand-off) finite (the model-level
    consequence: tests/test_model_gpu.py::test_fused_handoff_timeout_reaches_the_loss).  Two 2-s spins
    at most."""
    k = K()
    B, H, nf, tpf, D = 1, 2, 16, 64, 64
    L = nf * tpf
    q, kk, v, do = _inputs(B, H, L, D, 300)
    mask = k.FrameMask(tpf, None, True)
    o, lse = k.attn_fwd(q, kk, v, H, D, mask)
    monkeypatch.setenv("OWLK_BWD_FUSED", variant_env)
    monkeypatch.setattr(k, "FUSED_FAIL_TEST", True)
    dq, dk, dv = (torch.zeros_like(q) for _ in range(3))
    k.attn_bwd(q, kk, v, o, do, lse, H, D, mask, dq, dk, dv)
    torch.cuda.synchronize()
    dq0 = dq.view(B, L, H, D)[:, :, 0]  # chain 0 = head 0
    # block 1 (keys 256..511) sweeps query tiles 4.. (causal): their dQ is void
    assert torch.isnan(dq0[:, 256:].float()).any(), "timed-out hand-off left no NaN in dQ"
    assert torch.isfinite(dk.float()).all() and torch.isfinite(dv.float()).all()
    # the raw entry reports it in the error word
    delta = _delta(o, do, H, D)
    ws = k.attn_bwd_fused(q, kk, v, do, lse, delta, H, D, mask, dq, dk, dv, D ** -0.5,
                          k.fused_bwd_variant(D, mask))
    torch.cuda.synchronize()
    assert _hdr(ws)[8].item() == 1


@pytest.mark.parametrize("case", [(2, 8, 48, 64, True, None), (1, 2, 40, 64, False, None), (1, 1, 300, 1, True, None),
                                  (1, 2, 48, 64, True, 16)])
def test_attention_bwd_fused_deterministic(case):
    """Every query tile receives its key blocks' dQ parts in key-block order, so two runs -- and the
    write-through and the XCD-local hand-offs, which differ only in where the sums live, and the
    chain-group dequeue orders (variant bits 2-5) -- give the same bits.  So does the one-wave-per-SIMD
    kernel (bit 7): its hand-placed step forms every product in the 8-wave kernel's order."""
    k = K()
    B, H, nf, tpf, causal, window = case
    D, L = 64, nf * tpf
    q, kk, v, do = _inputs(B, H, L, D, 200)
    mask = k.FrameMask(tpf, window, causal)
    o, lse = k.attn_fwd(q, kk, v, H, D, mask)
    delta = _delta(o, do, H, D)
    runs = []
    for variant in (0, 0, 1, 1, 5, 9, 128, 129, 133):
        g = [torch.full_like(q, float("nan")) for _ in range(3)]
        ws = k.attn_bwd_fused(q, kk, v, do, lse, delta, H, D, mask, *g, D ** -0.5, variant)
        torch.cuda.synchronize()
        assert _hdr(ws)[8].item() == 0
        runs.append(g)
    for r in runs[1:]:
        for a, b in zip(runs[0], r):
            assert torch.equal(a, b)


@pytest.mark.parametrize("variant", [1, 129])
def test_attention_bwd_fused_cu_reserve(variant):
    """owlk_set_cu_reserve (the gradient all-reduce's room, utils/grad_reducer.py): the persistent grid
    shrinks to (CUs - k) workgroups per CU-slot, at least one per XCD, so every per-XCD queue is still
    drained (error word 0) and the ordered hand-off gives the full grid's bits at k = 8, 16 and a k
    past the CU count (clamped to 8 CUs)."""
    from owl_wms import _lib
    k = K()
    B, H, nf, tpf = 1, 4, 48, 64
    D, L = 64, nf * tpf
    q, kk, v, do = _inputs(B, H, L, D, 400)
    mask = k.FrameMask(tpf, None, True)
    o, lse = k.attn_fwd(q, kk, v, H, D, mask)
    delta = _delta(o, do, H, D)
    runs = []
    try:
        for cus in (0, 8, 16, 100000):
            _lib.call("owlk_set_cu_reserve", cus)
            g = [torch.full_like(q, float("nan")) for _ in range(3)]
            ws = k.attn_bwd_fused(q, kk, v, do, lse, delta, H, D, mask, *g, D ** -0.5, variant)
            torch.cuda.synchronize()
            assert _hdr(ws)[8].item() == 0, f"reserve {cus}: error word set"
            runs.append(g)
    finally:
        _lib.call("owlk_set_cu_reserve", 0)
    for r in runs[1:]:
        for a, b in zip(runs[0], r):
            assert torch.equal(a, b)
    with pytest.raises(RuntimeError):
        _lib.call("owlk_set_cu_reserve", -1)


@pytest.mark.parametrize("variant", [2, 3, 7, 131])
@pytest.mark.parametrize("shape", [(1, 24, 1536, 64, True, None), (2, 3, 20, 64, True, None), (1, 1, 300, 1, True, None),
                                   (1, 2, 40, 64, False, None), (1, 8, 96, 65, True, None),
                                   (1, 24, 1536, 64, True, 16), (1, 2, 30, 65, True, 4), (1, 2, 40, 64, False, 3),
                                   (1, 1, 600, 1, True, 100)])
def test_attention_bwd_fused_handoff_counts(shape, variant):
    """Counting form of the hand-off (variant bit 1): every key block adds 1.0 instead of its dQ
    part and the last one keeps the fp32 sum, so each of the 4,096 words of every query tile's sum
    must equal the number of key blocks that sweep the tile -- a stale read or a lost add anywhere
    shows as a smaller count, a hand-off that started from zeros too late or too early as another.
    Checked at the full dit_v4 shapes (24 heads x 98,304 tokens, 1,536 tiles x 384 key blocks per
    head, global and window 16), for both hand-off forms and the one-chain-at-a-time dequeue; the
    flags end at one past each tile's last contributor."""
    k = K()
    B, H, nf, tpf, causal, window = shape
    D, L = 64, nf * tpf
    q, kk, v, do = _inputs(B, H, L, D, 300)
    mask = k.FrameMask(tpf, window, causal)
    lse = torch.zeros(B, H, L, device=DEV)
    delta = torch.zeros(B, H, L, device=DEV)
    dq, dk, dv = (torch.empty_like(q) for _ in range(3))
    ws = k.attn_bwd_fused(q, kk, v, do, lse, delta, H, D, mask, dq, dk, dv, D ** -0.5, variant)
    torch.cuda.synchronize()
    assert _hdr(ws)[8].item() == 0, "hand-off wait timed out"
    nchain, nt = B * H, (L + FQT - 1) // FQT
    fkb = _hdr(ws)[9].item()
    assert fkb in (128, 256)
    jlo, jhi = _jrange(L, tpf, causal, window, fkb)
    want_flag = (jhi + 1).to(DEV)
    want_sum = (jhi - jlo + 1).to(DEV)  # every contributor adds 1.0, the first onto zeros
    flags = ws[256:256 + nchain * nt * 64].view(torch.int32).view(nchain, nt, 16)[:, :, 0]
    assert torch.equal(flags, want_flag[None, :].to(torch.int32).expand(nchain, nt))
    acc = ws[256 + nchain * nt * 64:256 + nchain * nt * (64 + FQT * 64 * 4)].view(torch.float32)
    acc = acc.view(nchain, nt, FQT * 64)
    bad = (acc != want_sum[None, :, None].float()).sum().item()
    assert bad == 0, f"{bad} accumulator words off"


def _runs_doc(B, nf, lens, seed):
    """[B, nf] doc ids as contiguous runs (sequence packing): sample b's documents have the lengths
    lens[b] (frames), the last one filling the rest"""
    doc = torch.zeros(B, nf, dtype=torch.int64)
    for b in range(B):
        f, d = 0, 0
        for n in lens[b]:
            doc[b, f:f + n] = d
            f, d = f + n, d + 1
        doc[b, f:] = d
    return doc


DOC_CASES = [
    # (B, H, n_frames, tpf, window, document lengths per sample)
    (1, 2, 24, 64, None, [[5, 9, 3]]),  # four documents, runs across key-block and tile seams
    (2, 3, 20, 64, None, [[7], [2, 2, 11]]),  # per-sample layouts (each chain its own runs)
    (1, 2, 30, 65, 4, [[10, 13]]),  # window folded into kv_lo / q_hi, 65-token frames
    (1, 1, 300, 1, None, [[37, 100, 1, 62]]),  # token-causal: documents of 1..100 tokens
    (2, 8, 48, 64, 16, [[12, 12, 12], [30]]),  # dit_v4's local layers over packed documents
]


@pytest.mark.parametrize("variant", [0, 5, 129])
@pytest.mark.parametrize("case", DOC_CASES)
def test_attention_bwd_fused_packed_documents(case, variant, monkeypatch):
    """Causal masks of packed documents (kv_lo / q_hi, the runs form): the single pass against the
    fp32 oracle with the document predicate (attn.py:24-62) and against the two-kernel backward,
    and bitwise equal across hand-off forms."""
    k = K()
    B, H, nf, tpf, window, lens = case
    D, L = 64, nf * tpf
    q, kk, v, do = _inputs(B, H, L, D, 400)
    doc = _runs_doc(B, nf, lens, 0)
    arrays = k.frame_arrays(doc.to(DEV), nf, window)
    assert arrays["runs"]
    mask = k.FrameMask(tpf, window, True, arrays=arrays)
    assert k.fused_bwd_variant(D, mask) is not None
    o, lse = k.attn_fwd(q, kk, v, H, D, mask)
    delta = _delta(o, do, H, D)
    got = [torch.full_like(q, float("nan")) for _ in range(3)]
    ws = k.attn_bwd_fused(q, kk, v, do, lse, delta, H, D, mask, *got, D ** -0.5, variant)
    torch.cuda.synchronize()
    assert _hdr(ws)[8].item() == 0, "hand-off wait timed out"
    again = [torch.full_like(q, float("nan")) for _ in range(3)]
    k.attn_bwd_fused(q, kk, v, do, lse, delta, H, D, mask, *again, D ** -0.5, 1 - (variant & 1))
    torch.cuda.synchronize()
    for a, b in zip(got, again):
        assert torch.equal(a, b)
    monkeypatch.setenv("OWLK_BWD_FUSED", "0")
    split = [torch.empty_like(q) for _ in range(3)]
    k.attn_bwd(q, kk, v, o, do, lse, H, D, mask, *split)
    qr, kr, vr = (t.cpu().float().view(B, L, H, D).transpose(1, 2).requires_grad_() for t in (q, kk, v))
    m = R.frame_mask(L, L, tpf, window, doc, causal=True)
    oref = R.attention(qr, kr, vr, m)
    oref.backward(do.cpu().float().view(B, L, H, D).transpose(1, 2))
    for name, g, s, ref in zip(("dq", "dk", "dv"), got, split, (qr.grad, kr.grad, vr.grad)):
        assert torch.isfinite(g).all(), name
        assert rel(g.view(B, L, H, D).transpose(1, 2), ref) < 1e-2, name
        assert rel(g, s) < 5e-3, name
