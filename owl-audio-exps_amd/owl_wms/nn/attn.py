"""attn.py (reference: owl_wms/nn/attn.py) -- DiT backbone on libowlk.

``get_block_mask`` returns a :class:`FrameMask` (analytic frame/window/doc description consumed
by the attention kernels) instead of a dense-evaluated flex BlockMask: same mask semantics
(attn.py:24-62), O(frames) host work instead of 2 x T^2 predicate evaluations per step.

Training path: ``DiTBlock.forward`` -> ``DiTBlockFn`` (whole block fwd+bwd fused on libowlk).
Sampling path (``kv_cache`` given): a no-grad functional path with the reference's cache
semantics (attn.py:86-107): cached K/V prepended, local layers keep the last
``local_window * tokens_per_frame`` keys when decoding unmasked.
"""
import torch
import weakref
from torch import nn
from torch.utils.checkpoint import checkpoint as torch_checkpoint

from .. import kernels as K
from .fused import (BlockGeometry, DiTBlockFn, ModFn, adaln_mod, bf16_weight, cond_silu, linear,
                    stacked_modulation_weights)
from .mlp import MLP
from .modulation import AdaLN, Gate
from .rope import get_rope_cls


def checkpoint(function, *args, **kwargs):
    kwargs.setdefault("use_reentrant", False)
    return torch_checkpoint(function, *args, **kwargs)


def get_block_mask(n_tokens, tokens_per_frame, window_len=None, doc_id=None, q_offset=0, is_causal=True,
                   device="cuda"):
    """attn.py:24-62 -> FrameMask (Q_LEN = n_tokens - q_offset, KV_LEN = n_tokens)."""
    assert 0 <= q_offset < n_tokens, "kv cache cannot exceed total tokens"
    if not is_causal:
        assert q_offset == 0, "kv caching not supported with bidirectional"
    arrays = None
    if doc_id is not None:
        n_frames = (n_tokens + tokens_per_frame - 1) // tokens_per_frame
        # one document per sample (the unpacked case): the doc_id predicate of mask_mod is always
        # true, so the kernels take the document-free path (analytic FULL-tile ranges, no
        # per-frame array reads in the tile loop)
        if not _single_document(doc_id, n_frames):
            arrays = K.frame_arrays(doc_id.to(device)[:, :n_frames], n_frames, window_len, is_causal)
    return K.FrameMask(tokens_per_frame, window_len, is_causal, q_offset, arrays)


_single_doc_cache = {}  # id(tensor) -> (weakref, version, n_frames, result)


def _single_document(doc_id, n_frames):
    """True when every sample's frames [0, n_frames) carry one doc id.  Evaluated on the host for
    a CPU tensor; for a device tensor once per tensor object and version (checked through a weak
    reference, so a new tensor at a recycled address or id never hits): the local and global
    masks of a forward, and a batch reused across micro-steps, share one device -> host sync."""
    doc = doc_id[:, :n_frames]
    if doc.device.type == "cpu":
        return bool((doc == doc[:, :1]).all())
    hit = _single_doc_cache.get(id(doc_id))
    if hit is not None and hit[0]() is doc_id and hit[1] == doc_id._version and hit[2] == n_frames:
        return hit[3]
    if len(_single_doc_cache) > 64:
        _single_doc_cache.clear()
    res = bool((doc == doc[:, :1]).all())
    _single_doc_cache[id(doc_id)] = (weakref.ref(doc_id), doc_id._version, n_frames, res)
    return res


def check_rope_rows(rope, offset, n):
    """Positions offset .. offset + n - 1 must lie in the RoPE table (config.n_frames frames): the
    reference slices cos[offset:offset + n] and its rotation fails on the short slice (rope.py:46-49);
    the kernels would read past the table instead, so this raises first, as the reference does."""
    rows = rope.cos.shape[0]
    if offset < 0 or offset + n > rows:
        raise RuntimeError(f"RoPE positions {offset}..{offset + n - 1} lie past the {rows}-row table "
                           f"(config.n_frames frames); decode at most n_frames frames of context + new frames")


class Attn(nn.Module):
    def __init__(self, config, layer_idx, local=False, rope=None):
        super().__init__()
        self.config = config
        self.layer_idx = layer_idx
        self.n_heads = config.n_heads
        self.qkv = nn.Linear(config.d_model, 3 * config.d_model)
        self.out = nn.Linear(config.d_model, config.d_model)
        # one RoPE table per model (non-persistent buffers, rope.py:40-41), shared by every layer
        object.__setattr__(self, "rope", rope if rope is not None else
                           get_rope_cls(getattr(config, "rope_impl", "ortho"))(config))
        self.local = local
        self.local_offset = config.local_window * config.tokens_per_frame

    def forward(self, x, block_mask, kv_cache=None):
        """Stand-alone attention (x already modulated) -- reference API; no-grad cache path."""
        B, L, d = x.shape
        H = self.n_heads
        D = d // H
        x2 = x.reshape(B * L, d).to(torch.bfloat16).contiguous()
        qkv = K.gemm(x2, bf16_weight(self.qkv.weight), bias=self.qkv.bias)
        o = self._attend(qkv, B, L, block_mask, kv_cache)
        return K.gemm(o.reshape(B * L, d), bf16_weight(self.out.weight), bias=self.out.bias).view(B, L, d)

    def _attend(self, qkv, B, L, block_mask, kv_cache):
        d = self.config.d_model
        H = self.n_heads
        D = d // H
        offset = kv_cache.get_offset(self.layer_idx) if kv_cache is not None else 0
        check_rope_rows(self.rope, offset, L)
        if block_mask is None and getattr(kv_cache, "dev", None) is not None and offset > 0 and \
                K.decode_dev_supported(D, L):
            # decode with the cache position on the device (one captured graph for every frame)
            kb, vb = kv_cache.bufs[self.layer_idx]
            q = torch.empty(B, L, d, device=qkv.device, dtype=torch.bfloat16)
            K.qk_rope_fwd_kv_dev(qkv, B, L, H, D, self.rope.cos, self.rope.sin, kv_cache.dev, q, kb, vb)
            o, _ = K.attn_decode_fwd(q, kb, vb, H, D, kv_cache.dev, L, self.local_offset if self.local else 0,
                                     score_bound=K.qk_norm_bound(D))
            if kv_cache.should_update:
                kv_cache.commit_device(self.layer_idx, L)
            return o
        if offset > 0 and kv_cache.noise_caches == 0.0 and hasattr(kv_cache, "extend_slots"):
            # decode: rotated k and v written straight into the cache's slots behind its window
            q = torch.empty(B, L, d, device=qkv.device, dtype=torch.bfloat16)
            ks, vs = kv_cache.extend_slots(self.layer_idx, L, q)
            K.qk_rope_fwd_kv(qkv, B, L, H, D, self.rope.cos, self.rope.sin, offset, q, ks, vs)
            k, v = kv_cache.extended(self.layer_idx, L)
            offset = -1  # the [cache | new] views are in hand
        else:
            qkr, _ = K.qk_rope_fwd(qkv, H, D, self.rope.cos, self.rope.sin, offset, L)
            q = qkr.view(B, L, 2 * d)[:, :, :d]
            k = qkr.view(B, L, 2 * d)[:, :, d:]
            v = qkv.view(B, L, 3 * d)[:, :, 2 * d:]
        if offset > 0:
            if kv_cache.noise_caches == 0.0 and hasattr(kv_cache, "extend"):
                k, v = kv_cache.extend(self.layer_idx, k, v)  # [cache | new] in place, no torch.cat
            else:
                old_k, old_v = kv_cache.get(self.layer_idx)
                k = torch.cat([old_k, k], dim=1)
                v = torch.cat([old_v, v], dim=1)
        if kv_cache is not None and kv_cache.should_update:
            kv_cache.update(k, v, self.layer_idx)
        if block_mask is None:  # decoding: unmasked over [cache | new] (attn.py:101-107)
            if self.local:
                k, v = k[:, -self.local_offset:], v[:, -self.local_offset:]
            mask = K.FrameMask(1, None, False, 0, None)
        else:
            mask = block_mask
        o, _ = K.attn_fwd(q, k, v, H, D, mask, score_bound=K.qk_norm_bound(D))  # q, k RMS-normalised
        return o


class DiTBlock(nn.Module):
    def __init__(self, config, layer_idx, local=False, rope=None):
        super().__init__()
        dim = config.d_model
        self.attn = Attn(config, layer_idx, local, rope)
        self.mlp = MLP(config)
        self.adaln1 = AdaLN(dim)
        self.gate1 = Gate(dim)
        self.adaln2 = AdaLN(dim)
        self.gate2 = Gate(dim)
        self.config = config
        # GradReducer lays these four weights' gradient views out back to back in this order, a [6d, d]
        # stack: the block's backward then forms their gradients as ONE weight-gradient GEMM
        for i, w in enumerate(self.mod_params()[0]):
            w._owl_grad_stack = (id(self), i)

    def modulation(self, cond):
        """(adaln1 [2d], gate1 [d], adaln2 [2d], gate2 [d]) per frame from silu(cond): one stacked GEMM
        (fused.ModFn) instead of the four Linears."""
        ws, bs = self.mod_params()
        params = [t for pair in zip(ws, bs) for t in pair]
        W, bvec = stacked_modulation_weights(self, params)
        return ModFn.apply(cond_silu(cond), W, bvec, *params)

    def mod_params(self):
        """(weights, biases) of the four per-frame modulation Linears, in the column order of
        modulation()'s outputs: adaln1 [2d] | gate1 [d] | adaln2 [2d] | gate2 [d]."""
        fcs = (self.adaln1.fc, self.gate1.fc_c, self.adaln2.fc, self.gate2.fc_c)
        return [f.weight for f in fcs], [f.bias for f in fcs]

    def forward(self, x, cond, block_mask, kv_cache=None, mods=None, scond=None):
        """scond: silu(cond) from fused.cond_silu / cond.CondFn (computed here when not given)."""
        if kv_cache is not None:
            with torch.no_grad():
                return self._forward_cached(x, cond, block_mask, kv_cache, mods, scond)
        cfg = self.config
        if scond is None:
            scond = cond_silu(cond)
        ws, bs = self.mod_params()
        mparams = [t for pair in zip(ws, bs) for t in pair]
        W, bvec = stacked_modulation_weights(self, mparams)
        H = cfg.n_heads
        rope = self.attn.rope
        ck = getattr(self, "_checkpointed", False)
        geo = BlockGeometry(H, cfg.d_model // H, cfg.tokens_per_frame, block_mask, rope.cos, rope.sin, 0,
                            keep_attn=id(self) if ck else None,
                            lean=bool(getattr(cfg, "lean_activations", False)) and not ck)
        a, m = self.attn, self.mlp
        return DiTBlockFn.apply(x.to(torch.bfloat16).contiguous(), scond, W, bvec, geo, a.qkv.weight, a.qkv.bias,
                                a.out.weight, a.out.bias, m.fc1.weight, m.fc1.bias, m.fc2.weight, m.fc2.bias,
                                *mparams)

    def _forward_cached(self, x, cond, block_mask, kv_cache, mods=None, scond=None):
        """No-grad forward of the decode path (attn.py:86-107 cache branch).  mods: this block's
        [rows, 6d] column slice of DiT._decode_modulation, else computed here."""
        cfg = self.config
        d, tpf = cfg.d_model, cfg.tokens_per_frame
        B, L, _ = x.shape
        if mods is None:
            ws, bs = self.mod_params()
            W, bvec = stacked_modulation_weights(self, [t for pair in zip(ws, bs) for t in pair])
            s = scond if scond is not None else cond_silu(cond)
            mods = K.gemm(s.reshape(-1, d).to(torch.bfloat16).contiguous(), W, bias=bvec)
        ab1, g1, ab2, g2 = mods[:, :2 * d], mods[:, 2 * d:3 * d], mods[:, 3 * d:5 * d], mods[:, 5 * d:]
        xx = x.reshape(B * L, d).to(torch.bfloat16).contiguous()
        ab1, ab2 = ab1.reshape(-1, 2 * d), ab2.reshape(-1, 2 * d)
        h1, _ = K.adaln_fwd(xx, ab1[:, :d], ab1[:, d:], tpf)
        qkv = K.gemm(h1, bf16_weight(self.attn.qkv.weight), bias=self.attn.qkv.bias)
        o = self.attn._attend(qkv, B, L, block_mask, kv_cache)
        x1 = K.gemm(o.reshape(B * L, d), bf16_weight(self.attn.out.weight), bias=self.attn.out.bias,
                    epi=K.EPI_GATE_RESID, gate=g1.reshape(-1, d), tpf=tpf, resid=xx)
        h2, _ = K.adaln_fwd(x1, ab2[:, :d], ab2[:, d:], tpf)
        a_pre = torch.empty(B * L, 4 * d, device=x.device, dtype=torch.bfloat16)
        a = K.gemm(h2, bf16_weight(self.mlp.fc1.weight), bias=self.mlp.fc1.bias, epi=K.EPI_SILU, aux=a_pre)
        out = K.gemm(a, bf16_weight(self.mlp.fc2.weight), bias=self.mlp.fc2.bias, epi=K.EPI_GATE_RESID,
                     gate=g2.reshape(-1, d), tpf=tpf, resid=x1)
        return out.view(B, L, d)


class DiT(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.config = config
        if not hasattr(config, "local_idx"):
            config.local_idx = 4
        self.rope = get_rope_cls(getattr(config, "rope_impl", "ortho"))(config)
        self.local_layers = [(i % config.local_idx != 0) for i in range(config.n_layers)]
        self.blocks = nn.ModuleList([DiTBlock(config, i, loc, self.rope) for i, loc in enumerate(self.local_layers)])
        self.decoding = False

    def enable_decoding(self):
        self.decoding = True

    def disable_decoding(self):
        self.decoding = False

    def get_block_mask(self, seq_len, doc_id, window_len, q_offset, device):
        return get_block_mask(seq_len + q_offset, self.config.tokens_per_frame, window_len, doc_id, q_offset,
                              self.config.causal, device)

    def forward(self, x, cond, doc_id=None, kv_cache=None, local_block_mask=None, global_block_mask=None,
                scond=None):
        """scond: silu(cond) as produced by cond.CondFn (GameRFTCore) -- every block's modulation reads
        it and sums its gradient into one fp32 accumulator (fused.CondGrad); computed here from cond
        when not given."""
        seq_len, device = x.size(1), x.device
        q_offset = kv_cache.length_at(0) if kv_cache is not None else 0
        if local_block_mask is None and not self.decoding:
            local_block_mask = self.get_block_mask(seq_len, doc_id, self.config.local_window, q_offset, device)
        if global_block_mask is None and not self.decoding:
            global_block_mask = self.get_block_mask(seq_len, doc_id, getattr(self.config, "global_window", None),
                                                    q_offset, device)
        ckpt = self.training and getattr(self.config, "gradient_checkpointing", False) and kv_cache is None
        # optional: checkpoint only the first `checkpoint_layers` blocks and keep the rest's activations
        # (HBM headroom on a 288 GB MI355X trades for the recompute); default = every block, as the reference
        n_ck = getattr(self.config, "checkpoint_layers", None)
        if scond is None:
            scond = cond_silu(cond)
        mods = self._decode_modulation(scond) if kv_cache is not None else None
        d6 = 6 * self.config.d_model
        for i, block in enumerate(self.blocks):
            mask = local_block_mask if self.local_layers[i] else global_block_mask
            if mods is not None:
                x = block(x, cond, mask, kv_cache, mods[:, i * d6:(i + 1) * d6])
                continue
            ck = ckpt and (n_ck is None or i < n_ck)
            block._checkpointed = ck  # the re-run inside backward reuses the kept attention output
            x = checkpoint(block, x, cond, mask, kv_cache, None, scond) if ck else \
                block(x, cond, mask, kv_cache, None, scond)
        if kv_cache is not None and kv_cache.should_update and getattr(kv_cache, "dev", None) is not None:
            kv_cache.sync_device_state()  # every layer committed the frame
        return x

    @torch.no_grad()
    def _decode_modulation(self, scond):
        """Every block's per-frame modulation (DiTBlock.modulation) for a no-grad KV-cache forward
        as ONE GEMM: scond = silu(cond) [rows, d] against all blocks' modulation weights stacked
        [L x 6d, d].  Decode has 1-2 rows per call, so the 4 x L per-block GEMMs were each a
        latency-bound launch pair; the stacked GEMM streams the same 28 MB/block of weights once.
        The bf16 stack is rebuilt when any of its parameters changes (version counters)."""
        ws, bs = zip(*(b.mod_params() for b in self.blocks))
        ws, bs = [w for g in ws for w in g], [b for g in bs for b in g]
        key = (scond.device,) + tuple(p._version for p in ws + bs) + tuple(id(p) for p in ws)
        ent = getattr(self, "_mod_stack", None)
        if ent is None or ent[0] != key:
            W = torch.cat([w.detach().to(torch.bfloat16) for w in ws]).contiguous()
            bias = torch.cat([b.detach().float() for b in bs]).contiguous()
            ent = (key, W, bias)
            object.__setattr__(self, "_mod_stack", ent)
        d = self.config.d_model
        return K.gemm(scond.reshape(-1, d).to(torch.bfloat16).contiguous(), ent[1], bias=ent[2])


class FinalLayer(nn.Module):
    """attn.py:264-277: proj(silu(AdaLN(x, cond))) with AdaLN + SiLU fused in one kernel."""

    def __init__(self, sample_size, d_model, channels=3, patch_size=1):
        super().__init__()
        self.norm = AdaLN(d_model)
        self.act = nn.SiLU()
        self.proj = nn.Linear(d_model, channels * patch_size * patch_size)

    def forward(self, x, cond, scond=None):
        """scond: silu(cond) (fused.cond_silu / cond.CondFn), computed here when not given."""
        s = scond if scond is not None else cond_silu(cond)
        h = adaln_mod(x, s, self.norm.fc.weight, self.norm.fc.bias, x.shape[1] // s.shape[1], act=True)
        return linear(h, self.proj.weight, self.proj.bias)
