"""Muon + AdamW (reference: owl_wms/muon.py:11-179) with Newton-Schulz on libowlk.

``zeropower_via_newtonschulz5`` keeps the reference signature and runs as one library entry
(owlk_newton_schulz_bf16): X = bf16(G)/(||X||_F+eps), transposed when rows > cols, then per
iteration A = X X^T, B = b A + (c A) A, X = a X + B X on bf16 MFMA GEMMs, rounded in the eager
reference's order (the A GEMM also emits bf16(c A); the other two apply the scalar
combination in their AXPBY epilogue).

Inside Muon.step, same-shape parameters are orthogonalised as one batch: momentum + Nesterov +
stacking + the Frobenius norm are one fused pass per shape (owlk_muon_momentum), then the scale
pass (owlk_ns_scale) and the batched iterations (owlk_ns_iterate); decoupled weight decay + the
scaled update is another fused pass (owlk_muon_apply) reading the NS iterate in its transposed
layout.

Distributed (muon.py:86-115): NS work is dealt round-robin over ranks by parameter index.  Each
rank orthogonalises all the parameters it owns in a group as shape batches, then ONE bf16
all_gather_into_tensor per parameter group exchanges them (RCCL over xGMI, async_op=True, so the
gather of a group overlaps the next group's NS); every rank then applies every update, so
replicas stay bit-identical.
"""
import torch
import torch.distributed as dist
from torch import Tensor
from torch.optim import AdamW
from torch.optim.optimizer import Optimizer

from . import kernels as K

NS_A, NS_B, NS_C = K.NS_COEFFS


def _pad8(G: Tensor) -> Tensor:
    # the GEMMs need dims that are multiples of 8: zero-pad (exact -- zero rows/columns add nothing
    # to ||X||_F or X X^T and stay zero through every iteration), e.g. mouse angle_proj [256, 2]
    r, c = G.shape[-2:]
    pr, pc = (-r) % 8, (-c) % 8
    return torch.nn.functional.pad(G, (0, pc, 0, pr)) if (pr or pc) else G


def newton_schulz_bf16(G: Tensor, steps: int = 5) -> Tensor:
    """G [b, r, c] (fp32 or bf16, on the GPU) -> bf16 [b, r, c] quintic NS orthogonalisation."""
    assert G.dim() == 3
    return K.newton_schulz(G, steps)


def momentum_update(grads, bufs, momentum, nesterov, out, sumsq):
    """muon.py:67-73 for same-numel fp32 grads, fused (owlk_muon_momentum): bufs updated in place,
    the Nesterov-combined gradients written to out [len, numel] (not back into p.grad), sumsq[i] =
    the partial sums of ||bf16(g'_i)||^2 [len, K.NORM_PARTS]."""
    K.muon_momentum(grads, bufs, momentum, nesterov, out, sumsq)


def ns_orthogonalize(G: Tensor, sumsq: Tensor, steps: int, out: Tensor = None):
    """muon.py:23-34 on a batch of momentum-combined fp32 matrices G [n, r, c] whose sum(bf16(g)^2)
    partials are already in sumsq [n, K.NORM_PARTS]: -> (U, tr), U bf16 contiguous [n, c, r] when tr (the iterate before its
    transpose back, r > c) else [n, r, c]; written into `out` when given (same shape)."""
    n, r, c = G.shape
    tr = r > c
    Gp = _pad8(G)
    if Gp is G and out is not None:
        return K.ns_iterate(K.ns_scale(G, tr, sumsq, out=out), steps), tr
    X = K.ns_iterate(K.ns_scale(Gp.contiguous(), tr, sumsq), steps)
    if Gp is not G:  # zero-padded matrix: crop
        X = (X[:, :c, :r] if tr else X[:, :r, :c]).contiguous()
    if out is not None:
        out.copy_(X)
        X = out
    return X, tr


def apply_update(params, u, rows, cols, transpose, decay, alpha):
    """muon.py:80-84 fused (owlk_muon_apply): p = p * decay - alpha * u."""
    K.muon_apply(params, u, rows, cols, transpose, decay, alpha)


def zeropower_via_newtonschulz5(G: Tensor, steps: int) -> Tensor:
    """muon.py:11-38 API: [..., m, n] -> bf16 of the same shape."""
    shp = G.shape
    out = newton_schulz_bf16(G.reshape(-1, shp[-2], shp[-1]), steps)
    return out.reshape(shp)


def _all_gather_async(out, inp):
    """all_gather_into_tensor(async_op=True) (RCCL); list form where the backend lacks it (gloo)."""
    if dist.get_backend() == "nccl":
        return dist.all_gather_into_tensor(out, inp, async_op=True)
    return dist.all_gather(list(out.view(dist.get_world_size(), -1).unbind(0)), inp, async_op=True)


def _shape2(p):
    return p.shape[0], p[0].numel()


def _runs(items, key):
    """consecutive runs of items with equal key -> [(key, [items])]"""
    out = []
    for it in items:
        k = key(it)
        if out and out[-1][0] == k:
            out[-1][1].append(it)
        else:
            out.append((k, [it]))
    return out


class Muon(torch.optim.Optimizer):
    """muon.py:40-115: momentum (lerp) + Nesterov, NS, decoupled weight decay, shape-scaled lr."""

    def __init__(self, params, lr=0.02, weight_decay=0.01, momentum=0.95, nesterov=True, ns_steps=5, rank=None,
                 world_size=None):
        if rank is None or world_size is None:
            raise Exception("world_size and rank params required, if you want to use this optimizer on a single "
                            "GPU, pass rank=0 and world_size=1.")
        self.rank, self.world_size = rank, world_size
        defaults = dict(lr=lr, weight_decay=weight_decay, momentum=momentum, nesterov=nesterov, ns_steps=ns_steps)
        params = [*params]
        groups = []
        # the reference iterates a set of numels (muon.py:52): same group order, so that a reference
        # Muon state_dict loads onto the same parameters
        for size in {p.numel() for p in params}:
            groups.append(dict(params=[p for p in params if p.numel() == size]))
        super().__init__(groups, defaults)

    def _buffers(self, params):
        bufs = []
        for p in params:
            st = self.state[p]
            if "momentum_buffer" not in st:
                st["momentum_buffer"] = torch.zeros_like(p.grad, memory_format=torch.contiguous_format)
            bufs.append(st["momentum_buffer"])
        return bufs

    @staticmethod
    def _scales(group, rows, cols):
        return 1 - group["lr"] * group["weight_decay"], group["lr"] * max(1, rows / cols) ** 0.5

    def _orthogonalize(self, group, ps, out=None):
        """momentum + NS for same-shape params ps (one batch) -> (U, tr) as ns_orthogonalize"""
        for p in ps:  # the fused passes take flat fp32 storage
            if not p.grad.is_contiguous():
                p.grad = p.grad.contiguous()
        r, c = _shape2(ps[0])
        G = torch.empty(len(ps), r * c, device=ps[0].device, dtype=torch.float32)
        sumsq = torch.empty(len(ps), K.NORM_PARTS, device=G.device, dtype=torch.float32)
        momentum_update([p.grad for p in ps], self._buffers(ps), group["momentum"], group["nesterov"], G, sumsq)
        return ns_orthogonalize(G.view(len(ps), r, c), sumsq, group["ns_steps"], out=out)

    @torch.no_grad()
    def step(self):
        pending = []
        for group in self.param_groups:
            if self.world_size == 1:
                params = [p for p in group["params"] if p.grad is not None]
                by_shape = {}
                for p in params:
                    by_shape.setdefault(_shape2(p), []).append(p)
                for (r, c), ps in by_shape.items():
                    U, tr = self._orthogonalize(group, ps)
                    decay, alpha = self._scales(group, r, c)
                    apply_update(ps, U, r, c, tr, decay, alpha)
                continue
            pending.append(self._launch_group(group))
        for finish in pending:
            finish()

    def _launch_group(self, group):
        """multi-rank (muon.py:86-115): NS of the params this rank owns (index % world_size == rank)
        as shape batches into slot j of a [chunks, numel] bf16 buffer, then one async all_gather of
        it; returns the closure that waits and applies every rank's updates."""
        params, ws, rank = group["params"], self.world_size, self.rank
        numel = params[0].numel()
        nc = (len(params) + ws - 1) // ws
        dev = params[0].device
        mine = torch.zeros(nc, numel, device=dev, dtype=torch.bfloat16)
        owned = [(j, params[j * ws + rank]) for j in range(nc) if j * ws + rank < len(params)]
        for p in params:
            assert p.grad is not None
        for (r, c), run in _runs(owned, lambda jp: _shape2(jp[1])):
            j0 = run[0][0]
            slots = mine[j0:j0 + len(run)]  # owned params take consecutive slots j
            tr = r > c
            self._orthogonalize(group, [p for _, p in run], out=slots.view(len(run), *((c, r) if tr else (r, c))))
        out = torch.empty(ws, nc, numel, device=dev, dtype=torch.bfloat16)
        work = _all_gather_async(out.view(-1), mine.view(-1))

        def finish():
            work.wait()
            for src in range(ws):
                ps = [(j, params[j * ws + src]) for j in range(nc) if j * ws + src < len(params)]
                for (r, c), run in _runs(ps, lambda jp: _shape2(jp[1])):
                    j0 = run[0][0]
                    decay, alpha = self._scales(group, r, c)
                    apply_update([p for _, p in run], out[src, j0:j0 + len(run)], r, c, r > c, decay, alpha)

        return finish


class FusedAdamW(AdamW):
    """torch.optim.AdamW with the step in one libowlk pass (owlk_adamw): same
    hyper-parameters, same per-parameter state ('step', 'exp_avg', 'exp_avg_sq') and state_dict, so
    reference checkpoints load; same arithmetic order as torch's foreach implementation."""

    def __init__(self, params, **kw):
        super().__init__(params, **kw)
        for g in self.param_groups:
            if g["amsgrad"] or g["maximize"] or g.get("capturable") or g.get("differentiable"):
                raise NotImplementedError("FusedAdamW: amsgrad / maximize / capturable / differentiable")

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            by_step = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("FusedAdamW does not support sparse gradients")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0, dtype=torch.float32)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                by_step.setdefault(float(st["step"]), []).append(p)
            b1, b2 = group["betas"]
            for t, ps in by_step.items():
                grads = [p.grad if p.grad.is_contiguous() else p.grad.contiguous() for p in ps]
                K.adamw(ps, grads, [self.state[p]["exp_avg"] for p in ps], [self.state[p]["exp_avg_sq"] for p in ps],
                        group["lr"], b1, b2, group["weight_decay"], group["eps"], t)
        return loss


class CombinedOptimizer(Optimizer):
    """muon.py:117-176: AdamW for names containing an adamw_key or ndim < 2, Muon for the rest."""

    def __init__(self, model, rank=0, world_size=1, **kwargs):
        self.defaults = {}
        adamw_keys = kwargs.pop("adamw_keys", [])
        named = {n.replace("._orig_mod", "").replace("module.", "", 1) if n.startswith("module.") else
                 n.replace("._orig_mod", ""): p for n, p in model.named_parameters()}
        adamw_params = [p for n, p in named.items() if any(k in n for k in adamw_keys) or p.ndim < 2]
        muon_params = [p for n, p in named.items() if not any(k in n for k in adamw_keys) and p.ndim >= 2]
        names = list(named)
        for key in adamw_keys:
            assert any(key in n for n in names), f"AdamW key '{key}' not found in model parameters" + str(names)
        self.adamw = FusedAdamW(adamw_params, lr=kwargs.get("adamw_lr"), betas=tuple(kwargs.get("adamw_betas", (0.9, 0.999))),
                           weight_decay=kwargs.get("adamw_wd", 0.01), eps=kwargs.get("adamw_eps", 1.0e-15))
        # reference defect kept on purpose: Muon's weight decay is never forwarded
        self.muon = Muon(muon_params, lr=kwargs.get("lr"), momentum=kwargs.get("momentum"), rank=rank,
                         world_size=world_size)
        self.param_groups = self.adamw.param_groups + self.muon.param_groups
        self.state = {}

    def zero_grad(self, set_to_none: bool = False):
        self.adamw.zero_grad(set_to_none)
        self.muon.zero_grad(set_to_none)

    def step(self, closure=None):
        loss = closure() if closure is not None else None
        self.adamw.step()
        self.muon.step()
        return loss

    def state_dict(self):
        return {"adamw": self.adamw.state_dict(), "muon": self.muon.state_dict()}

    def load_state_dict(self, state_dict):
        self.adamw.load_state_dict(state_dict["adamw"])
        self.muon.load_state_dict(state_dict["muon"])


def init_muon(model, rank=0, world_size=1, **kwargs):
    return CombinedOptimizer(model, rank, world_size, **kwargs)
