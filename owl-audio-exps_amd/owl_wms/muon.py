"""Muon + AdamW (reference: owl_wms/muon.py:11-179) with Newton-Schulz on libowlk.

``zeropower_via_newtonschulz5`` keeps the reference signature.  Same-shape parameters are
orthogonalised as one batch (one set of batched GEMM launches per shape group instead of one
per parameter): X = bf16(G)/(||X||_F+eps) (owlk_ns_normalize, transposed when rows > cols),
then per iteration A = X X^T, B = b A + c A A, X = a X + B X on bf16 MFMA GEMMs whose AXPBY
epilogue applies the scalar combination in bf16 exactly as the eager reference rounds it.

Momentum + Nesterov + stacking + the Frobenius norm are one fused pass per shape group
(owlk_muon_momentum), and decoupled weight decay + the scaled update another (owlk_muon_apply),
reading the NS iterate in its transposed layout.

Distributed (muon.py:86-115): NS work is dealt round-robin over ranks by parameter index and
the bf16 updates are exchanged with all_gather_into_tensor (RCCL over xGMI on MI355X); every
rank then applies every update, so replicas stay bit-identical.
"""
import torch
import torch.distributed as dist
from torch import Tensor
from torch.optim import AdamW
from torch.optim.optimizer import Optimizer

from . import kernels as K

NS_A, NS_B, NS_C = 3.4445, -4.7750, 2.0315


def _pad8(G: Tensor) -> Tensor:
    # the GEMMs need dims that are multiples of 8: zero-pad (exact -- zero rows/columns add nothing
    # to ||X||_F or X X^T and stay zero through every iteration), e.g. mouse angle_proj [256, 2]
    r, c = G.shape[-2:]
    pr, pc = (-r) % 8, (-c) % 8
    return torch.nn.functional.pad(G, (0, pc, 0, pr)) if (pr or pc) else G


def _ns_iterate(X: Tensor, steps: int) -> Tensor:
    """Quintic iterations on a normalised bf16 X [b, m, k] (m <= k); returns the final iterate."""
    b, m, _ = X.shape
    A = torch.empty(b, m, m, device=X.device, dtype=torch.bfloat16)
    Bm = torch.empty_like(A)
    X2 = torch.empty_like(X)
    for _ in range(steps):
        K.bgemm(X, X, A)                                                      # A = X X^T
        K.bgemm(A, A, Bm, epi=K.EPI_AXPBY, alpha=NS_C, beta=NS_B, aux=A)      # B = b A + c A A
        K.bgemm(Bm, X, X2, b_trans=True, epi=K.EPI_AXPBY, alpha=1.0, beta=NS_A, aux=X)  # X = a X + B X
        X, X2 = X2, X
    return X


def newton_schulz_bf16(G: Tensor, steps: int = 5) -> Tensor:
    """G [b, r, c] (fp32 or bf16, on the GPU) -> bf16 [b, r, c] quintic NS orthogonalisation."""
    assert G.dim() == 3
    b, r, c = G.shape
    tr = r > c
    X = _ns_iterate(K.ns_normalize(_pad8(G), tr), steps)
    X = X.transpose(1, 2) if tr else X
    return X[:, :r, :c] if X.shape[1:] != (r, c) else X


def momentum_update(grads, bufs, momentum, nesterov, out, sumsq):
    """muon.py:67-73 for same-numel fp32 grads, fused (owlk_muon_momentum): bufs updated in place,
    the Nesterov-combined gradients written to out [len, numel] (not back into p.grad), sumsq[i] +=
    ||bf16(g'_i)||^2."""
    K.muon_momentum(grads, bufs, momentum, nesterov, out, sumsq)


def apply_update(params, u, rows, cols, transpose, decay, alpha):
    """muon.py:80-84 fused (owlk_muon_apply): p = p * decay - alpha * u."""
    K.muon_apply(params, u, rows, cols, transpose, decay, alpha)


def zeropower_via_newtonschulz5(G: Tensor, steps: int) -> Tensor:
    """muon.py:11-38 API: [..., m, n] -> bf16 of the same shape."""
    shp = G.shape
    out = newton_schulz_bf16(G.reshape(-1, shp[-2], shp[-1]), steps)
    return out.reshape(shp)


def _all_gather(out, inp):
    """all_gather_into_tensor (RCCL); list form where the backend lacks it (gloo tests)."""
    if dist.get_backend() == "nccl":
        dist.all_gather_into_tensor(out, inp)
    else:
        dist.all_gather(list(out.unbind(0)), inp)


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
        for size in sorted({p.numel() for p in params}):
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

    @torch.no_grad()
    def step(self):
        for group in self.param_groups:
            params = [p for p in group["params"] if p.grad is not None]
            if not params:
                continue
            for p in params:  # the fused passes take flat fp32 storage
                if not p.grad.is_contiguous():
                    p.grad = p.grad.contiguous()
            if self.world_size == 1:
                # all same-shape parameters of the group as one batch: one momentum pass (which also
                # stacks the NS input and reduces its norm), one NS launch sequence, one apply pass
                by_shape = {}
                for p in params:
                    by_shape.setdefault((p.grad.shape[0], p.grad[0].numel()), []).append(p)
                for (r, c), ps in by_shape.items():
                    G = torch.empty(len(ps), r * c, device=ps[0].device, dtype=torch.float32)
                    sumsq = torch.zeros(len(ps), device=G.device, dtype=torch.float32)
                    momentum_update([p.grad for p in ps], self._buffers(ps), group["momentum"], group["nesterov"],
                                    G, sumsq)
                    tr = r > c
                    X = _ns_iterate(K.ns_scale(_pad8(G.view(len(ps), r, c)).contiguous(), tr, sumsq),
                                    group["ns_steps"])
                    if X.shape[1:] != ((c, r) if tr else (r, c)):  # zero-padded matrix: crop first
                        X = (X.transpose(1, 2) if tr else X)[:, :r, :c].contiguous()
                        tr = False
                    decay, alpha = self._scales(group, r, c)
                    apply_update(ps, X, r, c, tr, decay, alpha)
                continue
            # multi-rank: round-robin NS + all_gather of the flat bf16 updates (muon.py:86-115)
            numel = params[0].numel()
            ws = self.world_size
            buf = torch.empty(ws, numel, device=params[0].device, dtype=torch.bfloat16)
            for base in range(0, len(params), ws):
                chunk = params[base:base + ws]
                if self.rank < len(chunk):
                    p = chunk[self.rank]
                    r = p.grad.shape[0]
                    G = torch.empty(1, numel, device=p.device, dtype=torch.float32)
                    sumsq = torch.zeros(1, device=p.device, dtype=torch.float32)
                    momentum_update([p.grad], self._buffers([p]), group["momentum"], group["nesterov"], G, sumsq)
                    mine = newton_schulz_bf16(G.view(1, r, numel // r), group["ns_steps"])[0].flatten()
                else:
                    mine = torch.zeros(numel, device=buf.device, dtype=torch.bfloat16)
                _all_gather(buf, mine.contiguous())
                for i, p in enumerate(chunk):
                    r = p.shape[0]
                    decay, alpha = self._scales(group, p.size(-2), p.size(-1))
                    apply_update([p.data], buf[i], r, numel // r, False, decay, alpha)


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
