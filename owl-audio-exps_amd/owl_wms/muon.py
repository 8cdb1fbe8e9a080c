"""Muon + AdamW (reference: owl_wms/muon.py:11-179) with Newton-Schulz on libowlk.

``zeropower_via_newtonschulz5`` keeps the reference signature.  Same-shape parameters are
orthogonalised as one batch (one set of batched GEMM launches per shape group instead of one
per parameter): X = bf16(G)/(||X||_F+eps) (owlk_ns_normalize, transposed when rows > cols),
then per iteration A = X X^T, B = b A + c A A, X = a X + B X on bf16 MFMA GEMMs whose AXPBY
epilogue applies the scalar combination in bf16 exactly as the eager reference rounds it.

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


def newton_schulz_bf16(G: Tensor, steps: int = 5) -> Tensor:
    """G [b, r, c] (fp32 or bf16, on the GPU) -> bf16 [b, r, c] quintic NS orthogonalisation."""
    assert G.dim() == 3
    b, r, c = G.shape
    tr = r > c
    # the GEMMs need dims that are multiples of 8: zero-pad (exact -- zero rows/columns add nothing
    # to ||X||_F or X X^T and stay zero through every iteration), e.g. mouse angle_proj [256, 2]
    pr, pc = (-r) % 8, (-c) % 8
    if pr or pc:
        G = torch.nn.functional.pad(G, (0, pc, 0, pr))
    X = K.ns_normalize(G, tr)
    m = X.shape[1]
    A = torch.empty(b, m, m, device=G.device, dtype=torch.bfloat16)
    Bm = torch.empty_like(A)
    X2 = torch.empty_like(X)
    for _ in range(steps):
        K.bgemm(X, X, A)                                                      # A = X X^T
        K.bgemm(A, A, Bm, epi=K.EPI_AXPBY, alpha=NS_C, beta=NS_B, aux=A)      # B = b A + c A A
        K.bgemm(Bm, X, X2, b_trans=True, epi=K.EPI_AXPBY, alpha=1.0, beta=NS_A, aux=X)  # X = a X + B X
        X, X2 = X2, X
    X = X.transpose(1, 2) if tr else X
    return X[:, :r, :c] if (pr or pc) else X


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

    @torch.no_grad()
    def _momentum(self, group, p):
        g = p.grad
        st = self.state[p]
        if "momentum_buffer" not in st:
            st["momentum_buffer"] = torch.zeros_like(g)
        buf = st["momentum_buffer"]
        buf.lerp_(g, 1 - group["momentum"])
        return g.lerp_(buf, group["momentum"]) if group["nesterov"] else buf

    @torch.no_grad()
    def _apply(self, group, p, u):
        p.mul_(1 - group["lr"] * group["weight_decay"])
        p.add_(u.view_as(p), alpha=-group["lr"] * max(1, p.size(-2) / p.size(-1)) ** 0.5)

    @torch.no_grad()
    def step(self):
        for group in self.param_groups:
            params = [p for p in group["params"] if p.grad is not None]
            if not params:
                continue
            if self.world_size == 1:
                gs = [self._momentum(group, p) for p in params]
                # batch all same-shape parameters of the group into one NS launch sequence
                by_shape = {}
                for p, g in zip(params, gs):
                    by_shape.setdefault(tuple(g.view(len(g), -1).shape if g.ndim == 4 else g.shape), []).append(
                        (p, g))
                for shape, items in by_shape.items():
                    G = torch.stack([g.reshape(shape) for _, g in items])
                    U = newton_schulz_bf16(G, group["ns_steps"])
                    for (p, _), u in zip(items, U):
                        self._apply(group, p, u)
                continue
            # multi-rank: round-robin NS + all_gather of the flat bf16 updates (muon.py:86-115)
            numel = params[0].numel()
            ws = self.world_size
            buf = torch.empty(ws, numel, device=params[0].device, dtype=torch.bfloat16)
            for base in range(0, len(params), ws):
                chunk = params[base:base + ws]
                if self.rank < len(chunk):
                    p = chunk[self.rank]
                    g = self._momentum(group, p)
                    g2 = g.view(len(g), -1) if g.ndim == 4 else g
                    mine = newton_schulz_bf16(g2[None], group["ns_steps"])[0].flatten()
                else:
                    mine = torch.zeros(numel, device=buf.device, dtype=torch.bfloat16)
                _all_gather(buf, mine.contiguous())
                for i, p in enumerate(chunk):
                    self._apply(group, p, buf[i])


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
        self.adamw = AdamW(adamw_params, lr=kwargs.get("adamw_lr"), betas=tuple(kwargs.get("adamw_betas", (0.9, 0.999))),
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
