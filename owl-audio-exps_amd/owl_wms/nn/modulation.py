"""modulation.py (reference: owl_wms/nn/modulation.py:7-63).

AdaLN / Gate keep the reference signature ``module(x, cond)``.  Inside DiTBlock the per-frame
modulation vectors are computed once from silu(cond) and the modulate/gate math is fused into
libowlk kernels (DiTBlockFn); these modules serve FinalLayer and any external caller.
"""
from torch import nn

from .fused import adaln, adaln_mod, cond_silu, linear


class AdaLN(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.fc = nn.Linear(dim, 2 * dim)

    def mod(self, scond):
        """per-frame [a | b] = fc(silu(cond)) given scond = silu(cond): [b, n, 2d] bf16"""
        return linear(scond, self.fc.weight, self.fc.bias)

    def forward(self, x, cond, act=False):
        """AdaLN(x) with its fc on silu(cond), fused (fused.AdaLNModFn)."""
        n = cond.shape[1]
        return adaln_mod(x, cond_silu(cond), self.fc.weight, self.fc.bias, x.shape[1] // n, act)


class Gate(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.fc_c = nn.Linear(dim, dim)

    def mod(self, scond):
        return linear(scond, self.fc_c.weight, self.fc_c.bias)

    def forward(self, x, cond):
        b, n, d = cond.shape
        c = self.mod(cond_silu(cond))
        m = x.shape[1] // n
        return c[:, :, None, :].expand(b, n, m, d).reshape(b, n * m, d) * x


def cond_adaln(x, scale, bias):
    """modulation.py:46-55 on the fused AdaLN kernel."""
    return adaln(x, scale, bias, x.shape[1] // scale.shape[1])


def cond_gate(x, gate):
    """modulation.py:57-63."""
    b, nm, d = x.shape
    n = gate.shape[1]
    return gate[:, :, None, :].expand(b, n, nm // n, d).reshape(b, nm, d) * x
