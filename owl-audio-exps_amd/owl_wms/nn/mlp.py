"""mlp.py (reference: owl_wms/nn/mlp.py:6-37).  Same init, same state_dict keys (fc1, fc2)."""
from torch import nn


class MLPCustom(nn.Module):
    def __init__(self, dim_in, dim_middle, dim_out):
        super().__init__()
        self.fc1 = nn.Linear(dim_in, dim_middle)
        self.fc2 = nn.Linear(dim_middle, dim_out)
        nn.init.kaiming_normal_(self.fc1.weight)
        nn.init.kaiming_normal_(self.fc2.weight)
        self.fc1.weight.data *= dim_in ** -0.5
        self.fc2.weight.data *= dim_middle ** -0.5
        nn.init.zeros_(self.fc1.bias)
        nn.init.zeros_(self.fc2.bias)

    def forward(self, x):
        # fc1 GEMM with the SiLU epilogue, fc2 GEMM (cond.MLPFn); the conditioning MLPs of the
        # training step run inside cond.CondFn instead
        from .cond import mlp_custom
        return mlp_custom(x, self)


class MLP(MLPCustom):
    def __init__(self, config):
        super().__init__(config.d_model, config.d_model * 4, config.d_model)
