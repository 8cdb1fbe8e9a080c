"""normalization.py (reference: owl_wms/nn/normalization.py:6-11).

rms_norm / layer_norm are kept as free functions for API compatibility; on the training hot path
RMSNorm is fused into the AdaLN and QK-RoPE kernels (owl_wms/nn/fused.py).
"""
import torch
import torch.nn.functional as F


def layer_norm(x: torch.Tensor) -> torch.Tensor:
    """normalization.py:6-7 (MMDiT head) on the libowlk layer_norm kernels."""
    from .fused import layer_norm as _ln
    return _ln(x)


def rms_norm(x: torch.Tensor) -> torch.Tensor:
    """normalization.py:10-11 -- weightless RMSNorm, fp32 eps, output in x.dtype."""
    return F.rms_norm(x, (x.size(-1),))
