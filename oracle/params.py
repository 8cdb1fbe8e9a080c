"""Deterministic parameter recipe shared by the golden-vector generator, the oracle and the tests.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Parameters are never stored in fixtures: every state_dict entry is regenerated from
``torch.Generator().manual_seed(base + i)`` where ``i`` is the index of the key in sorted
state_dict-key order, ``randn * scale``.  Biases get the same treatment so
that every path through the model carries a non-trivial value.
"""
import torch


def det_state(named_shapes, base_seed=0, scale=0.02):
    """named_shapes: iterable of (name, shape). Returns {name: fp32 tensor}."""
    out = {}
    for i, (name, shape) in enumerate(sorted(named_shapes, key=lambda t: t[0])):
        g = torch.Generator().manual_seed(base_seed + i)
        out[name] = torch.randn(tuple(shape), generator=g, dtype=torch.float32) * scale
    return out


def det_init_(module, base_seed=0, scale=0.02):
    """In-place deterministic init of every parameter of ``module`` (keys of state_dict)."""
    sd = module.state_dict()
    vals = det_state([(k, v.shape) for k, v in sd.items()], base_seed, scale)
    with torch.no_grad():
        for k, v in sd.items():
            v.copy_(vals[k].to(v.dtype))
    return module


def det_tensor(shape, seed, scale=1.0, dtype=torch.float32):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(tuple(shape), generator=g, dtype=torch.float32) * scale).to(dtype)
