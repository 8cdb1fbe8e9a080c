"""schedulers.py (reference: owl_wms/sampling/schedulers.py:5-13).

PARITY-UNPINNED: the reference builds the step sizes with diffusers'
FlowMatchEulerDiscreteScheduler(shift=3, num_train_timesteps=n_steps) (diffusers is absent here,
version unpinned).  Restated from that scheduler's published construction: timesteps
linspace(1, N, N) reversed, sigma = t / N, shifted sigma' = 3 sigma / (1 + 2 sigma); the sampler
uses ts = sigma' (timesteps / N) with a trailing 0 and dt = ts[:-1] - ts[1:].
"""
import numpy as np
import torch


def get_sd3_euler(n_steps, shift=3.0):
    t = np.linspace(1, n_steps, n_steps, dtype=np.float32)[::-1].copy()
    sigma = torch.from_numpy(t / n_steps)
    sigma = shift * sigma / (1 + (shift - 1) * sigma)
    ts = torch.cat([sigma.float(), torch.zeros(1)])
    return ts[:-1] - ts[1:]


def get_deltas(custom_schedule):
    """av_caching_v2.py:12-23: |differences| of a custom schedule (0.0 appended if missing)."""
    sched = list(custom_schedule)
    if sched[-1] != 0.0:
        sched.append(0.0)
    return [abs(b - a) for a, b in zip(sched[:-1], sched[1:])]
