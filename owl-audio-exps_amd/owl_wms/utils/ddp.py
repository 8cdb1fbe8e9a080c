"""utils/ddp.py (reference :5-28): one process per GPU; backend "nccl" is RCCL on ROCm."""
import datetime as dt
import os

import torch
import torch.distributed as dist


def setup(force=False, timeout=None):
    kw = dict(timeout=dt.timedelta(seconds=timeout)) if timeout else {}
    if "RANK" not in os.environ and not force:
        return 0, 0, 1  # single process (the reference's bare-except fallback, made explicit)
    backend = "nccl" if torch.cuda.is_available() else "gloo"
    dist.init_process_group(backend=backend, **kw)
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    if torch.cuda.is_available():
        torch.cuda.set_device(local_rank)
    return dist.get_rank(), local_rank, dist.get_world_size()


def cleanup():
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
