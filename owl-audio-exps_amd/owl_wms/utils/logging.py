"""LogHelper (reference: owl_wms/utils/logging.py:23-64) without wandb.

Same semantics: ``log(key, v)`` adds v / world_size to the key's running sum (the caller divides
by the accumulation steps beforehand); ``pop()`` sums over ranks and clears.  MI355X-side
difference: tensor values stay on the device until ``pop`` (the reference calls ``.item()`` per
micro-step, a host sync that idles the GPU while the next micro-step is enqueued), and the
cross-rank sum is one all_reduce of a small vector instead of all_gather_object.
"""
import torch
import torch.distributed as dist


class LogHelper:
    def __init__(self):
        self.world_size = dist.get_world_size() if dist.is_initialized() else 1
        self.data = {}

    def log(self, key, data):
        if isinstance(data, torch.Tensor):
            data = data.detach().float()
        val = data / self.world_size
        self.data[key] = self.data[key] + val if key in self.data else val

    def log_dict(self, d):
        for k, v in d.items():
            self.log(k, v)

    def pop(self):
        keys = list(self.data)
        if not keys:
            return {}
        dev = next((v.device for v in self.data.values() if isinstance(v, torch.Tensor)), torch.device("cpu"))
        if self.world_size > 1 and dist.get_backend() == "nccl" and dev.type == "cpu":
            dev = torch.device("cuda", torch.cuda.current_device())
        vals = torch.stack([torch.as_tensor(self.data[k], dtype=torch.float32, device=dev).reshape(()) for k in keys])
        if self.world_size > 1:
            dist.all_reduce(vals)
        self.data = {}
        return dict(zip(keys, vals.tolist()))
