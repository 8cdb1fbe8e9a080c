"""BaseTrainer (reference: owl_wms/trainers/base.py:10-75) without the wandb dependency."""
import os

import torch
import torch.distributed as dist


class BaseTrainer:
    def __init__(self, train_cfg, logging_cfg, model_cfg, global_rank=0, local_rank=0, world_size=1):
        self.rank, self.local_rank, self.world_size = global_rank, local_rank, world_size
        self.train_cfg, self.logging_cfg, self.model_cfg = train_cfg, logging_cfg, model_cfg
        self.device = f"cuda:{local_rank}"

    def barrier(self):
        if self.world_size > 1:
            dist.barrier()

    def save(self, save_dict):
        """base.py:61-72: checkpoint_dir/step_N.pt (+ EMA-only weights to output_path)."""
        os.makedirs(self.train_cfg.checkpoint_dir, exist_ok=True)
        torch.save(save_dict, os.path.join(self.train_cfg.checkpoint_dir, f"step_{self.total_step_counter}.pt"))
        out = getattr(self.train_cfg, "output_path", None)
        if "ema" in save_dict and out:
            prefix = "ema_model."
            d = {k[len(prefix):]: v for k, v in save_dict["ema"].items() if k.startswith(prefix)}
            os.makedirs(out, exist_ok=True)
            torch.save(d, os.path.join(out, f"step_{self.total_step_counter}.pt"))

    def load(self, path):
        return torch.load(path, map_location="cpu", weights_only=True)
