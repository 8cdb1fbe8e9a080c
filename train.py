"""Drop-in entry point (reference: train.py:9-29):
    python train.py --config_path configs/X.yml [--nccl_timeout S]
    torchrun --nproc_per_node=8 --master-addr 127.0.0.1 train.py --config_path configs/dit_v4.yml
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "owl-audio-exps_amd"))

from owl_wms.configs import Config  # noqa: E402
from owl_wms.trainers import get_trainer_cls  # noqa: E402
from owl_wms.utils.ddp import cleanup, setup  # noqa: E402

if __name__ == "__main__":
    parser = argparse.ArgumentParser()
    parser.add_argument("--config_path", type=str, help="Path to config YAML file")
    parser.add_argument("--nccl_timeout", type=int, default=None, help="NCCL process-group timeout in seconds")
    parser.add_argument("--max_steps", type=int, default=None, help="stop after N optimizer steps")
    args = parser.parse_args()
    cfg = Config.from_yaml(args.config_path)
    global_rank, local_rank, world_size = setup(timeout=args.nccl_timeout)
    trainer = get_trainer_cls(cfg.train.trainer_id)(cfg.train, cfg.wandb, cfg.model, global_rank, local_rank,
                                                    world_size)
    trainer.max_steps = args.max_steps
    trainer.train()
    cleanup()
