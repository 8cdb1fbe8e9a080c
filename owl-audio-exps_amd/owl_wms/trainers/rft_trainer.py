"""RFTTrainer (reference: owl_wms/trainers/rft_trainer.py:25-228) for MI355X.

Step semantics kept: accum = target_batch_size // batch_size // world_size micro-steps of
``loss / accum`` backward; then (AdamW only) clip_grad_norm 10, optimizer step, zero grads,
EMA update, barrier.  Differences (MI355X-first): no torch.compile/DDP wrapper -- the block
kernels are libowlk and the all-reduce is GradReducer (bucket views, one RCCL all-reduce per
bucket on the last micro-step, overlapped with backward); data is synthetic latents of the
configured shape (real loaders are out of scope); metrics go to stdout instead of wandb.
"""
import time

import torch
import torch.distributed as dist

from ..data import get_loader
from ..models import get_model_cls
from ..muon import FusedAdamW, init_muon
from ..utils import Timer, strip_prefixes
from ..utils.grad_reducer import EMA, GradReducer
from .base import BaseTrainer


class RFTTrainer(BaseTrainer):
    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.model = get_model_cls(self.model_cfg.model_id)(self.model_cfg).train()
        if self.rank == 0:
            print(f"Model has {sum(p.numel() for p in self.model.parameters()):,} parameters")
        self.ema = self.opt = self.scheduler = None
        self.total_step_counter = 0
        self.max_steps = None  # optional cap (plumbing runs)
        self.history = []

    def get_module(self, ema=False):
        return self.model

    def save(self):
        if self.rank != 0:
            return
        super().save({"model": self.model.state_dict(), "ema": self.ema.state_dict(), "opt": self.opt.state_dict(),
                      "steps": self.total_step_counter})

    def load(self):
        ckpt = getattr(self.train_cfg, "resume_ckpt", None)
        state = None
        if ckpt:
            state = super().load(ckpt)
            state["model"] = strip_prefixes(state["model"])
            self.model.load_state_dict(state["model"], strict=True)
            self.total_step_counter = state.get("steps", 0)
        self.model = self.model.cuda()
        if self.world_size > 1:  # identical initial weights on every rank (DDP's init broadcast)
            with torch.no_grad():
                for p in self.model.parameters():
                    dist.broadcast(p, 0)
        self.ema = EMA(self.model, beta=0.999, update_after_step=0, update_every=1)
        opt_kwargs = dict(self.train_cfg.opt_kwargs or {})
        if self.train_cfg.opt.lower() == "muon":
            self.opt = init_muon(self.model, rank=self.rank, world_size=self.world_size, **opt_kwargs)
        else:
            if "betas" in opt_kwargs:
                opt_kwargs["betas"] = tuple(opt_kwargs["betas"])
            cls = FusedAdamW if self.train_cfg.opt == "AdamW" else getattr(torch.optim, self.train_cfg.opt)
            self.opt = cls(self.model.parameters(), **opt_kwargs)
        self.reducer = GradReducer(self.model.parameters(), world_size=self.world_size)
        if ckpt:
            self.ema.load_state_dict(state["ema"])
            self.opt.load_state_dict(state["opt"])

    def batch_loss(self, batch):
        vid, mouse, btn, doc_id = [t.cuda(non_blocking=True) for t in batch]
        vid = vid / self.train_cfg.vae_scale
        return self.model(vid, mouse, btn, doc_id)

    def loader(self):
        """rft_trainer.py:148-151: ``data_id`` + ``data_kwargs``.  A ``sequence_packing`` config whose
        ``dataset_path`` holds an NpyTable reads it (packed windows with per-frame doc_id); without
        one the loader yields synthetic latents of the configured shape."""
        kw = dict(self.train_cfg.get("data_kwargs") or {})
        data_id = self.train_cfg.get("data_id") or "synthetic"
        kw.setdefault("batch_columns", ["depth_latent", "mouse", "buttons"])
        return get_loader(data_id, self.train_cfg.batch_size, model_cfg=self.model_cfg, **kw)

    def train(self):
        torch.cuda.set_device(self.local_rank)
        accum = max(1, self.train_cfg.target_batch_size // self.train_cfg.batch_size // self.world_size)
        self.load()
        timer = Timer()
        timer.reset()
        local_step, loss_sum = 0, torch.zeros((), device="cuda")
        loader = self.loader()  # built once: persistent workers survive epochs
        for epoch in range(self.train_cfg.epochs):
            for batch in loader:
                self.reducer.begin(sync=(local_step + 1) % accum == 0)
                loss = self.batch_loss(batch) / accum
                loss.backward()
                self.reducer.finish()
                loss_sum += loss.detach()
                local_step += 1
                if local_step % accum != 0:
                    continue
                if self.train_cfg.opt.lower() != "muon":
                    torch.nn.utils.clip_grad_norm_(self.model.parameters(), max_norm=10.0)
                self.opt.step()
                self.reducer.zero_grad()
                self.ema.update()
                if self.world_size > 1:
                    dist.all_reduce(loss_sum)
                    loss_sum /= self.world_size
                rec = {"step": self.total_step_counter, "diffusion_loss": loss_sum.item(), "time": timer.hit()}
                self.history.append(rec)
                if self.rank == 0:
                    print(rec, flush=True)
                timer.reset()
                loss_sum.zero_()
                self.total_step_counter += 1
                if self.total_step_counter % self.train_cfg.save_interval == 0:
                    self.save()
                self.barrier()
                if self.max_steps is not None and self.total_step_counter >= self.max_steps:
                    return


class AudioRFTTrainer(RFTTrainer):
    """audio_rft_trainer.py:23-292 minus the on-the-fly VAE encode (random latents, config 1)."""

    def batch_loss(self, batch):
        return self.model(batch.cuda(non_blocking=True))

    def loader(self):
        return get_loader("synthetic_audio", self.train_cfg.batch_size, model_cfg=self.model_cfg)


class AVRFTTrainer(RFTTrainer):
    """av_trainer.py:23-261: joint video + audio objective (MMDiT, config 4)."""

    def batch_loss(self, batch):
        vid, mouse, btn, doc_id = [t.cuda(non_blocking=True) for t in batch]
        g = torch.Generator().manual_seed(len(self.history))
        audio = torch.randn(vid.shape[0], vid.shape[1], self.model_cfg.audio_channels, generator=g).cuda()
        loss, _, _ = self.model(vid / self.train_cfg.vae_scale, audio, mouse, btn)
        return loss
