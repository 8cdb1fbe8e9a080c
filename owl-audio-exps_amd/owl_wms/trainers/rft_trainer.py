"""RFTTrainer (reference: owl_wms/trainers/rft_trainer.py:25-280) for MI355X.

Step semantics kept: accum = target_batch_size // batch_size // world_size micro-steps of
``loss / accum`` backward; then (non-Muon only) clip_grad_norm 10, optimizer step, zero grads,
scheduler step, EMA update; logging through LogHelper (the logged ``diffusion_loss`` is the sum of
the micro-steps' ``loss / accum``, averaged over ranks, utils/logging.py:33-64); the eval sampler
at every ``sample_interval`` (step 0 included, :213, :243-280); save every ``save_interval``.

Differences (MI355X-first): no torch.compile/DDP wrapper -- the block kernels are libowlk and the
all-reduce is GradReducer (bucket views, one RCCL all-reduce per bucket on the last micro-step,
overlapped with backward); metrics go to stdout instead of wandb, and eval returns summary
statistics of the sampled latents (no VAE decode or media: out of scope).  Optional
``train.seed`` seeds torch's RNG per micro-step (the reference seeds nothing),
which makes a resumed run bit-identical to an uninterrupted one.
"""
import gc
from pathlib import Path

import torch
import torch.distributed as dist

from ..data import get_loader
from ..models import get_model_cls
from ..muon import FusedAdamW, init_muon
from ..sampling import get_sampler_cls
from ..schedulers import get_scheduler_cls
from ..utils import Timer, batch_permute_to_length, strip_prefixes
from ..utils.grad_reducer import EMA, GradReducer
from ..utils.logging import LogHelper
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
        return self.ema.ema_model if ema else self.model

    def save(self):
        if self.rank != 0:
            return
        d = {"model": self.model.state_dict(), "ema": self.ema.state_dict(), "opt": self.opt.state_dict(),
             "steps": self.total_step_counter}
        if self.scheduler is not None:
            d["scheduler"] = self.scheduler.state_dict()
        super().save(d)

    def load(self):
        """rft_trainer.py:78-121: build model / EMA / optimizer / scheduler, then restore a checkpoint
        (``resume_ckpt``) with the legacy module. / _orig_mod. prefixes stripped from both the model
        and the EMA keys (:86-89), strict."""
        ckpt = getattr(self.train_cfg, "resume_ckpt", None)
        state = None
        if ckpt:
            state = super().load(ckpt)
            state["model"] = strip_prefixes(state["model"])
            state["ema"] = strip_prefixes(state["ema"])
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
        sched = self.train_cfg.get("scheduler")
        if sched:
            self.scheduler = get_scheduler_cls(sched)(self.opt, **dict(self.train_cfg.get("scheduler_kwargs") or {}))
        self.reducer = GradReducer(self.model.parameters(), world_size=self.world_size)
        if ckpt:
            self.ema.load_state_dict(state["ema"])
            self.opt.load_state_dict(state["opt"])
            if self.scheduler is not None and "scheduler" in state:
                self.scheduler.load_state_dict(state["scheduler"])
        del state

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

    # ------------------------------------------------------------------ eval (rft_trainer.py:243-280)
    def eval_setup(self):
        """sample loader + sampler (rft_trainer.py:155-170); None when the config names no sampler."""
        sid = self.train_cfg.get("sampler_id")
        if not sid:
            return None, None
        n = (int(self.train_cfg.get("n_samples") or 1) + self.world_size - 1) // self.world_size
        kw = dict(self.train_cfg.get("sample_data_kwargs") or {})
        sample_loader = iter(get_loader(self.train_cfg.get("sample_data_id") or "synthetic", n,
                                        model_cfg=self.model_cfg, **kw))
        skw = dict(self.train_cfg.get("sampler_kwargs") or {})
        self.sampler_only_return_generated = bool(skw.pop("only_return_generated", False))
        return sample_loader, get_sampler_cls(sid)(**skw)

    def _gather_concat_cpu(self, t, dim=0):
        if self.world_size == 1:
            return t.cpu()
        if self.rank == 0:
            parts, scratch = [t.cpu()], torch.empty_like(t)
            for src in range(1, self.world_size):
                dist.recv(scratch, src=src)
                parts.append(scratch.cpu())
            return torch.cat(parts, dim=dim)
        dist.send(t, dst=0)

    @torch.no_grad()
    def eval_step(self, sample_loader, sampler):
        ema_core = self.get_module(ema=True).core
        vid, mouse, btn = [x.cuda() for x in next(sample_loader)[:3]]
        mouses, btns = [mouse], [btn]
        for _ in range(15):
            _, m, b = [x.cuda() for x in next(sample_loader)[:3]]
            mouses.append(m)
            btns.append(b)
        mouse, button = batch_permute_to_length(torch.cat(mouses), torch.cat(btns), sampler.num_frames + vid.size(1))
        mouse, button = mouse[:vid.size(0)], button[:vid.size(0)]
        vid = vid / self.train_cfg.vae_scale
        latent = sampler(ema_core, vid, mouse, button)
        if self.sampler_only_return_generated:
            latent = latent[:, vid.size(1):]
        out = {"eval/samples": latent.shape[0] * self.world_size, "eval/frames": latent.shape[1],
               "eval/latent_std": latent.float().std().item()}
        if self.train_cfg.get("eval_sample_dir"):
            full = self._gather_concat_cpu(latent)
            if self.rank == 0:
                d = Path(self.train_cfg.eval_sample_dir)
                d.mkdir(parents=True, exist_ok=True)
                torch.save(full, d / f"vid.{self.total_step_counter}.pt")
        self.barrier()  # the reference's unconditional dist.barrier() (App. A.4), guarded for 1 rank
        return out if self.rank == 0 else None

    # ------------------------------------------------------------------ training loop
    def train(self):
        torch.cuda.set_device(self.local_rank)
        accum = max(1, self.train_cfg.target_batch_size // self.train_cfg.batch_size // self.world_size)
        self.load()
        timer = Timer()
        timer.reset()
        metrics = LogHelper()
        loader = self.loader()  # built once: persistent workers survive epochs
        sample_loader, sampler = self.eval_setup()
        seed = self.train_cfg.get("seed")
        local_step = 0
        for epoch in range(self.train_cfg.epochs):
            for batch in loader:
                if seed is not None:
                    torch.manual_seed(int(seed) + 7919 * (self.total_step_counter * accum + local_step % accum)
                                      + 104729 * self.rank)
                self.reducer.begin(sync=(local_step + 1) % accum == 0)
                loss = self.batch_loss(batch) / accum
                loss.backward()
                self.reducer.finish()
                metrics.log("diffusion_loss", loss)
                local_step += 1
                if local_step % accum != 0:
                    continue
                if self.train_cfg.opt.lower() != "muon":
                    torch.nn.utils.clip_grad_norm_(self.model.parameters(), max_norm=10.0)
                self.opt.step()
                self.reducer.zero_grad()
                if self.scheduler is not None:
                    self.scheduler.step()
                self.ema.update()
                rec = metrics.pop()
                rec["time"] = timer.hit()
                timer.reset()
                if sampler is not None and self.total_step_counter % self.train_cfg.sample_interval == 0:
                    ev = self.eval_step(sample_loader, sampler)
                    gc.collect()
                    torch.cuda.empty_cache()
                    if ev:
                        rec.update(ev)
                rec["step"] = self.total_step_counter
                self.history.append(rec)
                if self.rank == 0:
                    print(rec, flush=True)
                self.total_step_counter += 1
                if self.total_step_counter % self.train_cfg.save_interval == 0:
                    self.save()
                self.barrier()
                if self.max_steps is not None and len(self.history) >= self.max_steps:
                    return


class AudioRFTTrainer(RFTTrainer):
    """audio_rft_trainer.py:23-292 minus the on-the-fly VAE encode (random latents, config 1)."""

    def batch_loss(self, batch):
        return self.model(batch.cuda(non_blocking=True))

    def loader(self):
        return get_loader("synthetic_audio", self.train_cfg.batch_size, model_cfg=self.model_cfg)

    def eval_setup(self):
        return None, None


class AVRFTTrainer(RFTTrainer):
    """av_trainer.py:23-261: joint video + audio objective (MMDiT, config 4)."""

    def batch_loss(self, batch):
        vid, mouse, btn, doc_id = [t.cuda(non_blocking=True) for t in batch]
        g = torch.Generator().manual_seed(len(self.history))
        audio = torch.randn(vid.shape[0], vid.shape[1], self.model_cfg.audio_channels, generator=g).cuda()
        loss, _, _ = self.model(vid / self.train_cfg.vae_scale, audio, mouse, btn)
        return loss

    def eval_setup(self):
        return None, None
