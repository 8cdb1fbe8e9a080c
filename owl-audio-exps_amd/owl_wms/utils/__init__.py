"""utils (reference: owl_wms/utils/__init__.py): Timer, freeze, checkpoint-prefix handling."""
import re
import time

import torch


class Timer:
    def reset(self):
        self.t = time.time()

    def hit(self):
        return time.time() - self.t


def freeze(module):
    if module is None:
        return
    for p in module.parameters():
        p.requires_grad = False


_PREFIX = re.compile(r'^(?:(?:_orig_mod\.|module\.)+)?([^.]+\.)?(?:(?:_orig_mod\.|module\.)+)?')


def strip_prefixes(sd):
    """rft_trainer.py:86-89: legacy checkpoints may carry module./_orig_mod. prefixes."""
    return {_PREFIX.sub(r"\1", k): v for k, v in sd.items()}


def versatile_load(path):
    """utils/__init__.py:21-62 (model weights only; never unpickles arbitrary objects)."""
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if "ema" in sd:
        sd = sd["ema"]
        prefix = "ema_model.module." if any(k.startswith("ema_model.module.") for k in sd) else "ema_model."
        sd = {k[len(prefix):]: v for k, v in sd.items() if k.startswith(prefix)}
    elif "model" in sd:
        sd = sd["model"]
    return strip_prefixes(sd)


@torch.no_grad()
def batch_permute(mouse, button, factor=1):
    """utils/__init__.py:69-90: ``factor`` times, append a batch-permuted copy along time."""
    for _ in range(factor):
        inds = torch.randperm(mouse.size(0))
        mouse = torch.cat([mouse, mouse.clone()[inds]], dim=1)
        button = torch.cat([button, button.clone()[inds]], dim=1)
    return mouse, button


@torch.no_grad()
def batch_permute_to_length(mouse, button, length):
    """utils/__init__.py:93-118: double the controls by batch_permute until >= length, truncate."""
    factor, n = 0, mouse.shape[1]
    while n < length:
        factor += 1
        n *= 2
    mouse, button = batch_permute(mouse, button, factor=factor)
    return mouse[:, :length], button[:, :length]
