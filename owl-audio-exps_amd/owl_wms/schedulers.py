"""LR schedulers (reference: owl_wms/schedulers.py:1-2).

The reference's ``get_scheduler_cls`` is an empty stub (it returns None, so any non-null
``train.scheduler`` fails there at construction).  Here a name resolves to the torch.optim.lr_scheduler
class of that name (e.g. ``LinearLR``, ``CosineAnnealingLR``), built with ``train.scheduler_kwargs``
on the optimizer; anything else raises NotImplementedError instead of failing later.
"""
import torch


def get_scheduler_cls(scheduler_id):
    cls = getattr(torch.optim.lr_scheduler, str(scheduler_id), None)
    if isinstance(cls, type) and issubclass(cls, torch.optim.lr_scheduler.LRScheduler):
        return cls
    raise NotImplementedError(f"scheduler {scheduler_id!r}: the reference defines none "
                              "(owl_wms/schedulers.py); use a torch.optim.lr_scheduler class name")
