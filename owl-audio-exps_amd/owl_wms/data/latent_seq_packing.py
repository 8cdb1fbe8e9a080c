"""Sequence-packing loader over an NpyTable (reference: owl_wms/data/latent_seq_packing.py:13-164).

Documents (one NpyTable row each, ``seq_len`` frames) are laid end to end in a permuted order and
cut into fixed windows of ``window_length`` frames; a window that the stream does not fill (the
tail) is dropped.  Each sample is the concatenation of its document slices plus a per-frame
``doc_id`` (the document's position in the permutation), which the frame-masked attention kernels
take as their document array: frames attend only within their own document.

Packing is computed with cut points instead of the reference's per-window expansion: the union
of document boundaries and window boundaries splits the packed stream into segments that each lie
in exactly one document and one window.  The result is stored as two flat int64 arrays (segments
``[S, 3] = (doc, lo, hi)`` and a window -> segment CSR pointer), so a 10^6-document table packs
in milliseconds and pickles cheaply to loader workers.
"""
from functools import partial
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist
from torch.utils.data import DataLoader, Dataset, DistributedSampler

from .npy_table import NpyTable

META_COLUMNS = ("tarball", "pt_idx", "missing", "truncated", "seq_len")


def pack_windows(lens: np.ndarray, window: int) -> Tuple[np.ndarray, np.ndarray]:
    """Pack documents of ``lens`` frames (in the given order) into full windows of ``window`` frames.

    Returns ``(seg, ptr)``: ``seg[ptr[w]:ptr[w+1]]`` are the ``(doc, lo, hi)`` slices of window w,
    ``hi`` exclusive, in stream order.  Same windows as ``get_window_slices``
    (latent_seq_packing.py:102-135), including the dropped partial tail.
    """
    lens = np.asarray(lens, dtype=np.int64)
    if window <= 0:
        raise ValueError("window_length must be positive")
    if lens.size and (lens <= 0).any():
        raise ValueError("every document needs seq_len > 0")
    ends = np.cumsum(lens)
    total = int(ends[-1]) if lens.size else 0
    n_win = total // window
    if n_win == 0:
        return np.zeros((0, 3), np.int64), np.zeros(1, np.int64)
    limit = n_win * window
    starts = ends - lens
    cuts = np.unique(np.concatenate([starts, ends, np.arange(0, limit + 1, window, dtype=np.int64)]))
    cuts = cuts[cuts <= limit]
    a, b = cuts[:-1], cuts[1:]
    doc = np.searchsorted(ends, a, side="right")
    seg = np.stack([doc, a - starts[doc], b - starts[doc]], axis=1)
    ptr = np.searchsorted(a // window, np.arange(n_win + 1), side="left").astype(np.int64)
    return seg, ptr


class AutoEpochDistributedSampler(DistributedSampler):
    """latent_seq_packing.py:16-25: a fresh shuffle each time the sampler is iterated."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self._auto_epoch = 0

    def __iter__(self):
        self.set_epoch(self._auto_epoch)
        self._auto_epoch += 1
        return super().__iter__()


class WindowedViewDataset(Dataset):
    """Packed fixed-length windows over an NpyTable (latent_seq_packing.py:28-100)."""

    def __init__(self, table_dir: str, window_length: int, include_missing_features: bool = False,
                 include_truncated: bool = True, meta_cols: Sequence[str] = META_COLUMNS,
                 array_columns: Optional[List[str]] = None, verbose: bool = True):
        self.window_length = int(window_length)
        self.table = NpyTable(table_dir)
        self.array_columns = (list(array_columns) if array_columns is not None
                              else [c for c in self.table.columns if c not in meta_cols])
        seq_len, missing, truncated = (np.asarray(v) for v in self.table[["seq_len", "missing", "truncated"]])
        keep = np.ones(seq_len.shape, bool)
        if not include_missing_features:
            keep &= ~missing.astype(bool)
        if not include_truncated:
            keep &= ~truncated.astype(bool)
        self._docs = np.flatnonzero(keep)
        self._lens = seq_len[keep].astype(np.int64)
        if (self._lens <= 0).any():
            raise ValueError("NpyTable rows with seq_len <= 0")
        self._build_packing(np.arange(len(self._docs)))
        if verbose:
            print(f"{len(self)} packed windows over {len(self._docs)} documents")

    def set_epoch(self, epoch: int):
        """Re-pack under ``RandomState(epoch).permutation`` (same on every rank)."""
        self._build_packing(np.random.RandomState(epoch).permutation(len(self._docs)))

    def _build_packing(self, perm):
        perm = np.asarray(perm, dtype=np.int64)
        self._row_lookup = self._docs[perm]
        self._seg, self._ptr = pack_windows(self._lens[perm], self.window_length)

    def window_slices(self, idx: int) -> List[Tuple[int, int, int]]:
        s = self._seg[self._ptr[idx]:self._ptr[idx + 1]]
        return [tuple(int(v) for v in r) for r in s]

    def __len__(self):
        return len(self._ptr) - 1

    def __getitem__(self, idx):
        if not 0 <= idx < len(self):
            raise IndexError(idx)
        segs = self._seg[self._ptr[idx]:self._ptr[idx + 1]]
        out = {}
        for col in self.array_columns:
            first = self.table.array(col, int(self._row_lookup[segs[0, 0]]))
            buf = np.empty((self.window_length,) + first.shape[1:], dtype=first.dtype)
            at = 0
            for doc, lo, hi in segs:
                buf[at:at + hi - lo] = self.table.array(col, int(self._row_lookup[doc]))[lo:hi]
                at += hi - lo
            out[col] = torch.from_numpy(buf)
        out["doc_id"] = torch.from_numpy(np.repeat(segs[:, 0], segs[:, 2] - segs[:, 1]))
        return out


def collate_fn(batch, batch_columns: List[str]):
    """latent_seq_packing.py:138-146: stack, fp32 and buttons to bf16; ``batch_columns + [doc_id]``."""
    out = []
    for col in list(batch_columns) + ["doc_id"]:
        t = torch.stack([item[col] for item in batch])
        if t.dtype == torch.float32 or col == "buttons":
            t = t.bfloat16()
        out.append(t)
    return out


def get_loader(batch_size, dataset_path, window_length, batch_columns, num_workers: int = 2, **_):
    """latent_seq_packing.py:149-164."""
    assert batch_size == 1, "sequence packing yields one packed window per sample (batch_size 1)"
    world_size = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    ds = WindowedViewDataset(dataset_path, window_length, array_columns=list(batch_columns))
    if world_size > 1:
        kw = dict(sampler=AutoEpochDistributedSampler(ds, num_replicas=world_size, rank=rank, shuffle=True),
                  shuffle=False)
    else:
        kw = dict(shuffle=True)
    if num_workers > 0:
        kw.update(prefetch_factor=2, persistent_workers=True)
    return DataLoader(ds, batch_size=batch_size, collate_fn=partial(collate_fn, batch_columns=list(batch_columns)),
                      num_workers=num_workers, drop_last=True, pin_memory=torch.cuda.is_available(), **kw)
