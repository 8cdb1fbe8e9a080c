"""Data (reference: owl_wms/data/).  ``sequence_packing`` over an on-disk NpyTable is in
``latent_seq_packing`` / ``npy_table``; the S3 loaders are out of scope.
``synthetic`` yields batches of the configured latent shape for benchmarking and
plumbing runs, with the reference's batch tuple layout."""
import os

import torch


def synthetic_video_batch(cfg, batch_size, seed=1234, n_docs=1, device="cpu", n_frames=None):
    """(vid [b,n,c,h,w] bf16, mouse [b,n,2] bf16, btn [b,n,n_buttons] bf16, doc_id [b,n] int64);
    n = n_frames (a loader's window_length) or the model's n_frames."""
    g = torch.Generator().manual_seed(seed)
    n, c, s = n_frames or cfg.n_frames, cfg.channels, cfg.sample_size
    vid = torch.randn(batch_size, n, c, s, s, generator=g).to(torch.bfloat16)
    mouse = torch.randn(batch_size, n, 2, generator=g).to(torch.bfloat16)
    btn = (torch.rand(batch_size, n, cfg.n_buttons, generator=g) < 0.5).to(torch.bfloat16)
    doc = (torch.arange(n) * n_docs // n).expand(batch_size, n).contiguous()
    return [t.to(device) for t in (vid, mouse, btn, doc)]


def synthetic_audio_batch(cfg, batch_size, seed=1234, device="cpu"):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(batch_size, cfg.sample_size, cfg.channels, generator=g).to(device)


class SyntheticLoader:
    def __init__(self, make, n_batches):
        self.make, self.n = make, n_batches

    def __len__(self):
        return self.n

    def __iter__(self):
        for i in range(self.n):
            yield self.make(i)


def get_loader(data_id, batch_size, model_cfg=None, n_batches=10 ** 9, **kwargs):
    """data/__init__.py:1-19.  ``sequence_packing`` with an existing ``dataset_path`` reads a real
    NpyTable (latent_seq_packing.py); without one it falls back to synthetic latents of the shape."""
    path = kwargs.get("dataset_path")
    if data_id == "sequence_packing" and path and os.path.exists(os.path.join(path, "manifest.json")):
        from . import latent_seq_packing
        return latent_seq_packing.get_loader(batch_size, **kwargs)
    if data_id in ("synthetic", "sequence_packing", "cod", "synthetic_video"):
        return SyntheticLoader(lambda i: synthetic_video_batch(model_cfg, batch_size, seed=1234 + i,
                                                               n_docs=kwargs.get("n_docs", 1),
                                                               n_frames=kwargs.get("window_length")), n_batches)
    if data_id in ("synthetic_audio", "local_waveform"):
        return SyntheticLoader(lambda i: synthetic_audio_batch(model_cfg, batch_size, seed=1234 + i), n_batches)
    raise NotImplementedError(f"data_id {data_id!r}: only synthetic latents are supported on this build "
                              "(real S3/NpyTable loaders are out of scope, SURVEY.md §2.1)")
