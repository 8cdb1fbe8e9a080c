"""Config loading (reference: owl_wms/configs.py:7-84).

omegaconf is not available on MI355X boxes here, so YAML is loaded into permissive attribute
dicts: declared dataclass defaults first, then every YAML key (including the undeclared ones the
reference reads through getattr: backbone, rope_impl, local_window, has_audio, ...).
"""
from dataclasses import asdict, dataclass

import yaml


class AttrDict(dict):
    """dict with attribute access; missing attributes raise AttributeError (so getattr defaults work)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    def __delattr__(self, k):
        del self[k]


def _wrap(v):
    if isinstance(v, dict):
        return AttrDict({k: _wrap(x) for k, x in v.items()})
    if isinstance(v, list):
        return [_wrap(x) for x in v]
    return v


@dataclass
class TransformerConfig:
    model_id: str = None
    n_layers: int = 12
    n_heads: int = 12
    d_model: int = 384
    patch_size: int = 1
    channels: int = 128
    audio_channels: int = 64
    sample_size: int = 16
    cfg_prob: float = 0.1
    n_buttons: int = 8
    tokens_per_frame: int = 16
    audio_tokens: int = 0
    n_frames: int = 120
    causal: bool = False


@dataclass
class TrainingConfig:
    trainer_id: str = None
    data_id: str = None
    target_batch_size: int = 128
    batch_size: int = 2
    epochs: int = 200
    opt: str = "AdamW"
    opt_kwargs: dict = None
    loss_weights: dict = None
    scheduler: str = None
    scheduler_kwargs: dict = None
    checkpoint_dir: str = "checkpoints/v0"
    resume_ckpt: str = None
    teacher_ckpt: str = None
    teacher_cfg: str = None
    sample_interval: int = 1000
    save_interval: int = 1000
    n_samples: int = 8
    sampler_id: str = None
    sampler_kwargs: dict = None
    vae_id: str = None
    vae_cfg_path: str = None
    vae_ckpt_path: str = None
    vae_scale: float = 0.34
    vae_batch_size: int = 4


@dataclass
class WANDBConfig:
    name: str = None
    project: str = None
    run_name: str = None


def make_section(cls, raw):
    d = asdict(cls())
    d.update(raw or {})
    return _wrap(d)


def model_config(**kw):
    return make_section(TransformerConfig, kw)


class Config(AttrDict):
    @classmethod
    def from_yaml(cls, path):
        with open(path) as f:
            raw = yaml.safe_load(f)
        return cls(model=make_section(TransformerConfig, raw.get("model")),
                   train=make_section(TrainingConfig, raw.get("train")),
                   wandb=make_section(WANDBConfig, raw.get("wandb")))
