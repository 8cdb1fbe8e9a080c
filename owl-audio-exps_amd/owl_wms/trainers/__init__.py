"""Trainer registry (reference: owl_wms/trainers/__init__.py:1-37)."""


def get_trainer_cls(trainer_id):
    if trainer_id == "rft":
        from .rft_trainer import RFTTrainer
        return RFTTrainer
    if trainer_id == "audio_rft":
        from .rft_trainer import AudioRFTTrainer
        return AudioRFTTrainer
    if trainer_id == "av":
        from .rft_trainer import AVRFTTrainer
        return AVRFTTrainer
    raise NotImplementedError(f"trainer {trainer_id!r} is out of scope for the MI355X hot-path build "
                              "(distillation / self-forcing trainers, SURVEY.md §2.1)")
