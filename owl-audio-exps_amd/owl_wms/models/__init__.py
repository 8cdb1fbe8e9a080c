"""Model registry (reference: owl_wms/models/__init__.py:1-25)."""


def get_model_cls(model_id):
    if model_id == "game_rft":
        from .gamerft import GameRFT
        return GameRFT
    if model_id == "game_rft_audio":
        from .gamerft_audio import GameRFTAudio
        return GameRFTAudio
    if model_id == "audio_rft":
        from .audiorft import AudioRFT
        return AudioRFT
    if model_id == "game_mft_audio":
        raise NotImplementedError("game_mft_audio (Mean-Flow) is out of scope: no BASELINE config uses it and the "
                                  "reference's own import is broken (SURVEY.md §2.1)")
    raise ValueError(f"unknown model_id {model_id!r}")
