"""Samplers (reference: owl_wms/sampling/__init__.py:1-39).

Implemented on libowlk's KV-cache decode path: ``av_caching`` (AVCachingSamplerV2, the registry
entry the reference resolves it to) and ``audio_caching``.  The window / causal-window samplers
and the one-step variant are outside this build's hot-path scope.
"""


def get_sampler_cls(sampler_id):
    if sampler_id == "av_caching":
        from .av_caching_v2 import AVCachingSamplerV2
        return AVCachingSamplerV2
    if sampler_id == "audio_caching":
        from .audio_caching import AudioCachingSampler
        return AudioCachingSampler
    if sampler_id in ("av_window", "av_causal", "av_causal_no_cfg", "av_caching_one_step"):
        raise NotImplementedError(f"sampler {sampler_id!r} is out of scope for the MI355X build (SURVEY.md §8(f))")
    raise ValueError(f"unknown sampler_id {sampler_id!r}")
