"""ctypes binding of libowlk.so (the C ABI declared in include/owlk.h).

The library is built in-tree by ``owl-audio-exps_amd/csrc/Makefile`` (``__graft_entry__.build()``).
It is loaded after ``torch`` so it binds to the HIP runtime torch already loaded (same SONAME).
There is no fallback: if the library is missing or a call fails, a RuntimeError is raised.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libowlk.so")

L, I, F, P = ctypes.c_long, ctypes.c_int, ctypes.c_float, ctypes.c_void_p

_SIGS = {
    "owlk_gemm": [L, L, L, L, P, L, L, I, P, L, L, I, P, L, L, I, I, F, F, P, P, L, L, P, L, L, L, P, L, L, P, P, L,
                  P],
    "owlk_gemm_frames": [L, L, L, P, L, L, I, P, L, L, I, P, L, L, I, I, F, F, P, P, L, P, L, L, P, L, P, L, P],
    "owlk_gemm_splitk_bytes": [L, L, L, L, I, I, I, I, F],
    "owlk_gemm_ws_bytes": [L, L, L, L, I, I, I, I, F, I],
    "owlk_gemm_ws_counter_bytes": [L, L, L, L, I, I, I, I, F],
    "owlk_adaln_fwd": [P, L, P, P, L, L, L, I, P, L, P, P, P],
    "owlk_adaln_bwd": [P, L, P, L, P, P, L, L, L, I, P, L, P, L, P, P, L, P, I, P],
    "owlk_gate_bwd": [P, L, P, L, P, L, L, L, I, P, L, P, L, I, P, L, P],
    "owlk_adaln_gate_bwd": [P, L, P, L, P, P, L, L, L, I, P, L, P, L, P, P, L, I, P, L, P, L, P, L, P, L, I, P, L,
                            P],
    "owlk_cond_embed": [P, I, P, I, F, P, L, P, I, L, P, I, F, P, P, L, P, P, I, L, I, I, P, L, L, P],
    "owlk_cond_silu_fwd": [P, P, P, P, L, L, I, P, P, P],
    "owlk_cond_silu_bwd": [P, I, P, P, L, L, I, P, P, P],
    "owlk_small_k_wgrad": [P, L, P, L, L, L, I, P, L, F, P],
    "owlk_qk_rope_fwd": [P, L, L, I, I, P, P, L, L, L, L, P, L, P, P],
    "owlk_qk_rope_fwd_kv": [P, L, L, L, I, I, P, P, L, L, L, P, L, L, P, L, L, P, L, L, P],
    "owlk_qk_rope_fwd_kv_dev": [P, L, L, L, I, I, P, P, L, L, P, P, L, L, P, L, L, P, L, L, L, P],
    "owlk_attn_decode_fwd": [P, L, L, P, L, L, P, L, L, P, L, L, P, L, I, L, I, F, F, P, L, L, L, P],
    "owlk_qk_rope_bwd": [P, L, P, L, L, I, I, P, P, L, L, L, L, P, P, L, P],
    "owlk_qk_rope_bwd_ws_bytes": [L, I, I],
    "owlk_qk_rope_bwd_bias": [P, L, P, L, L, I, I, P, P, L, L, L, L, P, P, L, P, P, L, P],
    "owlk_attn_fwd": [P, L, L, P, L, L, P, L, L, P, L, L, P, L, I, L, L, I, F, F, L, I, I, L, P, P, P, P, L, P],
    "owlk_attn_delta": [P, P, L, L, L, I, I, P, P],
    "owlk_frame_mux": [I, L, I, I, I, P, L, P, L, P, L, P],
    "owlk_layernorm_fwd": [P, L, L, I, P, L, P, P, P],
    "owlk_layernorm_bwd": [P, L, P, L, P, P, L, I, P, L, P],
    "owlk_attn_bwd": [P, L, L, P, L, L, P, L, L, P, L, L, P, P, P, L, L, P, L, L, P, L, L, L, I, L, L, I, F, L, I, I,
                      P, P, P, P, L, P],
    "owlk_attn_bwd_dkdv": [P, L, L, P, L, L, P, L, L, P, L, L, P, P, P, L, L, P, L, L, P, L, L, L, I, L, L, I, F, L, I,
                           I, P, P, P, P, L, P],
    "owlk_attn_bwd_dq": [P, L, L, P, L, L, P, L, L, P, L, L, P, P, P, L, L, P, L, L, P, L, L, L, I, L, L, I, F, L, I, I,
                         P, P, P, P, L, P],
    "owlk_attn_bwd_fused_ws_bytes": [L, I, L, I],
    "owlk_attn_bwd_fused": [P, L, L, P, L, L, P, L, L, P, L, L, P, P, P, L, L, P, L, L, P, L, L, L, I, L, I, F, L, I, I,
                            P, P, P, P, L, P, L, I, P],
    "owlk_set_cu_reserve": [I],
    "owlk_gemm_attn_delta": [L, L, L, P, L, P, L, P, L, P, L, L, I, I, P, P],
    "owlk_gemm_qk_rope": [L, L, L, P, L, P, L, P, P, L, I, I, P, P, L, L, L, L, P, L, P, P],
    "owlk_flow_noise": [P, P, P, I, I, L, P, P, P, P],
    "owlk_unpatchify": [P, I, I, L, P, P],
    "owlk_mse": [P, P, L, F, P, P, I, P, P],
    "owlk_mse_grad": [P, P, L, F, P, P, P],
    "owlk_gate_resid": [P, L, P, L, P, L, L, L, I, P, L, P],
    "owlk_colsum_ws_bytes": [L, L],
    "owlk_colsum": [P, I, L, L, L, P, P, L, P],
    "owlk_colsum_frames": [P, I, L, L, L, L, P, P, L, P],
    "owlk_ns_normalize": [P, I, L, L, L, I, P, P, P],
    "owlk_ns_scale": [P, I, L, L, L, I, P, P, P],
    "owlk_ns_iterate_ws_bytes": [L, L, L],
    "owlk_ns_iterate": [P, L, L, L, I, F, F, F, P, L, P],
    "owlk_newton_schulz_ws_bytes": [L, L, L],
    "owlk_newton_schulz_bf16": [P, I, L, L, L, I, F, F, F, P, P, L, P],
    "owlk_muon_momentum": [I, P, P, L, F, I, P, P, P],
    "owlk_muon_apply": [I, P, P, L, L, I, F, F, P],
    "owlk_adamw": [I, P, P, P, P, P, F, F, F, F, F, F, F, P],
    "owlk_ema": [I, P, P, P, F, P],
}

# size queries; every other entry returns an int status
_RESTYPES = {n: ctypes.c_long for n in ("owlk_gemm_splitk_bytes", "owlk_gemm_ws_bytes", "owlk_gemm_ws_counter_bytes",
                                         "owlk_qk_rope_bwd_ws_bytes", "owlk_attn_bwd_fused_ws_bytes",
                                        "owlk_colsum_ws_bytes", "owlk_ns_iterate_ws_bytes",
                                        "owlk_newton_schulz_ws_bytes")}

_lib = None


def lib():
    global _lib
    if _lib is None:
        path = os.environ.get("OWLK_LIB", LIB_PATH)  # A/B builds (tools/); default: the in-tree library
        if not os.path.exists(path):
            raise RuntimeError(f"libowlk.so not built at {path}: run `make -C owl-audio-exps_amd/csrc` "
                               "(or __graft_entry__.build()); there is no non-HIP fallback")
        h = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        for name, args in _SIGS.items():
            if path != LIB_PATH and not hasattr(h, name):  # older A/B build: symbol not there
                continue
            fn = getattr(h, name)
            fn.argtypes = args
            fn.restype = _RESTYPES.get(name, ctypes.c_int)
        h.owlk_last_error.restype = ctypes.c_char_p
        h.owlk_last_error.argtypes = []
        h.owlk_version.restype = ctypes.c_int
        h.owlk_device_ok.restype = ctypes.c_int
        _lib = h
    return _lib


def exported_symbols():
    return ["owlk_last_error", "owlk_version", "owlk_device_ok"] + list(_SIGS)


_profile = None  # list of (key, flops, start_event, end_event) while a profile window is open


def profiling():
    """True while a profile window is open (its events time launches on the current stream)."""
    return _profile is not None


def profile_begin():
    global _profile
    _profile = []


def profile_end():
    """-> {key: (launches, total_ms, total_flops)} for the calls made since profile_begin()."""
    global _profile
    torch.cuda.synchronize()
    out = {}
    for key, flops, e0, e1 in _profile or []:
        n, ms, fl = out.get(key, (0, 0.0, 0.0))
        out[key] = (n + 1, ms + e0.elapsed_time(e1), fl + (flops or 0.0))
    _profile = None
    return out


def call(name, *args, key=None, flops=None):
    prof = _profile
    if prof is not None:
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed ({rc}): {lib().owlk_last_error().decode()}")
    if prof is not None:
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        prof.append((key or name, flops() if callable(flops) else flops, e0, e1))


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
