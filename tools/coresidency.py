"""Can a collective run beside the single-pass attention backward?

The global-layer attn_bwd_fused launch is a persistent grid of one workgroup per CU (round 6: the
one-wave-per-SIMD kernel, 4 waves x 512 registers, 147.5 KiB of LDS: nothing else fits beside it).
RCCL's all-reduce kernels run on their own stream (utils/grad_reducer.py).  This probe launches, on a
second stream, a kernel with an RCCL-like footprint (tools/coresid_kernel.hip: 32 persistent
workgroups of 256 threads, 8 KiB LDS, streaming a 256 MiB gradient bucket) while the fused kernel
runs, and the other way round, and reads the 100 MHz real-time clock stamped by every workgroup and
around the fused launch -- once per CU reserve in RESERVE (owlk_set_cu_reserve: the grid shrinks to
CUs - k).

    RESERVE=0,8,16 python tools/coresidency.py
    (build: hipcc -O3 --offload-arch=gfx950 -shared -fPIC tools/coresid_kernel.hip -o tools/_coresid.so)
"""
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "owl-audio-exps_amd")]
import torch  # noqa: E402

from owl_wms import _lib  # noqa: E402
from owl_wms import kernels as K  # noqa: E402

CO = ctypes.CDLL(os.path.join(REPO, "tools", "_coresid.so"))
CO.coresid_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_void_p,
                            ctypes.c_void_p]
CO.coresid_now.argtypes = [ctypes.c_void_p, ctypes.c_void_p]


def main():
    H, D, tpf, nf = 24, 64, 64, 1536
    L = nf * tpf
    torch.manual_seed(0)
    qkv = torch.randn(1, L, 3 * H * D, device="cuda", dtype=torch.bfloat16)
    qk = qkv[:, :, :2 * H * D].view(1, L, 2 * H, D)
    qk.copy_((qk.float() * torch.rsqrt(qk.float().pow(2).mean(-1, keepdim=True))).bfloat16())
    q, k, v = qkv[:, :, :H * D], qkv[:, :, H * D:2 * H * D], qkv[:, :, 2 * H * D:]
    do = torch.randn(1, L, H * D, device="cuda", dtype=torch.bfloat16)
    dq, dk, dv = (torch.empty(1, L, H * D, device="cuda", dtype=torch.bfloat16) for _ in range(3))
    mask = K.FrameMask(tpf, None)
    o, lse = K.attn_fwd(q, k, v, H, D, mask)
    delta = torch.empty(1, H, L, device="cuda", dtype=torch.float32)
    _lib.call("owlk_attn_delta", _lib.ptr(o), _lib.ptr(do), o.stride(1), 1, L, H, D, _lib.ptr(delta), _lib.stream())
    ws = torch.empty(_lib.lib().owlk_attn_bwd_fused_ws_bytes(1, H, L, D), device="cuda", dtype=torch.uint8)
    var = K.fused_bwd_variant(D, mask)
    n4 = (256 << 20) // 16  # one 256 MiB bucket of float4
    src = torch.randn(n4 * 4, device="cuda")
    dst = torch.empty_like(src)
    NWG = 32
    stamps = torch.zeros(2 * NWG, dtype=torch.int64, device="cuda")
    marks = torch.zeros(4, dtype=torch.int64, device="cuda")
    side = torch.cuda.Stream()
    main_s = torch.cuda.current_stream()

    def fused():
        K.attn_bwd_fused(q, k, v, do, lse, delta, H, D, mask, dq, dk, dv, D ** -0.5, var, ws)

    def copy(stream):
        assert CO.coresid_copy(src.data_ptr(), dst.data_ptr(), n4, NWG, stamps.data_ptr(), stream.cuda_stream) == 0

    def now(i, stream):
        assert CO.coresid_now(marks[i:i + 1].data_ptr(), stream.cuda_stream) == 0

    fused()
    copy(main_s)
    torch.cuda.synchronize()
    out = {}
    for cus in [int(x) for x in os.environ.get("RESERVE", "0").split(",")]:
        _lib.call("owlk_set_cu_reserve", cus)  # the grid the all-reduce micro-step launches (grad_reducer.py)
        out[f"reserve_{cus}"] = probe(fused, copy, now, marks, stamps, NWG, side, main_s)
    _lib.call("owlk_set_cu_reserve", 0)
    print(json.dumps(out, indent=1))


def probe(fused, copy, now, marks, stamps, NWG, side, main_s):
    fused()
    torch.cuda.synchronize()
    res = {}
    # alone
    now(0, main_s); fused(); now(1, main_s); torch.cuda.synchronize()
    res["fused_alone_ms"] = (marks[1] - marks[0]).item() / 1e5
    now(0, main_s); copy(main_s); now(1, main_s); torch.cuda.synchronize()
    res["copy_alone_ms"] = (marks[1] - marks[0]).item() / 1e5
    # 1: the collective is launched while the fused kernel runs (its stream waits for the fused start)
    for rep in range(2):
        now(0, main_s)
        fused()
        now(1, main_s)
        time.sleep(0.01)  # the fused kernel (~73 ms) is running when the collective is enqueued
        with torch.cuda.stream(side):
            copy(side)
        torch.cuda.synchronize()
        m = marks.tolist()
        st = stamps.view(NWG, 2).tolist()
        first = min(a for a, _ in st)
        last = max(b for _, b in st)
        res[f"during_{rep}"] = {
            "fused_ms": (m[1] - m[0]) / 1e5,
            "copy_first_wg_start_after_fused_start_ms": (first - m[0]) / 1e5,
            "copy_last_wg_end_after_fused_end_ms": (last - m[1]) / 1e5,
            "copy_wgs_started_before_fused_end": sum(1 for a, _ in st if a < m[1]),
            "copy_wgs_ended_before_fused_end": sum(1 for _, b in st if b < m[1]),
            "copy_wg_end_ms_after_first_start": sorted(round((b - first) / 1e5, 2) for _, b in st),
        }
    # 2: the collective is in flight when the fused kernel is launched
    for rep in range(2):
        with torch.cuda.stream(side):
            now(2, side)
            copy(side)
            now(3, side)
        ev = torch.cuda.Event()
        ev.record(side)
        now(0, main_s)
        fused()
        now(1, main_s)
        torch.cuda.synchronize()
        m = marks.tolist()
        res[f"before_{rep}"] = {"fused_ms": (m[1] - m[0]) / 1e5, "copy_ms": (m[3] - m[2]) / 1e5,
                                "fused_start_after_copy_start_ms": (m[0] - m[2]) / 1e5,
                                "copy_end_after_fused_start_ms": (m[3] - m[0]) / 1e5}
    return res


if __name__ == "__main__":
    main()
