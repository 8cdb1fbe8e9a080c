"""Launch only the dit_v4 global-layer attention forward (for PMC profiling)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "owl-audio-exps_amd")]
import torch  # noqa: E402

from owl_wms import kernels as K  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "fwd"
H, D, tpf, nf = int(os.environ.get("HEADS", "24")), int(os.environ.get("DIM", "64")), 64, int(os.environ.get("FRAMES", "512"))
L = nf * tpf
torch.manual_seed(0)
qkv = torch.randn(1, L, 3 * H * D, device="cuda", dtype=torch.bfloat16)
qk = qkv[:, :, :2 * H * D].view(1, L, 2 * H, D)  # QK-RMSNorm'd, as in the model
qk.copy_((qk.float() * torch.rsqrt(qk.float().pow(2).mean(-1, keepdim=True))).bfloat16())
q, k, v = qkv[:, :, :H * D], qkv[:, :, H * D:2 * H * D], qkv[:, :, 2 * H * D:]
mask = K.FrameMask(tpf, int(os.environ["WINDOW"]) if os.environ.get("WINDOW") else None)
o, lse = K.attn_fwd(q, k, v, H, D, mask, score_bound=K.qk_norm_bound(D))
if which == "bwd":
    do = torch.randn_like(o)
    dq, dk, dv = (torch.empty_like(o) for _ in range(3))
    K.attn_bwd(q, k, v, o, do, lse, H, D, mask, dq, dk, dv)
torch.cuda.synchronize()
