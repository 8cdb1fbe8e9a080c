"""Launch the dit_v4 fc1 forward GEMM shape (98304 x 6144 x 1536, SiLU epilogue) a few times (PMC target)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "owl-audio-exps_amd")]
import torch  # noqa: E402

from owl_wms import kernels as K  # noqa: E402

M, N, Kd = 98304, 6144, 1536
torch.manual_seed(0)
a = torch.randn(M, Kd, device="cuda", dtype=torch.bfloat16)
w = torch.randn(N, Kd, device="cuda", dtype=torch.bfloat16) * 0.02
b = torch.zeros(N, device="cuda")
aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(3):
    K.gemm(a, w, bias=b, epi=K.EPI_SILU, aux=aux)
torch.cuda.synchronize()
