"""torch.matmul (hipBLASLt) at the dit_v4 forward shapes, for a rocprofv3 kernel trace of the
library's kernel names (their Tensile parameters: macro tile, depth, store remap, ...)."""
import torch

T, d = 98304, 1536
r = lambda *s: (torch.randn(*s, device="cuda") * 0.5).to(torch.bfloat16)
x, w1, w2, wo = r(T, d), r(4 * d, d), r(d, 4 * d), r(d, d)
h = r(T, 4 * d)
for _ in range(3):
    torch.matmul(x, w1.T)
    torch.matmul(h, w2.T)
    torch.matmul(x, wo.T)
torch.cuda.synchronize()
