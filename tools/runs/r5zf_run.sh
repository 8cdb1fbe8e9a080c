# r5zf: PMC of the 256^2 ping-pong GEMM at the dit_v4 shapes (tools/gemm_bench.py: forward, dX, dW and
# fused-epilogue forms; three passes of SQ counters), to compare the weight-gradient (both operands
# transposed) main loop with the dX / forward ones
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PROG=gemm_bench.py WHICH=--wgrad-only bash tools/pmc_attn.sh || exit 1
python tools/pmc_csv.py "gpurun_out/pmc_--wgrad-only" > gpurun_out/r5zf_pmc_wgrad.txt
cat > /tmp/dx.py <<'PY'
import os, sys
R = os.environ["GRAFT_REPO_ROOT"]; sys.path[:0] = [R, R + "/owl-audio-exps_amd"]
import torch
from owl_wms import kernels as K
T, d = 98304, 1536
r = lambda *s: (torch.randn(*s, device="cuda") * 0.5).to(torch.bfloat16)
a, w2, w1 = r(T, d), r(d, 4 * d), r(4 * d, d)
for _ in range(3):
    K.gemm(a, w2, b_trans=True)   # fc2 dX plain [98304 x 6144 x 1536], B transposed
    K.gemm(a, w1)                 # fc1 forward plain [98304 x 6144 x 1536]
torch.cuda.synchronize()
PY
cp /tmp/dx.py tools/_dx_pmc.py
PROG=_dx_pmc.py WHICH=x bash tools/pmc_attn.sh || exit 1
python tools/pmc_csv.py gpurun_out/pmc_x > gpurun_out/r5zf_pmc_dx.txt
rm -f tools/_dx_pmc.py
cat gpurun_out/r5zf_pmc_wgrad.txt gpurun_out/r5zf_pmc_dx.txt
