# r5r: scheduler flags and the D = 128 attention kernels: a0 = no flags, a1 = flags on every file,
# a2 = flags on gemm.hip and attn_bwd_fused.hip only (production); D = 128 forward and dK/dV + dQ
# pair (dit_v4_5B shape), then the D = 64 single pass (dit_v4), interleaved
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; rm -f gpurun_out/libs_*.log
bash tools/ab_libs.sh "a0 a1 a2" 2 --dim 128 --heads 20 --windows none,16 --iters 2 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "  fwd \|dkdv\|  dq \|bwd pair" $f | cut -c1-60; done | tee gpurun_out/r5r_ab.txt
rm -f gpurun_out/libs_*.log
FUSED_VARIANTS="5" bash tools/ab_libs.sh "a0 a1 a2" 2 --windows none,16 --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "fused\|  fwd " $f | cut -c1-40; done | tee -a gpurun_out/r5r_ab.txt
