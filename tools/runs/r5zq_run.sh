# r5zq: single pass with static issue priority: pr1 / pr2 = s_setprio 1 / 2 on the dQ waves (each
# step's critical path), prm1 = s_setprio 1 on the other waves; pr0 production; interleaved x3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; rm -f gpurun_out/libs_*.log
FUSED_VARIANTS=1 bash tools/ab_libs.sh "pr0 pr1 pr2 prm1" 3 --bwd-only --windows none,16 --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "fused" $f | cut -c1-40; done | tee gpurun_out/r5zq_ab.txt
rm -f gpurun_out/libs_*.log
