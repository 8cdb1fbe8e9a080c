# fused backward: issue priority of the dQ waves (s_setprio 1 / 2 / 3) against equal (pr0)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -f gpurun_out/libs_*.log
FUSED_VARIANTS="5" bash tools/ab_libs.sh "pr0 pr1 pr2 pr3" 2 --bwd-only --windows 16,none --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "fused" $f | cut -c1-60; done > gpurun_out/r4ab_summary.txt; cat gpurun_out/r4ab_summary.txt
