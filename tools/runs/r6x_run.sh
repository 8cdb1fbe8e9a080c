# r6x: timing-only: ring DMA from a fixed (cache-resident) tile every step (dc) vs none (nd) vs base
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; rm -f gpurun_out/libs_*.log
FUSED_VARIANTS=129 bash tools/ab_libs.sh "base dc nd" 2 --bwd-only --windows none --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "fused" $f | cut -c1-60; done | tee gpurun_out/r6x_ab.txt
