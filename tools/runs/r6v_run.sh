# r6v: timing-only upper bounds inside the steady run (results wrong): no landing-zone wait (xp), no
# end-of-step vmcnt (xe), v_exp -> v_mov (xx), no ring DMA (nd)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; rm -f gpurun_out/libs_*.log
FUSED_VARIANTS=129 bash tools/ab_libs.sh "base xp xe xx nd" 2 --bwd-only --windows none --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "fused" $f | cut -c1-60; done | tee gpurun_out/r6v_ab.txt
