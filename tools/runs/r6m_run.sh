# r6m: ring DMA placement A/B: M1_0 (base), M1_1 (d34), M2_0 (d66), late M1_0 (d18)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; rm -f gpurun_out/libs_*.log
FUSED_VARIANTS=129 bash tools/ab_libs.sh "base d34 d66 d18" 2 --bwd-only --windows none,16 --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "fused" $f | cut -c1-60; done | tee gpurun_out/r6m_ab.txt
