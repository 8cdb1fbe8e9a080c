# r6i: one-wave-per-SIMD step schedule A/B: hand-off check at M2_0 (c64) / M2_1 (c96) top, ring DMA spacing
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; rm -f gpurun_out/libs_*.log
FUSED_VARIANTS=129 bash tools/ab_libs.sh "c64 c96 c96d6" 2 --bwd-only --windows none,16 --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "fused" $f | cut -c1-60; done | tee gpurun_out/r6i_ab.txt
