# r6l: one-wave-per-SIMD step schedule A/B: prologue order (p1), 5-slot dQ ring (s5), ring DMA in M2_1 (dm)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; rm -f gpurun_out/libs_*.log
FUSED_VARIANTS=129 bash tools/ab_libs.sh "base p1 s5 p1s5 dm" 2 --bwd-only --windows none,16 --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "fused" $f | cut -c1-60; done | tee gpurun_out/r6l_ab.txt
