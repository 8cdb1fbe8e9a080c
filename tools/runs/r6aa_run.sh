# r6aa: timing-only upper bounds of the one-wave-per-SIMD forward: no ring DMA (fnd), v_exp -> v_mov (fxe)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; rm -f gpurun_out/libs_*.log
bash tools/ab_libs.sh "base fnd fxe" 2 --fwd-only --windows none --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "fwd " $f | cut -c1-60; done | tee gpurun_out/r6aa_ab.txt
