# r6n: fused-backward GPU tests (incl. the one-wave-per-SIMD variants), then a ring-DMA-first A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; rm -f gpurun_out/libs_*.log
timeout -k 10 900 python -u -m pytest tests/test_attn_fused_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6n_tests.log 2>&1 || exit 1
FUSED_VARIANTS=129 bash tools/ab_libs.sh "base e0 e1 nd nq" 2 --bwd-only --windows none,16 --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "fused" $f | cut -c1-60; done | tee gpurun_out/r6n_ab.txt
