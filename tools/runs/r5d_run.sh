# r5d: ring DMA by waves 4-7 (d1) vs all 8 waves (d0): fused parity tests with d1, then interleaved A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; rm -f gpurun_out/libs_*.log
timeout -k 10 400 python -u -m pytest tests/test_attn_fused_gpu.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r5d_tests.log 2>&1 || { tail -30 gpurun_out/r5d_tests.log; exit 1; }
tail -2 gpurun_out/r5d_tests.log
FUSED_VARIANTS="5" bash tools/ab_libs.sh "d0 d1" 2 --bwd-only --windows none,16,4 --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "fused" $f | cut -c1-40; done | tee gpurun_out/r5d_ab.txt
