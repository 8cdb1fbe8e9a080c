# windowed single-pass backward: tests, window 16 / 4 / global timing against the two-kernel pair
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_attn_fused_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r4l_tests.log 2>&1; rc=$?; echo "fused tests rc=$rc"; tail -3 gpurun_out/r4l_tests.log
[ $rc -eq 0 ] || exit 1
FUSED_VARIANTS="1,5" timeout -k 10 300 python -u tools/attn_bench.py --bwd-only --windows 16,4 --iters 5 > gpurun_out/r4l_ab.log 2>&1 || exit 1
grep "window=\|fused\|dkdv\|dq \|bwd pair" gpurun_out/r4l_ab.log
