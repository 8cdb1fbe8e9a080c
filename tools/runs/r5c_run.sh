# r5c: the one-wave-per-SIMD single pass (variant bit 7): parity (oracle + counting), then timing against the 8-wave form
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_attn_fused_gpu.py -x -q --timeout 200 --timeout-method thread \
  -k "133 or 135" > gpurun_out/r5c_tests.log 2>&1 || { tail -30 gpurun_out/r5c_tests.log; exit 1; }
tail -2 gpurun_out/r5c_tests.log
FUSED_VARIANTS="5,133" timeout -k 10 300 python -u tools/attn_bench.py --bwd-only --windows none,16 --iters 3 > gpurun_out/r5c_bench.log 2>&1 || exit 1
grep -E "window|fused" gpurun_out/r5c_bench.log
