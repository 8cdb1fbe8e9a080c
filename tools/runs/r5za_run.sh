# r5za: GEMM GPU tests after the K <= 4096 grouping rule, then the dit_v4_5B bench (1 timed step)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5za_tests.log 2>&1 && tail -2 gpurun_out/r5za_tests.log &&
timeout -k 10 600 python -u bench.py --config configs/dit_v4_5B.yml --steps 1 --warmup 1 --no-cpu-baseline --no-traffic > gpurun_out/r5za_bench_5B.log 2>&1 && tail -1 gpurun_out/r5za_bench_5B.log | cut -c1-300
