# Other BASELINE configs through bench.py (1 timed step, 1 warm-up; no CPU baseline / PMC passes)
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r}
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -q -m gpu -x -k "stacked_modulation" --timeout 120 --timeout-method thread > gpurun_out/${TAG}_modtest.log 2>&1
timeout -k 10 500 python -u bench.py --config configs/mmdit_v2.yml --steps 1 --warmup 1 --no-cpu-baseline --no-traffic > gpurun_out/${TAG}_bench_mmdit_v2.log 2>&1
timeout -k 10 700 python -u bench.py --config configs/dit_v4_5B.yml --steps 1 --warmup 1 --no-cpu-baseline --no-traffic > gpurun_out/${TAG}_bench_dit_v4_5B.log 2>&1
