# r6ai: full GPU suite after the long-window W4 default, then mmdit_v2 and docs-4 bench lines
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6ai_gputests.log 2>&1 || { tail -30 gpurun_out/r6ai_gputests.log; exit 1; }
tail -1 gpurun_out/r6ai_gputests.log
timeout -k 10 500 python -u bench.py --config configs/mmdit_v2.yml --steps 1 --warmup 1 --no-cpu-baseline --no-traffic > gpurun_out/r6ai_bench_mmdit_v2.log 2>&1 || exit 1
tail -1 gpurun_out/r6ai_bench_mmdit_v2.log | cut -c1-200
timeout -k 10 500 python -u bench.py --docs 4 --steps 1 --warmup 1 --no-cpu-baseline --no-traffic > gpurun_out/r6ai_bench_docs4.log 2>&1 || exit 1
tail -1 gpurun_out/r6ai_bench_docs4.log | cut -c1-200
