# final round-4 library: smoke, bench (dit_v4, live traffic, cpu_baseline), rocprofv3 stats (tests: r4ah)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/round_check.sh r4end skip-tests || exit 1
tail -1 gpurun_out/r4end_smoke.log; tail -1 gpurun_out/r4end_bench.log | cut -c1-300
grep -A 16 "per-kernel time in one micro-step" gpurun_out/r4end_bench.log
