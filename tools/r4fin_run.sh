# final round-4 tree: GPU tests, smoke, bench (dit_v4, live traffic, cpu_baseline), rocprofv3 stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/round_check.sh r4fin || exit 1
tail -3 gpurun_out/r4fin_gputests.log; tail -1 gpurun_out/r4fin_smoke.log; tail -1 gpurun_out/r4fin_bench.log | cut -c1-300
grep -A 16 "per-kernel time in one micro-step" gpurun_out/r4fin_bench.log
