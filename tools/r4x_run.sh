# round check with dK / dV and forward O rows stored whole through LDS: GPU tests, smoke, bench, profile
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/round_check.sh r4x || exit 1
tail -3 gpurun_out/r4x_gputests.log; tail -1 gpurun_out/r4x_smoke.log; tail -1 gpurun_out/r4x_bench.log | cut -c1-300
grep -A 16 "per-kernel time in one micro-step" gpurun_out/r4x_bench.log
