# round check with the next item claimed during the epilogue: GPU tests, smoke, bench, profile
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/round_check.sh r4t || exit 1
tail -3 gpurun_out/r4t_gputests.log; tail -1 gpurun_out/r4t_smoke.log; tail -1 gpurun_out/r4t_bench.log | cut -c1-300
grep -A 16 "per-kernel time in one micro-step" gpurun_out/r4t_bench.log
