# end-to-end check with the single pass on every dit_v4 layer: GPU tests, smoke, bench, profile
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/round_check.sh r4m || exit 1
tail -3 gpurun_out/r4m_gputests.log; tail -1 gpurun_out/r4m_smoke.log; tail -1 gpurun_out/r4m_bench.log | cut -c1-300
grep -A 16 "per-kernel time in one micro-step" gpurun_out/r4m_bench.log
