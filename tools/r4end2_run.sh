# final round-4 library: mmdit_v2 bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u bench.py --config configs/mmdit_v2.yml --no-traffic --no-cpu-baseline > gpurun_out/r4end_mmdit.log 2>&1 || exit 1
tail -1 gpurun_out/r4end_mmdit.log | cut -c1-200
grep -A 6 "per-kernel time in one micro-step" gpurun_out/r4end_mmdit.log
