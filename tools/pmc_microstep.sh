# HBM traffic (FETCH_SIZE, WRITE_SIZE in separate --pmc passes) of one kernel over one dit_v4 micro-step.
# Usage (on the box): bash tools/pmc_microstep.sh KERNEL_REGEX TAG
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
K=${1:-attn_bwd_dkdv_k}
TAG=${2:-pmc}
for c in FETCH_SIZE WRITE_SIZE; do
  echo "pass $c" >> $R/gpurun_out/${TAG}_pmc.log
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "$K" -f csv -d $R/gpurun_out/${TAG}_pmc -o $c \
    -- python3 $R/bench.py --microsteps 1 >> $R/gpurun_out/${TAG}_pmc.log 2>&1
done
