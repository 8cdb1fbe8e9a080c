# HBM traffic of the bench's dominant kernel (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE
# in separate --pmc passes, only the kernel matching $KREGEX, on the bench command itself.
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
K=${KREGEX:-attn_bwd_dkdv}
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c --kernel-include-regex "$K" -f csv -d $R/gpurun_out/traffic -o $c \
    -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile > $R/gpurun_out/traffic_$c.log 2>&1
done
