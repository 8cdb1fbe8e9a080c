# rocprofv3 kernel-trace stats of the N=1 bench, then the HBM-traffic PMC passes (tools/pmc_traffic.sh).
#   bash tools/prof_only.sh TAG
set -e
TAG=${1:-r}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/${TAG}_prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/${TAG}_profbench.log 2>&1
python tools/rocpd_stats.py $O/${TAG}_prof/run_results.db > $O/${TAG}_kernel_stats.csv
bash tools/pmc_traffic.sh
