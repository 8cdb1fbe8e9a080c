# One GPU call: GPU parity tests, smoke, bench (N=1 defaults, live PMC traffic), rocprofv3 kernel-trace
# stats of the bench.  Usage (on the box):  bash tools/round_check.sh TAG [skip-tests]
set -e
TAG=${1:-r}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/${TAG}_gputests.log 2>&1
fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1
timeout -k 10 600 python -u bench.py > $O/${TAG}_bench.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/${TAG}_prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-traffic > $O/${TAG}_profbench.log 2>&1
# rocprofv3 writes a rocpd database on this image: summarise it like --stats' kernel_stats.csv
python tools/rocpd_stats.py $O/${TAG}_prof/run_results.db > $O/${TAG}_kernel_stats.csv
