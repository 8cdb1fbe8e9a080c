# Whole-step A/B of an env toggle on one box: GPU tests once, then interleaved bench.py runs.
#   bash tools/ab_bench_env.sh VAR VAL_A VAL_B [rounds]
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/abb_tests.log 2>&1
for i in $(seq 1 ${4:-2}); do
  env $1=$2 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/abb_A_$i.log 2>&1
  env $1=$3 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/abb_B_$i.log 2>&1
done
