# A/B of an env toggle on one library: tests with the toggle at its default, then interleaved timing.
#   bash tools/ab_env.sh "pytest-k-expr" tool.py VAR VAL_A VAL_B [rounds]
set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "$1" --timeout 120 --timeout-method thread > gpurun_out/abe_test.log 2>&1
for i in $(seq 1 ${6:-2}); do
  env $3=$4 timeout -k 10 200 python tools/$2 > gpurun_out/abe_A_$i.log 2>&1
  env $3=$5 timeout -k 10 200 python tools/$2 > gpurun_out/abe_B_$i.log 2>&1
done
