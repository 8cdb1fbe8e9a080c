# r6aq: the four modulation weight gradients as one [6d, d] GEMM: model tests, bench A/B (stack on / off)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_model_gpu.py > gpurun_out/r6aq_model_tests.log 2>&1 || exit 1
for i in 1 2; do
  OWL_MOD_STACK_GEMM=0 timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-traffic > gpurun_out/r6aq_off_$i.log 2>&1 || exit 1
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-traffic > gpurun_out/r6aq_on_$i.log 2>&1 || exit 1
done
