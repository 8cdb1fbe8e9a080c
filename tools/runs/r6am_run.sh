# r6am: fused AdaLN + gate backward: parity, micro timing, model tests
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "adaln or gate" > gpurun_out/r6am_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/adaln_gate_bench.py > gpurun_out/r6am_micro.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_model_gpu.py > gpurun_out/r6am_model_tests.log 2>&1
