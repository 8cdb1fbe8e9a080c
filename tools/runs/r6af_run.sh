# r6af: GEMM dispatch tests (split-256 weight-gradient plan, 216-tile ping-pong) and the graphed decode
# tests after the deferred graph release
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_epi_exact_gpu.py "tests/test_kernels_gpu.py::test_gemm_splitk_without_workspace" -x -v --timeout 200 --timeout-method thread > gpurun_out/r6af_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r6af_tests.log | tail -30; exit $rc
