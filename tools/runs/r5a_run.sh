# r5a: the r4ac subset once with the production library (the rope-table fix), plus the new bound tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "gemm or mlp or block or model or bounded" > gpurun_out/r5a_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5a_tests.log; exit $rc
