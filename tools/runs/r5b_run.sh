# r5b: the whole GPU suite with the rope-table bounds, the hand-off timeout poisoning and the drain check
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/r5b_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5b_tests.log; exit $rc
