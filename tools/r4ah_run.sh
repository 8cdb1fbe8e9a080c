# the production library with the dQ reads three k-steps ahead: every GPU test and smoke, once
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4ah_gputests.log 2>&1; rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/r4ah_gputests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4ah_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r4ah_smoke.log
