# Generic A/B: in-tree lib vs libowlk_prev.so on a tool script, interleaved rounds.
#   bash tools/ab_lib.sh "pytest-k-expr" tool.py [rounds]
set -e
cd "$GRAFT_REPO_ROOT"
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "$1" --timeout 120 --timeout-method thread > gpurun_out/ab_test.log 2>&1
for i in $(seq 1 ${3:-2}); do
  OWLK_LIB=$L/libowlk_prev.so timeout -k 10 200 python tools/$2 > gpurun_out/ab_prev_$i.log 2>&1
  timeout -k 10 200 python tools/$2 > gpurun_out/ab_new_$i.log 2>&1
done
