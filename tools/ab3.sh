# three-way A/B: libowlk_prev.so / in-tree libowlk.so / libowlk_w2.so, interleaved rounds of a tool
#   bash tools/ab3.sh "pytest-k-expr" tool.py [rounds]
set -e
cd "$GRAFT_REPO_ROOT"
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "$1" --timeout 120 --timeout-method thread > gpurun_out/ab3_test.log 2>&1
OWLK_LIB=$L/libowlk_w2.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "$1" --timeout 120 --timeout-method thread > gpurun_out/ab3_test_w2.log 2>&1
for i in $(seq 1 ${3:-2}); do
  OWLK_LIB=$L/libowlk_prev.so timeout -k 10 200 python tools/$2 > gpurun_out/ab3_prev_$i.log 2>&1
  timeout -k 10 200 python tools/$2 > gpurun_out/ab3_new_$i.log 2>&1
  OWLK_LIB=$L/libowlk_w2.so timeout -k 10 200 python tools/$2 > gpurun_out/ab3_w2_$i.log 2>&1
done
