set -e
cd "$GRAFT_REPO_ROOT"
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "adaln" --timeout 120 --timeout-method thread > gpurun_out/ew_test.log 2>&1
for i in 1 2; do
  OWLK_LIB=$L/libowlk_prev.so timeout -k 10 200 python tools/ew_bench.py > gpurun_out/ew_prev_$i.log 2>&1
  timeout -k 10 200 python tools/ew_bench.py > gpurun_out/ew_new_$i.log 2>&1
done
