# HBM-bound fused passes: libowlk_prev.so (before) vs the tree's libowlk.so, interleaved; parity first
set -e
cd "$GRAFT_REPO_ROOT"
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -q -m gpu -x -k "adaln or gate or gamerft_loss" --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | tail -1
for i in 1 2; do
  echo "== prev $i"; OWLK_LIB=$L/libowlk_prev.so timeout -k 10 200 python tools/ew_bench.py
  echo "== new $i"; timeout -k 10 200 python tools/ew_bench.py
done
