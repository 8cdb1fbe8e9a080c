# attention A/B: parity tests on the in-tree lib, then interleaved timing of prev / new / w2
set -e
cd "$GRAFT_REPO_ROOT"
L=owl-audio-exps_amd/owl_wms/_lib
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "attn or attention" --timeout 120 --timeout-method thread > gpurun_out/a3_test.log 2>&1
OWLK_LIB=$PWD/$L/libowlk_w2.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "attn or attention" --timeout 120 --timeout-method thread > gpurun_out/a3_test_w2.log 2>&1
for i in 1 2; do
  for v in prev new w2; do
    case $v in prev) LIB=$PWD/$L/libowlk_prev.so;; new) LIB=$PWD/$L/libowlk.so;; w2) LIB=$PWD/$L/libowlk_w2.so;; esac
    OWLK_LIB=$LIB timeout -k 10 200 python tools/attn_bench.py --iters 3 > gpurun_out/a3_${v}_$i.log 2>&1
  done
done
