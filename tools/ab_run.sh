# A/B helper for gpurun: previous library (OWLK_LIB) vs the in-tree one, plus GEMM tile variants.
set -e
PREV=$PWD/owl-audio-exps_amd/owl_wms/_lib/libowlk_prev.so
OWLK_GEMM_BN=128 timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -m gpu -k "gemm" -x > gpurun_out/ab_gemmtest.log 2>&1
for i in 1 2; do
  OWLK_LIB=$PREV timeout -k 10 200 python tools/attn_bench.py --iters 3 > gpurun_out/ab_prev$i.log 2>&1
  timeout -k 10 200 python tools/attn_bench.py --iters 3 > gpurun_out/ab_new$i.log 2>&1
done
timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/gb256.log 2>&1
OWLK_GEMM_BN=128 timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/gb128.log 2>&1
