set -e
OWLK_GEMM_HALFK=1 timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "gemm" > gpurun_out/ab_gemmtest.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/gb_base$i.log 2>&1
  OWLK_GEMM_HALFK=1 timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/gb_half$i.log 2>&1
done
