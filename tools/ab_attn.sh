set -e
PREV=$PWD/owl-audio-exps_amd/owl_wms/_lib/libowlk_prev.so
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -q -m gpu -x > gpurun_out/kt.log 2>&1
for i in 1 2; do
  OWLK_LIB=$PREV timeout -k 10 200 python tools/attn_bench.py --iters 3 > gpurun_out/ab_prev$i.log 2>&1
  timeout -k 10 200 python tools/attn_bench.py --iters 3 > gpurun_out/ab_new$i.log 2>&1
done
