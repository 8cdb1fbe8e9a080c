# r5ze: GEMM epilogue inputs of strips 0-3 by LDS-DMA during the last K step (OWLK_GEMM_XPF) + the dSiLU
# epilogue without the activation output when none is asked for; v1 = new, v0 = HEAD: kernel GPU tests
# (v1), bit-exact epilogue outputs v1 vs v0, then interleaved timing at d 1536 and 2560
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out /tmp/r5ze
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5ze_tests.log 2>&1 && tail -1 gpurun_out/r5ze_tests.log || exit 1
for v in v0 v1; do
  OWLK_LIB=$L/libowlk_$v.so timeout -k 10 300 python -u tools/gemm_epi_bench.py --save /tmp/r5ze/$v.pt --iters 3 > gpurun_out/r5ze_save_$v.log 2>&1 || { tail -20 gpurun_out/r5ze_save_$v.log; exit 1; }
done
python tools/gemm_epi_bench.py --compare /tmp/r5ze/v0.pt /tmp/r5ze/v1.pt | tee gpurun_out/r5ze_compare.txt
for i in 1 2 3; do for v in v0 v1; do for d in 1536 2560; do
  echo "== $v d$d $i"; OWLK_LIB=$L/libowlk_$v.so timeout -k 10 300 python -u tools/gemm_epi_bench.py --d $d 2>&1 | grep "TF/s" || exit 1
done; done; done | tee gpurun_out/r5ze_ab.txt
