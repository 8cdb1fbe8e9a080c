# r5zh: GEMM ping-pong A-tile LDS-DMA placement: v0 HEAD (both 128-row halves of the next K step's A in
# phase 0, beside 12 fragment reads), v1 one half in phase 0 and one in phase 1, v2 both in phase 1;
# bit-exact epilogue outputs, then interleaved timing x3 at d 1536 and the dW shapes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out /tmp/r5zh
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
for v in v0 v1 v2; do
  OWLK_LIB=$L/libowlk_$v.so timeout -k 10 300 python -u tools/gemm_epi_bench.py --save /tmp/r5zh/$v.pt --iters 3 > gpurun_out/r5zh_save_$v.log 2>&1 || { tail -20 gpurun_out/r5zh_save_$v.log; exit 1; }
done
{ python tools/gemm_epi_bench.py --compare /tmp/r5zh/v0.pt /tmp/r5zh/v1.pt | tail -1; python tools/gemm_epi_bench.py --compare /tmp/r5zh/v0.pt /tmp/r5zh/v2.pt | tail -1; } | tee gpurun_out/r5zh_compare.txt
for i in 1 2 3; do for v in v0 v1 v2; do
  echo "== $v $i"; OWLK_LIB=$L/libowlk_$v.so timeout -k 10 300 python -u tools/gemm_epi_bench.py 2>&1 | grep "TF/s" || exit 1
  OWLK_LIB=$L/libowlk_$v.so timeout -k 10 300 python -u tools/gemm_bench.py --wgrad-only 2>&1 | grep "TF/s" || exit 1
done; done | tee gpurun_out/r5zh_ab.txt
