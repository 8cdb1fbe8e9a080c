# r5u: AdaLN forward with 1 / 2 / 4 rows per wave (r1 = the previous kernel): adaln parity tests of
# r2 and r4, then tools/ew_bench.py interleaved x3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
for v in r2 r4; do
  OWLK_LIB=$L/libowlk_$v.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "adaln" --timeout 120 --timeout-method thread \
    > gpurun_out/r5u_tests_$v.log 2>&1 || { tail -20 gpurun_out/r5u_tests_$v.log; exit 1; }
  tail -1 gpurun_out/r5u_tests_$v.log
done
for i in 1 2 3; do for v in r1 r2 r4; do
  echo "== $v $i"; OWLK_LIB=$L/libowlk_$v.so timeout -k 10 200 python -u tools/ew_bench.py 2>&1 | grep "adaln_fwd" || exit 1
done; done | tee gpurun_out/r5u_ab.txt
# the per-frame modulation GEMM on the 256^2 kernel (production, 216 tiles >= 192) vs 128^2 (OWLK_GEMM_MIN256=256)
for i in 1 2; do for m in 192 256; do
  echo "== min256 $m $i"; OWLK_GEMM_MIN256=$m timeout -k 10 200 python -u tools/gemm_epi_bench.py 2>&1 | grep "modulation" || exit 1
done; done | tee -a gpurun_out/r5u_ab.txt
