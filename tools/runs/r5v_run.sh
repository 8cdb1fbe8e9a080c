# r5v: small per-frame GEMMs -- the modulation forward on the 256^2 kernel at >= 192 tiles and the cond
# gradient as one round of 256^2 split-K (k1, production) against the previous dispatch (k0): GEMM /
# block / model GPU tests of k1, then interleaved timing
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
OWLK_LIB=$L/libowlk_k1.so timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -k "gemm or cond or block or model or muon" --timeout 200 --timeout-method thread \
  > gpurun_out/r5v_tests.log 2>&1 || { tail -30 gpurun_out/r5v_tests.log; exit 1; }
tail -1 gpurun_out/r5v_tests.log
for i in 1 2; do for v in k0 k1; do
  echo "== $v $i"; OWLK_LIB=$L/libowlk_$v.so timeout -k 10 200 python -u tools/gemm_epi_bench.py 2>&1 | grep "modulation\|cond grad" || exit 1
done; done | tee gpurun_out/r5v_ab.txt
