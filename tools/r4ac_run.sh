# GEMM epilogue without the strip lgkmcnt drains (g1) against with (g0): GEMM tests with g1, gemm_bench A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
OWLK_LIB=$L/libowlk_g1.so timeout -k 10 400 python -u -m pytest tests -m gpu -q -x -k "gemm or mlp or block or model" --timeout 120 --timeout-method thread > gpurun_out/r4ac_tests.log 2>&1; rc=$?; echo "tests (g1) rc=$rc"; tail -2 gpurun_out/r4ac_tests.log
[ $rc -eq 0 ] || exit 1
for i in 1 2; do for v in g0 g1; do
OWLK_LIB=$L/libowlk_$v.so timeout -k 10 200 python -u tools/gemm_bench.py > gpurun_out/r4ac_${v}_$i.log 2>&1 || exit 1
done; done
for f in gpurun_out/r4ac_g*_*.log; do echo "== $f"; cut -c1-50 $f; done > gpurun_out/r4ac_summary.txt; cat gpurun_out/r4ac_summary.txt
