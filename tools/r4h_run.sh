set -o pipefail
cd $GRAFT_REPO_ROOT
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
for v in m1 m2; do
  OWLK_LIB=$L/libowlk_$v.so timeout -k 10 300 python -u -m pytest tests/test_attn_fused_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r4h_tests_$v.log 2>&1; rc=$?; echo "tests $v rc=$rc"; tail -2 gpurun_out/r4h_tests_$v.log
  [ $rc -eq 0 ] || exit 1
done
rm -f gpurun_out/libs_*.log
bash tools/ab_libs.sh "m0 m1 m2" 2 --bwd-only --windows none --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "fused\|dkdv\|dq " $f; done
OWLK_LIB=$L/libowlk_m1pf.so timeout -k 10 200 python -u tools/attn_bench.py --bwd-only --windows none --iters 2 > gpurun_out/r4h_prof.log 2>&1 || exit 1
grep "fused" gpurun_out/r4h_prof.log
