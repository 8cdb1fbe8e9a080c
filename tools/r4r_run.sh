# fused backward: fewer spilled lane constants in the sweep (pb) and + the next item claimed in the epilogue (pc) against HEAD (pa)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
for v in pb pc; do
OWLK_LIB=$L/libowlk_$v.so timeout -k 10 400 python -u -m pytest tests/test_attn_fused_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r4r_tests_$v.log 2>&1; rc=$?; echo "fused tests ($v) rc=$rc"; tail -2 gpurun_out/r4r_tests_$v.log
[ $rc -eq 0 ] || exit 1
done
rm -f gpurun_out/libs_*.log
FUSED_VARIANTS="5" bash tools/ab_libs.sh "pa pb pc" 3 --bwd-only --windows none,16,4 --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "window=\|fused" $f; done
