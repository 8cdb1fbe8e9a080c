# fused backward: waves without dQ work store their dK / dV during the dQ epilogue (pe) against after it (pa)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
OWLK_LIB=$L/libowlk_pe.so timeout -k 10 400 python -u -m pytest tests/test_attn_fused_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r4aa_tests.log 2>&1; rc=$?; echo "fused tests (pe) rc=$rc"; tail -2 gpurun_out/r4aa_tests.log
[ $rc -eq 0 ] || exit 1
rm -f gpurun_out/libs_*.log
FUSED_VARIANTS="5" bash tools/ab_libs.sh "pa pe" 3 --bwd-only --windows 16,4,none --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "fused" $f | cut -c1-60; done > gpurun_out/r4aa_summary.txt; cat gpurun_out/r4aa_summary.txt
