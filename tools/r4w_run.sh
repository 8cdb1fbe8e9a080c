# forward: D = 64 output rows stored whole through LDS (f1) against lane pieces (f0); attention tests with f1
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
OWLK_LIB=$L/libowlk_f1.so timeout -k 10 500 python -u -m pytest tests -m gpu -q -x -k "attn or sampler or decode" --timeout 120 --timeout-method thread > gpurun_out/r4w_tests.log 2>&1; rc=$?; echo "attention tests (f1) rc=$rc"; tail -2 gpurun_out/r4w_tests.log
[ $rc -eq 0 ] || exit 1
rm -f gpurun_out/libs_*.log
bash tools/ab_libs.sh "f0 f1" 3 --fwd-only --windows 16,4,none --iters 5 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "fwd" $f | cut -c1-70; done > gpurun_out/r4w_summary.txt
cat gpurun_out/r4w_summary.txt
