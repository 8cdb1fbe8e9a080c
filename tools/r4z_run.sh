# single-pass backward with packed documents: fused tests (incl. documents), every GPU test, the
# 4-documents dit_v4 bench with the single pass and with the two-kernel backward (OWLK_BWD_FUSED_DOCS=0)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_attn_fused_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r4z_fused_tests.log 2>&1; rc=$?; echo "fused tests rc=$rc"; tail -2 gpurun_out/r4z_fused_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4z_gputests.log 2>&1; rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/r4z_gputests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u bench.py --docs 4 --no-traffic --no-cpu-baseline > gpurun_out/r4z_docs_fused.log 2>&1 || exit 1
OWLK_BWD_FUSED_DOCS=0 timeout -k 10 400 python -u bench.py --docs 4 --no-traffic --no-cpu-baseline > gpurun_out/r4z_docs_pair.log 2>&1 || exit 1
for f in gpurun_out/r4z_docs_fused.log gpurun_out/r4z_docs_pair.log; do echo "== $f"; tail -1 $f | cut -c1-200; grep -A6 "per-kernel time" $f | grep attn; done
