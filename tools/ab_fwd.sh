# attention A/B: in-tree lib vs libowlk_prev.so; attention parity tests first, then interleaved
# attn_bench rounds (args: extra attn_bench flags)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out; L=$PWD/owl-audio-exps_amd/owl_wms/_lib
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -m gpu -x --timeout 120 --timeout-method thread -k "attention" > $O/ab_tests.log 2>&1
for i in 1 2; do
  OWLK_LIB=$L/libowlk_prev.so timeout -k 10 200 python -u tools/attn_bench.py --iters 5 --windows none,16 "$@" > $O/ab_prev_$i.log 2>&1
  timeout -k 10 200 python -u tools/attn_bench.py --iters 5 --windows none,16 "$@" > $O/ab_new_$i.log 2>&1
done
