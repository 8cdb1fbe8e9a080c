# Interleaved A/B of libowlk variants (abvar/*.so) on the attention kernels at the dit_v4 shape.
#   bash tools/r3_ab_lib.sh TAG "lib1 lib2 ..." [attn_bench args]   (parity tests first with each variant)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out
TAG=$1; LIBS=$2; shift 2
for L in $LIBS; do
  OWLK_LIB=$PWD/abvar/$L.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -m gpu -x --timeout 120 --timeout-method thread -k "attention" > $O/${TAG}_tests_$L.log 2>&1
  echo "$L tests: $(tail -1 $O/${TAG}_tests_$L.log)"
done
for r in 1 2; do
  for L in $LIBS; do
    echo "== $L round $r"
    OWLK_LIB=$PWD/abvar/$L.so timeout -k 10 300 python -u tools/attn_bench.py "$@" 2>&1 | grep -E "window|dkdv|dq |fwd "
  done
done
