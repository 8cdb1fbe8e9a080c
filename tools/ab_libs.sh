# A/B of prebuilt library variants (libowlk_v*.so) on attn_bench: interleaved rounds.
#   bash tools/ab_libs.sh "v0 v1 ..." [rounds] [attn_bench args...]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out; L=$PWD/owl-audio-exps_amd/owl_wms/_lib
VARS=$1; R=${2:-2}; shift 2
for i in $(seq 1 $R); do
  for v in $VARS; do
    OWLK_LIB=$L/libowlk_$v.so timeout -k 10 200 python -u tools/attn_bench.py "$@" > $O/libs_${v}_$i.log 2>&1
  done
done
