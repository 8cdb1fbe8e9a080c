# Same-box A/B of the GEMM tile-row grouping (OWLK_GEMM_GROUP) at the dit_v4 shapes: interleaved rounds.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out
for i in 1 2; do
  for g in auto 0 2 4 8 16; do
    if [ $g = auto ]; then unset OWLK_GEMM_GROUP; else export OWLK_GEMM_GROUP=$g; fi
    echo "== group $g round $i" >> $O/r3_group_ab.log
    timeout -k 10 240 python -u tools/gemm_bench.py >> $O/r3_group_ab.log 2>&1
  done
done
