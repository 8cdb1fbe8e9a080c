# r5z: tile-row grouping (OWLK_GEMM_GROUP) at the dit_v4_5B shapes (d = 2,560, K = 2,560 / 10,240):
# the automatic rule (4 for K <= 2,048, else none) against 4 and 8, interleaved x2
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2; do for gr in auto 4 8; do
  echo "== group $gr $i"
  if [ $gr = auto ]; then timeout -k 10 300 python -u tools/gemm_epi_bench.py --d 2560 2>&1 | grep "TF/s" || exit 1
  else OWLK_GEMM_GROUP=$gr timeout -k 10 300 python -u tools/gemm_epi_bench.py --d 2560 2>&1 | grep "TF/s" || exit 1; fi
done; done | tee gpurun_out/r5z_ab.txt
