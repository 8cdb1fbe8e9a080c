# r5t: scheduler options on the HBM-bound passes (e0 production, e1 trackers + max-ilp, e2 trackers;
# each on every file): tools/ew_bench.py, interleaved x3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
for i in 1 2 3; do for v in e0 e1 e2; do
  echo "== $v $i"; OWLK_LIB=$L/libowlk_$v.so timeout -k 10 200 python -u tools/ew_bench.py 2>&1 | grep "TB/s" || exit 1
done; done | tee gpurun_out/r5t_ab.txt
