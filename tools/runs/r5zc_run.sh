# r5zc: attention forward FULL tiles software-pipelined over 32-key parts (OWLK_FWD_PIPE, v1) vs HEAD (v0):
# D = 64 global + window 16 (v1 with 64-key tiles: OWLK_FWD_KT128=0), D = 128 global (v1 with 32-query
# waves: OWLK_FWD_NQ3=0), interleaved x3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; L=$PWD/owl-audio-exps_amd/owl_wms/_lib
for i in 1 2 3; do
  echo "== v0 $i"; OWLK_LIB=$L/libowlk_v0.so timeout -k 10 200 python -u tools/attn_bench.py --fwd-only --windows none,16 --iters 3 2>&1 | grep "  fwd " | cut -c1-40 || exit 1
  echo "== v1 kt64 $i"; OWLK_FWD_KT128=0 OWLK_LIB=$L/libowlk_v1.so timeout -k 10 200 python -u tools/attn_bench.py --fwd-only --windows none,16 --iters 3 2>&1 | grep "  fwd " | cut -c1-40 || exit 1
  echo "== v0 d128 $i"; OWLK_LIB=$L/libowlk_v0.so timeout -k 10 200 python -u tools/attn_bench.py --fwd-only --dim 128 --heads 20 --windows none --iters 3 2>&1 | grep "  fwd " | cut -c1-40 || exit 1
  echo "== v1 d128 nq2 $i"; OWLK_FWD_NQ3=0 OWLK_LIB=$L/libowlk_v1.so timeout -k 10 200 python -u tools/attn_bench.py --fwd-only --dim 128 --heads 20 --windows none --iters 3 2>&1 | grep "  fwd " | cut -c1-40 || exit 1
done | tee gpurun_out/r5zc_ab.txt
