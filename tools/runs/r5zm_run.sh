# r5zm: single-pass backward, per-phase shader-clock shares (OWLK_FUSED_PROF build p1) and the share of
# hand-offs that found the predecessor's flag down at mid-step (OWLK_FUSED_STATS build s1), production
# kernel otherwise; global and window-16 layers, XCD-local form
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
for v in p1 s1; do
  echo "== $v"; FUSED_VARIANTS=1 OWLK_LIB=$L/libowlk_$v.so timeout -k 10 200 python -u tools/attn_bench.py --bwd-only --windows none,16 --iters 2 2>&1 | grep "fused\|window\|frames" | cut -c1-260 || exit 1
done | tee gpurun_out/r5zm_phases.txt
