# r6ak: how often the W4 backward's run finds the predecessor's flag down (stats build)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
FUSED_VARIANTS=129 OWLK_LIB=$L/libowlk_stats.so timeout -k 10 200 python -u tools/attn_bench.py --bwd-only --windows none,16,256 --iters 3 > gpurun_out/r6ak_stats.log 2>&1 || exit 1
FUSED_VARIANTS=1 OWLK_LIB=$L/libowlk_stats.so timeout -k 10 200 python -u tools/attn_bench.py --bwd-only --windows none --iters 3 >> gpurun_out/r6ak_stats.log 2>&1
