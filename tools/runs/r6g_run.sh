# r6g: phase profile of the one-wave-per-SIMD single pass with in-statement stamps (timing-only build)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OWLK_LIB=$PWD/owl-audio-exps_amd/owl_wms/_lib/libowlk_prof.so FUSED_VARIANTS=129 timeout -k 10 200 python -u tools/attn_bench.py --bwd-only --windows none,16 --iters 2 > gpurun_out/r6g_prof.log 2>&1
