# r6ah: one-wave-per-SIMD backward vs the 8-wave kernel (both XCD-local) on mmdit_v2's long windows
# (tpf 65, window 256 frames = 16,640 keys) and window 16, 24 heads x 1000 frames
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
FUSED_VARIANTS=1,129 timeout -k 10 300 python -u tools/attn_bench.py --bwd-only --frames 1000 --tpf 65 --windows 256,64,16 --iters 3 > gpurun_out/r6ah_mmdit.log 2>&1 || exit 1
grep -E "window=|fused" gpurun_out/r6ah_mmdit.log | cut -c1-150
