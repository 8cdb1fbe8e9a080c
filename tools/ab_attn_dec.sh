set -e
cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
OWLK_FWD_SPLIT=0 timeout -k 10 120 python tools/attn_decode_bench.py > gpurun_out/ad_old_$i.log 2>&1
timeout -k 10 120 python tools/attn_decode_bench.py > gpurun_out/ad_new_$i.log 2>&1
done
