# Decode (AVCachingSamplerV2, CFG as one B = 2 forward) wall time and rocprofv3 kernel stats.
#   bash tools/prof_decode.sh TAG
set -e
TAG=${1:-r}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out
timeout -k 10 300 python -u tools/decode_bench.py > $O/${TAG}_decode_bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${TAG}_dprof -o run -- python3 tools/decode_bench.py --frames 2 > $O/${TAG}_decode_prof.log 2>&1
python tools/rocpd_stats.py $O/${TAG}_dprof/run_results.db > $O/${TAG}_decode_kernel_stats.csv
rm -rf $O/${TAG}_dprof
