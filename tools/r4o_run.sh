# mmdit_v2 with / without the single-pass backward (its windows: 16 and 256 frames, tpf 65), and the
# dit_v4_5B line of round 4 (D = 128: two-kernel backward)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 500 python -u bench.py --config configs/mmdit_v2.yml --no-traffic --no-cpu-baseline > $O/r4o_mmdit_fused.log 2>&1 || exit 1
tail -1 $O/r4o_mmdit_fused.log | cut -c1-200
OWLK_BWD_FUSED=0 timeout -k 10 500 python -u bench.py --config configs/mmdit_v2.yml --no-traffic --no-cpu-baseline > $O/r4o_mmdit_pair.log 2>&1 || exit 1
tail -1 $O/r4o_mmdit_pair.log | cut -c1-200
grep -A 12 "per-kernel time in one micro-step" $O/r4o_mmdit_fused.log
grep -A 12 "per-kernel time in one micro-step" $O/r4o_mmdit_pair.log
timeout -k 10 600 python -u bench.py --config configs/dit_v4_5B.yml --no-traffic --no-cpu-baseline > $O/r4o_5b.log 2>&1 || exit 1
tail -1 $O/r4o_5b.log | cut -c1-200
