# Build libowlk variants of the one-wave-per-SIMD step schedule (tools/gen_fused4_asm.py knobs).
#   bash tools/build_f4_variants.sh NAME "F4_CHECK=64 F4_DMA0=3" [NAME "ENV..."]...
# -> owl-audio-exps_amd/owl_wms/_lib/libowlk_NAME.so; the tree's .inc is regenerated with defaults after.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
while [ $# -ge 2 ]; do
  env $2 python3 $R/tools/gen_fused4_asm.py 2>/dev/null
  bash $R/tools/build_variant.sh $R/owl-audio-exps_amd/owl_wms/_lib/libowlk_$1.so - ${EXTRA:-} | tail -1
  shift 2
done
python3 $R/tools/gen_fused4_asm.py 2>/dev/null
