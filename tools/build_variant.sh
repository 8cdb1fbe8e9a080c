# Build an A/B variant of libowlk.so outside the tree's build/ dir.
#   tools/build_variant.sh OUT.so [git-rev|-] [extra hipcc flags...]
# git-rev: build that commit's csrc (e.g. HEAD for "previous"); "-" = the working tree.
# DEVFLAGS (env, may be empty) replaces the Makefile's device-only scheduler flags.
set -e
OUT=$(realpath -m "$1"); REV=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
W=$(mktemp -d /tmp/owlk_var.XXXX)
if [ "$REV" = "-" ]; then mkdir -p "$W/x"; cp -r "$R/owl-audio-exps_amd/csrc" "$W/x/"; cp -r "$R/include" "$W/";
else git -C "$R" archive "$REV" owl-audio-exps_amd/csrc include | tar -x -C "$W"; mkdir -p "$W/x"; mv "$W/owl-audio-exps_amd/csrc" "$W/x/"; fi
rm -rf "$W/x/csrc/build"
make -s -C "$W/x/csrc" -j8 OUT="$OUT" ${DEVFLAGS+DEVFLAGS="$DEVFLAGS"} CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -Wno-unused-function -Wno-unused-variable -Wno-unused-but-set-variable $*" 2>&1 | grep -E "error" || true
rm -rf "$W"
ls -la "$OUT"
