# Compile attn_bwd_fused.hip (working tree or a given file) with -save-temps and print the production
# instantiation's register / spill figures and the main loop's instruction mix.
#   tools/isa_fused_stats.sh [file.hip] [extra hipcc flags...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
SRC=${1:-$R/owl-audio-exps_amd/csrc/attn_bwd_fused.hip}; shift || true
W=$(mktemp -d /tmp/isafs.XXXX)
cp "$SRC" $W/attn_bwd_fused.hip; cp $R/owl-audio-exps_amd/csrc/*.hpp $W/
cd $W && /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$R/include -fno-slp-vectorize \
  -Wno-unused-function -Wno-unused-variable -Wno-unused-but-set-variable -Wno-inline-asm -save-temps -c attn_bwd_fused.hip -o x.o "$@" > build.log 2>&1 || { cat build.log; exit 1; }
python3 - "$W/attn_bwd_fused-hip-amdgcn-amd-amdhsa-gfx950.s" <<'PY'
import re, sys
from collections import Counter
s = open(sys.argv[1]).read()
name = '_ZN12_GLOBAL__N_116attn_bwd_fused_kILb1ELb0ELb0EEEvNS_6FusedPE'
m = re.search(r'^' + re.escape(name) + r':', s, re.M)
end = s.find('.Lfunc_end', m.end())
meta = s[s.find(name + '\n', end) if False else 0:]
lines = [l.strip() for l in s[m.end():end].split('\n')]
labels = {re.match(r'^(\.LBB\S+):', l).group(1): i for i, l in enumerate(lines) if re.match(r'^\.LBB\S+:', l)}
# the innermost loop containing the most MFMAs = the step loop
best = None
for i, l in enumerate(lines):
    mm = re.match(r'^s_c?branch\S*\s+(\.LBB\S+)', l)
    if mm and mm.group(1) in labels and labels[mm.group(1)] < i:
        a = labels[mm.group(1)]
        n = sum(1 for x in lines[a:i] if x.startswith('v_mfma'))
        if 70 <= n <= 90 and (best is None or i - a < best[1] - best[0]):
            best = (a, i)
c = Counter(x.split()[0] for x in lines[best[0]:best[1]] if x and not x.startswith((';', '.')))
tail = s[end:end + 4000]
g = lambda k: (re.search(k + r':\s*(\d+)', tail) or [None, '?'])[1]
i0 = s.find('.name:           ' + name)
md = s[i0:i0 + 1500]
sp = re.findall(r'\.sgpr_spill_count:\s*(\d+)', md)[:1] or ['?']
vs = re.findall(r'\.vgpr_spill_count:\s*(\d+)', md)[:1] or ['?']
valu = sum(v for k, v in c.items() if k.startswith('v_') and not k.startswith('v_mfma'))
print(f"sgpr={g('; TotalNumSgprs')} vgpr={g('; NumVgprs')} scratch={g('; ScratchSize')} sgpr_spill={sp[0]} vgpr_spill={vs[0]}")
print(f"loop[{best[1]-best[0]} lines]: valu={valu} readlane={c['v_readlane_b32']} writelane={c['v_writelane_b32']} "
      f"mov_b64={c['v_mov_b64_e32']} mov_b32={c['v_mov_b32_e32']} nop={c['s_nop']} salu={sum(v for k,v in c.items() if k.startswith('s_'))} "
      f"scratch={sum(v for k,v in c.items() if k.startswith('scratch_'))} mfma={sum(v for k,v in c.items() if k.startswith('v_mfma'))} "
      f"ds_read={sum(v for k,v in c.items() if k.startswith('ds_read'))} waitcnt={c['s_waitcnt']}")
PY
rm -rf $W
