"""Per-kernel ISA summary of a hipcc -save-temps .s file: VGPR/AGPR/scratch and instruction counts.

    python tools/isa_summary.py file.s [name-substring]
"""
import re
import sys


def main(path, pat=""):
    s = open(path).read()
    for m in re.finditer(r"^(_Z\S+):\s*;\s*@", s, re.M):
        name = m.group(1)
        if pat not in name:
            continue
        end = s.find(".Lfunc_end", m.end())
        body = s[m.end():end]
        V0 = r"vmcnt\(0\)"

        def cnt(r):
            return len(re.findall(r, body))
        vg = re.search(r"; NumVgprs: (\d+)", s[end:end + 3000])
        ag = re.search(r"; NumAgprs: (\d+)", s[end:end + 3000])
        sc = re.search(r"; ScratchSize: (\d+)", s[end:end + 3000])
        occ = re.search(r"; Occupancy: (\d+)", s[end:end + 3000])
        print(f"{name[:90]}\n   vgpr={vg and vg.group(1)} agpr={ag and ag.group(1)} scratch={sc and sc.group(1)} "
              f"occ={occ and occ.group(1)} mfma={cnt(r'v_mfma')} ds_read={cnt(r'ds_read')} glds={cnt(r'global_load_lds')} "
              f"vmcnt={cnt(r'vmcnt')} vmcnt0={cnt(V0)} barrier={cnt(r's_barrier')} scratch_ops={cnt(r'scratch_')}")


if __name__ == "__main__":
    main(*sys.argv[1:])
