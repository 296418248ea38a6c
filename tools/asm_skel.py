"""Memory-op / wait / branch skeleton of one kernel in a device .s file
(developer tool): python tools/asm_skel.py file.s kernel_substring"""
import re
import sys

lines = open(sys.argv[1]).read().splitlines()
pat = sys.argv[2]
starts = [i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and pat in l]
for st in starts:
    print("==", lines[st][:100])
    for l in lines[st + 1:]:
        t = l.strip()
        if t.startswith("s_endpgm"):
            print("ENDPGM")
            break
        if t.startswith(".LBB"):
            print(t.split()[0])
        elif any(k in t for k in ("_load", "s_waitcnt", "s_cbranch", "s_barrier", "_store", "s_branch", "scratch", "mfma", "ds_bpermute")):
            if "s_load" in t:
                continue
            print("   " + t[:72])
