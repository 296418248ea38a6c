"""Per-kernel, per-grid median durations from a rocprofv3 kernel trace (prof_mb.sh output)."""
import collections
import csv
import glob
import sys

for tag in sys.argv[1:]:
    print("==", tag)
    f = glob.glob(f"gpurun_out/prof_mb_{tag}/**/*kernel_trace.csv", recursive=True)[0]
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "gs::" not in n:
            continue
        k = n.split("(")[0][-34:] + f" grid=({r['Grid_Size_X']},{r['Grid_Size_Y']},{r['Grid_Size_Z']})"
        d[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, v in sorted(d.items()):
        v.sort()
        print(f"{k:72s} med={v[len(v) // 2]:6.2f} min={v[0]:6.2f}")
