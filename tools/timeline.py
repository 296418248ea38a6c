"""Median step timeline from a rocprofv3 kernel trace of bench.py: for each
main-stream kernel of a step (its last launch to the next step's: the sgd,
or the slab sum with the deferred update), its start offset, duration and the
idle gap before it, plus which side-stream kernels overlapped it.  Steps from
the middle third of the run (calibration-free when --sustain covers it).
Developer tool:  python3 tools/timeline.py gpurun_out/<dir>/run_kernel_trace.csv [first_frac last_frac]"""
import csv
import sys

import numpy as np

rows = list(csv.DictReader(open(sys.argv[1])))
lo, hi = (float(sys.argv[2]), float(sys.argv[3])) if len(sys.argv) > 3 else (0.5, 0.95)
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "")[-40:],
             r["Queue_Id"]) for r in rows if "gs::" in r["Kernel_Name"])
queues = {}
for e in ev:
    queues.setdefault(e[3], []).append(e)
last = "sgd" if any("sgd" in e[2] for e in ev) else "sum_slabs_pair"
main_q = max(queues, key=lambda q: sum(1 for e in queues[q] if last in e[2]))
main = queues[main_q]
side = [e for q, v in queues.items() if q != main_q for e in v]
sgd = [i for i, e in enumerate(main) if last in e[2]]
steps = []
for a, b in zip(sgd, sgd[1:]):
    steps.append(main[a + 1:b + 1])
steps = steps[int(len(steps) * lo):int(len(steps) * hi)]
period = [s[-1][1] - s[0][0] for s in steps]
print(f"{len(steps)} steps; first-kernel start to {last} end: median {np.median(period)/1e3:.2f} us")
n = min(len(s) for s in steps)
for i in range(n):
    name = steps[0][i][2]
    off = [(s[i][0] - s[0][0]) / 1e3 for s in steps]
    dur = [(s[i][1] - s[i][0]) / 1e3 for s in steps]
    gap = [((s[i][0] - s[i - 1][1]) / 1e3) if i else 0.0 for s in steps]
    ov = {}
    for s in steps:
        a, b = s[i][0], s[i][1]
        for e in side:
            o = min(b, e[1]) - max(a, e[0])
            if o > 0:
                ov[e[2].strip()] = ov.get(e[2].strip(), 0) + o / 1e3 / len(steps)
    ovs = ", ".join(f"{k[-24:]} {v:.1f}" for k, v in sorted(ov.items(), key=lambda x: -x[1]) if v > 0.3)
    print(f"{np.median(off):7.2f} +{np.median(dur):6.2f} (gap {np.median(gap):5.2f})  {name.strip():40s} | {ovs}")
for k in sorted({e[2] for e in side}):
    d = [(e[1] - e[0]) / 1e3 for e in side if e[2] == k]
    print(f"side: {k.strip():40s} median {np.median(d):.2f} us")
