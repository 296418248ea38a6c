"""Step-timeline statistics from a rocprofv3 kernel trace of bench.py:
per-step period, the main-stream gap from the update (sgd) to the next
step's first kernel, and mean kernel durations, for the first, middle and
last third of the steps (bench phases: warmup+timed, calibration, sustained).
Developer tool:  python3 tools/gaps.py gpurun_out/<dir>/run_kernel_trace.csv"""
import csv
import sys

import numpy as np

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-34:], r["Queue_Id"])
            for r in rows if "gs::" in r["Kernel_Name"])
queues = {}
for e in ev:
    queues.setdefault(e[3], []).append(e)
main = max(queues.values(), key=lambda q: sum(1 for e in q if "sgd" in e[2]))
sgd = [i for i, e in enumerate(main) if "sgd" in e[2]]
steps = []
for a, b in zip(sgd, sgd[1:]):
    k = main[a + 1:b + 1]
    steps.append(dict(period=(main[b][1] - main[a][1]) / 1e3, gap=(main[a + 1][0] - main[a][1]) / 1e3,
                      durs={e[2]: (e[1] - e[0]) / 1e3 for e in k}))
n = len(steps)
for name, part in (("first", steps[: n // 3]), ("middle", steps[n // 3: 2 * n // 3]), ("last", steps[2 * n // 3:])):
    per = np.median([s["period"] for s in part])
    gap = np.median([s["gap"] for s in part])
    print(f"{name:6s} steps {len(part):3d}: period med {per:6.2f} us, sgd->next gap med {gap:5.2f} us")
    names = {}
    for s in part:
        for k, v in s["durs"].items():
            names.setdefault(k, []).append(v)
    print("        " + ", ".join(f"{k.strip()} {np.median(v):.2f}" for k, v in names.items()))
