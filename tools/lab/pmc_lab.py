"""Per-kernel means of a rocprofv3 --pmc pass over a lab binary
(tools/gpu_r05*.sh): SQ wave-cycle buckets as fractions of SQ_WAVE_CYCLES
(quad-cycles; WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES) and
the matrix-core busy fraction against GRBM_GUI_ACTIVE / 8 (MI355X_MICROARCH.md
§rocprofv3 PMC slots).  Developer tool:  python tools/lab/pmc_lab.py DIR"""
import collections
import csv
import glob
import sys


def main():
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:70]
            acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in sorted(acc.items()):
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        n = len(next(iter(cs.values())))
        wc = m.get("SQ_WAVE_CYCLES")
        parts = [f"{k} ({n} dispatches)"]
        for c, v in sorted(m.items()):
            frac = f" ({v / wc:.3f} of wave cycles)" if wc and c.startswith("SQ_") and c not in (
                "SQ_WAVE_CYCLES", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_WAVES", "SQ_BUSY_CYCLES") else ""
            parts.append(f"  {c} = {v:.0f}{frac}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
            parts.append(f"  mfma busy / (1024 SIMDs x GRBM/8) = "
                         f"{m['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * m['GRBM_GUI_ACTIVE'] / 8):.3f}")
        print("\n".join(parts))


if __name__ == "__main__":
    main()
