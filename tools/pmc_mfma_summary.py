"""MFMA utilisation per kernel from a rocprofv3 --pmc pass of
SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, SQ_WAVE_CYCLES, SQ_WAVES and
GRBM_GUI_ACTIVE (tools/pmc_mfma.sh).

  kernel cycles   = GRBM_GUI_ACTIVE / 8           (summed over the 8 XCDs)
  MFMA util       = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x kernel cycles)
SQ_VALU_MFMA_BUSY_CYCLES counts matrix-core busy cycles summed over SIMDs
(MI355X_MICROARCH.md: 32 per v_mfma_f32_32x32x16_bf16); on a dispatch
shorter than ~0.3 ms GRBM_GUI_ACTIVE reads high (launch ramp included), so
the utilisation is a lower bound.  Means per dispatch."""
import collections
import csv
import glob
import json
import sys

SIMDS = 1024


def main():
    out_dir = sys.argv[1]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{out_dir}/pmc/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    bench = {}
    for line in open(f"{out_dir}/bench.log"):
        if line.startswith('{"metric"'):
            bench = json.loads(line)
    kernels = {}
    for k, cs in sorted(acc.items()):
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        cyc = m.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        busy = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        kernels[k] = {"dispatches": len(next(iter(cs.values()))), **{c: round(v) for c, v in m.items()},
                      "kernel_cycles": round(cyc),
                      "mfma_util": round(busy / (SIMDS * cyc), 4) if cyc else None}
    print(json.dumps({"what": "per-dispatch means; mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x "
                              "GRBM_GUI_ACTIVE / 8)", "bench_value": bench.get("value"),
                      "kernels": kernels}, indent=1))


if __name__ == "__main__":
    main()
