#!/bin/bash
# Stall / cache / MFMA counters for a microbenchmark ($MB, default the linear
# one), three --pmc passes, summarised per kernel and grid shape.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/pmck_${TAG:-x}
mkdir -p "$OUT"
cd "$ROOT"
i=0
for SET in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "TCC_HIT TCC_MISS TCP_TCC_READ_REQ_LATENCY SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $SET -d "$OUT/p$i" -o run --output-format csv -- \
      python3 ${MB:-tools/mb_linear.py} ${MB_ARGS} > "$OUT/mb$i.log" 2>&1 || exit $?
done
python3 - "$OUT" <<'PY'
import collections, csv, glob, sys
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "gs::" not in n:
            continue
        k = n.split("(")[0][-42:] + " g" + r.get("Grid_Size", r.get("Grid_Size_X", "?"))
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in acc.items():
    m = {n: sum(v) / len(v) for n, v in c.items()}
    print(k)
    print("   " + "  ".join(f"{n}={m[n]:.4g}" for n in sorted(m)))
PY
