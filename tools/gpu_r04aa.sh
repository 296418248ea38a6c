#!/bin/bash
# Round-4 pass AA: rocprofv3 kernel stats of the final defaults (300-step fp32
# MEAN and bf16 MAX benches), for the bench's committed summaries.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r04aa
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_rmat2m" -o run --output-format csv -- python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline --ref-stream-steps 0 > "$OUT/prof_rmat2m.log" 2>&1 || exit $?
cp "$OUT/prof_rmat2m/run_kernel_stats.csv" "$OUT/kernel_stats_rmat2m_steps300.csv" || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_bf16" -o run --output-format csv -- python3 bench.py --config rmat2m-max-bf16 --steps 300 --warmup 5 --no-cpu-baseline --ref-stream-steps 0 > "$OUT/prof_bf16.log" 2>&1 || exit $?
cp "$OUT/prof_bf16/run_kernel_stats.csv" "$OUT/kernel_stats_rmat2m_max_bf16_steps300.csv" || exit 1
rm -rf "$OUT/prof_rmat2m" "$OUT/prof_bf16"
for f in kernel_stats_rmat2m_steps300 kernel_stats_rmat2m_max_bf16_steps300; do
python3 - "$OUT/$f.csv" <<'PY'
import csv, sys
tot = 0
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "gs::" in n and int(r["Calls"]) > 100:
        a = float(r["AverageNs"]) / 1e3
        print(f"  {n.split('(')[0][-50:]:50s} avg {a:7.2f} min {float(r['MinNs'])/1e3:7.2f}")
        if not any(x in n for x in ("agg_ids", "pull_pack", "resolve")):
            tot += a
print("  main-stream sum", round(tot, 2))
PY
done
