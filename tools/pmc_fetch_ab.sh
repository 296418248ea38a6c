#!/bin/bash
# FETCH_SIZE of one bench run per runtime switch (no trace domains beside --pmc):
# bash tools/pmc_fetch_ab.sh "VAR=a" "VAR=b"; prints raw FETCH bytes per dispatch of the top kernels
set -o pipefail
export TMPDIR=/tmp
for e in "$@"; do
  D=gpurun_out/pmcab_${e//[=\/]/_}; mkdir -p $D
  env $e timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $D -o run --output-format csv -- \
      python3 bench.py --steps 30 --warmup 5 --sustain 0 --no-cpu-baseline > $D/bench.log 2>&1 || exit $?
  python3 - "$D" "$e" <<'PY'
import csv, glob, sys, collections
rows = []
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
acc = collections.defaultdict(list)
for r in rows:
    acc[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1]) / len(kv[1]))[:6]:
    print(sys.argv[2], k[:50], "FETCH raw MB/dispatch %.2f" % (sum(v) / len(v) / 1e6))
PY
done
