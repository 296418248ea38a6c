#!/bin/bash
# Device sampler pass: parity tests, the rmat2m lab (latency / throughput),
# and rocprofv3 kernel stats of the lab.  TAG names the output directory.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
TAG=${TAG:-ds}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u -m pytest -x -v -p no:cacheprovider --timeout 200 --timeout-method thread \
    tests/test_gpu_dsampler.py ${EXTRA_TESTS} > "$OUT/tests.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/lab/ds_time.py > "$OUT/ds_time.log" 2>&1
rc=$?; echo "ds_time rc=$rc"; tail -6 "$OUT/ds_time.log"; [ $rc -eq 0 ] || exit $rc
mkdir -p "$OUT/prof"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python3 tools/lab/ds_time.py > "$OUT/prof/ds_time.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
rm -f "$OUT"/prof/*/*kernel_trace.csv "$OUT"/prof/*kernel_trace.csv
python3 - "$OUT/prof" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for x in csv.DictReader(open(f)):
    print("%-34s %6s %9.1f us avg %8.1f min" % (x["Name"].split("(")[0][-34:], x["Calls"],
          float(x["AverageNs"]) / 1e3, float(x["MinNs"]) / 1e3))
PY
