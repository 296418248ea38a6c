#!/bin/bash
# Round-4 pass C: the device-sampler capacity fallback alone first (the test
# whose run faulted before the GS_DS_BAIL fix), then the sampler A/B, the
# -m gpu suite, smoke() and the driver's default bench command.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r04c
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
    "tests/test_gpu_fullsize.py::test_fullsize_device_sampler_past_capacity_falls_back" > "$OUT/fallback.log" 2>&1
rc=$?; tail -3 "$OUT/fallback.log"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 120 tools/bin/sampler_bench_r03 1 300 1 >> "$OUT/sampler_ab.txt" 2>&1 || exit $?
  timeout -k 10 120 tools/bin/sampler_bench_new2 1 300 1 >> "$OUT/sampler_ab.txt" 2>&1 || exit $?
done
timeout -k 10 200 tools/bin/sampler_bench_new2 1 200 7 >> "$OUT/sampler_ab.txt" 2>&1 || exit $?
grep -E "helpers|phases" "$OUT/sampler_ab.txt"
timeout -k 10 1100 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > "$OUT/gpu_tests.log" 2>&1
rc=$?; tail -3 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
echo smoke ok
timeout -k 10 400 python3 bench.py > "$OUT/bench_rmat2m_steps20.json" 2> "$OUT/bench_rmat2m_steps20.err" || exit $?
python3 - "$OUT/bench_rmat2m_steps20.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d["config"]
print("value", d["value"], "ms", d["ms_per_step"], "sampler", c["sampler"], "sustained", {k: d["sustained"][k] for k in ("value", "lookahead_misses", "max_step_ms")})
print("reference_stream", d.get("reference_stream"))
PY
