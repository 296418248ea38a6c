#!/bin/bash
# r06 pass h: GPU tests on the DPP wave_sum build, then the rocprofv3 kernel stats of the 300-step rmat2m bench.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$PWD}"
O=gpurun_out/r06h
mkdir -p $O
TESTS="tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_dp.py tests/test_gpu_fullsize.py::test_fullsize_timed_step_embeddings_and_grads_vs_oracle tests/test_gpu_fullsize.py::test_fullsize_timed_step_bf16_max_vs_oracle tests/test_gpu_pubmed.py tests/test_apply_model.py" \
  TAG=r06h bash tools/gpu_pass.sh || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/ks_rmat2m -o run --output-format csv -- \
    python3 bench.py --steps 300 --warmup 10 --sustain 300 --no-cpu-baseline --ref-stream-steps 0 \
    > $O/ks_rmat2m.log 2>&1 || { tail -5 $O/ks_rmat2m.log; exit 1; }
tail -1 $O/ks_rmat2m.log | cut -c1-200
f=$(find $O/ks_rmat2m -name "*kernel_stats.csv" | head -1); echo "stats: $f"
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print(f'{float(r["AverageNs"])/1e3:8.2f} us avg {float(r["MinNs"])/1e3:8.2f} min {int(r["Calls"]):6d} calls  {r["Name"][:110]}')
PY
