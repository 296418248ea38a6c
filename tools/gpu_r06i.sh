#!/bin/bash
# r06 pass i: top lab v11 vs v12 (logits + softmax in one 4-wave stage; dZ beside the slab);
# parity tests on v12; rocprofv3 kernel stats for the bf16 MAX and rmat16m configs.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$PWD}"
O=gpurun_out/r06i
mkdir -p $O
for v in v11 v12 v11 v12; do
  timeout -k 10 120 tools/bin/top_lab_$v tids > $O/top_lab_$v.txt 2>&1; echo "lab $v rc=$?"; grep "v2 top kernel\|v2:" $O/top_lab_$v.txt | tail -2; grep -A9 "stamped launch 2" $O/top_lab_$v.txt
done
TESTS="tests/test_gpu_model.py tests/test_gpu_dp.py tests/test_gpu_fullsize.py::test_fullsize_timed_step_embeddings_and_grads_vs_oracle tests/test_gpu_fullsize.py::test_fullsize_timed_step_bf16_max_vs_oracle tests/test_gpu_fullsize.py::test_fullsize_timed_step_fp32_max_vs_oracle tests/test_apply_model.py" \
  TAG=r06i bash tools/gpu_pass.sh || exit $?
for c in rmat2m-max-bf16 rmat16m; do
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/ks_$c -o run --output-format csv -- \
      python3 bench.py --config $c --steps 300 --warmup 10 --sustain 300 --no-cpu-baseline --ref-stream-steps 0 \
      > $O/ks_$c.log 2>&1 || { tail -5 $O/ks_$c.log; exit 1; }
  tail -1 $O/ks_$c.log | cut -c1-160
  f=$(find $O/ks_$c -name "*kernel_stats.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:9]:
    print(f'{float(r["AverageNs"])/1e3:8.2f} us avg {float(r["MinNs"])/1e3:8.2f} min {int(r["Calls"]):6d} calls  {r["Name"][:100]}')
PY
done
