#!/bin/bash
# r06 pass f: top lab v10 vs v11 (unconditional dZ / slab operand reads); GPU tests on the library
# (two-round gather, single-round transposed backward, top v11); bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$PWD}"
O=gpurun_out/r06f
mkdir -p $O
for v in v10 v11 v10 v11; do
  timeout -k 10 120 tools/bin/top_lab_$v tids > $O/top_lab_$v.txt 2>&1; echo "lab $v rc=$?"; grep "v2 top kernel\|v2:" $O/top_lab_$v.txt | tail -2; grep -A10 "stamped launch 2" $O/top_lab_$v.txt
done
TESTS="tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_dp.py tests/test_gpu_fullsize.py tests/test_gpu_fullsize16m.py" \
  TEST_TIMEOUT=1000 BENCH=default TAG=r06f bash tools/gpu_pass.sh || exit $?
run() {  # name, timeout, bench args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python3 bench.py "$@" > $O/bench_$n.log 2>&1 || { tail -5 $O/bench_$n.log; return 1; }
  grep '^{"metric"' $O/bench_$n.log | tail -1 > $O/bench_$n.json; cut -c1-200 $O/bench_$n.json
}
run max_bf16 300 --config rmat2m-max-bf16 --steps 100 --no-cpu-baseline --ref-stream-steps 0 && \
run rmat16m 500 --config rmat16m --steps 100 --no-cpu-baseline --ref-stream-steps 0
