#!/bin/bash
# A/B of the XCD-mapped weight-gradient grid against the (k, h, slab) grid (GS_DW_GRID3=1).
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
run() {
  timeout -k 10 200 env $1 python bench.py --steps 400 --warmup 10 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/ab.log').read().splitlines()[-1]);print('$1', d['ms_per_step'], d['value'], d['roofline_mfma']['dw']['avg_launch_us'])"
}
for i in 1 2; do for m in GS_DW_GRID3=1 GS_X=0; do run "$m"; done; done
rm -rf gpurun_out/pmc_xcd; mkdir -p gpurun_out/pmc_xcd
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_xcd/FETCH_SIZE -o run --output-format csv -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/pmc_xcd/bench_FETCH_SIZE.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_xcd/WRITE_SIZE -o run --output-format csv -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/pmc_xcd/bench_WRITE_SIZE.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_xcd rmat2m > gpurun_out/pmc_xcd/summary.json
