#!/bin/bash
# A/B of the package's Python files: tools/lab/abpy_old/*.py (the old copies)
# against the tree's, alternating bench runs; BENCH_ARGS picks the config.
P=graphsage-pytorch_amd
O=${OUT:-gpurun_out/ab_py}
mkdir -p $O/new
for f in tools/lab/abpy_old/*.py; do cp $P/$(basename $f) $O/new/; done
swap() { for f in $1/*.py; do cp $f $P/$(basename $f); done; }
for i in $(seq 1 ${ROUNDS:-3}); do
  for v in old new; do
    if [ $v = old ]; then swap tools/lab/abpy_old; else swap $O/new; fi
    timeout -k 10 300 python3 bench.py ${BENCH_ARGS} --no-cpu-baseline > $O/${v}_${i}.log 2>&1 || { swap $O/new; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[2], d['ms_per_step'], d['value'], d['config'].get('final_loss'))" $O/${v}_${i}.log $v | tee -a $O/runs.txt
  done
done
swap $O/new
