#!/bin/bash
# A/B of library builds under rocprofv3 kernel stats: ROUNDS alternating
# bench runs (300 steps + 300 sustained) per .so, then per-build medians of
# each step kernel's rocprof average and of the main-stream sum.
#   ROUNDS=2 bash tools/ab_prof.sh graphsage-pytorch_amd/libgraphsage_amd.so other.so ...
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/ab_prof}
mkdir -p $OUT
P=graphsage-pytorch_amd
cp $P/libgraphsage_amd.so /tmp/lib_main.so
: > $OUT/runs.txt
for i in $(seq 1 ${ROUNDS:-2}); do
  for so in "$@"; do
    src=$so; [ "$so" = "$P/libgraphsage_amd.so" ] && src=/tmp/lib_main.so
    cp $src $P/libgraphsage_amd.so
    tag=$(basename $so .so)_$i
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$tag -o run --output-format csv -- \
        python3 bench.py --steps ${STEPS:-300} --warmup 10 --sustain ${SUSTAIN:-300} --no-cpu-baseline \
        --ref-stream-steps 0 ${BENCH_ARGS} > $OUT/$tag.log 2>&1 || { cp /tmp/lib_main.so $P/libgraphsage_amd.so; exit 1; }
    python3 tools/ab_prof_line.py $(basename $so) $OUT/$tag $OUT/$tag.log | tee -a $OUT/runs.txt
  done
done
cp /tmp/lib_main.so $P/libgraphsage_amd.so
python3 tools/ab_prof_line.py --summary $OUT/runs.txt
