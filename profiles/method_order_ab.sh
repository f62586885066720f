#!/bin/bash
# Are the many-to-all copy launches (m2, m4) slower because of their pattern or because of the
# launch before them?  Bench under rocprofv3 kernel traces with the methods in two orders;
# per-position launch durations (bench_per_method.py labels positions 1..4).
# usage: profiles/method_order_ab.sh <outdir>
out=${1:-gpurun_out/method_order}; mkdir -p $out
export TMPDIR=/tmp
for ord in 1,2,3,4 2,1,4,3 1,3,2,4; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $out/kt_$ord -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --methods $ord > $out/bench_$ord.json 2> /dev/null || exit 1
  echo "methods in order $ord (positions 1..4 below)" >> $out/summary.txt
  python3 profiles/bench_per_method.py $(find $out/kt_$ord -name run_kernel_trace.csv | head -1) >> $out/summary.txt || exit 1
done
KINDS=9,16 SIZES_MIB=448 timeout -k 10 100 python3 profiles/copy_ceiling.py >> $out/summary.txt 2>&1
echo done
