#!/bin/bash
# round 4: A/B of the XCD-dealt piece order (XG_XCD_ORDER=1) against destination order on the bench
# (configs[1]), interleaved, 3 runs each; bench verifies every byte before timing
set -o pipefail
O=gpurun_out/r04_xcd
mkdir -p $O
for rep in 1 2 3; do
  for x in 0 1; do
    XG_XCD_ORDER=$x timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench_x${x}_$rep.json 2> $O/bench_x${x}_$rep.err || exit 1
    python3 -c "import json,sys; d=json.load(open('$O/bench_x${x}_$rep.json')); print('xcd_order=$x rep $rep', d['value'], d['roofline']['avg_launch_us'], d['max_total_time_s'])" >> $O/summary.txt
  done
done
