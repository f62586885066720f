#!/bin/bash
# round 4: A/B of a gap after every rank's buffer (XG_REGION_SKEW bytes) on the bench (configs[1]):
# aggregator buffers are 32 MiB (P32 x 1 MiB) and rank buffers 14 MiB; interleaved, 2 runs each
set -o pipefail
O=gpurun_out/r04_skew
mkdir -p $O
for rep in 1 2; do
  for k in 0 4096 65536 1052672; do
    XG_REGION_SKEW=$k timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench_k${k}_$rep.json 2> $O/bench_k${k}_$rep.err || exit 1
    python3 -c "import json; d=json.load(open('$O/bench_k${k}_$rep.json')); print('skew=$k rep $rep', d['value'], d['roofline']['avg_launch_us'], ' '.join('m%s %.1f' % (m, t * 1e6) for m, t in sorted(d['max_total_time_s'].items())))" >> $O/summary.txt
  done
done
