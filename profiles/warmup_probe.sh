#!/bin/bash
# bench value vs warmup length and timed steps (sustained load before / during the timed region)
for r in 1 2; do for ws in "5 20" "200 20" "2000 20" "5 200" "200 200"; do
  set -- $ws
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --warmup $1 --steps $2 > gpurun_out/wu_$1_$2.json || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/wu_$1_$2.json'));print('warmup=$1 steps=$2', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
done; done
