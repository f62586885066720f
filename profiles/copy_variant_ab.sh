#!/bin/bash
# interleaved A/B of copy-kernel variants inside the bench (value GB/s, copy launch us)
for r in 1 2 3; do for v in ${VARIANTS:-5 12 13}; do
  timeout -k 10 120 python3 bench.py --no-cpu-baseline --copy-variant $v > gpurun_out/cv_$v.json || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/cv_$v.json'));print('variant=$v', d['value'], d['roofline']['avg_launch_us'])"
done; done
