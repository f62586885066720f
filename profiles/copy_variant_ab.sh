#!/bin/bash
# interleaved A/B of copy-kernel variants x piece sizes inside the bench (value GB/s, copy launch us)
# usage: VARIANTS="5 14" CHUNKS="32768 65536" REPS=3 profiles/copy_variant_ab.sh
for r in $(seq ${REPS:-3}); do for v in ${VARIANTS:-5 12 13}; do for ch in ${CHUNKS:-32768}; do
  timeout -k 10 120 python3 bench.py --no-cpu-baseline --copy-variant $v --chunk $ch > gpurun_out/cv_${v}_$ch.json || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/cv_${v}_$ch.json'));print('variant=$v chunk=$ch', d['value'], d['roofline']['avg_launch_us'])"
done; done; done
