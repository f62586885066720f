#!/bin/bash
# round 4, call I: three more draws of the widened random sweep (seeds 1..3)
set -o pipefail
O=gpurun_out/r04i
mkdir -p $O
for seed in 1 2 3; do
  XG_RANDOM_SEED=$seed XG_RANDOM_N1=400 XG_RANDOM_NV=200 XG_RANDOM_NL=120 timeout -k 10 600 python -u -m pytest \
      tests/test_gpu_random.py -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/random_seed$seed.log 2>&1 || exit 1
  tail -1 $O/random_seed$seed.log
done
