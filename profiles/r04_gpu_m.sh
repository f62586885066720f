#!/bin/bash
# round 4, call M: two draws after virtual jobs took the mark mask too (seeds 16..17; 1000 one-GPU + 500
# virtual 2/3/4/8-GPU + 200 virtual P = 48-256 configurations each)
set -o pipefail
O=gpurun_out/r04m
mkdir -p $O
for seed in 16 17; do
  XG_RANDOM_SEED=$seed XG_RANDOM_N1=1000 XG_RANDOM_NV=500 XG_RANDOM_NL=200 timeout -k 10 600 python -u -m pytest \
      tests/test_gpu_random.py -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/random_seed$seed.log 2>&1 || exit 1
  tail -n 1 $O/random_seed$seed.log
done
