#!/bin/bash
# round 4: the bench's gather pattern (kind 16, 448 MiB) against piece size, pipeline depth and the
# loads' / stores' cache policy, beside the contiguous nt copy of the same bytes (kind 9).
# PASSES x KINDS (defaults: the first A/B, two passes)
set -o pipefail
O=gpurun_out/r04_gather_ab${TAG:+_$TAG}
mkdir -p $O
export KINDS=${KINDS:-9,16,28,29,30,31,32,33,34,35,36,37} SIZES_MIB=448
for p in $(seq 1 ${PASSES:-2}); do
  timeout -k 10 240 python3 profiles/copy_ceiling.py > $O/pass$p.txt 2>&1 || exit $?
done
