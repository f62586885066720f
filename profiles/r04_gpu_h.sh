#!/bin/bash
# round 4, call H: the bench's BASELINE-configs phase on one GPU (--baseline-configs on): configs[2]
# and configs[3] run with every rank on this GPU; configs[4]'s 64 MiB segments (2 TiB on one GPU)
# must fail to allocate and be recorded, the line still printed
set -o pipefail
O=gpurun_out/r04h
mkdir -p $O
timeout -k 10 600 python3 bench.py --baseline-configs on --steps 5 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
