#!/bin/bash
# round 4 probe: can two bench ranks (two processes, one RCCL communicator) share the one GPU of
# this box (XG_DEVICE=0 for both)?  If RCCL accepts it, this is a real 2-process RCCL run of the
# N = 2 path; if it refuses (duplicate device), the log says so.  Bounded: watchdog 90 s, timeout 150 s.
set -o pipefail
O=gpurun_out/r04_two_ranks
mkdir -p $O
XG_DEVICE=0 NCCL_DEBUG=WARN timeout -k 10 150 python3 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline \
    --watchdog 90 --child-timeout 120 > $O/bench.json 2> $O/bench.err
echo "rc=$?" > $O/rc.txt
