#!/bin/bash
# Round 6: the driver's N = 8 command form, verbatim but for XG_SHARE_GPU=1 (every rank on this
# box's one GPU): python -m torch.distributed.run ... bench.py --gpus 8 --steps K --warmup W with
# the default phases (CPU baselines, xGMI phases, BASELINE configs), under a time limit.
set -o pipefail
out=${OUT:-gpurun_out/r06_torchrun8b}
mkdir -p $out
export XG_SHARE_GPU=1 GPU_MAX_HW_QUEUES=1
t0=$(date +%s)
timeout -k 10 700 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 8 --steps 10 --warmup 2 > $out/bench8.json 2> $out/bench8.err
rc=$?; echo "rc=$rc wall=$(( $(date +%s) - t0 )) s"; tail -c 800 $out/bench8.json; exit $rc
