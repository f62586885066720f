#!/bin/bash
# Round 5: the driver's N = 4 and N = 2 command forms, verbatim but for XG_SHARE_GPU=1 (every rank
# on this box's one GPU): python -m torch.distributed.run ... bench.py --gpus N --steps K --warmup W
# with the default phases, each under its own time limit; stops at the first failure.
set -o pipefail
out=gpurun_out/r05_torchrun24
mkdir -p $out
export XG_SHARE_GPU=1 GPU_MAX_HW_QUEUES=1
for n in 4 2; do
    t0=$(date +%s)
    timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
        --master-port $((29520 + n)) bench.py --gpus $n --steps 10 --warmup 2 > $out/bench$n.json 2> $out/bench$n.err
    rc=$?
    echo "N=$n rc=$rc wall=$(( $(date +%s) - t0 )) s"
    tail -c 600 $out/bench$n.json; echo
    [ $rc -eq 0 ] || exit $rc
done
