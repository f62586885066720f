#!/bin/bash
# round 6, last code: the driver's N = 2, 4 and 8 command forms (python -m torch.distributed.run ...
# bench.py --gpus N), every rank on this box's one GPU (XG_SHARE_GPU=1), each under its own limit;
# stops at the first failure.
set -o pipefail
out=${OUT:-gpurun_out/r06_rehearse}
mkdir -p $out
export XG_SHARE_GPU=1 GPU_MAX_HW_QUEUES=1
for n in ${NS:-2 4 8}; do
    t0=$(date +%s)
    timeout -k 10 640 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
        --master-port $((29530 + n)) bench.py --gpus $n --steps 10 --warmup 2 > $out/bench$n.json 2> $out/bench$n.err
    rc=$?
    echo "N=$n rc=$rc wall=$(( $(date +%s) - t0 )) s"
    tail -c 400 $out/bench$n.json; echo
    [ $rc -eq 0 ] || exit $rc
done
