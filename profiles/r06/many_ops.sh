#!/bin/bash
# round 6: profiles/r06/many_ops.py as an 8-rank job on this GPU (each rank its own program)
set -o pipefail
out=$PWD/gpurun_out/r06/many_ops
mkdir -p $out/mr
rm -f $out/mr/uid.bin
pids=()
for r in 1 2 3 4 5 6 7; do
    RANK=$r WORLD_SIZE=8 XG_SHARE_GPU=1 XG_MR_DIR=$out/mr GPU_MAX_HW_QUEUES=1 \
        timeout -k 10 150 python3 -u profiles/r06/many_ops.py > $out/rank$r.out 2> $out/rank$r.err &
    pids+=($!)
done
RANK=0 WORLD_SIZE=8 XG_SHARE_GPU=1 XG_MR_DIR=$out/mr GPU_MAX_HW_QUEUES=1 \
    timeout -k 10 150 python3 -u profiles/r06/many_ops.py > $out/rank0.out 2> $out/rank0.err
rc=$?
for p in "${pids[@]}"; do wait $p || rc=$?; done
cat $out/rank0.out; [ $rc -eq 0 ] || tail -5 $out/rank0.err
exit $rc
