#!/bin/bash
# round 6: (a) why copy_kernel_w's 4 MiB launch stays at ~4.8 us whatever its
# piece size -- GPU 0's configs[2]-shape share at -d 64 KiB .. 1 MiB (local part 1-16 MiB, packs and
# unpacks 7-112 MiB), rocprofv3 kernel trace per -d, duration against bytes; (b) one rank of a real
# 8-rank job (configs[2], m5 / m8, XG_SHARE_GPU) under rocprofv3: do the side-stream local copies run
# inside the RCCL kernel?  The other 7 ranks run beside it, unprofiled, as programs of their own.
set -o pipefail
export TMPDIR=/tmp
out=$PWD/gpurun_out/r06/launch_floor
mkdir -p $out
for dk in 64 128 256 512 1024; do
    D_KIB=$dk REPS=50 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $out/d$dk -o run -- \
        python3 profiles/share_launches.py > $out/d$dk.log 2>&1 || { echo "d $dk rc=$?"; tail -5 $out/d$dk.log; exit 1; }
    f=$(find $out/d$dk -name 'run_kernel_trace.csv' | head -1)
    { echo "== -d $dk KiB"; python3 profiles/kernel_classes.py $f; } >> $out/summary.txt
done
ov=$PWD/gpurun_out/r06/overlap
mkdir -p $ov/mr
rm -f $ov/mr/uid.bin
case='[{"shape": [64, 16, 262144, 200000000], "methods": [5, 8], "forms": [[4194304, 0], [4194304, 1], [0, -1]]}]'
pids=()
for r in 1 2 3 4 5 6 7; do
    RANK=$r WORLD_SIZE=8 LOCAL_RANK=$r XG_SHARE_GPU=1 XG_MR_DIR=$ov/mr GPU_MAX_HW_QUEUES=1 XG_MR_DEADLINE=100 \
        timeout -k 10 130 python3 -u tests/multirank_worker.py "$case" > $ov/rank$r.out 2> $ov/rank$r.err &
    pids+=($!)
done
RANK=0 WORLD_SIZE=8 LOCAL_RANK=0 XG_SHARE_GPU=1 XG_MR_DIR=$ov/mr GPU_MAX_HW_QUEUES=2 XG_MR_DEADLINE=100 \
    timeout -k 10 130 rocprofv3 --kernel-trace --output-format csv -d $ov/prof -o run -- \
    python3 -u tests/multirank_worker.py "$case" > $ov/rank0.out 2> $ov/rank0.err
rc=$?
for p in "${pids[@]}"; do wait $p || rc=$?; done
[ $rc -eq 0 ] || { echo "8-rank job rc=$rc"; tail -3 $ov/rank0.err; exit $rc; }
f=$(find $ov/prof -name 'run_kernel_trace.csv' | head -1)
python3 profiles/r06/overlap_summary.py $f > $ov/summary.txt
cat $out/summary.txt $ov/summary.txt; tail -4 $ov/rank0.out
