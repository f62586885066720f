#!/bin/bash
# Round 3: the cross-GPU step's copy launches of the 8-GPU configs[2] plans (P64 A16 -d 256 KiB,
# m5 + m8) on one MI355X (virtual GPUs).  Kernel trace per launch class with the round-3 piece
# size rule (launches too small for 2 x CUs workgroups of 32 KiB get smaller pieces: the 4 MiB
# local gather is now 512 workgroups of 8 KiB, was 128 of 32 KiB), PMC per class, and the
# device time of a whole virtual run packed vs direct with the pairs through RCCL.
export TMPDIR=/tmp
o=${1:-$PWD/gpurun_out/r03_pack}; mkdir -p $o
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $o/kt -o run --output-format csv -- python3 profiles/pack_virtual.py > $o/run.txt 2> $o/run.err || exit 1
python3 profiles/pack_summary.py $(find $o/kt -name run_kernel_trace.csv) > $o/summary.txt || exit 1
rm -rf $o/kt
for pack in 1073741824 0; do
  PACK=$pack RCCL=1 REPS=20 timeout -k 10 120 python3 profiles/pack_virtual.py > $o/time_rccl_$pack.txt 2>&1 || exit 1
done
REPS=3 timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $o/fetch -o run --output-format csv -- python3 profiles/pack_virtual.py > /dev/null 2>&1 || exit 1
REPS=3 timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $o/write -o run --output-format csv -- python3 profiles/pack_virtual.py > /dev/null 2>&1 || exit 1
python3 profiles/pack_pmc.py $(find $o/fetch -name run_counter_collection.csv) $(find $o/write -name run_counter_collection.csv) > $o/pmc.txt || exit 1
rm -rf $o/fetch $o/write
echo done
