#!/bin/bash
# Round 3, call J: wave-persistent copy (copy_kernel_w) against the product's one-piece-per-
# workgroup copy_kernel_g on (a) one GPU's configs[2] pack launch (28 MiB, cache-resident)
# and (b) the bench's many-to-all gather (448 MiB, non-temporal), interleaved 3 times, then
# under rocprofv3 --kernel-trace --stats.
export TMPDIR=/tmp
o=$PWD/gpurun_out/r03j; mkdir -p $o
for rep in 1 2 3; do
  KINDS=18,20,22 SIZES_MIB=32 timeout -k 10 120 python3 profiles/copy_ceiling.py >> $o/probe.txt 2>&1 || { cat $o/probe.txt; exit 1; }
  KINDS=16,23,24,25 SIZES_MIB=512 timeout -k 10 120 python3 profiles/copy_ceiling.py >> $o/probe.txt 2>&1 || { cat $o/probe.txt; exit 1; }
done
cat $o/probe.txt
KINDS=16,23,24,25 SIZES_MIB=512 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $o/kt -o run --output-format csv -- python3 profiles/copy_ceiling.py > $o/probe_rocprof.txt 2>&1 || { tail -20 $o/probe_rocprof.txt; exit 1; }
find $o/kt -name 'run_kernel_stats.csv' -exec cp {} $o/probe_kernel_stats.csv \;
rm -rf $o/kt
cut -c1-160 $o/probe_kernel_stats.csv
echo done
