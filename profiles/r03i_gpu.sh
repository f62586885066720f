#!/bin/bash
# Round 3, call I: one GPU's configs[2] pack launch as it runs on a real 8-GPU node (28 MiB
# gathered out of the GPU's own 32 MiB of segments: source + staging fit the Infinity Cache),
# the product's copy_kernel_g<4> over 16 KiB pieces against a persistent-workgroup probe
# (copy_kernel_p<U>), interleaved 3 times; then the same under rocprofv3 --kernel-trace --stats.
export TMPDIR=/tmp
o=$PWD/gpurun_out/r03i; mkdir -p $o
for rep in 1 2 3; do
  KINDS=18,19,20,21 SIZES_MIB=32 timeout -k 10 120 python3 profiles/copy_ceiling.py >> $o/pack_probe.txt 2>&1 || { cat $o/pack_probe.txt; exit 1; }
done
cat $o/pack_probe.txt
KINDS=18,19,20,21 SIZES_MIB=32 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $o/kt -o run --output-format csv -- python3 profiles/copy_ceiling.py > $o/pack_probe_rocprof.txt 2>&1 || { tail -20 $o/pack_probe_rocprof.txt; exit 1; }
find $o/kt -name 'run_kernel_stats.csv' -exec cp {} $o/pack_probe_kernel_stats.csv \;
rm -rf $o/kt
cut -c1-160 $o/pack_probe_kernel_stats.csv
echo done
