#!/bin/bash
# Round 3, call K: the wave-persistent copy on cross-GPU launches.  The -m gpu suite (every virtual-GPU test now runs
# direct, packed one-sided and packed two-sided), then the three forms of the configs[2] 8-GPU
# plans on this device (profiles/pack_forms.py), plain and under rocprofv3 --kernel-trace --stats.
export TMPDIR=/tmp
o=$PWD/gpurun_out/r03k; mkdir -p $o
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1 || { tail -30 $o/gpu_tests.log; exit 1; }
tail -3 $o/gpu_tests.log
timeout -k 10 240 python3 -u profiles/pack_forms.py > $o/pack_forms.txt 2>&1 || { cat $o/pack_forms.txt; exit 1; }
cat $o/pack_forms.txt
REPS=10 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $o/kt -o run --output-format csv -- python3 profiles/pack_forms.py > $o/pack_forms_rocprof.txt 2>&1 || { tail -20 $o/pack_forms_rocprof.txt; exit 1; }
find $o/kt -name 'run_kernel_stats.csv' -exec cp {} $o/pack_forms_kernel_stats.csv \;
rm -rf $o/kt
echo done
