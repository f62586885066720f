#!/bin/bash
# round 6: (a) copy_kernel_w piece size per launch (XG_WAVE_KIB 8 = round 5, 4, 2, 0 = by launch
# bytes) on one GPU's share of the configs[2] 8-GPU plans, rocprofv3 kernel trace per setting;
# (b) the relay form's per-call cost (relay_cost.py); (c) the wave-copy parity tests.
set -o pipefail
export TMPDIR=/tmp
out=$PWD/gpurun_out/r06/wave_kib
mkdir -p $out
for kib in 8 4 2 0; do
    XG_WAVE_KIB=$kib FORM=0 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $out/k$kib -o run -- \
        python3 profiles/share_launches.py > $out/k$kib.log 2>&1 || { echo "kib $kib rc=$?"; tail -5 $out/k$kib.log; exit 1; }
    f=$(find $out/k$kib -name 'run_kernel_trace.csv' | head -1)
    { echo "== XG_WAVE_KIB=$kib"; python3 profiles/kernel_classes.py $f; } >> $out/summary.txt
done
timeout -k 10 300 python3 -u profiles/r06/relay_cost.py > gpurun_out/r06/relay_cost.log 2>&1 || { echo "relay_cost rc=$?"; tail -5 gpurun_out/r06/relay_cost.log; exit 1; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_virtual.py -k "wave_copy" --durations=5 > gpurun_out/r06/wave_tests.log 2>&1
