#!/bin/bash
# Round 3, second GPU call: the -m gpu suite, the cross-GPU step forms (hybrid), the pack
# launch classes, and the configs[4] reference cells at -d 4096 on the box's CPUs.
out=${1:-gpurun_out/r03b}; mkdir -p $out
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  > $out/gpu_tests.log 2>&1; rc=$?
tail -5 $out/gpu_tests.log; grep FAILED $out/gpu_tests.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash profiles/r03_hybrid.sh $PWD/$out/hybrid > /dev/null || exit 1
cat $out/hybrid/run_*.txt
bash profiles/r03_pack.sh $PWD/$out/pack > /dev/null || exit 1
cat $out/pack/summary.txt $out/pack/time_*.txt $out/pack/pmc.txt
[ -n "$C4REF" ] && { bash profiles/configs4_ref.sh $out/configs4_ref 4096 120 > /dev/null; cat $out/configs4_ref/ref_d4096.txt; }
exit $rc
