#!/bin/bash
# Round 3, call E: the -m gpu suite at HEAD, configs[4] on one GPU at -d 8 MiB, the pack launch
# classes with 32 KiB pieces again, and the copy ceiling at the cross-GPU launch sizes.
out=${1:-gpurun_out/r03e}; mkdir -p $out
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  > $out/gpu_tests.log 2>&1; rc=$?
tail -3 $out/gpu_tests.log; grep FAILED $out/gpu_tests.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python3 -u profiles/configs4_sweep.py > $out/configs4_gpu_d8m.txt 2> $out/configs4.err || exit 1
cat $out/configs4_gpu_d8m.txt
bash profiles/r03_pack.sh $PWD/$out/pack > /dev/null || exit 1
cat $out/pack/summary.txt $out/pack/pmc.txt
KINDS=0,1,8,9,14,15 SIZES_MIB=4,14,28,56,448 timeout -k 10 300 python3 -u profiles/copy_ceiling.py > $out/copy_ceiling_mid.txt 2>&1 || exit 1
cat $out/copy_ceiling_mid.txt
XG_SELF_COMM=1 timeout -k 10 120 python3 -u profiles/rccl_self_floor.py > $out/rccl_self_floor.txt 2>&1 || exit 1
cat $out/rccl_self_floor.txt
exit $rc
