#!/bin/bash
# Round 3, call F: the -m gpu suite at HEAD, a widened random sweep (600 one-GPU + 300 virtual
# multi-GPU configurations, every method, against the oracle), smoke, the bench line.
out=${1:-gpurun_out/r03f}; mkdir -p $out
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  > $out/gpu_tests.log 2>&1; rc=$?
tail -3 $out/gpu_tests.log; grep FAILED $out/gpu_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
XG_RANDOM_N1=600 XG_RANDOM_NV=300 timeout -k 10 900 python3 -u -m pytest tests/test_gpu_random.py -m gpu -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > $out/random_sweep.log 2>&1 || { tail -20 $out/random_sweep.log; exit 1; }
tail -3 $out/random_sweep.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as G; G.smoke()" > $out/smoke.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py > $out/bench.json 2> $out/bench.err || exit 1
cat $out/smoke.txt $out/bench.json
