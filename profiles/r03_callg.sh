#!/bin/bash
# Round 3, call G: the -m gpu suite at HEAD (graph replay on by default for launch-bound one-GPU
# runs, init/finalize error paths), the README configuration per mode, smoke, bench.
out=${1:-gpurun_out/r03g}; mkdir -p $out
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  > $out/gpu_tests.log 2>&1; rc=$?
tail -3 $out/gpu_tests.log; grep FAILED $out/gpu_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
bash profiles/chain_modes.sh $out/readme_cli 3 > /dev/null || exit 1
python3 profiles/chain_summary.py $out/readme_cli > $out/readme_cli/summary.txt || exit 1
cat $out/readme_cli/summary.txt
timeout -k 10 300 python3 -u -c "import __graft_entry__ as G; G.smoke()" > $out/smoke.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py > $out/bench.json 2> $out/bench.err || exit 1
cat $out/smoke.txt $out/bench.json
