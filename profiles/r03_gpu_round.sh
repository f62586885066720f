#!/bin/bash
# One GPU call: the -m gpu suite, smoke, the N = 1 bench line, and the README configuration
# through the CLI in each engine mode beside the reference.  usage: profiles/r03_gpu_round.sh <outdir>
out=${1:-gpurun_out/r03}; mkdir -p $out
timeout -k 10 120 mpi-asynchronous-communication-test_amd/tools/bin/graph_probe 38 > $out/graph_probe.txt 2>&1; cat $out/graph_probe.txt
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  > $out/gpu_tests.log 2>&1; rc=$?
tail -5 $out/gpu_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc          # 1 = failures (read the log); anything else: stop
timeout -k 10 300 python3 -u -c "import __graft_entry__ as G; G.smoke()" > $out/smoke.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py > $out/bench.json 2> $out/bench.err || exit 1
cat $out/bench.json
bash profiles/chain_modes.sh $out/readme_cli 3 > /dev/null || exit 1
python3 profiles/chain_summary.py $out/readme_cli > $out/readme_cli/summary.txt || exit 1
cat $out/readme_cli/summary.txt
[ -n "$HYBRID" ] && { bash profiles/r03_hybrid.sh $PWD/$out/hybrid > /dev/null || exit 1; cat $out/hybrid/run_*.txt; }
exit $rc
