#!/bin/bash
# Round 3, third GPU call: the bench line under rocprofv3 (kernel stats + the two PMC passes),
# and the README configuration through the CLI per mode (graph replay included).
out=${1:-gpurun_out/r03c}; mkdir -p $out
bash profiles/bench_rocprof.sh r03 > $out/bench_rocprof.log 2>&1 || { tail -20 $out/bench_rocprof.log; exit 1; }
cat gpurun_out/prof_r03/bench.json; cat gpurun_out/prof_r03/kernel_stats.csv | head -5; cat gpurun_out/prof_r03/pmc_traffic.json
bash profiles/chain_modes.sh $out/readme_cli 3 > /dev/null || exit 1
python3 profiles/chain_summary.py $out/readme_cli > $out/readme_cli/summary.txt || exit 1
cat $out/readme_cli/summary.txt
