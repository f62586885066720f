#!/bin/bash
# Round 3, last check at HEAD (TAM stage fusion on top of final2): the -m gpu suite, the README
# configuration per mode beside the reference, smoke, the bench.
export TMPDIR=/tmp
out=${1:-$PWD/gpurun_out/r03_final3}; mkdir -p $out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
bash profiles/chain_modes.sh $out/readme_cli 3 > /dev/null || exit 1
python3 profiles/chain_summary.py $out/readme_cli > $out/readme_cli/summary.txt || exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as G; G.smoke()" > $out/smoke.txt 2>&1 || exit 1
cat $out/smoke.txt
timeout -k 10 300 python3 -u bench.py > $out/bench.json 2> $out/bench.err || exit 1
cut -c1-200 $out/bench.json
grep TAM $out/readme_cli/summary.txt
