#!/bin/bash
# Round 6 check: the driver's three commands (-m gpu suite, smoke, bench), then the bench
# under rocprofv3 (kernel trace + stats, csv) and the two PMC passes (profiles/bench_rocprof.sh).
set -o pipefail
out=${OUT:-gpurun_out/r06_final}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=25 > $out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "passed|failed" $out/gpu_tests.log | tail -1; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $out/smoke.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py > $out/bench.json 2> $out/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 300 $out/bench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 bash profiles/bench_rocprof.sh r06
rc=$?; echo "rocprof rc=$rc"; exit $rc
