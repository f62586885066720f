#!/bin/bash
# Round 5: the whole -m gpu suite as the driver runs it, smoke(), the N = 1 bench, and the
# rocprofv3 kernel-trace summary of the bench (profiles/r05/bench/).
set -o pipefail
out=gpurun_out/r05_full
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -5 $out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $out/smoke.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py > $out/bench.json 2> $out/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 600 $out/bench.json; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 64 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/$out/bench_under_rocprof.json 2> $GRAFT_REPO_ROOT/$out/rocprof.err
rc=$?; echo "rocprof rc=$rc"; exit $rc
