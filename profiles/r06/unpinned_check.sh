#!/bin/bash
# round 6: the reference baselines unpinned again (bench.reference_cpus) -- the N = 1 line, then the
# driver's N = 8 command form with every rank on this GPU
set -o pipefail
mkdir -p gpurun_out/r06_unpinned
timeout -k 10 300 python3 bench.py > gpurun_out/r06_unpinned/bench.json 2> gpurun_out/r06_unpinned/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 700 gpurun_out/r06_unpinned/bench.json; [ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/r06_torchrun8d bash profiles/r06/torchrun8.sh
