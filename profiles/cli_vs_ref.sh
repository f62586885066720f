#!/bin/bash
# README configuration (BASELINE configs[0]) through the drop-in CLI on one MI355X and through
# the reference under MPICH on the same box's host cores; reports side by side.
# usage: profiles/cli_vs_ref.sh <outdir> [extra test args]
out=${1:-gpurun_out/cli}; shift; mkdir -p $out
args=${@:-"-a 14 -d 2048 -c 3 -m 0 -i 2 -k 1"}
cd $out
timeout -k 10 120 ../../mpi-asynchronous-communication-test_amd/bin/test --procs 32 $args > gpu.txt 2> gpu.err || exit 1
if [ -x ../../oracle/_ref/test ]; then
  timeout -k 10 300 /opt/conda/bin/mpiexec -launcher fork -n 32 ../../oracle/_ref/test $args > ref.txt 2> ref.err || echo "reference run failed"
fi
