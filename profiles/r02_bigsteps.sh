#!/bin/bash
# Per-step copy launches of a plan with large steps (configs[4] shape at -d 1 MiB, m12 c1:
# 256 steps of 64 MiB; m7 c1: 64 steps of 256 MiB), timed with an event after every step
# launch (XG_STEP_CHAIN=0) or as chains (default: in-kernel start stamps, one event per
# chain): kernel trace -> launch durations and the gaps between consecutive launches, plus
# the CLI's max total time.  usage: <outdir>
out=${1:-gpurun_out/r02_bigsteps}; mkdir -p $out
B=$PWD/mpi-asynchronous-communication-test_amd/bin/test
export TMPDIR=/tmp
for ev in 0 1; do
  for m in 12 7; do
    XG_STEP_CHAIN=$ev timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/kt_chain${ev}_m$m -o run --output-format csv -- \
      $B --procs 256 -a 64 -d 1048576 -c 1 -m $m -i 3 -k 1 > $out/cli_chain${ev}_m$m.txt 2> $out/cli_chain${ev}_m$m.err || exit 1
    python3 profiles/trace_gaps.py $(find $out/kt_chain${ev}_m$m -name run_kernel_trace.csv | head -1) copy_kernel \
      > $out/gaps_chain${ev}_m$m.txt || exit 1
  done
done
echo done
