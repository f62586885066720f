#!/bin/bash
# rocprofv3 kernel trace of the README configuration through the CLI (all 20 methods, solo
# engine on rails by default): per-kernel statistics, solo_engine_kernel durations included.
# usage: profiles/r02_rails_trace.sh <outdir>
out=${1:-gpurun_out/r02_rails_trace}; mkdir -p $out
export TMPDIR=/tmp
B=$PWD/mpi-asynchronous-communication-test_amd/bin/test
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/kt -o run --output-format csv -- \
  $B --procs 32 -a 14 -d 2048 -c 3 -m 0 -i 2 -k 1 > $out/cli.txt 2> $out/cli.err || exit 1
cp $(find $out/kt -name run_kernel_stats.csv | head -1) $out/kernel_stats.csv
python3 profiles/trace_gaps.py $(find $out/kt -name run_kernel_trace.csv | head -1) solo_engine > $out/solo_launches.txt || exit 1
echo done
