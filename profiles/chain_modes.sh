#!/bin/bash
# README configuration (configs[0]) through the drop-in CLI under the step-engine modes,
# interleaved, plus the reference under MPICH on the same box: max total time per method.
#   solo_armed  default: one-workgroup engine for small plans, launch before the timed region
#   grid_armed  XG_ENGINE_SOLO_STEP=0 (grid-barrier engine), armed
#   solo_launch XG_ENGINE_ARM=0 (launch inside the timed region)
#   grid_launch both off = the round-1 engine
# usage: profiles/chain_modes.sh <outdir> [reps]
out=${1:-gpurun_out/chain}; reps=${2:-3}; mkdir -p $out
args="-a 14 -d 2048 -c 3 -m 0 -i 2 -k 1"
bin=$PWD/mpi-asynchronous-communication-test_amd/bin/test
cd $out
for r in $(seq 1 $reps); do
  timeout -k 10 120 $bin --procs 32 $args > solo_armed_$r.txt 2>> err.txt || exit 1
  XG_ENGINE_SOLO_STEP=0 timeout -k 10 120 $bin --procs 32 $args > grid_armed_$r.txt 2>> err.txt || exit 1
  XG_ENGINE_ARM=0 timeout -k 10 120 $bin --procs 32 $args > solo_launch_$r.txt 2>> err.txt || exit 1
  XG_ENGINE_ARM=0 XG_ENGINE_SOLO_STEP=0 timeout -k 10 120 $bin --procs 32 $args > grid_launch_$r.txt 2>> err.txt || exit 1
done
if [ -x ../../oracle/_ref/test ]; then
  timeout -k 10 300 /opt/conda/bin/mpiexec -launcher fork -n 32 ../../oracle/_ref/test $args > ref.txt 2> ref.err || echo "reference run failed"
fi
echo done
