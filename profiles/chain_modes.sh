#!/bin/bash
# README configuration (configs[0]) through the drop-in CLI under the step-engine modes,
# interleaved, plus the reference under MPICH on the same box: max total time per method.
#   solo_armed  default: solo engine (256 one-wave rails) for small plans, launch before the timed region
#   solo1_armed XG_SOLO_WAVES=16 XG_SOLO_RAILS=1 (one 16-wave workgroup, the round-2 start)
#   grid_armed  XG_ENGINE_SOLO=0 (grid-barrier engine), armed
#   solo_launch XG_ENGINE_ARM=0 (launch inside the timed region)
# usage: profiles/chain_modes.sh <outdir> [reps]
out=${1:-gpurun_out/chain}; reps=${2:-3}; mkdir -p $out
args="-a 14 -d 2048 -c 3 -m 0 -i 2 -k 1"
repo=$PWD; bin=$repo/mpi-asynchronous-communication-test_amd/bin/test
cd $out
for r in $(seq 1 $reps); do
  timeout -k 10 120 $bin --procs 32 $args > solo_armed_$r.txt 2>> err.txt || exit 1
  XG_ENGINE_SOLO=0 timeout -k 10 120 $bin --procs 32 $args > grid_armed_$r.txt 2>> err.txt || exit 1
  XG_ENGINE_ARM=0 timeout -k 10 120 $bin --procs 32 $args > solo_launch_$r.txt 2>> err.txt || exit 1
  XG_SOLO_WAVES=16 XG_SOLO_RAILS=1 timeout -k 10 120 $bin --procs 32 $args > solo1_armed_$r.txt 2>> err.txt || exit 1
done
if [ -x $repo/oracle/_ref/test ] && [ -z "$NOREF" ]; then
  for r in $(seq 1 $reps); do
    timeout -k 10 300 /opt/conda/bin/mpiexec -launcher fork -n 32 $repo/oracle/_ref/test $args > ref_$r.txt 2>> ref.err || echo "reference run failed"
  done
fi
echo done
