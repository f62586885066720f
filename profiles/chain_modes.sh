#!/bin/bash
# HISTORICAL RECIPE: it sets XG_* knobs folded into constants by commit 88b890f (round 4);
# rerun now, those arms are identical (libxg warns about each such variable).  Kept as the record.
# README configuration (configs[0]) through the drop-in CLI under the step-engine modes,
# interleaved, plus the reference under MPICH on the same box: max total time per method.
#   launch      default: engine segments launched inside the timed region (like-for-like with
#               the reference's total_time, which brackets its request posts)
#   armed       XG_ENGINE_ARM=1: single-segment plans launched before the timed region and
#               started by the host's doorbell ring (the launch stays outside the time)
#   grid_launch XG_ENGINE_SOLO=0 (grid-barrier engine), launched
#   copy1       XG_SOLO_MIN_STEPS=2: a one-step plan runs as an event-timed copy launch
#   nograph     XG_GRAPH=0: launch-bound one-GPU runs (TAM chains) launched, not replayed as a graph
# usage: profiles/chain_modes.sh <outdir> [reps]
out=${1:-gpurun_out/chain}; reps=${2:-3}; mkdir -p $out
args="-a 14 -d 2048 -c 3 -m 0 -i 2 -k 1"
repo=$PWD; bin=$repo/mpi-asynchronous-communication-test_amd/bin/test
cd $out
for r in $(seq 1 $reps); do
  timeout -k 10 120 $bin --procs 32 $args > launch_$r.txt 2>> err.txt || exit 1
  XG_ENGINE_ARM=1 timeout -k 10 120 $bin --procs 32 $args > armed_$r.txt 2>> err.txt || exit 1
  XG_ENGINE_SOLO=0 timeout -k 10 120 $bin --procs 32 $args > grid_launch_$r.txt 2>> err.txt || exit 1
  XG_SOLO_MIN_STEPS=2 timeout -k 10 120 $bin --procs 32 $args > copy1_$r.txt 2>> err.txt || exit 1
  XG_GRAPH=0 timeout -k 10 120 $bin --procs 32 $args > nograph_$r.txt 2>> err.txt || exit 1
done
if [ -x $repo/oracle/_ref/test ] && [ -z "$NOREF" ]; then
  for r in $(seq 1 $reps); do
    timeout -k 10 300 /opt/conda/bin/mpiexec -launcher fork -n 32 $repo/oracle/_ref/test $args > ref_$r.txt 2>> ref.err || echo "reference run failed"
  done
fi
echo done
