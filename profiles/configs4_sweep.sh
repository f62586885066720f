#!/bin/bash
# BASELINE configs[4] (P256 A64, half-sync m7 / m11 / m12, -c 1..8) through the drop-in CLI on
# ONE MI355X at the largest -d it holds (8 MiB: 128 GiB SEND + 128 GiB RECV), every byte
# verified (--verify), and the reference under MPICH on the box's host cores at a REDUCED
# -d (64 KiB: 256 MPI processes on the box's CPU share are oversubscribed; labelled so).
# usage: profiles/configs4_sweep.sh <outdir>
out=${1:-gpurun_out/configs4}; mkdir -p $out
bin=$PWD/mpi-asynchronous-communication-test_amd/bin/test
cd $out
for c in 1 2 3 4 5 6 7 8; do
  for m in 7 11 12; do
    timeout -k 10 120 $bin --procs 256 --verify -a 64 -d 8388608 -c $c -m $m -i 1 -k 1 > gpu_m${m}_c$c.txt 2>> err.txt || exit 1
  done
done
if [ -x ../../oracle/_ref/test ]; then
  for c in 1 2 3 4 5 6 7 8; do
    for m in 7 11 12; do
      timeout -k 10 120 /opt/conda/bin/mpiexec -launcher fork -n 256 ../../oracle/_ref/test -a 64 -d 65536 -c $c -m $m -i 1 -k 1 > ref_m${m}_c$c.txt 2>> ref.err || echo "reference m$m c$c failed or timed out" >> ref.err
    done
  done
fi
echo done
