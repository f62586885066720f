#!/bin/bash
# one-launch exchanges (m1/m2, default -c: a single step) on one MI355X, P32 A14, one copy launch per run (step engine off):
# max total time vs XG_COPY_MIN_PIECES -- an experiment knob since removed (profiles/r01_min_pieces_ab.txt)
B=$PWD/mpi-asynchronous-communication-test_amd/bin/test
for d in 4096 16384 65536 262144; do for r in 1 2; do for mp in 1 1024 4096; do
  t=$(cd /tmp && XG_ENGINE_MAX_STEP=0 XG_COPY_MIN_PIECES=$mp timeout -k 5 60 $B --procs 32 -a 14 -d $d -m 1 -i 1 -k 20 | grep "max total" | sed 's/.*= //') || exit 1
  t2=$(cd /tmp && XG_ENGINE_MAX_STEP=0 XG_COPY_MIN_PIECES=$mp timeout -k 5 60 $B --procs 32 -a 14 -d $d -m 2 -i 1 -k 20 | grep "max total" | sed 's/.*= //') || exit 1
  echo "d=$d launch_MiB=$((32*14*d/1048576)) min_pieces=$mp m1=$t m2=$t2"
done; done; done
