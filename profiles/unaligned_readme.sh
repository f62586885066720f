#!/bin/bash
out=gpurun_out/unaligned; mkdir -p $out; cd $out
bin=$GRAFT_REPO_ROOT/mpi-asynchronous-communication-test_amd/bin/test
for d in 1000 2048 24; do
  timeout -k 10 120 $bin --procs 32 -a 14 -d $d -c 3 -m 0 -i 2 -k 1 > cli_d$d.txt 2>> err.txt || exit 1
  timeout -k 10 300 /opt/conda/bin/mpiexec -launcher fork -n 32 $GRAFT_REPO_ROOT/oracle/_ref/test -a 14 -d $d -c 3 -m 0 -i 2 -k 1 > ref_d$d.txt 2>> ref.err || echo "ref failed d=$d"
done
echo done
