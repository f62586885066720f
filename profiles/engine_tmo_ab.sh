#!/bin/bash
# step-engine A/B: barrier waiters read the timeout word every poll (1, the old engine) or every 64 polls (64)
B=$PWD/mpi-asynchronous-communication-test_amd/bin/test
for trial in 1 2 3; do for m in 6 9 11 12 1; do for p in 1 64; do
 t=$(cd /tmp && XG_ENGINE_TMO_EVERY=$p timeout -k 5 60 $B --procs 32 -a 14 -d 2048 -c 3 -m $m -i 2 -k 3 | grep "max total" | sed 's/.*= //' | tr '\n' ' ') || exit 1
 echo "t$trial m$m tmo_every=$p $t"
done; done; done
