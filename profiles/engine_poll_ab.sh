#!/bin/bash
# step-engine barrier A/B: waiters poll the arrival counter (count) or a release word on its
# own cache line written by the last arriver (gen); README size, max total time (s), -k 3
B=$PWD/mpi-asynchronous-communication-test_amd/bin/test
for trial in 1 2 3; do for m in 6 9 11 12 1; do for p in count gen; do
 t=$(cd /tmp && XG_ENGINE_POLL=$p timeout -k 5 60 $B --procs 32 -a 14 -d 2048 -c 3 -m $m -i 2 -k 3 | grep "max total" | sed 's/.*= //' | tr '\n' ' ') || exit 1
 echo "t$trial m$m poll=$p $t"
done; done; done
