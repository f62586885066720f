#!/bin/bash
# HISTORICAL RECIPE: it sets XG_* knobs folded into constants by commit 88b890f (round 4);
# rerun now, those arms are identical (libxg warns about each such variable).  Kept as the record.
B=$PWD/mpi-asynchronous-communication-test_amd/bin/test
for m in 6 9 11 12 1; do for w in 1 2 4 8 16 256; do
 t=$(cd /tmp && XG_ENGINE_WG=$w timeout -k 5 60 $B --procs 32 -a 14 -d 2048 -c 3 -m $m -i 2 -k 3 | grep "max total" | sed 's/.*= //' | tr '\n' ' ') || exit 1
 echo "m$m wg=$w $t"
done; done
