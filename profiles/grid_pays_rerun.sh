#!/bin/bash
# HISTORICAL RECIPE: it sets XG_* knobs folded into constants by commit 88b890f (round 4);
# rerun now, those arms are identical (libxg warns about each such variable).  Kept as the record.
# grid_pays used solo_max (1 GiB since a9cb48e) as "larger than the 256 MiB
# Infinity Cache", so engine runs of 256 MiB .. 1 GiB that do not go solo always took the grid
# engine.  Round 3 gives the cache its own constant (XG_GRID_CACHE_MAX, 256 MiB).  Re-run: a
# 512 MiB engine-eligible run with the solo engine off (P4096 A64 -d 2048 m1, -c 8: 512 steps of
# 1 MiB; -c 64: 64 steps of 8 MiB), old rule (XG_GRID_CACHE_MAX=1 GiB: always grid) vs new
# (cost model: grid vs chained launches), every byte verified.
out=${1:-gpurun_out/grid_pays}; mkdir -p $out
bin=$PWD/mpi-asynchronous-communication-test_amd/bin/test
for c in 8 64; do
  for rule in old new; do
    for r in 1 2 3; do
      if [ $rule = old ]; then export XG_GRID_CACHE_MAX=1073741824; else unset XG_GRID_CACHE_MAX; fi
      XG_ENGINE_SOLO=0 timeout -k 10 120 $bin --procs 4096 -a 64 -d 2048 -c $c -m 1 -i 1 -k 1 --verify > $out/c${c}_${rule}_$r.txt 2>> $out/err.txt || exit 1
      echo "c$c $rule run $r: $(grep -E 'max total time|verify' $out/c${c}_${rule}_$r.txt | tr '\n' ' ')" >> $out/summary.txt
    done
  done
done
unset XG_GRID_CACHE_MAX
cat $out/summary.txt
