#!/bin/bash
# HISTORICAL RECIPE: it sets XG_* knobs folded into constants by commit 88b890f (round 4);
# rerun now, those arms are identical (libxg warns about each such variable).  Kept as the record.
# One-step GPU-local plans (m5 / m8 alltoallw, m1 / m2 with -c >= P) at README size: a copy launch
# timed by events (XG_SOLO_MIN_STEPS=2, default) vs an armed solo launch (XG_SOLO_MIN_STEPS=1),
# interleaved, through the CLI.  usage: profiles/one_step_ab.sh <outdir>
out=${1:-gpurun_out/one_step}; mkdir -p $out; cd $out
bin=$GRAFT_REPO_ROOT/mpi-asynchronous-communication-test_amd/bin/test
for r in 1 2 3; do
  for d in 2048 1000; do
    for ms in 2 1; do
      XG_SOLO_MIN_STEPS=$ms timeout -k 10 60 $bin --procs 32 -a 14 -d $d -m 5 -i 3 -k 1 > m5_d${d}_min${ms}_$r.txt 2>> err.txt || exit 1
      XG_SOLO_MIN_STEPS=$ms timeout -k 10 60 $bin --procs 32 -a 14 -d $d -m 8 -i 3 -k 1 > m8_d${d}_min${ms}_$r.txt 2>> err.txt || exit 1
      XG_SOLO_MIN_STEPS=$ms timeout -k 10 60 $bin --procs 32 -a 14 -d $d -m 1 -i 3 -k 1 > m1_d${d}_min${ms}_$r.txt 2>> err.txt || exit 1
    done
  done
done
for f in *.txt; do [ "$f" = err.txt ] || echo "$f $(grep 'max total time' $f | sed 's/.*= //' | tr '\n' ' ')"; done > summary.txt
echo done
