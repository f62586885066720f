#!/bin/bash
# Very large copy launches as one launch (XG_COPY_LAUNCH_MAX=0) or as back-to-back launches of
# about 512 MiB (default), interleaved x2, through the CLI: BASELINE configs[3] m1 / m2 (one 32 GiB
# step of 4 MiB segments) and the Theta shape at -c 16384 (one 8 GiB step of 2 KiB segments).
# usage: profiles/launch_split_ab.sh <outdir>
out=${1:-gpurun_out/launch_split}; mkdir -p $out; cd $out
bin=$GRAFT_REPO_ROOT/mpi-asynchronous-communication-test_amd/bin/test
for r in 1 2; do
  for lm in 0 536870912; do
    for m in 1 2; do
      XG_COPY_LAUNCH_MAX=$lm timeout -k 10 120 $bin --procs 256 -a 32 -d 4194304 -m $m -i 2 > cfg3_m${m}_max${lm}_$r.txt 2>>err.txt || exit 1
    done
    XG_COPY_LAUNCH_MAX=$lm timeout -k 10 120 $bin --procs 16384 -a 256 -d 2048 -c 16384 -m 1 -i 2 > theta_max${lm}_$r.txt 2>>err.txt || exit 1
  done
done
for f in cfg3_*.txt theta_*.txt; do echo "$f $(grep 'max total time' $f | sed 's/.*= //' | tr '\n' ' ')"; done | sort > summary.txt
echo done
