#!/bin/bash
# configs[4] host-MPI baseline: the reference ./test (oracle/_ref/test) under MPICH, mpiexec -n 256,
# for m7 / m11 / m12 at every -c in 1..8, at a REDUCED -d (configs[4]'s 64 MiB is 1 TiB per
# direction: no host holds it).  256 MPI processes on the host's CPU share are oversubscribed
# (MPICH busy-polls); each cell gets its own time limit and a cell that does not finish says so.
# usage: profiles/configs4_ref.sh <outdir> <d> <limit_s>
out=${1:-gpurun_out/configs4_ref}; d=${2:-4096}; lim=${3:-120}
mkdir -p $out; repo=$PWD
echo "# host: $(nproc) CPUs visible, $(python3 -c 'import bench; print(bench.host_cpus())' 2>/dev/null)" > $out/ref_d$d.txt
cd /tmp
for c in 1 2 3 4 5 6 7 8; do
  for m in 7 11 12; do
    t0=$(date +%s.%N)
    r=$(timeout -k 5 $lim /opt/conda/bin/mpiexec -launcher fork -n 256 $repo/oracle/_ref/test -a 64 -d $d -c $c -m $m -i 1 -k 1 2>> $repo/$out/ref.err | grep "max total time")
    rc=$?; t1=$(date +%s.%N)
    if [ -n "$r" ]; then echo "m$m c$c d$d: $r  (wall $(python3 -c "print('%.1f' % ($t1 - $t0))") s)" >> $repo/$out/ref_d$d.txt
    else echo "m$m c$c d$d: did not finish in $lim s (exit $rc)" >> $repo/$out/ref_d$d.txt; fi
  done
done
echo done
