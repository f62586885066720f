#!/bin/bash
# configs[4] -c sweep: the HIP path at -d 8 MiB (profiles/configs4_sweep.py) and the reference
# under MPICH on the box's host cores at a REDUCED -d 64 KiB (1 TiB per direction does not fit a
# host; 256 MPI processes share the box's CPUs, so these are oversubscribed -- labelled so).
out=${1:-gpurun_out/configs4}; mkdir -p $out
timeout -k 10 300 python3 profiles/configs4_sweep.py > $out/gpu_d8m.txt 2> $out/gpu.err || exit 1
if [ -x oracle/_ref/test ]; then
  nproc > $out/host_cpus.txt
  cd /tmp
  for c in 1 2 3 4 5 6 7 8; do
    for m in 7 11 12; do
      timeout -k 5 60 /opt/conda/bin/mpiexec -launcher fork -n 256 $OLDPWD/oracle/_ref/test -a 64 -d 65536 -c $c -m $m -i 1 -k 1 \
        > $OLDPWD/$out/ref_m${m}_c$c.txt 2>> $OLDPWD/$out/ref.err || echo "m$m c$c: no result (exit $?)" >> $OLDPWD/$out/ref.err
    done
  done
fi
echo done
