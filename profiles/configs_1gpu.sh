#!/bin/bash
# BASELINE.json configs 1-4 (0-based) through the drop-in CLI with every logical rank on ONE MI355X,
# beside the reference under MPICH on the same box's host cores where the process count allows
# (P <= 64; 256 MPI processes on the box's CPU share would only measure oversubscription).
# Prints: config method d c | GPU max total (s), GB/s | reference max total (s), GB/s
B=$PWD/mpi-asynchronous-communication-test_amd/bin/test
REF=$PWD/oracle/_ref/test
MPIEXEC=$(command -v mpiexec || echo /opt/conda/bin/mpiexec)
row() {   # name P A d c k method
  local name=$1 P=$2 A=$3 d=$4 c=$5 k=$6 m=$7 g r gb rb
  g=$(cd /tmp && timeout -k 10 300 $B --procs $P -a $A -d $d -c $c -m $m -i 1 -k $k | grep "max total" | sed 's/.*= //') || return 1
  gb=$(python3 -c "print('%.1f' % ($P*$A*$d*$k/$g/1e9))")
  r="-"; rb="-"
  if [ $P -le 64 ] && [ -x $REF ]; then
    r=$(cd /tmp && timeout -k 10 300 $MPIEXEC -launcher fork -n $P $REF -a $A -d $d -c $c -m $m -i 1 -k $k 2>/dev/null | grep "max total" | sed 's/.*= //')
    [ -n "$r" ] && rb=$(python3 -c "print('%.2f' % ($P*$A*$d*$k/$r/1e9))") || r="failed"
  fi
  printf "%-28s m%-2s d=%-9s c=%-9s gpu_max_total=%-10s gpu_GBps=%-8s ref_max_total=%-10s ref_GBps=%s\n" $name $m $d $c $g $gb $r $rb
}
for m in 1 2 3 4; do row "cfg1_p32_a14_d1M_k3" 32 14 1048576 200000000 3 $m || exit 1; done
for m in 5 8; do row "cfg2_p64_a16_d256K_k3" 64 16 262144 200000000 3 $m || exit 1; done
for m in 1 2 9 10; do row "cfg3_p256_a32_d4M_k1" 256 32 4194304 200000000 1 $m || exit 1; done
for c in 1 3 8; do for m in 7 11 12; do row "cfg4_p256_a64_d1M(reduced)_k1" 256 64 1048576 $c 1 $m || exit 1; done; done
