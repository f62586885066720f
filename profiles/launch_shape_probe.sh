#!/bin/bash
# one-launch exchange copy rate vs launch size and segment size (m1, A14, -k 10, step engine off)
B=$PWD/mpi-asynchronous-communication-test_amd/bin/test
run() { # P d
  t=$(cd /tmp && XG_ENGINE_MAX_STEP=0 timeout -k 5 120 $B --procs $1 -a 14 -d $2 -m 1 -i 1 -k 10 | grep "max total" | sed 's/.*= //') || exit 1
  python3 -c "P,d,t=$1,$2,$t; B=P*14*d; print('P=%-4d d=%-9d seg=%5.2f MiB launch=%6.0f MiB HBM_GBps=%.0f' % (P,d,d/2**20,B/2**20,2*B*10/t/1e9))"
}
for r in 1 2; do
  run 512 1048576; run 256 1048576
  run 64 4194304; run 64 8388608; run 32 16777216
  run 32 1048576; run 32 2097152; run 16 4194304
done
