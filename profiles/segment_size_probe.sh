#!/bin/bash
# one-launch exchange copy rate vs segment size at P32 A14 (m1, -k 10, step engine off)
B=$PWD/mpi-asynchronous-communication-test_amd/bin/test
for r in 1 2; do for d in 524288 1048576 1572864 2097152 3145728 4194304 6291456 8388608 12582912 16777216; do
  t=$(cd /tmp && XG_ENGINE_MAX_STEP=0 timeout -k 5 120 $B --procs 32 -a 14 -d $d -m 1 -i 1 -k 10 | grep "max total" | sed 's/.*= //') || exit 1
  python3 -c "P,d,t=32,$d,$t; B=P*14*d; print('seg=%5.2f MiB launch=%6.0f MiB HBM_GBps=%.0f' % (d/2**20,B/2**20,2*B*10/t/1e9))"
done; done
