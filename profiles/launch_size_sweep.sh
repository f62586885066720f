#!/bin/bash
# copy rate of one exchange launch vs its size: m1 (default -c: one step, one copy_kernel launch),
# A14, -k 5, step engine off; delivered GB/s = P*A*d*k / max total (HBM traffic = 2x)
B=$PWD/mpi-asynchronous-communication-test_amd/bin/test
for pd in "32 1048576" "64 1048576" "128 1048576" "256 1048576" "32 4194304" "32 262144" "256 4194304"; do
  set -- $pd
  t=$(cd /tmp && XG_ENGINE_MAX_STEP=0 timeout -k 5 120 $B --procs $1 -a 14 -d $2 -m 1 -i 1 -k 5 | grep "max total" | sed 's/.*= //') || exit 1
  python3 -c "P,d,t=$1,$2,$t; B=P*14*d; print('P=%d d=%d launch=%.0f MiB  per_launch_us=%.1f  delivered_GBps=%.0f  HBM_GBps=%.0f' % (P,d,B/2**20,t/5*1e6,B*5/t/1e9,2*B*5/t/1e9))"
done
