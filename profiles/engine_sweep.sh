#!/bin/bash
# Step engine (one persistent launch per plan) vs one launch + event per step, on the
# multi-step GPU-local schedules, P32 A14 -c 3 on one MI355X.
# Prints: method d  auto(built-in choice)  engine(step engine at every step size)
#         eager(one launch per step)   (max total time, s, -k 3)
out=${1:-gpurun_out/engine_sweep.txt}; : > $out
B=$PWD/mpi-asynchronous-communication-test_amd/bin/test
run() { (cd /tmp && env "$@" timeout -k 5 60 $B --procs 32 -a 14 -d $d -c 3 -m $m -i 1 -k 3 | grep "max total" | sed 's/.*= //'); }
for m in ${METHODS:-1 6 9 11 12}; do for d in ${SIZES:-2048 16384 65536 262144 1048576}; do
  [ $m = 6 ] && [ $d -gt 65424 ] && continue      # the reference deadlocks there (refused)
  au=$(run XG_UNUSED=0) || exit 1
  gr=$(run XG_ENGINE_MAX_STEP=1073741824) || exit 1
  g=$(run XG_ENGINE_MAX_STEP=0) || exit 1
  echo "m$m d=$d auto=$au engine=$gr eager=$g" | tee -a $out
done; done
