#!/bin/bash
# Round 5 probe: several ranks of one job on the box's ONE GPU over RCCL (XG_SHARE_GPU=1:
# every rank names a host of its own, so RCCL pairs them over its socket transport).
# Exercises the real multi-rank path: ncclCommInitRank with nranks > 1, enqueue_step's
# groups to real peers, xg_barrier / xg_allreduce_max across processes.
set -o pipefail
out=gpurun_out/r05_share
mkdir -p $out
B=mpi-asynchronous-communication-test_amd/bin
export XG_SHARE_GPU=1 NCCL_DEBUG=WARN
stop() { case $1 in 124|137|134|139) echo "stopping after rc=$1"; exit $1;; esac; }
echo "== bin/test --gpus 2 README config, every method, verify" | tee $out/summary.txt
timeout -k 10 180 $B/test --gpus 2 --procs 32 -a 14 -d 2048 -c 3 -m 0 -i 1 -k 1 --verify > $out/cli2.txt 2> $out/cli2.err
rc=$?; echo "rc=$rc" | tee -a $out/summary.txt; grep -c "verify = OK" $out/cli2.txt | tee -a $out/summary.txt; stop $rc
tail -5 $out/cli2.err
echo "== bench.py --gpus 2" | tee -a $out/summary.txt
timeout -k 10 400 python3 -u bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --baseline-configs off > $out/bench2.json 2> $out/bench2.err
rc=$?; echo "rc=$rc" | tee -a $out/summary.txt; stop $rc
tail -c 3000 $out/bench2.json; tail -5 $out/bench2.err
