#!/bin/bash
# two RCCL ranks on GPU 0 (experiment): does RCCL accept it?
export MASTER_PORT=29555 TORCHELASTIC_RUN_ID=mp2test XG_DEVICE=0 WORLD_SIZE=2
RANK=0 LOCAL_RANK=0 timeout -k 5 120 python3 -u bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/mp2_r0.txt 2>&1 &
p0=$!
RANK=1 LOCAL_RANK=1 timeout -k 5 120 python3 -u bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/mp2_r1.txt 2>&1 &
p1=$!
wait $p0; r0=$?; wait $p1; r1=$?
echo "rc $r0 $r1"
