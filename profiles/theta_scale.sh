#!/bin/bash
# The reference's own Theta sweep (script_theta_all_to_many_256.sh: 16384 processes = 256 KNL
# nodes x 64, -a 256 -d 2048 -m 1 -i 5, -c 1 .. 16384) with all 16384 logical ranks on ONE
# MI355X through the drop-in CLI (-i 2 here), every -c of the script.  usage: profiles/theta_scale.sh <outdir>
out=${1:-gpurun_out/theta}; mkdir -p $out; cd $out
bin=$GRAFT_REPO_ROOT/mpi-asynchronous-communication-test_amd/bin/test
m=${THETA_METHOD:-1}      # 1: script_theta_all_to_many_256.sh, 2: script_theta_many_to_all_256.sh
cs=${THETA_CS:-"1 2 4 8 16 32 64 128 256 512 1024 2048 4096 8192 16384"}
for c in $cs; do
  t0=$(date +%s.%N)
  timeout -k 10 240 $bin --procs 16384 -a 256 -d 2048 -c $c -m $m -i 2 > theta_c$c.txt 2>> err.txt || { echo "c=$c failed"; exit 1; }
  python3 -c "import sys; print(\"c=%s wall %.1f s\" % (sys.argv[1], float(sys.argv[3]) - float(sys.argv[2])))" $c $t0 $(date +%s.%N) >> theta_c$c.txt
done
grep -H "max total time\|wall" theta_c*.txt err.txt > summary.txt
echo done
