#!/bin/bash
# Copy-kernel tuning sweep on the bench workload (configs[1]); one JSON line per point.
# usage: profiles/sweep_copy.sh <out file> "<variants>" "<chunks>"
out=${1:-gpurun_out/sweep.txt}; variants=${2:-"0 1 2 3 4"}; chunks=${3:-"16384 32768 65536 131072 229376 262144"}
for v in $variants; do for ch in $chunks; do
  r=$(timeout -k 5 60 python3 bench.py --no-cpu-baseline --steps 20 --warmup 3 --copy-variant $v --chunk $ch) || exit 1
  python3 -c "import json,sys; d=json.loads(sys.argv[1]); print('variant=%s chunk=%s value=%.1f achieved=%.1f avg_us=%.1f' % (sys.argv[2], sys.argv[3], d['value'], d['roofline']['achieved'], d['roofline']['avg_launch_us']))" "$r" $v $ch | tee -a $out
done; done
