#!/bin/bash
# Solo engine on rails: per-step stamps of the README chains under every rail count / engine
# form (solo_probe.py), then the README configuration through the CLI beside the reference
# under MPICH on the same box (chain_modes.sh, 3 runs each).  usage: profiles/r02_rails.sh <outdir>
out=${1:-gpurun_out/r02_rails}; mkdir -p $out
timeout -k 10 150 python3 -u profiles/solo_probe.py > $out/solo_probe.txt 2>&1 || exit 1
bash profiles/chain_modes.sh $out/chain 3 || exit 1
python3 profiles/chain_summary.py $out/chain > $out/chain_summary.txt || exit 1
echo done
