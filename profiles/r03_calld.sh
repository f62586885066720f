#!/bin/bash
# Round 3, call D: the CLI-default cross-GPU form on the virtual 8-GPU README job, the ADVICE
# grid_pays re-run, then the missing configs[4] reference cells on the box's CPUs.
out=${1:-gpurun_out/r03d}; mkdir -p $out
FORMS="self_in_group" bash profiles/r03_hybrid.sh $PWD/$out/hybrid_default > /dev/null || exit 1
for pm in 65536; do
  XG_SELF_MAX=262144 PACK=4194304 PACK_MIN=$pm REPS=20 timeout -k 10 180 python3 profiles/hybrid_virtual.py > $out/hybrid_cli_default.txt 2>&1 || exit 1
done
cat $out/hybrid_default/run_*.txt $out/hybrid_cli_default.txt
bash profiles/grid_pays_rerun.sh $out/grid_pays || exit 1
mkdir -p $out/configs4_ref && cp profiles/r03/configs4_ref_box/ref_d4096.txt $out/configs4_ref/ref_d4096.txt
timeout -k 10 900 python3 -u profiles/configs4_ref.py $out/configs4_ref/ref_d4096.txt 4096 100
