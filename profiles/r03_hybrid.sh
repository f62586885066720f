#!/bin/bash
# Cross-GPU step forms on the README configuration as a virtual 8-GPU job (RCCL self send/recv
# on one MI355X), packed and direct, rocprofv3 kernel traces (launches the device saw):
#   split           round 2: local gather on the side stream (fork/join events): XG_SELF_MAX=0 XG_SPLIT_MIN=0
#   local_in_fused  XG_SELF_MAX=0 XG_SPLIT_MIN=huge: the local part joins the step's (fused) pack launch
#   self_in_group   XG_SELF_MAX=huge: the local part goes in the step's RCCL group as self send/recv
#                   (the round-3 default at these sizes: local parts <= 256 KiB)
#   *_graph         the same with XG_GRAPH=1: the job captured once into a hipGraph and replayed
export TMPDIR=/tmp
o=${1:-$PWD/gpurun_out/r03_hybrid}; mkdir -p $o
for form in ${FORMS:-split local_in_fused self_in_group split_graph local_in_fused_graph self_in_group_graph}; do
  unset XG_GRAPH; export XG_SELF_MAX=0 XG_SPLIT_MIN=0
  case $form in local_in_fused*) export XG_SPLIT_MIN=1099511627776;; esac
  case $form in self_in_group*) export XG_SELF_MAX=1073741824;; esac
  case $form in *_graph) export XG_GRAPH=1;; esac
  for pack in 4194304 0; do
    PACK=$pack REPS=20 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $o/kt_${form}_$pack -o run --output-format csv -- \
      python3 profiles/hybrid_virtual.py > $o/run_${form}_$pack.txt 2> $o/run_${form}_$pack.err || exit 1
    cp $(find $o/kt_${form}_$pack -name run_kernel_stats.csv) $o/stats_${form}_$pack.csv
    rm -rf $o/kt_${form}_$pack
  done
done
echo done
