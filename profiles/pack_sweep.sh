#!/bin/bash
# HISTORICAL RECIPE: it sets XG_* knobs folded into constants by commit 88b890f (round 4);
# rerun now, those arms are identical (libxg warns about each such variable).  Kept as the record.
# pack/unpack launch rate vs copy piece size and kernel variant (profiles/pack_virtual.py under rocprofv3)
export TMPDIR=/tmp
for v in ${VARIANTS:-5 13}; do for ch in ${CHUNKS:-16384 32768 65536}; do
  o=$PWD/gpurun_out/packsw_${v}_$ch; mkdir -p $o
  XG_COPY_VARIANT=$v XG_COPY_CHUNK=$ch REPS=5 timeout -k 10 120 rocprofv3 --kernel-trace -d $o/kt -o run --output-format csv -- python3 profiles/pack_virtual.py > $o/run.txt 2>&1 || exit 1
  echo "variant=$v chunk=$ch"; XG_COPY_CHUNK=$ch python3 profiles/pack_summary.py $(find $o/kt -name run_kernel_trace.csv | head -1) || exit 1
done; done
