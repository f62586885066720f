#!/bin/bash
# HISTORICAL RECIPE: it sets XG_* knobs folded into constants by commit 88b890f (round 4);
# rerun now, those arms are identical (libxg warns about each such variable).  Kept as the record.
# Bench copy launches per method by piece size (XG_COPY_CHUNK; pieces in destination order),
# rocprofv3 kernel traces.  usage: profiles/chunk_ab.sh <outdir>
out=${1:-gpurun_out/chunk_ab}; mkdir -p $out
export TMPDIR=/tmp
for ch in 32768 65536 131072 16384; do
  XG_COPY_CHUNK=$ch timeout -k 10 300 rocprofv3 --kernel-trace -d $out/kt$ch -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline > $out/bench_$ch.json 2> /dev/null || exit 1
  echo "chunk $ch" >> $out/summary.txt
  python3 profiles/bench_per_method.py $(find $out/kt$ch -name run_kernel_trace.csv | head -1) >> $out/summary.txt || exit 1
done
echo done
