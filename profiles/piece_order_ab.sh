#!/bin/bash
# HISTORICAL RECIPE: it sets XG_* knobs folded into constants by commit 88b890f (round 4);
# rerun now, those arms are identical (libxg warns about each such variable).  Kept as the record.
# Bench copy launches per method under each local-piece order (XG_PIECE_ORDER 0 message order,
# 1 by destination, 2 by source), rocprofv3 kernel traces; the contiguous copy ceiling of the
# same box beside it.  usage: profiles/piece_order_ab.sh <outdir>
out=${1:-gpurun_out/piece_order}; mkdir -p $out
export TMPDIR=/tmp
for o in 0 1 2; do
  XG_PIECE_ORDER=$o timeout -k 10 300 rocprofv3 --kernel-trace -d $out/kt$o -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline > $out/bench_$o.json 2> /dev/null || exit 1
  echo "order $o" >> $out/summary.txt
  python3 profiles/bench_per_method.py $(find $out/kt$o -name run_kernel_trace.csv | head -1) >> $out/summary.txt || exit 1
done
KINDS=9 SIZES_MIB=448 timeout -k 10 100 python3 profiles/copy_ceiling.py >> $out/summary.txt 2>&1
echo done
