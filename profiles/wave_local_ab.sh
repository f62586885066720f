#!/bin/bash
# HISTORICAL RECIPE: it sets XG_* knobs folded into constants by commit 88b890f (round 4);
# rerun now, those arms are identical (libxg warns about each such variable).  Kept as the record.
# One-off GPU-local launches larger than the step engine's 16 MiB steps and below the 128 MiB
# non-temporal switch: m1 / m2 at P32 A14, one launch of 448 x d per -k repetition, d = 64 KiB
# .. 256 KiB (28 .. 112 MiB per launch; regions 56 .. 224 MiB, so the -k repetitions stay in the
# 256 MiB Infinity Cache), rocprofv3 kernel durations: mode nt = XG_COPY_VARIANT=6 (non-temporal
# copy_kernel_g<4>, what these launches ran before the footprint rule), g = XG_COPY_WAVE=0
# (plain copy_kernel_g<4>, balanced pieces), w = the default (copy_kernel_w<8>); interleaved
# twice; --verify checks every byte.
export TMPDIR=/tmp
o=${1:-$PWD/gpurun_out/wave_local}; mkdir -p $o
bin=$PWD/mpi-asynchronous-communication-test_amd/bin/test
for rep in 1 2; do
for d in 65536 131072 262144; do
  for w in nt g w; do
    for m in 1 2; do
      case $w in nt) ev="XG_COPY_VARIANT=6";; g) ev="XG_COPY_WAVE=0";; w) ev="XG_COPY_WAVE=1";; esac
      ( export $ev; timeout -k 10 120 rocprofv3 --kernel-trace -d $o/kt_${d}_${w}_$m -o run --output-format csv -- \
        $bin --procs 32 -a 14 -d $d -m $m -k 50 -i 1 --verify > $o/cli_${d}_${w}_$m.txt 2>> $o/err.txt ) || exit 1
      python3 - $(find $o/kt_${d}_${w}_$m -name run_kernel_trace.csv) $d $w $m >> $o/summary.txt <<'PY' || exit 1
import csv, statistics, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "copy_kernel" in r["Kernel_Name"]]
d, w, m = int(sys.argv[2]), sys.argv[3], int(sys.argv[4])
ds = sorted(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows)[5:]   # warm launches
names = sorted({r["Kernel_Name"].split("(")[0].replace("void ", "") for r in rows})
med = statistics.median(ds) / 1e3
print("m%d d=%-6d mode=%-2s %s launches=%d median_us=%.2f HBM_GBps=%.0f" % (
    m, d, w, names, len(ds), med, 2 * 448 * d / med / 1e3))
PY
      rm -rf $o/kt_${d}_${w}_$m
      grep -q "verify = OK" $o/cli_${d}_${w}_$m.txt || { echo "verify failed"; cat $o/cli_${d}_${w}_$m.txt; exit 1; }
    done
  done
done
done
cat $o/summary.txt
