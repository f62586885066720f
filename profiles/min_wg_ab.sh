#!/bin/bash
# (historical: the XG_COPY_MIN_WG rule was measured slower and removed after this A/B; run it at commit daa5908 or earlier)
# Piece size of small copy launches (XG_COPY_MIN_WG): standalone copy launches of m1 / m2 at
# P32 A14 (one launch of 448 x d per -k repetition; step engine off, so every repetition is a
# copy launch) for d = 8 KiB .. 128 KiB (3.5 .. 56 MiB per launch), rocprofv3 kernel durations
# with pieces of 32 KiB (XG_COPY_MIN_WG=0) and with the round-3 rule (>= 2 x CUs workgroups).
export TMPDIR=/tmp
o=${1:-$PWD/gpurun_out/min_wg}; mkdir -p $o
bin=$PWD/mpi-asynchronous-communication-test_amd/bin/test
for d in 8192 32768 131072; do
  for mw in 0 512; do
    for m in 1 2; do
      XG_ENGINE_MAX_STEP=0 XG_COPY_MIN_WG=$mw timeout -k 10 120 rocprofv3 --kernel-trace -d $o/kt_${d}_${mw}_$m -o run --output-format csv -- \
        $bin --procs 32 -a 14 -d $d -m $m -k 100 -i 1 > /dev/null 2>> $o/err.txt || exit 1
      python3 - $(find $o/kt_${d}_${mw}_$m -name run_kernel_trace.csv) $d $mw $m >> $o/summary.txt <<'PY' || exit 1
import csv, statistics, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "copy_kernel" in r["Kernel_Name"]]
d, mw, m = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
ds = sorted(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows)[5:]   # warm launches
wg = {int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]) for r in rows}
med = statistics.median(ds) / 1e3
print("m%d d=%-6d min_wg=%-3d workgroups=%s launches=%d median_us=%.2f HBM_GBps=%.0f" % (
    m, d, mw, sorted(wg), len(ds), med, 2 * 448 * d / med / 1e3))
PY
      rm -rf $o/kt_${d}_${mw}_$m
    done
  done
done
cat $o/summary.txt
