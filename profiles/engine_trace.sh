#!/bin/bash
# README config through the CLI under rocprofv3 --kernel-trace: step-engine kernel duration
# vs the reported max total time, -k 1 and -k 3, methods 1 6 9 12
export TMPDIR=/tmp
B=$PWD/mpi-asynchronous-communication-test_amd/bin/test
o=$PWD/gpurun_out/etrace; mkdir -p $o
for m in 1 6 9 12; do for k in 1 3; do
  (cd /tmp && timeout -k 10 60 rocprofv3 --kernel-trace -d $o/m${m}k$k -o run --output-format csv -- \
     $B --procs 32 -a 14 -d 2048 -c 3 -m $m -i 2 -k $k > $o/m${m}k$k.txt 2>&1) || exit 1
  f=$(find $o/m${m}k$k -name run_kernel_trace.csv)
  python3 - "$f" "$o/m${m}k$k.txt" "$m" "$k" <<'PY'
import csv, re, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "step_engine" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
tot = re.findall(r"max total time = ([0-9.]+)", open(sys.argv[2]).read())
print("m%s k%s engine_us=%s reported_total=%s" % (sys.argv[3], sys.argv[4], d, tot))
PY
done; done
