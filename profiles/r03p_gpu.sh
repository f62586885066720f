#!/bin/bash
# Round 3, call P: TAM stage copies sharing the local launch (XG_FUSE_STAGE).  GPU tests (the new
# one, TAM parity, golden configs), then the README configuration's m15 / m16 through the CLI with
# the fusion off and on, interleaved 5 times (max total time per experiment).
export TMPDIR=/tmp
o=$PWD/gpurun_out/r03p; mkdir -p $o
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "tam or golden_all or graph_replay" --timeout 200 \
  --timeout-method thread -p no:cacheprovider > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
bin=$PWD/mpi-asynchronous-communication-test_amd/bin/test
cd $o
for r in 1 2 3 4 5; do
  for f in 0 1; do
    for m in 15 16; do
      XG_FUSE_STAGE=$f timeout -k 10 60 $bin --procs 32 -a 14 -d 2048 -c 3 -m $m -i 2 -k 1 --verify > cli_f${f}_m${m}_$r.txt 2>> err.txt || exit 1
      grep -q "verify = OK" cli_f${f}_m${m}_$r.txt || { cat cli_f${f}_m${m}_$r.txt; exit 1; }
      grep "max total_time\|max total time" cli_f${f}_m${m}_$r.txt | sed "s/^/fuse=$f m=$m run=$r /" >> summary.txt
    done
  done
done
cat summary.txt
