#!/bin/bash
# round 4: configs[4]'s GPU-0 share (P256 A64 -d 64 MiB, 256 GiB of regions) for m11 -c 1 and
# m12 -c 8 under rocprofv3 --kernel-trace --stats (3 runs each), and one run each under the two
# PMC passes (FETCH_SIZE, WRITE_SIZE: separate runs) -> gpurun_out/r04_share/
set -o pipefail
O=$PWD/gpurun_out/r04_share
mkdir -p $O
export TMPDIR=/tmp
for cell in 11:1 12:8; do
  t=${cell/:/_c}
  CELLS=$cell REPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_m$t -o run --output-format csv -- \
      python3 profiles/configs4_share.py > $O/share_m$t.txt 2>&1 || exit 1
  CELLS=$cell REPS=1 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_m$t -o run --output-format csv -- \
      python3 profiles/configs4_share.py > $O/share_m${t}_fetch.txt 2>&1 || exit 1
  CELLS=$cell REPS=1 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/write_m$t -o run --output-format csv -- \
      python3 profiles/configs4_share.py > $O/share_m${t}_write.txt 2>&1 || exit 1
done
echo done > $O/done.txt
