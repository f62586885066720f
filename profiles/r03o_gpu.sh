#!/bin/bash
# Round 3, call O: traffic of the product's cross-GPU copy launches at a real GPU's footprint --
# GPU 0's configs[2] share alone (profiles/share_launches.py, two-sided), separate FETCH_SIZE /
# WRITE_SIZE passes reduced per launch class (896 workgroups: the 28 MiB pack / unpack launches,
# 128: the 4 MiB local part).
export TMPDIR=/tmp
o=$PWD/gpurun_out/r03o; mkdir -p $o
REPS=10 timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $o/fetch -o run --output-format csv -- python3 profiles/share_launches.py > $o/fetch.txt 2>&1 || { tail $o/fetch.txt; exit 1; }
REPS=10 timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $o/write -o run --output-format csv -- python3 profiles/share_launches.py > $o/write.txt 2>&1 || { tail $o/write.txt; exit 1; }
PACK_CLASSES="896=29360128,128=4194304" python3 profiles/pack_pmc.py $(find $o/fetch -name run_counter_collection.csv) $(find $o/write -name run_counter_collection.csv) > $o/pmc.txt || exit 1
rm -rf $o/fetch $o/write
cat $o/pmc.txt
