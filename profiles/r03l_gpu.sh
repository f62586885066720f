#!/bin/bash
# HISTORICAL RECIPE: it sets XG_* knobs folded into constants by commit 88b890f (round 4);
# rerun now, those arms are identical (libxg warns about each such variable).  Kept as the record.
# Round 3, call L: the wave-persistent copy (copy_kernel_w) A/B.  (1) one GPU's configs[2] pack
# launch standalone (28 MiB out of its own 32 MiB: cache-resident as on a real 8-GPU node), both
# pack orders, product copy_kernel_g<4> 16 KiB vs copy_kernel_w<8> 8 KiB, interleaved 3 times;
# (2) the configs[2] 8-GPU plans on this device under rocprofv3 kernel traces, XG_COPY_WAVE=0 vs 1,
# reduced to launch classes; (3) the N = 1 bench (its 448 MiB launches are non-temporal and stay
# copy_kernel_g: no change expected).
export TMPDIR=/tmp
o=$PWD/gpurun_out/r03l; mkdir -p $o
for rep in 1 2 3; do
  KINDS=18,22,26,27 SIZES_MIB=32 timeout -k 10 120 python3 profiles/copy_ceiling.py >> $o/probe.txt 2>&1 || { cat $o/probe.txt; exit 1; }
done
cat $o/probe.txt
for w in 0 1; do
  XG_COPY_WAVE=$w FORMS=packed_two_sided,packed_one_sided REPS=10 timeout -k 10 240 rocprofv3 --kernel-trace -d $o/kt$w -o run --output-format csv -- python3 profiles/pack_forms.py > $o/pack_forms_wave$w.txt 2>&1 || { tail -20 $o/pack_forms_wave$w.txt; exit 1; }
  python3 profiles/kernel_classes.py $(find $o/kt$w -name run_kernel_trace.csv) > $o/classes_wave$w.txt || exit 1
  rm -rf $o/kt$w
  echo "== XG_COPY_WAVE=$w"; grep "^m" $o/pack_forms_wave$w.txt; cat $o/classes_wave$w.txt
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $o/bench.json 2> $o/bench.err || { tail -20 $o/bench.err; exit 1; }
cut -c1-400 $o/bench.json
echo done
