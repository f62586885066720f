#!/bin/bash
# Round 3, final evidence at HEAD (one-sided pack form, wave-persistent copy): the -m gpu suite,
# the widened random sweep (default thresholds, then every cross-GPU launch on the wave copy),
# the README configuration per mode, smoke, the bench, and the bench under rocprofv3 with the
# two PMC passes.
export TMPDIR=/tmp
out=${1:-$PWD/gpurun_out/r03_final2}; mkdir -p $out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; grep FAILED $out/gpu_tests.log | head; exit 1; }
tail -1 $out/gpu_tests.log
XG_RANDOM_N1=600 XG_RANDOM_NV=300 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_random.py -m gpu -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > $out/random_sweep_600_300.log 2>&1 || { tail -30 $out/random_sweep_600_300.log; exit 1; }
tail -1 $out/random_sweep_600_300.log
XG_COPY_WAVE_MIN=0 XG_RANDOM_NV=300 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_random.py -m gpu -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider -k virtual > $out/random_sweep_wave_all.log 2>&1 || { tail -30 $out/random_sweep_wave_all.log; exit 1; }
tail -1 $out/random_sweep_wave_all.log
bash profiles/chain_modes.sh $out/readme_cli 3 > /dev/null || exit 1
python3 profiles/chain_summary.py $out/readme_cli > $out/readme_cli/summary.txt || exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as G; G.smoke()" > $out/smoke.txt 2>&1 || exit 1
cat $out/smoke.txt
timeout -k 10 300 python3 -u bench.py > $out/bench.json 2> $out/bench.err || exit 1
cut -c1-300 $out/bench.json
bash profiles/bench_rocprof.sh r03final > $out/bench_rocprof.txt 2>&1 || { cat $out/bench_rocprof.txt; exit 1; }
cp -r gpurun_out/prof_r03final $out/ 2>/dev/null; rm -rf $out/prof_r03final/kt $out/prof_r03final/fetch $out/prof_r03final/write
echo done
