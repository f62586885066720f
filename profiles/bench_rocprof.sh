#!/bin/bash
# The bench line and the rocprofv3 kernel summary of the same command (one run), plus the two
# PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs) reduced to HBM bytes per copy launch.
# usage: profiles/bench_rocprof.sh <round tag, e.g. r01>
tag=${1:-r01}; out=$PWD/gpurun_out/prof_$tag; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/kt -o run --output-format csv -- \
  python3 bench.py ${BENCH_ARGS:-} > $out/bench.json 2> $out/bench.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o run --output-format csv -- \
  python3 bench.py ${BENCH_ARGS:-} --no-cpu-baseline --steps 5 --warmup 1 > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $out/write -o run --output-format csv -- \
  python3 bench.py ${BENCH_ARGS:-} --no-cpu-baseline --steps 5 --warmup 1 > /dev/null 2>&1 || exit 1
f=$(find $out/fetch -name run_counter_collection.csv | head -1); w=$(find $out/write -name run_counter_collection.csv | head -1)
python3 profiles/pmc_summary.py $(dirname $f) $(dirname $w) $out/pmc_traffic.json "$tag: bench.py ${BENCH_ARGS:-} (rocprofv3 --pmc, separate passes)" > /dev/null || exit 1
cp $(find $out/kt -name run_kernel_stats.csv | head -1) $out/kernel_stats.csv
echo done
