#!/bin/bash
# Round 2: copy-kernel store policy A/B inside the bench (interleaved, 2 rounds), then a
# rocprofv3 kernel trace of the bench per variant (launch durations and back-to-back gaps).
#   0 by size (nt >= 128 MiB)  1 copy_kernel_g<4> plain  2 copy_kernel_b<4> plain  3 sc1  4 nt
#   5 copy_kernel_b<8> nt   6 copy_kernel_g<4> nt loads + nt stores
out=gpurun_out/r02_copy_ab; mkdir -p $out
export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in 0 1 6 0 1 6; do
    timeout -k 10 120 python3 bench.py --no-cpu-baseline --copy-variant $v > $out/bench_v${v}_$rep.json || exit 1
  done
done
for v in 0 1; do
  timeout -k 10 180 rocprofv3 --kernel-trace -d $out/kt$v -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --copy-variant $v > $out/kt_bench_v$v.json 2> $out/kt_v$v.err || exit 1
  python3 profiles/trace_gaps.py $(find $out/kt$v -name run_kernel_trace.csv) copy_kernel > $out/gaps_v$v.txt || exit 1
done
echo done
