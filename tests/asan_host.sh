#!/bin/bash
# Host half (libxghost: placement, per-rank programs, matching, step compiler, device plans)
# under AddressSanitizer + UndefinedBehaviorSanitizer, driven by the CPU tests.  CPU only.
# usage: tests/asan_host.sh            (exit 0 = no sanitizer report, all tests passed)
set -e
REPO=$(cd "$(dirname "$0")/.." && pwd)
OUT=$(mktemp -d /tmp/xg_asan.XXXXXX)
gcc -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=all \
    -Wall -Wextra -fPIC -std=c99 -D_POSIX_C_SOURCE=200809L -I"$REPO/include" -shared -o "$OUT/libxghost.so" \
    "$REPO/mpi-asynchronous-communication-test_amd/csrc/host/programs.c" "$REPO/mpi-asynchronous-communication-test_amd/csrc/host/sched.c" "$REPO/mpi-asynchronous-communication-test_amd/csrc/host/devplan.c" \
    "$REPO/mpi-asynchronous-communication-test_amd/csrc/host/report.c" \
    "$REPO/mpi-asynchronous-communication-test_amd/csrc/host/hazard.c" "$REPO/mpi-asynchronous-communication-test_amd/csrc/host/solo.c" \
    "$REPO/mpi-asynchronous-communication-test_amd/csrc/host/calls.c" "$REPO/mpi-asynchronous-communication-test_amd/csrc/host/pieces.c"
cd "$REPO/tests"
# the sanitizer runtimes go first in LD_PRELOAD (ASan must be the first DSO); whatever the
# environment already preloads stays after them
LD_PRELOAD="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libubsan.so)${LD_PRELOAD:+ $LD_PRELOAD}" ASAN_OPTIONS=detect_leaks=0 \
    XG_LIBDIR="$OUT" python -m pytest test_host_sched.py test_devplan.py test_oracle.py test_engine_hazards.py test_hbm_fit.py test_solo_tables.py test_rccl_calls.py test_relay.py test_baseline_golden.py test_timed_steps.py -q -s -m "not gpu" -p no:cacheprovider
rm -rf "$OUT"
