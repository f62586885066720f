#!/bin/bash
# round 4, call E: the XCD-order A/B, then the bench under rocprofv3 + the two PMC passes
set -o pipefail
bash profiles/r04_xcd_ab.sh && bash profiles/bench_rocprof.sh r04
