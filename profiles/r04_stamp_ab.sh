#!/bin/bash
# round 4: step marks as events vs clock stamps (profiles/stamp_marks_ab.py)
set -o pipefail
O=gpurun_out/r04_stamp_ab
mkdir -p $O
timeout -k 10 300 python3 -u profiles/stamp_marks_ab.py > $O/ab.txt 2>&1
