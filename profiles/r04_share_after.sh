#!/bin/bash
# round 4: configs[4]'s stated-size GPU-0 share after the step-mark changes (every -c)
set -o pipefail
O=gpurun_out/r04_share_after
mkdir -p $O
timeout -k 10 600 python3 -u profiles/configs4_share.py > $O/configs4_share.txt 2>&1
