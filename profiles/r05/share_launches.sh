#!/bin/bash
# Round 5: one GPU's share of the 8-GPU configs[2] plans (profiles/share_launches.py: packs, the
# local part, unpacks; RCCL left out) at the current code, two-sided and one-sided, under
# rocprofv3 --kernel-trace (csv), reduced per launch class by kernel_classes.py.
set -o pipefail
export TMPDIR=/tmp
out=$PWD/gpurun_out/r05_share_launches
mkdir -p $out
for form in 0 1; do
    FORM=$form timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $out/f$form -o run -- \
        python3 profiles/share_launches.py > $out/f$form.log 2>&1 || { echo "form $form rc=$?"; tail -5 $out/f$form.log; exit 1; }
    f=$(find $out/f$form -name 'run_kernel_trace.csv' | head -1)
    { echo "== FORM=$form"; grep "GPU 0 alone" $out/f$form.log; python3 profiles/kernel_classes.py $f; } | tee -a $out/summary.txt
done
