#!/bin/bash
# A/B: bench value with and without the per-launch kernel-timing events in the timed region
for i in 1 2 3; do
  timeout -k 10 120 python3 bench.py --no-cpu-baseline > gpurun_out/kt_on_$i.json || exit 1
  timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-ktime > gpurun_out/kt_off_$i.json || exit 1
done
python3 - <<'PY'
import json
for k in ("on", "off"):
    for i in (1, 2, 3):
        d = json.load(open("gpurun_out/kt_%s_%d.json" % (k, i)))
        r = d.get("roofline") or {}
        print(k, i, d["value"], d["ms_per_step"], r.get("avg_launch_us"), d["max_total_time_s"])
PY
