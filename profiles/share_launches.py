#!/usr/bin/env python3
"""One GPU's share of the 8-GPU configs[2] plans (P64 A16 -d 256 KiB, m5 / m8) run alone on
this device (xg_plan_set_local_only: the product's copy launches -- pack, the local part on the
side stream, unpack -- with its RCCL calls left out), so its regions are one real GPU's (32 MiB
of segments, staging, slots: resident in the Infinity Cache as on the 8-GPU node).  REPS
back-to-back runs; run under rocprofv3 --kernel-trace and reduce with kernel_classes.py.
FORM: 0 two-sided (default) / 1 one-sided.  D_KIB: -d in KiB (default 256: GPU 0 has 16 local segments
of -d and packs / unpacks 112 of them)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as G  # noqa: E402

xg = G.load_package().xg
P, A, GPUS, REPS = 64, 16, 8, int(os.environ.get("REPS", "50"))
d = int(os.environ.get("D_KIB", "256")) << 10      # -d (configs[2]: 256 KiB)
FORM = int(os.environ.get("FORM", "0"))
rl = xg.aggregator_list(P, A)
ctx = xg.Context.virtual(0, GPUS, device=0)
for m in (5, 8):
    s = xg.Schedule(m, P, A, d, 200000000, rl, ntimes=1)
    run = xg.MethodRun(ctx, s, it=0, mode=0, pack_max_seg=4 << 20, pack_form=FORM)
    try:
        run.set_local_only()
        for _ in range(REPS):
            run.enqueue()
        ctx.device_sync()
        run.check()
        v = run.view
        pk = sum(c[4] for c in v.copies if c[2] == 2)
        up = sum(c[4] for c in v.copies if c[0] == 3)
        print("m%d form %d: GPU 0 alone, %d runs; per run: local %d B, packs %d B, unpacks %d B, launches %d" % (
            m, FORM, REPS, v.local_bytes, pk, up, run.launches), flush=True)
    finally:
        run.close()
ctx.close()
print("share_launches ok", flush=True)
