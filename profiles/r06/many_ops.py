#!/usr/bin/env python3
"""Round 6: does one RCCL group take the call counts the relay forms post at configs[4]'s stated
size (the coalesced form's weighted m7 steps: up to 505 send/recv calls per GPU and step)?  One rank
of an 8-rank job (XG_SHARE_GPU=1, every rank on this GPU; started 8 times by many_ops.sh): all pairs
at once, 1 MiB to every peer cut into 1, 8, 32 and 72 calls -- 14, 112, 448 and 1008 send + receive
calls in one group per rank -- each timed; rank 0 prints one JSON line per count."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import __graft_entry__ as G  # noqa: E402

xg = G.load_package().xg
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
d = os.environ["XG_MR_DIR"]
path = os.path.join(d, "uid.bin")
if rank == 0:
    with open(path + ".tmp", "wb") as f:
        f.write(xg.unique_id())
    os.replace(path + ".tmp", path)
t0 = time.time()
while True:
    try:
        uid = open(path, "rb").read()
        if len(uid) == 128:
            break
    except FileNotFoundError:
        pass
    if time.time() - t0 > 60:
        raise SystemExit("rank %d: no RCCL id" % rank)
    time.sleep(0.01)
ctx = xg.Context(rank=rank, nranks=world, device=0, uid=uid)
try:
    ctx.barrier()
    for calls in (1, 8, 32, 72):
        _g, sec = ctx.p2p_split_bench(1 << 20, calls, 2)
        t = ctx.allreduce_max([sec])[0]
        if rank == 0:
            print(json.dumps({"calls_per_peer": calls, "calls_per_group": 2 * calls * (world - 1),
                              "ms_per_rep_max": round(t * 1e3, 3)}), flush=True)
finally:
    ctx.close()
if rank == 0:
    print("many_ops ok", flush=True)
