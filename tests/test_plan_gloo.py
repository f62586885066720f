"""world_size-2 run of the multi-GPU exchange on CPU: each process executes its
GPU's device plan on numpy regions and posts exactly the calls the runtime posts
(xg_devplan_step_calls: cross-GPU sends/receives with torch.distributed (gloo) in the
per-peer issue order RCCL matches on, self send/recv pairs as local copies, the in-loop
barrier as dist.barrier), with and without the local part in the group (self_max).
Same bytes as the oracle.

torch is imported only in the two worker processes, never in the pytest process: collecting or
running this module in the same process as the -m gpu tests must not load torch's bundled ROCm
runtime (its
libamdhip64.so.7 / librccl.so.1 carry the same sonames as /opt/rocm's, so libxg.so would bind
to them -- the full GPU suite hung in RCCL that way, profiles/r04/torch_runtime/)."""
import os
import socket

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, results):
    import sys
    import torch
    import torch.distributed as dist
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import __graft_entry__ as G
    import xg_oracle as O
    from plan_exec import copies, make_regions, step_parts
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    xg = G.load_package().xg
    ok = True
    try:
        for (P, A, d, c, k, m) in [(12, 5, 64, 3, 2, 1), (12, 5, 64, 3, 2, 2), (16, 5, 100, 4, 1, 4),
                                   (16, 4, 32, 200000000, 1, 5), (12, 5, 48, 2, 1, 6), (16, 6, 40, 3, 1, 9),
                                   (12, 5, 16, 2, 2, 11), (16, 5, 56, 3, 1, 12), (12, 5, 32, 3, 2, 13),
                                   (12, 4, 24, 5, 1, 14), (16, 5, 40, 3, 1, 17), (12, 5, 48, 4, 2, 18),
                                   (12, 5, 16, 3, 1, 19), (16, 6, 40, 5, 1, 20), (12, 5, 40, 3, 2, 15),
                                   (16, 5, 24, 3, 1, 16)]:
            rl = xg.aggregator_list(P, A)
            s = xg.Schedule(m, P, A, d, c, rl, ntimes=k, proc_node=3, barrier_type=2, iteration=2)
            for pack, self_max, form in ((0, 0, -1), (1 << 20, 0, 0), (0, 1 << 30, -1), (1 << 20, 1 << 30, 0),
                                         (1 << 20, 0, 1), (1 << 20, 1 << 30, 1)):   # form 1: one-sided packing
                v = s.devplan(world, rank, pack, 0, form)
                reg = make_regions(s, v, world, rank, 2, 1)
                seq = {}
                for st in range(v.nsteps):
                    stage, pre, _p2p, post = step_parts(v, st)
                    # exactly the calls the runtime posts (xg_devplan_step_calls): with self_max the
                    # step's local copies travel in the group as self send/recv pairs instead
                    calls = v.calls(st, self_max)
                    selfs = [c for c in calls if c[0] != 3 and c[1] == rank]
                    copies(reg, stage)
                    copies(reg, [cp for cp in pre if cp[2] == 2] if selfs else pre)   # packs only
                    reqs, bufs = [], []
                    for (s_kind, _, sb, so, sl), (r_kind, _, rb, ro, rl_) in zip(selfs[0::2], selfs[1::2]):
                        assert (s_kind, r_kind) == (1, 2) and sl == rl_      # send then receive, one copy
                        bufs.append((torch.from_numpy(reg[sb][so:so + sl].copy()), rb, ro, rl_))
                    for kind, peer, buf, off, ln in calls:
                        if kind == 3 or peer == rank:
                            continue
                        key = (peer, kind == 1)
                        tag = seq.get(key, 0)
                        seq[key] = tag + 1
                        if kind == 1:
                            t = torch.from_numpy(reg[buf][off:off + ln].copy())
                            reqs.append(dist.isend(t, dst=peer, tag=tag))
                        else:
                            t = torch.empty(ln, dtype=torch.uint8)
                            reqs.append(dist.irecv(t, src=peer, tag=tag))
                            bufs.append((t, buf, off, ln))
                    for q in reqs:
                        q.wait()
                    for t, buf, off, ln in bufs:
                        reg[buf][off:off + ln] = t.numpy()
                    copies(reg, post)
                    if calls and calls[-1][0] == 3:                # the step's in-loop barrier
                        dist.barrier()
                exp = O.expected_recv(m, P, A, d, rl, 2, 1)
                lo, hi = s.block_range(world, rank)
                for r in range(lo, hi):
                    off = s.recv_offset(world, r)
                    if off < 0:
                        continue
                    got = reg[1][off: off + exp[r].size]
                    ok &= bool((got == exp[r]).all())
        dist.barrier()
    finally:
        results[rank] = ok
        dist.destroy_process_group()


def test_two_process_exchange():
    # two spawned processes (stdlib multiprocessing: this pytest process never imports torch)
    import multiprocessing
    ctx = multiprocessing.get_context("spawn")
    mgr = ctx.Manager()
    results = mgr.dict()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, results)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=600)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert results[0] and results[1]
