"""One rank of a real multi-rank job on the box's GPU (tests/test_gpu_multirank.py).

Started G times by the test (RANK / WORLD_SIZE / XG_MR_DIR / XG_SHARE_GPU=1 set): every rank is
its own process with its own RCCL communicator rank, all on device 0 -- RCCL then pairs the ranks
over its network transport instead of xGMI (XG_SHARE_GPU, runtime/ctx.hip), but every call is
the real rank's: ncclCommInitRank with nranks > 1, enqueue_step's groups to real peers,
xg_barrier / xg_allreduce_max across processes.

argv[1]: JSON list of cases {"golden": <dir under tests/golden>, "methods": [...] (default: every
method the capture holds), "forms": [[pack_max_seg, pack_form], ...], "iters": [...] (default:
the last)}.  Per case, method, form and iteration every rank runs its plan once through
xg_plan_run, verifies its receive slots on the device and compares each slot's checksum with the
one the REFERENCE's receive buffer had (tests/golden, captured by oracle/pmpi_capture.c); counts
are gathered with MAX reductions, rank 0 prints one JSON line per run and a last {"done": true}.
Failures are agreed on before anything collective follows them (as bench.py does), so one bad
rank cannot leave the others waiting in RCCL.
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(REPO, "oracle"))      # the checker (xg_oracle.direction)


def rendezvous(xg, rank, world, d):
    path = os.path.join(d, "uid.bin")
    if rank == 0:
        uid = xg.unique_id()
        with open(path + ".tmp", "wb") as f:
            f.write(uid)
        os.replace(path + ".tmp", path)
        return uid
    t0 = time.time()
    while time.time() - t0 < 60:
        try:
            with open(path, "rb") as f:
                uid = f.read()
            if len(uid) == 128:
                return uid
        except FileNotFoundError:
            pass
        time.sleep(0.01)
    raise SystemExit("rank %d: no RCCL id" % rank)


def load(case):
    """-> (meta, want(it, direction, src, seed, dst, chk) -> bool, fingerprint mode, expected slot count(it, direction)):
    a reference capture (case["golden"]: every slot's checksum as the REFERENCE's receive buffer
    had it), or an explicit shape {"shape": [P, A, d, c]} on the collision-free fingerprint (mode 1):
    the device's own byte check of every slot plus a sample of slots against the oracle's closed form"""
    import xg_oracle as O
    from conftest import load_baseline, load_golden
    if "shape" in case:
        P, A, d, c = case["shape"]
        rl = list(O.aggregator_list(P, A))
        meta = {"P": P, "A": A, "d": d, "c": c, "aggregators": rl, "ntimes": 1, "proc_node": 1, "iters": 2,
                "method_list": case["methods"]}
        sample = max(1, P * A // 64)
        seen = [0]

        def want(it, direction, src, seed, dst, chk):
            seen[0] += 1
            return seen[0] % sample or chk == O.chk64(O.fingerprint(1, src, seed, it, d))
        return meta, want, 1, lambda it, direction: P * A
    name = case["golden"]
    if name.startswith("baseline/"):
        meta, _t, data = load_baseline(name.split("/", 1)[1])
    else:
        meta, _t, data = load_golden(name)

    def want(it, direction, src, seed, dst, chk):
        glen, gchk = data[direction][(it, src, dst)]
        return glen == meta["d"] and chk == gchk
    return meta, want, 0, lambda it, direction: sum(1 for k in data[direction] if k[0] == it)


NOW = ["start"]


def deadline_watch(xg, rank, seconds):
    """a rank still running after `seconds` says which run it is in and where libxg's host thread
    is (xg_debug_where), then exits 5: the test reads it from stderr (no hang without a diagnosis)"""
    import threading

    def fire():
        try:
            dev = xg.device()
            dev.xg_debug_where.restype = __import__("ctypes").c_char_p
            where = dev.xg_debug_where().decode()
        except Exception as e:        # the diagnosis must not mask the hang
            where = "unavailable (%s)" % e
        sys.stderr.write("rank %d: still in %s after %.0f s; libxg: %s\n" % (rank, NOW[0], seconds, where))
        sys.stderr.flush()
        os._exit(5)

    t = threading.Timer(seconds, fire)
    t.daemon = True
    t.start()


def main():
    import __graft_entry__ as G
    import xg_oracle as O
    xg = G.load_package().xg
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    deadline_watch(xg, rank, float(os.environ.get("XG_MR_DEADLINE", "100")))
    cases = json.loads(sys.argv[1])
    uid = rendezvous(xg, rank, world, os.environ["XG_MR_DIR"])
    ctx = xg.Context(rank=rank, nranks=world, device=0, uid=uid)
    ctx.barrier()
    for case in cases:
        meta, want, mode, nslots = load(case)
        label = case.get("golden") or "shape %s" % case["shape"]
        P, A, d = meta["P"], meta["A"], meta["d"]
        rl = meta["aggregators"]
        methods = case.get("methods") or meta["method_list"]
        iters = case.get("iters") or [meta["iters"] - 1]
        for method in methods:
            direction = O.direction(method)
            for it in iters:
                try:
                    s = xg.Schedule(method, P, A, d, meta["c"], rl, ntimes=meta["ntimes"],
                                    proc_node=meta["proc_node"], barrier_type=meta.get("barrier", 0), iteration=it)
                except xg.XGError as e:      # the schedule deadlocks under MPI (every rank computes the same)
                    if rank == 0:
                        print(json.dumps({"case": label, "method": method, "it": it, "error": "schedule: %s" % e}),
                              flush=True)
                    continue
                for pack, form in case["forms"]:
                    run, err = None, ""
                    t0 = time.time()
                    NOW[0] = "%s m%d it%d form %s" % (label, method, it, [pack, form])
                    sys.stderr.write("rank %d: %s\n" % (rank, NOW[0]))
                    try:
                        run = xg.MethodRun(ctx, s, it=it, mode=mode, pack_max_seg=pack, pack_form=form)
                    except xg.XGError as e:
                        err = str(e)
                    if ctx.allreduce_max([1.0 if err else 0.0])[0]:
                        if rank == 0:
                            print(json.dumps({"case": label, "method": method, "it": it, "form": [pack, form],
                                              "error": err or "plan failed on another rank"}), flush=True)
                        if run is not None:
                            run.close()
                        continue
                    try:
                        ctx.barrier()
                        done, post, _wall = run.run_timed()
                        chk, bad, _first = run.verify()
                        lo, hi = s.block_range(world, rank)
                        tot = max((s.rank_timer(q, done, post, world).total_time for q in range(lo, hi)), default=0.0)
                        wrong = 0
                        for (src, seed, dst, _off), ck, nb in zip(run.slots, chk, bad):
                            wrong += nb != 0 or not want(it, direction, src, seed, dst, ck)
                        counts = [0.0] * world
                        counts[rank] = float(len(run.slots))
                        red = ctx.allreduce_max(counts + [float(wrong), tot])
                    finally:
                        run.close()
                    if rank == 0:
                        # steps of this rank's plan with a second RCCL group (the relay form's forwards)
                        v = s.devplan(world, rank, pack, 0, form)
                        relayed = sum(1 for st in range(v.nsteps)
                                      if any(k == xg.CALL_FENCE for k, *_ in v.calls(st)))
                        print(json.dumps({"case": label, "method": method, "it": it, "form": [pack, form],
                                          "slots": int(sum(red[:world])), "want": nslots(it, direction),
                                          "wrong": int(red[world]), "relayed_steps": relayed,
                                          "max_total_time_s": red[world + 1], "wall_s": round(time.time() - t0, 3)}),
                              flush=True)
    ctx.barrier()
    ctx.close()
    if rank == 0:
        print(json.dumps({"done": True}), flush=True)


if __name__ == "__main__":
    main()
