"""Round 5: random shapes as REAL multi-rank jobs on one GPU (XG_SHARE_GPU=1): per job a random
P, A, -d (aligned and not), -c and G in {2, 3, 4, 8}, every method 1-12, direct / two-sided / relay,
every slot byte-checked on the device and a sample against the oracle's closed form
(tests/multirank_worker.py).  usage: mr_random.py <seed> <jobs> [big]; a summary line per job.
"big": 8 ranks, P 64-256, A 8-64, -d 64 KiB - 4 MiB + 48 (BASELINE-like shapes, where the relay
form applies), at most 1 GiB of segments per job (8 ranks share one GPU's HBM and sockets)."""
import json, os, random, signal, subprocess, sys, tempfile, time
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
W = os.path.join(REPO, "tests", "multirank_worker.py")
rng = random.Random(int(sys.argv[1]))
njobs = int(sys.argv[2])
big = len(sys.argv) > 3 and sys.argv[3] == "big"
tot = {"runs": 0, "bad": 0, "refused": 0}
for j in range(njobs):
    if big:
        G = 8
        while True:
            d = rng.choice([65536, 1 << 20, (1 << 20) + 48, 4 << 20])
            P = rng.choice([64, 96, 128, 200, 256])
            A = rng.choice([1, 2, 4, 8, 16, 32, 64])
            if P * A * d <= 1 << 30 and A <= P:
                break
        c = rng.choice([1, 2, 8, 200000000])
    else:
        G = rng.choice([2, 3, 4, 8])
        P = rng.randint(max(G, 6), 64)
        A = rng.randint(1, min(P, 20))
        d = rng.choice([24, 1000, 4096, 65536, (1 << 20) + 16, 1 << 20])
        c = rng.choice([1, 2, 3, 5, 8, 200000000])
    cases = [{"shape": [P, A, d, c], "methods": list(range(1, 13)), "forms": [[0, -1], [1 << 30, 0], [0, 2]]}]
    tmp = tempfile.mkdtemp()
    env = dict(os.environ, XG_SHARE_GPU="1", NCCL_DEBUG="WARN", XG_MR_DIR=tmp, XG_MR_DEADLINE="200" if big else "100",
               WORLD_SIZE=str(G), GPU_MAX_HW_QUEUES="1")
    t0 = time.time()
    procs = []
    for r in range(G):
        fo, fe = open(os.path.join(tmp, "r%d.out" % r), "w"), open(os.path.join(tmp, "r%d.err" % r), "w")
        procs.append(subprocess.Popen([sys.executable, "-u", W, json.dumps(cases)], env=dict(env, RANK=str(r), LOCAL_RANK=str(r)),
                                      stdout=fo, stderr=fe, start_new_session=True))
    hung = False
    for p in procs:
        try:
            p.wait(timeout=220 if big else 110)
        except subprocess.TimeoutExpired:
            hung = True
    if hung:
        for p in procs:
            if p.poll() is None:
                os.killpg(p.pid, signal.SIGKILL)
        for p in procs:
            p.wait()
    rows = [json.loads(x) for x in open(os.path.join(tmp, "r0.out")).read().splitlines() if x.startswith("{")]
    rows = [x for x in rows if "done" not in x]
    bad = [x for x in rows if "error" not in x and (x["wrong"] or x["slots"] != x["want"])]
    refused = [x for x in rows if "error" in x]
    tot["runs"] += len(rows); tot["bad"] += len(bad); tot["refused"] += len(refused)
    print("job %d G=%d P=%d A=%d d=%d c=%d: %d runs, %d bad, %d refused (deadlocked under MPI), rcs %s, %.1f s"
          % (j, G, P, A, d, c, len(rows), len(bad), len(refused), [p.returncode for p in procs], time.time() - t0))
    if bad or hung or any(p.returncode for p in procs):
        print("   ", bad[:2], open(os.path.join(tmp, "r0.err")).read()[-500:].replace("\n", " | "))
    sys.stdout.flush()
    if hung:
        break
print("TOTAL", json.dumps(tot))
