"""Round 5 probe: the 8-rank hang of tests/test_gpu_multirank.py at p64_a16_d256 m16 (direct),
run alone under a few settings; every rank's last stderr lines (xg_debug_where) printed."""
import json, os, signal, subprocess, sys, tempfile, time
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
W = os.path.join(REPO, "tests", "multirank_worker.py")
variants = [("default", {}), ("self_max_0", {"XG_SELF_MAX": "0"}), ("no_engine", {"XG_ENGINE_MAX_STEP": "0"})]
cases = [{"golden": "p64_a16_d256", "methods": [int(x) for x in sys.argv[2].split(",")], "forms": [[0, -1]]}]
for G in [int(x) for x in sys.argv[1].split(",")]:
    for name, extra in variants:
        d = tempfile.mkdtemp()
        env = dict(os.environ, XG_SHARE_GPU="1", NCCL_DEBUG="WARN", XG_MR_DIR=d, XG_MR_DEADLINE="25",
                   WORLD_SIZE=str(G), **extra)
        t0 = time.time()
        ps = [subprocess.Popen([sys.executable, "-u", W, json.dumps(cases)],
                               env=dict(env, RANK=str(r), LOCAL_RANK=str(r)), stdout=subprocess.PIPE,
                               stderr=subprocess.PIPE, text=True, start_new_session=True) for r in range(G)]
        res = []
        for p in ps:
            try:
                out, err = p.communicate(timeout=45)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                out, err = p.communicate()
            res.append((p.returncode, out, err))
        print("G=%d %s: wall %.1f s rcs %s" % (G, name, time.time() - t0, [x[0] for x in res]))
        for line in res[0][1].splitlines():
            if line.startswith("{"):
                print("   ", line[:220])
        for r, (rc, out, err) in enumerate(res):
            if rc:
                tail = [x for x in err.splitlines() if "LL cutoff" not in x and "Could not read" not in x and x.strip()]
                print("  rank %d: %s" % (r, " | ".join(tail[-2:])[:400]))
        sys.stdout.flush()
