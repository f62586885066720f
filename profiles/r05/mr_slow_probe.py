"""Round 5 probe: is the 8-rank shared-GPU job at configs[4]'s P256 A64 -d 4 KiB -c 2 m7 hung or
slow?  The case alone at G = 2, 4, 8 (GPU_MAX_HW_QUEUES=2), per-run wall and Timer total."""
import json, os, signal, subprocess, sys, tempfile, time
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
W = os.path.join(REPO, "tests", "multirank_worker.py")
cases = [{"golden": "baseline/cfg4_p256_a64_d4k_c2", "methods": [7, 11], "forms": [[0, -1]]},
         {"golden": "baseline/cfg3_p256_a32_d64k", "methods": [9], "forms": [[0, -1]]}]
for G in [int(x) for x in sys.argv[1].split(",")]:
    d = tempfile.mkdtemp()
    env = dict(os.environ, XG_SHARE_GPU="1", NCCL_DEBUG="WARN", XG_MR_DIR=d, XG_MR_DEADLINE="80",
               WORLD_SIZE=str(G), GPU_MAX_HW_QUEUES="2")
    t0 = time.time()
    ps = [subprocess.Popen([sys.executable, "-u", W, json.dumps(cases)], env=dict(env, RANK=str(r), LOCAL_RANK=str(r)),
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, start_new_session=True)
          for r in range(G)]
    res = []
    for p in ps:
        try:
            out, err = p.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            out, err = p.communicate()
        res.append((p.returncode, out, err))
    print("G=%d wall %.1f s rcs %s" % (G, time.time() - t0, [x[0] for x in res]))
    for line in res[0][1].splitlines():
        if line.startswith("{"):
            print("   ", line[:240])
    for r, (rc, out, err) in enumerate(res):
        if rc:
            tail = [x for x in err.splitlines() if "LL cutoff" not in x and "Could not read" not in x and x.strip()]
            print("  rank %d: %s" % (r, " | ".join(tail[-2:])[:400]))
    sys.stdout.flush()
