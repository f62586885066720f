"""Round 5 probe: how a G-rank job on one GPU (XG_SHARE_GPU=1) behaves as G grows --
one small case (README golden, m1 and m9, direct), per-run wall time, stderr tails."""
import json, os, signal, subprocess, sys, tempfile, time
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
W = os.path.join(REPO, "tests", "multirank_worker.py")
cases = [{"golden": "readme_p32_a14", "methods": [1, 9, 12], "forms": [[0, -1]]}]
for G in [int(x) for x in sys.argv[1].split(",")]:
    d = tempfile.mkdtemp()
    env = dict(os.environ, XG_SHARE_GPU="1", NCCL_DEBUG="WARN", XG_MR_DIR=d, XG_MR_DEADLINE="50", WORLD_SIZE=str(G))
    t0 = time.time()
    ps = [subprocess.Popen([sys.executable, "-u", W, json.dumps(cases)], env=dict(env, RANK=str(r), LOCAL_RANK=str(r)),
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, start_new_session=True)
          for r in range(G)]
    res = []
    for r, p in enumerate(ps):
        try:
            out, err = p.communicate(timeout=70)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            out, err = p.communicate()
        res.append((p.returncode, out, err))
    print("G=%d wall %.1f s rcs %s" % (G, time.time() - t0, [x[0] for x in res]))
    print(res[0][1][-1500:])
    for r, (rc, out, err) in enumerate(res):
        if rc:
            print("  rank %d stderr tail: %s" % (r, err[-700:].replace("\n", " | ")))
    sys.stdout.flush()
