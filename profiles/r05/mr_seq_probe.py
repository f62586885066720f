"""Round 5 probe: the 8-rank baseline job of tests/test_gpu_multirank.py in sequence, with a long
deadline and every run's wall time -- a stall, or just slow?"""
import json, os, signal, subprocess, sys, tempfile, time
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
W = os.path.join(REPO, "tests", "multirank_worker.py")
names = sys.argv[2].split(",")
cases = [{"golden": "baseline/" + n, "forms": [[0, -1]]} for n in names]
G = int(sys.argv[1])
d = tempfile.mkdtemp()
env = dict(os.environ, XG_SHARE_GPU="1", NCCL_DEBUG="WARN", XG_MR_DIR=d, XG_MR_DEADLINE="240",
           WORLD_SIZE=str(G), GPU_MAX_HW_QUEUES="2")
t0 = time.time()
ps = [subprocess.Popen([sys.executable, "-u", W, json.dumps(cases)], env=dict(env, RANK=str(r), LOCAL_RANK=str(r)),
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, start_new_session=True)
      for r in range(G)]
res = []
for p in ps:
    try:
        out, err = p.communicate(timeout=260)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        out, err = p.communicate()
    res.append((p.returncode, out, err))
print("G=%d wall %.1f s rcs %s" % (G, time.time() - t0, [x[0] for x in res]))
for line in res[0][1].splitlines():
    if line.startswith("{"):
        x = json.loads(line)
        print("   ", x.get("case"), x.get("method"), "wrong", x.get("wrong"), "wall_s", x.get("wall_s"), "tot", x.get("max_total_time_s"))
for r, (rc, out, err) in enumerate(res):
    if rc:
        tail = [x for x in err.splitlines() if "LL cutoff" not in x and "Could not read" not in x and x.strip()]
        print("  rank %d: %s" % (r, " | ".join(tail[-3:])[:500]))
