import gzip
import json
import os
import sys
import threading

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))      # the checker (xg_oracle)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box)")


@pytest.fixture(autouse=True)
def _gpu_test_watchdog(request):
    """A -m gpu test still running after XG_TEST_WATCHDOG seconds (default 150; the slowest test
    takes ~20 s) names itself and where the device library's host thread is (xg_debug_where: the
    entry point, the step, posting or waiting for the device), dumps every Python thread's stack
    and ends the run (exit 3) -- a hang then leaves a diagnosis instead of a silent timeout."""
    if request.node.get_closest_marker("gpu") is None:
        yield
        return
    secs = float(os.environ.get("XG_TEST_WATCHDOG", "150"))

    def fire():
        import faulthandler
        where = "?"
        try:
            mod = sys.modules.get("xgamd")
            dev = getattr(getattr(mod, "xg", None), "_dev", None)
            if dev is not None:
                dev.xg_debug_where.restype = __import__("ctypes").c_char_p
                where = dev.xg_debug_where().decode()
        except Exception as e:            # a diagnostic must not mask the hang
            where = "unavailable (%s)" % e
        msg = "\nwatchdog: %s still running after %.0f s; libxg host thread: %s\n" % (request.node.nodeid, secs, where)
        # pytest captures fd 2 during the test: write the diagnosis to a file as well
        # (XG_WATCHDOG_LOG, default gpurun_out/watchdog.txt under the repository)
        path = os.environ.get("XG_WATCHDOG_LOG") or os.path.join(REPO, "gpurun_out", "watchdog.txt")
        try:
            os.makedirs(os.path.dirname(path), exist_ok=True)
            with open(path, "a") as f:
                f.write(msg)
                f.flush()
                faulthandler.dump_traceback(file=f, all_threads=True)
        except OSError:
            pass
        sys.stderr.write(msg)
        sys.stderr.flush()
        faulthandler.dump_traceback(all_threads=True)
        sys.stderr.flush()
        os._exit(3)

    t = threading.Timer(secs, fire)
    t.daemon = True
    t.start()
    yield
    t.cancel()


@pytest.fixture(scope="session")
def pkg():
    import __graft_entry__ as G
    return G.load_package()


@pytest.fixture(scope="session")
def xg(pkg):
    return pkg.xg


def golden_configs():
    """the ./test configurations (tests/golden/pt2pt holds the pt2pt_test goldens)"""
    return sorted(n for n in os.listdir(GOLDEN)
                  if os.path.isdir(os.path.join(GOLDEN, n)) and os.path.exists(os.path.join(GOLDEN, n, "trace.txt.gz")))


def load_golden(name):
    p = os.path.join(GOLDEN, name)
    meta = json.load(open(os.path.join(p, "meta.json")))
    opts = dict(zip(meta["args"].split()[0::2], meta["args"].split()[1::2]))
    meta["barrier"] = int(opts.get("-b", 0))
    meta["method_list"] = sorted(int(m) for m, v in meta["methods"].items() if v.get("status") == "ok")
    traces = {}
    for line in gzip.open(os.path.join(p, "trace.txt.gz"), "rt"):
        head, _, toks = line.rstrip("\n").partition(": ")
        m, r = head.split()
        traces[(int(m[1:]), int(r[1:]))] = toks
    data = {}
    for direction in ("a2m", "m2a"):
        rows = gzip.open(os.path.join(p, "data_%s.csv.gz" % direction), "rt").read().split("\n")[1:]
        data[direction] = {tuple(map(int, r.split(",")[:3])): (int(r.split(",")[3]), int(r.split(",")[4], 16))
                           for r in rows if r}
    if meta["d"] == 0:
        # -d 0: every message carries 0 bytes, which PMPI has nothing to checksum; the golden
        # row of every (rank, aggregator) pair is the empty segment (closed form, like the
        # self-memcpy pairs): length 0, checksum of no bytes
        import numpy as np
        import xg_oracle as O
        e = O.chk64(np.zeros(0, np.uint8))
        for it in range(meta["iters"]):
            for g in meta["aggregators"]:
                for r in range(meta["P"]):
                    data["a2m"][(it, r, g)] = (0, e)
                    data["m2a"][(it, g, r)] = (0, e)
    # m15/m16 (TAM): per (method, iter, rank) the received messages in completion order
    data["tam"] = {}
    tp = os.path.join(p, "data_tam.csv.gz")
    if os.path.exists(tp):
        for r in gzip.open(tp, "rt").read().split("\n")[1:]:
            if r:
                m, it, rank, _k, src, cnt, chk = r.split(",")
                data["tam"].setdefault((int(m), int(it), int(rank)), []).append((int(src), int(cnt), int(chk, 16)))
    return meta, traces, data


BASELINE = os.path.join(GOLDEN, "baseline")


def baseline_configs(prefix=""):
    """the reference captured at the BASELINE.json configuration shapes
    (tests/golden/make_baseline.py): cfg1 / cfg2 at full size, cfg3 / cfg4 at reduced -d"""
    if not os.path.isdir(BASELINE):
        return []
    return sorted(n for n in os.listdir(BASELINE)
                  if n.startswith(prefix) and os.path.exists(os.path.join(BASELINE, n, "meta.json")))


def load_baseline(name):
    """-> meta (+ barrier, method_list), sampled full traces {(m, r): tokens}, data {direction: {(it, src, dst):
    (len, chk)}}; meta["trace_sha1"][str(m)][r] is the sha1 of rank r's whole token string"""
    p = os.path.join(BASELINE, name)
    meta = json.load(open(os.path.join(p, "meta.json")))
    meta["barrier"] = 0
    meta["method_list"] = sorted(int(m) for m, v in meta["methods"].items() if v.get("status") == "ok")
    traces = {}
    for line in gzip.open(os.path.join(p, "trace_sample.txt.gz"), "rt"):
        if line.strip():
            head, _, toks = line.rstrip("\n").partition(": ")
            m, r = head.split()
            traces[(int(m[1:]), int(r[1:]))] = toks
    data = {}
    src_dir = os.path.join(BASELINE, meta["data_from"])
    for direction in ("a2m", "m2a"):
        rows = gzip.open(os.path.join(src_dir, "data_%s.csv.gz" % direction), "rt").read().split("\n")[1:]
        data[direction] = {tuple(map(int, r.split(",")[:3])): (int(r.split(",")[3]), int(r.split(",")[4], 16))
                           for r in rows if r}
    return meta, traces, data
