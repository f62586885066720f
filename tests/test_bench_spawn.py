"""bench.py --gpus N without a launcher: the parent starts one child per GPU.

The driver may run `python3 bench.py --gpus N` with no RANK / WORLD_SIZE in the
environment.  Then bench.py must not become rank 0 of an N-rank job whose peers
nobody started (it would wait forever in ncclCommInitRank): it becomes a parent
that never touches the GPU, starts N children (subprocess, not exec), hands
them one rendezvous key, and exits with the highest child exit code.
"""
import json
import os
import subprocess
import sys
import time

from conftest import REPO

BENCH = os.path.join(REPO, "bench.py")


def _run(n, env_extra, timeout=120):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env.update(env_extra)
    return subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--no-cpu-baseline"], env=env,
                          capture_output=True, text=True, timeout=timeout)


def test_parent_starts_one_child_per_gpu():
    p = _run(4, {"XG_BENCH_CHILD_STUB": "1"})
    assert p.returncode == 0, p.stderr
    out = json.loads(p.stdout.strip().splitlines()[-1])
    kids = out["children"]
    assert len(kids) == 4
    assert sorted(int(k["LOCAL_RANK"]) for k in kids) == [0, 1, 2, 3]
    assert sorted(int(k["RANK"]) for k in kids) == [0, 1, 2, 3]
    assert {k["WORLD_SIZE"] for k in kids} == {"4"}
    assert len({k["XG_RDZV_KEY"] for k in kids}) == 1          # one rendezvous for the job
    assert {k["XG_BENCH_PARENT"] for k in kids} != {str(os.getpid())}


def test_parent_exit_code_is_the_highest_child_code():
    p = _run(4, {"XG_BENCH_CHILD_STUB": "1", "XG_BENCH_STUB_RC": "0,5,3,0"})
    assert p.returncode == 5
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["rcs"] == [0, 5, 3, 0] and out["rc"] == 5


def test_failed_rank_stops_the_job():
    """Without a GPU (this container) every child fails at device init; ranks waiting
    for the RCCL id would wait long -- the parent must stop them and fail, not hang."""
    t0 = time.time()
    p = _run(2, {"HIP_VISIBLE_DEVICES": "", "XG_BENCH_PARENT_TEST": "1"}, timeout=240)
    assert p.returncode != 0
    assert time.time() - t0 < 200
    assert "failed" in p.stderr
    out = json.loads(p.stdout.strip().splitlines()[-1])     # rank 0's line, passed on by the parent
    assert out["value"] is None and "init failed" in out["error"] and out["child_exit_codes"]


TEST_BIN = os.path.join(REPO, "mpi-asynchronous-communication-test_amd", "bin", "test")


def test_cli_gpus_flag_starts_one_process_per_gpu():
    """bin/test --gpus N (the ./test drop-in) without a launcher: N child processes,
    distinct ranks, one rendezvous key."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env["XG_SPAWN_STUB"] = "1"
    p = subprocess.run([TEST_BIN, "--gpus", "4", "-a", "2", "-d", "64", "-m", "1"], env=env,
                       capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    lines = [l for l in p.stdout.splitlines() if l.startswith("spawn-stub")]
    assert len(lines) == 4
    kv = [dict(t.split("=", 1) for t in l.split()[1:]) for l in lines]
    assert sorted(int(x["RANK"]) for x in kv) == [0, 1, 2, 3]
    assert sorted(int(x["LOCAL_RANK"]) for x in kv) == [0, 1, 2, 3]
    assert {x["WORLD_SIZE"] for x in kv} == {"4"} and len({x["XG_RDZV_KEY"] for x in kv}) == 1


def test_cli_failed_rank_stops_the_job():
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env.update({"XG_GPUS": "3", "HIP_VISIBLE_DEVICES": ""})
    t0 = time.time()
    p = subprocess.run([TEST_BIN, "-a", "2", "-d", "64", "-m", "1", "--procs", "6"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and time.time() - t0 < 100
    assert "stopping the job" in p.stderr
