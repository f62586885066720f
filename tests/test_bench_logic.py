"""bench.py's N > 1 control flow on the CPU, against a fake device layer (tests/fake_xg.py)
with the REAL host scheduler: per-method direct-vs-packed tuning, the per-launch roofline
pass, the xGMI object, the JSON line -- the code path only the driver's multi-GPU run
executes on hardware, checked here for crashes and for the line's schema."""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO

DRIVER = r'''
import os, sys, json
sys.path.insert(0, {repo!r}); sys.path.insert(0, os.path.join({repo!r}, "tests"))
import __graft_entry__ as G
import fake_xg
real = G.load_package()
fx = fake_xg.install(real)
sys.argv = ["bench.py"] + {argv!r}
import bench
rc = bench.main()
print("CALLS " + json.dumps({{"p2p": fx.calls["p2p_bench"], "ktime": fx.calls["ktime"], "runs": fx.calls["runs"]}}))
sys.exit(rc)
'''


def _run(world, rank, argv, tmp_path):
    env = dict(os.environ, RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
               XG_RDZV_KEY="logic_%s_%d" % (tmp_path.name, world))
    code = DRIVER.format(repo=REPO, argv=argv)
    return subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)


@pytest.mark.parametrize("world", [2, 8])
def test_bench_multi_gpu_rank0_line(world, tmp_path):
    p = _run(world, 0, ["--gpus", str(world), "--steps", "3", "--warmup", "1", "--no-cpu-baseline"], tmp_path)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0])
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "xgmi", "cpu_baseline"):
        assert key in out, key
    assert out["n_gpus"] == world and out["steps"] == 3 and out["unit"] == "GB/s"
    assert out["xgmi"]["peak"] > 0 and out["xgmi"]["cross_gpu_bytes_per_step"] > 0
    assert out["roofline"] and out["roofline"]["bound"] == "hbm"
    assert set(out["pack_autotune_ms_per_run"]) == {"1", "2", "3", "4"}
    forms = ("direct", "packed_one_sided", "packed_two_sided")
    for m, tune in out["pack_autotune_ms_per_run"].items():      # every form timed, the fastest kept
        assert set(tune) == {f + "_ms" for f in forms} | {"chosen"}, tune
        assert tune["chosen"] in forms and tune[tune["chosen"] + "_ms"] == min(tune[f + "_ms"] for f in forms)
    calls = json.loads([l for l in p.stdout.splitlines() if l.startswith("CALLS ")][0][6:])
    sweep = out["xgmi"]["sweep"]          # the pt2pt_test analogue: 1 -> 0 latency + all pairs, 4 sizes
    assert calls["p2p"] == 1 + len(sweep) == 9
    assert [(r["mode"], r["bytes"]) for r in sweep] == [(m, b) for b in (4096, 65536, 1 << 20, 16 << 20)
                                                        for m in ("one_way_1_to_0", "all_pairs")]
    for r in sweep:
        assert r["us_per_rep"] > 0 and r["reps"] >= 5
        assert r["GBps"] > 0 if r["mode"] == "one_way_1_to_0" else r["GBps_aggregate"] == pytest.approx(r["GBps_per_gpu_egress_min"] * world, rel=1e-3)
    assert calls["ktime"] and calls["ktime"][0][1] is True      # N > 1: per-launch roofline pass


def test_bench_multi_gpu_other_rank(tmp_path):
    """a non-zero rank waits for rank 0's RCCL id, runs everything, prints nothing"""
    key = "logic_%s_%d" % (tmp_path.name, 4)
    with open("/tmp/xg_bench_rdzv_%s.bin" % key, "wb") as f:
        f.write(b"\x02" * 128)
    try:
        p = _run(4, 3, ["--gpus", "4", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"], tmp_path)
    finally:
        if os.path.exists("/tmp/xg_bench_rdzv_%s.bin" % key):
            os.unlink("/tmp/xg_bench_rdzv_%s.bin" % key)
    assert p.returncode == 0, p.stderr[-2000:]
    assert not [l for l in p.stdout.splitlines() if l.startswith("{")]


def test_bench_single_gpu_line(tmp_path):
    p = _run(1, 0, ["--steps", "2", "--warmup", "1", "--no-cpu-baseline"], tmp_path)
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][0])
    assert out["n_gpus"] == 1 and out["xgmi"] is None
    assert out["roofline"]["measured"].startswith("one HIP event pair")
    assert out["roofline"]["avg_launch_us"] * out["roofline"]["launches_per_step"] <= out["ms_per_step"] * 1e3 * 1.001


def test_watchdog_ends_a_rank_whose_peers_never_come(tmp_path):
    """rank 1 of a 2-GPU job whose rank 0 never writes the RCCL id: instead of waiting in
    the rendezvous (or, on hardware, in ncclCommInitRank) forever, the watchdog names the
    phase and exits 124"""
    p = _run(2, 1, ["--gpus", "2", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--watchdog", "3"], tmp_path)
    assert p.returncode == 124, (p.returncode, p.stderr[-2000:])
    assert "rank 1 still in phase 'rendezvous" in p.stderr


def test_bench_under_torchrun_launch_form(tmp_path):
    """The driver's N > 1 command form: torch.distributed.run starts the ranks (RANK /
    WORLD_SIZE / MASTER_PORT / TORCHELASTIC_RUN_ID set, no XG_RDZV_KEY), so the RCCL id
    travels through the launcher-keyed file; fake device layer, real host scheduler.
    Rank 0 prints the one JSON line, the other rank nothing, both exit 0."""
    import socket
    script = tmp_path / "bench_fake.py"
    script.write_text(DRIVER.format(repo=REPO, argv=["--gpus", "2", "--steps", "2", "--warmup", "1",
                                                     "--no-cpu-baseline", "--watchdog", "120"]))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "XG_RDZV_KEY")}
    env["XG_FAKE_BARRIER_DIR"] = str(tmp_path)      # barriers (and the comm init) really wait for the peer
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), str(script)],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["xgmi"]["cross_gpu_bytes_per_step"] > 0
