"""bench.py's N > 1 control flow on the CPU, against a fake device layer (tests/fake_xg.py)
with the REAL host scheduler: per-method direct-vs-packed tuning, the per-launch roofline
pass, the xGMI object, the JSON line -- the code path only the driver's multi-GPU run
executes on hardware, checked here for crashes and for the line's schema."""
import json
import time
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


def _run_job(world, argv, tmp_path, extra_env):
    """all `world` ranks as processes whose barriers and MAX reductions really span the job
    (XG_FAKE_BARRIER_DIR), so a failure on one rank reaches every rank's decisions"""
    procs = []
    for rank in range(world):
        env = dict(os.environ, RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                   XG_RDZV_KEY="fault_%s_%d" % (tmp_path.name, world), XG_FAKE_BARRIER_DIR=str(tmp_path),
                   **extra_env)
        procs.append(subprocess.Popen([sys.executable, "-c", DRIVER.format(repo=REPO, argv=argv)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=300) for p in procs]
    return [p.returncode for p in procs], outs


ARGV2 = ["--gpus", "2", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--methods", "1,2"]


def test_bench_excludes_a_form_that_fails_verification_on_one_gpu(tmp_path):
    """packed one-sided m1 delivers a wrong slot on GPU 1 only: both ranks drop that form (MAX
    over the GPUs), the line names why, and is printed from the forms that passed"""
    rcs, outs = _run_job(2, ARGV2, tmp_path, {"XG_FAKE_VERIFY_FAIL": "1:%d:1" % (4 << 20), "XG_FAKE_FAIL_RANK": "1"})
    assert rcs == [0, 0], [o[1][-1500:] for o in outs]
    out = json.loads([l for l in outs[0][0].splitlines() if l.startswith("{")][0])
    t1 = out["pack_autotune_ms_per_run"]["1"]
    assert t1["packed_one_sided"].startswith("verify failed: 1 slots")
    assert t1["chosen"] in ("direct", "packed_two_sided") and "packed_one_sided_ms" not in t1
    assert set(out["pack_autotune_ms_per_run"]["2"]) >= {"direct_ms", "packed_one_sided_ms", "packed_two_sided_ms"}
    assert out["value"] > 0 and out["xgmi"]["sweep"] and out["xgmi"]["sweep_error"] is None


def test_bench_fails_with_a_line_when_every_form_of_a_method_fails(tmp_path):
    bad = ",".join("2:%d:%d" % f for f in ((0, -1), (4 << 20, 1), (4 << 20, 0)))
    rcs, outs = _run_job(2, ARGV2, tmp_path, {"XG_FAKE_VERIFY_FAIL": bad, "XG_FAKE_FAIL_RANK": "0"})
    assert rcs == [1, 1], [o[1][-1500:] for o in outs]
    lines = [l for l in outs[0][0].splitlines() if l.startswith("{")]
    assert len(lines) == 1 and not [l for l in outs[1][0].splitlines() if l.startswith("{")]
    out = json.loads(lines[0])
    assert out["value"] is None and "method(s) 2" in out["error"]
    assert set(out["failed_methods"]["2"]) == {"direct", "packed_one_sided", "packed_two_sided"}


def test_bench_survives_a_failing_ceiling_and_sweep(tmp_path):
    """an RCCL error on GPU 1 in the xGMI ceiling (p2p_bench call 0) and in the sweep's 1 MiB
    all-pairs case (call 6): the line still comes, with null + the error for each, and the
    sweep rows before the failing case"""
    rcs, outs = _run_job(2, ARGV2, tmp_path, {"XG_FAKE_P2P_FAIL": "0,6", "XG_FAKE_FAIL_RANK": "1"})
    assert rcs == [0, 0], [o[1][-1500:] for o in outs]
    out = json.loads([l for l in outs[0][0].splitlines() if l.startswith("{")][0])
    x = out["xgmi"]
    assert x["peak"] is None and x["frac"] is None and x["ceiling_error"] == "failed on another GPU"
    assert x["achieved"] > 0 and out["value"] > 0
    assert x["sweep_error"] == "all_pairs 1048576 B: failed on another GPU"
    assert [(r["mode"], r["bytes"]) for r in x["sweep"]] == [("one_way_1_to_0", 4096), ("all_pairs", 4096),
                                                             ("one_way_1_to_0", 65536), ("all_pairs", 65536),
                                                             ("one_way_1_to_0", 1 << 20)]


def test_bench_runs_the_8gpu_baseline_configs_after_the_line(tmp_path):
    """--baseline-configs on (the default at 8 GPUs): after the line's own measurements every method
    of configs[2], [3] and [4] (stated sizes) runs on the job, one verified and one timed run each,
    and lands in the line; a plan that fails on one GPU (injected: m9 on GPU 1) is recorded for that
    cell on every rank and the rest go on"""
    argv = ARGV2 + ["--baseline-configs", "on", "--no-ktime"]
    rcs, outs = _run_job(2, argv, tmp_path, {"XG_FAKE_PLAN_FAIL": "9:1"})
    assert rcs == [0, 0], [o[1][-1500:] for o in outs]
    out = json.loads([l for l in outs[0][0].splitlines() if l.startswith("{")][0])
    assert out["value"] > 0 and out["xgmi"]["peak"] > 0
    ex = out["baseline_configs_8gpu"]
    cells = ex["cells"]
    want = ["configs[2] m5", "configs[2] m8"] + ["configs[3] m%d" % m for m in (1, 2, 9, 10)] + \
           ["configs[4] -c %d m%d" % (c, m) for c in range(1, 9) for m in (7, 11, 12)]
    assert list(cells) == want
    assert cells["configs[3] m9"].startswith("failed")
    for k, v in cells.items():
        if k != "configs[3] m9":
            assert v["verified"] and v["ms_per_run"] > 0 and v["GBps_cross_gpu"] > 0, (k, v)
    assert cells["configs[4] -c 1 m7"]["cross_gpu_bytes"] == 256 * 64 * (64 << 20) // 2   # half the pairs cross
    assert "error" not in ex and ex["spent_s"] >= 0


def test_bench_baseline_configs_phase_keeps_to_its_budget(tmp_path):
    argv = ARGV2 + ["--baseline-configs", "on", "--baseline-budget", "0", "--no-ktime"]
    rcs, outs = _run_job(2, argv, tmp_path, {})
    assert rcs == [0, 0], [o[1][-1500:] for o in outs]
    out = json.loads([l for l in outs[0][0].splitlines() if l.startswith("{")][0])
    cells = out["baseline_configs_8gpu"]["cells"]
    assert len(cells) == 2 + 4 + 24 and all(str(v).startswith("skipped: phase budget") for v in cells.values())


def test_bench_baseline_configs_phase_skips_a_configuration_that_does_not_fit(tmp_path):
    """GPU 1 cannot allocate configs[4]'s regions (injected past 64 GiB): the first -c 1 cell
    records the failure on every rank, the other 23 cells of that configuration are skipped without
    another allocation attempt, and configs[2] / [3] still run"""
    argv = ARGV2 + ["--baseline-configs", "on", "--no-ktime"]
    rcs, outs = _run_job(2, argv, tmp_path, {"XG_FAKE_REGIONS_FAIL": "%d:1" % (64 << 30)})
    assert rcs == [0, 0], [o[1][-1500:] for o in outs]
    out = json.loads([l for l in outs[0][0].splitlines() if l.startswith("{")][0])
    cells = out["baseline_configs_8gpu"]["cells"]
    assert cells["configs[4] -c 1 m7"].startswith("failed: ")
    rest = [k for k in cells if k.startswith("configs[4]") and k != "configs[4] -c 1 m7"]
    assert len(rest) == 23 and all(cells[k] == "skipped: this configuration's regions did not fit" for k in rest)
    assert all(cells[k]["verified"] for k in cells if not k.startswith("configs[4]"))


def test_bench_line_survives_a_hang_in_the_xgmi_phase(tmp_path):
    """the line's value is measured, then one GPU never returns from the sweep's second call (a
    peer lost inside RCCL): after --xgmi-budget seconds rank 0 prints the line as measured -- the
    value, the ceiling, the sweep rows so far -- with xgmi_error naming the phase, and every rank
    ends (exit 0) instead of waiting for the 420 s watchdog"""
    argv = ARGV2 + ["--xgmi-budget", "8", "--no-ktime"]
    t0 = time.time()
    rcs, outs = _run_job(2, argv, tmp_path, {"XG_FAKE_P2P_HANG": "2", "XG_FAKE_FAIL_RANK": "1"})
    assert rcs == [0, 0], [o[1][-1500:] for o in outs]
    assert time.time() - t0 < 100
    out = json.loads([l for l in outs[0][0].splitlines() if l.startswith("{")][0])
    assert out["value"] > 0 and out["xgmi"]["peak"] > 0 and out["xgmi"]["ceiling_error"] is None
    assert out["xgmi_error"].startswith("still in phase 'xGMI p2p sweep' 8 s after it started")
    assert "sweep" not in out["xgmi"]          # the sweep never finished


def test_watchdog_on_rank0_prints_a_line_naming_the_phase(tmp_path):
    """rank 0 of a 2-GPU job whose rank 1 never comes waits in the communicator init: the watchdog
    prints a line with value null and the phase it stopped in, then exits 124"""
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="2", XG_FAKE_BARRIER_DIR=str(tmp_path),
               XG_RDZV_KEY="wd0_%s" % tmp_path.name)
    code = DRIVER.format(repo=REPO, argv=["--gpus", "2", "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
                                          "--watchdog", "3"])
    try:
        p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    finally:
        rdzv = "/tmp/xg_bench_rdzv_wd0_%s.bin" % tmp_path.name
        if os.path.exists(rdzv):
            os.unlink(rdzv)
    assert p.returncode == 124, (p.returncode, p.stderr[-2000:])
    out = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][0])
    assert out["value"] is None and out["error"].startswith("rank 0 still in phase 'RCCL communicator init")


def test_failed_communicator_init_still_prints_a_line(tmp_path):
    """RCCL refuses the communicator on every rank (as it does for two ranks on one GPU,
    profiles/r04/two_ranks/): no rank hangs, rank 0 prints a line with value null naming the
    failure, and the job exits 1"""
    rcs, outs = _run_job(2, ARGV2, tmp_path, {"XG_FAKE_INIT_FAIL": "1"})
    assert rcs == [1, 1], [o[1][-1500:] for o in outs]
    lines = [l for l in outs[0][0].splitlines() if l.startswith("{")]
    assert len(lines) == 1 and not [l for l in outs[1][0].splitlines() if l.startswith("{")]
    out = json.loads(lines[0])
    assert out["value"] is None and out["error"].startswith("device / RCCL init failed on rank 0 (RCCL communicator init")
