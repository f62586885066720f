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


def _key(prefix, tmp_path, *extra):
    """a rendezvous key unique to this test's directory (tmp_path.name alone is cut to 30 characters
    and numbered per xdist worker, so two tests running at once could share one RCCL id file)"""
    import hashlib
    h = hashlib.sha1(str(tmp_path).encode()).hexdigest()[:10]
    return "_".join([prefix, tmp_path.name, h] + [str(x) for x in extra])


def _run(world, rank, argv, tmp_path):
    env = dict(os.environ, RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
               XG_RDZV_KEY=_key("logic", tmp_path, world))
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
    for m, tune in out["pack_autotune_ms_per_run"].items():      # every form timed FORM_REPS times
        # the relay form is a candidate where it reroutes a step: >= 3 GPUs, and configs[1]'s m3 / m4
        forms = ("direct", "packed_one_sided", "packed_two_sided") + (("relay",) if "relay_ms" in tune else ())
        assert set(tune) == {f + "_ms" for f in forms} | {"chosen", "margin", "stats", "choice_rule"}, tune
        assert tune["chosen"] in forms and set(tune["stats"]) == set(forms)
        for f in forms:
            st = tune["stats"][f]
            assert st["min_ms"] <= st["median_ms"] == tune[f + "_ms"] <= st["max_ms"]
        assert tune["margin"] is not None
    # configs[1]'s methods 1-4 have no step the relay form reroutes, at any G (tests below: where it does)
    assert not [m for m, tune in out["pack_autotune_ms_per_run"].items() if "relay_ms" in tune]
    # the timed steps against their link bound (busiest-link bytes per step at the median link rate)
    lb = out["xgmi"]["link_bound"]
    assert lb["busiest_link_bytes_per_step"] > 0 and lb["link_GBps"] > 0 and lb["ms_per_step"] > 0
    # (frac comes from the unrounded step time; ms_per_step carries 4 decimals)
    assert lb["frac"] > 0 and abs(lb["ms_per_step"] / lb["frac"] - out["ms_per_step"]) <= 1e-4 + 0.02 * out["ms_per_step"]
    # the self-diagnosing fields: RCCL's version, each phase's wall time, the per-link sweep
    assert out["rccl_version"] == 22703 and "not xGMI" not in out["transport"]
    pw = out["phase_wall_s"]
    for ph in ("start", "RCCL communicator init (ncclCommInitRank, %d ranks)" % world, "methods: verify + plan choice",
               "warm-up", "timed steps", "xGMI ceiling (RCCL all-pairs send/recv)", "xGMI p2p sweep",
               "xGMI per-link sweep", "xGMI per-call cost"):
        assert ph in pw and pw[ph] >= 0, (ph, pw)
    links = out["xgmi"]["links"]
    assert out["xgmi"]["links_error"] is None and links["rounds"] == world - 1
    assert all((links["GBps"][r][q] is None) == (r == q) for r in range(world) for q in range(world))
    # (one process here: the MAX reduction holds this rank's row only; a real job's in the fault tests)
    assert all(links["GBps"][0][q] == 40.0 + q for q in range(1, world)) and links["max"] == 40.0 + world - 1
    assert "rccl_log_tail" not in out                 # nothing failed
    calls = json.loads([l for l in p.stdout.splitlines() if l.startswith("CALLS ")][0][6:])
    sweep = out["xgmi"]["sweep"]          # the pt2pt_test analogue: 1 -> 0 latency + all pairs, 4 sizes
    assert calls["p2p"] == 1 + len(sweep) == 9
    # RCCL's cost per call: 1 and `world` calls per peer at 1 and 16 MiB (the fake charges 5 us a call)
    pc = out["xgmi"]["per_call"]
    assert out["xgmi"]["per_call_error"] is None and len(pc["rows"]) == 4
    assert [(r["bytes"], r["calls_per_peer"]) for r in pc["rows"]] == [(b, c) for b in (1 << 20, 16 << 20) for c in (1, world)]
    for b in ("1048576", "16777216"):
        assert pc["us_per_extra_call"][b] == pytest.approx(5.0 / (world - 1), rel=0.01)
    assert lb["link_bytes_per_step"] >= out["xgmi"]["cross_gpu_bytes_per_step"]
    assert [(r["mode"], r["bytes"]) for r in sweep] == [(m, b) for b in (4096, 65536, 1 << 20, 16 << 20)
                                                        for m in ("one_way_1_to_0", "all_pairs")]
    for r in sweep:
        assert r["us_per_rep"] > 0 and r["reps"] >= 5
        assert r["GBps"] > 0 if r["mode"] == "one_way_1_to_0" else r["GBps_aggregate"] == pytest.approx(r["GBps_per_gpu_egress_min"] * world, rel=1e-3)
    assert calls["ktime"] and calls["ktime"][0][1] is True      # N > 1: per-launch roofline pass


def test_bench_multi_gpu_other_rank(tmp_path):
    """a non-zero rank waits for rank 0's RCCL id, runs everything, prints nothing"""
    key = _key("logic", tmp_path, 4)
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
    for key in ("phase_wall_s", "rccl_version", "transport", "rccl_log_tail", "cpu_baseline_configs"):
        assert key not in out, key           # the N = 1 line is unchanged
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
                   XG_RDZV_KEY=_key("fault", tmp_path, world), XG_FAKE_BARRIER_DIR=str(tmp_path),
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
    links = out["xgmi"]["links"]          # both ranks' rows, through the real MAX reduction
    assert links["GBps"] == [[None, 41.0], [41.0, None]] and links["spread"] == 1.0


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
    # GPU 1's RCCL warnings (its NCCL_DEBUG_FILE) are attached to rank 0's line
    tail = out["rccl_log_tail"]
    assert list(tail) == ["1"] and "injected RCCL failure on rank 1" in tail["1"][-1], tail
    assert [(r["mode"], r["bytes"]) for r in x["sweep"]] == [("one_way_1_to_0", 4096), ("all_pairs", 4096),
                                                             ("one_way_1_to_0", 65536), ("all_pairs", 65536),
                                                             ("one_way_1_to_0", 1 << 20)]


def test_bench_runs_the_8gpu_baseline_configs_after_the_line(tmp_path):
    """--baseline-configs on (the default at 8 GPUs): after the line's own measurements every method
    of configs[2], [3] and [4] (stated sizes) runs on the job, one verified and one timed run each,
    and lands in the line; a plan that fails on one GPU (injected: m9 on GPU 1) is recorded for that
    cell on every rank and the rest go on"""
    import bench
    argv = ARGV2 + ["--baseline-configs", "on", "--no-ktime"]
    rcs, outs = _run_job(2, argv, tmp_path, {"XG_FAKE_PLAN_FAIL": "9:1"})
    assert rcs == [0, 0], [o[1][-1500:] for o in outs]
    out = json.loads([l for l in outs[0][0].splitlines() if l.startswith("{")][0])
    assert out["value"] > 0 and out["xgmi"]["peak"] > 0
    ex = out["baseline_configs_8gpu"]
    cells = ex["cells"]
    want = ["two-hop probe P8 A8 -d 16 MiB m9", "configs[2] m5", "configs[2] m8"] + \
           ["configs[3] m%d" % m for m in (1, 2, 9, 10)] + \
           ["configs[3] at -d 4 KiB m%d" % m for m in (1, 2, 9, 10)] + \
           ["configs[4] -c %d at -d 4 KiB m%d" % (c, m) for c in (1, 8) for m in (7, 11, 12)] + \
           ["configs[4] -c %d m%d" % (c, m) for c in (1, 8, 2, 3, 4, 5, 6, 7) for m in (7, 11, 12)]
    assert list(cells) == want
    # every reference cell run on the host has a GPU cell of the same key (side_by_side)
    assert {k for k, *_ in bench.CPU_CELLS} <= set(want)
    def failed(v):       # one form: its failure; several: every form's failure under "forms"
        return str(v).startswith("failed") or (isinstance(v, dict) and "verified" not in v and
                                                all(str(x).startswith("failed") for x in v["forms"].values()))
    m9 = ("two-hop probe P8 A8 -d 16 MiB m9", "configs[3] m9", "configs[3] at -d 4 KiB m9")
    assert all(failed(cells[k]) for k in m9)
    assert "injected" in str(out["rccl_log_tail"]) or out.get("rccl_log_tail") is None
    for k, v in cells.items():
        if k not in m9:
            assert v["verified"] and v["ms_per_run"] > 0 and v["GBps_cross_gpu"] > 0, (k, v)
            # FORM_REPS timed runs of the chosen form, its median the figure; the bytes its calls put
            # on the links beside the logical payload (a relayed byte crosses two links)
            assert len(v["runs_ms"]) == bench.FORM_REPS and v["ms_per_run"] == sorted(v["runs_ms"])[1], (k, v)
            assert v["link_bytes"] >= v["cross_gpu_bytes"] and v["GBps_link"] >= v["GBps_cross_gpu"], (k, v)
    assert cells["configs[4] -c 1 m7"]["cross_gpu_bytes"] == 256 * 64 * (64 << 20) // 2   # half the pairs cross
    assert "error" not in ex and ex["spent_s"] >= 0
    # each cell's link bound: its busiest-link bytes at the per-link sweep's median rate
    assert ex["link_GBps"] == bench.link_rate(out) and ex["link_GBps"] > 0
    for k, v in cells.items():
        if isinstance(v, dict) and "verified" in v:
            assert v["busiest_link_bytes"] > 0, (k, v)
            want_ms = v["busiest_link_bytes"] / (ex["link_GBps"] * 1e9) * 1e3
            assert abs(v["link_bound_ms"] - want_ms) <= 1e-4 + 1e-6 * want_ms, (k, v)
            # (from the unrounded run time: ms_per_run carries 4 decimals)
            assert v["link_bound_frac"] > 0 and \
                abs(v["link_bound_ms"] / v["link_bound_frac"] - v["ms_per_run"]) <= 1e-4 + 0.02 * v["ms_per_run"], (k, v)


def test_bench_baseline_configs_phase_keeps_to_its_budget(tmp_path):
    argv = ARGV2 + ["--baseline-configs", "on", "--baseline-budget", "0", "--no-ktime"]
    rcs, outs = _run_job(2, argv, tmp_path, {})
    assert rcs == [0, 0], [o[1][-1500:] for o in outs]
    out = json.loads([l for l in outs[0][0].splitlines() if l.startswith("{")][0])
    cells = out["baseline_configs_8gpu"]["cells"]
    assert len(cells) == 1 + 2 + 4 + 4 + 6 + 24 and all(str(v).startswith("skipped: phase budget") for v in cells.values())


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
    stated = [k for k in cells if k.startswith("configs[4]") and "at -d" not in k]
    rest = [k for k in stated if k != "configs[4] -c 1 m7"]
    assert len(rest) == 23 and all(cells[k] == "skipped: this configuration's regions did not fit" for k in rest)
    assert all(cells[k]["verified"] for k in cells if k not in stated)


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
               XG_RDZV_KEY=_key("wd0", tmp_path))
    code = DRIVER.format(repo=REPO, argv=["--gpus", "2", "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
                                          "--watchdog", "3"])
    try:
        p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    finally:
        rdzv = "/tmp/xg_bench_rdzv_%s.bin" % _key("wd0", tmp_path)
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


def test_measured_line_outlives_a_short_watchdog(tmp_path):
    """the watchdog guards the road to the value only.  With --watchdog 6 and the sweep
    hanging on GPU 1 under a 12 s xGMI budget, the watchdog (cancelled once the value is measured)
    must not replace the line with a null one: the xGMI LineGuard prints the measured line, exit 0"""
    argv = ARGV2 + ["--xgmi-budget", "12", "--no-ktime", "--watchdog", "6"]
    rcs, outs = _run_job(2, argv, tmp_path, {"XG_FAKE_P2P_HANG": "2", "XG_FAKE_FAIL_RANK": "1"})
    assert rcs == [0, 0], [o[1][-1500:] for o in outs]
    out = json.loads([l for l in outs[0][0].splitlines() if l.startswith("{")][0])
    assert out["value"] > 0 and out["xgmi_error"].startswith("still in phase 'xGMI p2p sweep' 12 s")
    assert out["phase_wall_s"]["xGMI p2p sweep"] >= 0


def test_pair_rounds_cover_every_link_once():
    import bench
    for n in range(2, 10):
        seen = set()
        rounds = bench.pair_rounds(n)
        assert len(rounds) == (n - 1 if n % 2 == 0 else n)
        for partner in rounds:
            for r, q in enumerate(partner):
                assert q == -1 or partner[q] == r
                if q >= 0:
                    assert (r, q) not in seen
                    seen.add((r, q))
        assert seen == {(r, q) for r in range(n) for q in range(n) if r != q}


def test_wall_bound_of_the_driver_runs():
    """the longest a rank of the driver's runs can take with every phase at its budget and every
    guard firing: N = 1 the watchdog only; N = 8 under torch.distributed.run rank 0
    runs both CPU phases first (the others allow for them), then watchdog + xGMI + BASELINE phases"""
    import bench
    sys.argv = ["bench.py"]
    a = bench.parse()
    assert bench.wall_bound(a, 1) == a.watchdog == 110
    b8 = bench.wall_bound(a, 8)
    assert b8 == a.cpu_budget + a.cpu_configs_budget + bench.CPU_GRACE + a.watchdog + a.xgmi_budget + \
        a.baseline_budget + bench.GUARD_GRACE
    # the only driver timeout on record is 600 s (BENCH_r05.json): 30 s of headroom for the launcher
    assert b8 <= 570, b8
    assert bench.wall_bound(a, 2) == a.cpu_budget + a.watchdog + a.xgmi_budget <= 570
    # every guard fires after its phase's own budget, never before
    assert bench.GUARD_GRACE > 0 and bench.pre_value_allowance(a, 1, 8, parent=True) == 0


def test_cpu_baseline_configs_budget_and_schema(tmp_path):
    """the reference itself at BASELINE's 8-GPU cells: a zero budget skips every cell; one real cell
    (configs[2] m5 at full size, 64 MPI processes) when the reference build is here; side_by_side
    pairs it with the GPU cell of the same key"""
    import bench
    sys.argv = ["bench.py", "--cpu-configs-budget", "0"]
    a = bench.parse()
    r = bench.cpu_baseline_configs(a)
    assert list(r["cells"]) == [k for k, *_ in bench.CPU_CELLS] and len(r["cells"]) == 12
    # every BASELINE 8-GPU method once before any -c repeats: configs[2] m5 / m8, configs[3] m1 / m2 /
    # m9 / m10, configs[4] m7 / m11 / m12, a2m / m2a / half-sync / pairwise in the first five
    first9 = [(k.split(" ")[0], m) for k, *_x, m in bench.CPU_CELLS[:9]]
    assert {"%s m%d" % km for km in first9} == \
        {"configs[2] m5", "configs[2] m8", "configs[3] m1", "configs[3] m2", "configs[3] m9", "configs[3] m10",
         "configs[4] m7", "configs[4] m11", "configs[4] m12"}
    assert [m for _k, m in first9[1:6]] == [1, 2, 7, 11, 9]
    assert r["cell_cap_s"] == bench.cell_cap(a) and "pinning" in r
    assert all(v.startswith("skipped: budget") for v in r["cells"].values())
    if not os.path.exists(os.path.join(REPO, "oracle", "_ref", "test")):
        pytest.skip("no reference build here")
    sys.argv = ["bench.py", "--cpu-configs-budget", "100"]
    a = bench.parse()
    r = bench.cpu_baseline_configs(a, cells=bench.CPU_CELLS[:1])
    c = r["cells"]["configs[2] m5"]
    assert c["P"] == 64 and c["d"] == 256 << 10 and c["max_total_time_s"] > 0 and c["GBps_delivered"] > 0, c
    out = {"cpu_baseline_configs": r,
           "baseline_configs_8gpu": {"cells": {"configs[2] m5": {"max_total_time_s": c["max_total_time_s"] / 100}}}}
    assert bench.side_by_side(out)["configs[2] m5"]["speedup"] == 100.0


def test_link_sweep_failure_is_recorded_with_the_rccl_tail(tmp_path):
    """an RCCL error on GPU 1 in the per-link sweep's second round: every rank stops the sweep at
    that round, the line records links_error and the rounds before it, and GPU 1's RCCL warning"""
    rcs, outs = _run_job(3, ["--gpus", "3", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--methods", "1"],
                         tmp_path, {"XG_FAKE_PAIR_FAIL": "1", "XG_FAKE_FAIL_RANK": "1"})
    assert rcs == [0, 0, 0], [o[1][-1500:] for o in outs]
    out = json.loads([l for l in outs[0][0].splitlines() if l.startswith("{")][0])
    x = out["xgmi"]
    assert x["links"]["rounds"] >= 1 and x["links_error"].startswith("round ")
    assert "1" in out["rccl_log_tail"] and "pair_bench" in out["rccl_log_tail"]["1"][-1]


def test_bench_baseline_configs_time_the_relay_form_where_it_applies(tmp_path):
    """a 4-GPU job with the BASELINE phase on: configs[3]'s pairwise m9 / m10 (permutation rounds of
    >= 1 MiB per GPU pair) are verified and timed in the direct and both relay forms and the faster is
    kept; m1 / m2 (every GPU to every GPU) have one form only"""
    argv = ["--gpus", "4", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--methods", "1",
            "--baseline-configs", "on", "--no-ktime"]
    rcs, outs = _run_job(4, argv, tmp_path, {})
    assert rcs == [0] * 4, [o[1][-1500:] for o in outs]
    cells = json.loads([l for l in outs[0][0].splitlines() if l.startswith("{")][0])["baseline_configs_8gpu"]["cells"]
    for m in (9, 10):
        c = cells["configs[3] m%d" % m]
        assert {"direct", "relay", "relay_coalesced"} <= set(c["forms"]) and c["chosen"] in c["forms"], c
        assert c["verified"], c
        for f in ("direct", "relay", "relay_coalesced"):
            st = c["forms"][f]
            assert st["min_ms"] <= st["median_ms"] <= st["max_ms"], c
        assert c["ms_per_run"] == c["forms"][c["chosen"]]["median_ms"] and c["margin"] is not None, c
        # the relay form's calls put (G - 2) / G of every relayed byte on two links
        if c["chosen"] in ("relay", "relay_coalesced"):
            assert c["link_bytes"] > c["cross_gpu_bytes"], c
    for m in (1, 2):
        assert not {"relay", "relay_coalesced"} & set(cells["configs[3] m%d" % m].get("forms", {}))
    # configs[4]'s 64 MiB segments are never packed: direct, and the relay forms where they reroute
    for k, c in cells.items():
        if k.startswith("configs[4] -c") and "at -d" not in k and isinstance(c, dict):
            assert set(c.get("forms", {"direct": 0})) <= {"direct", "relay", "relay_coalesced"}, (k, c)


def test_bench_cell_forms_are_the_librarys():
    """bench.CELL_FORMS names the library's forms (xg.py mirrors xg_sched.h)"""
    import bench
    import __graft_entry__ as G
    xg = G.load_package().xg
    assert dict(bench.CELL_FORMS) == {"direct": (0, -1), "packed_one_sided": (4 << 20, xg.PACK_ONE_SIDED),
                                      "packed_two_sided": (4 << 20, xg.PACK_TWO_SIDED), "relay": (0, xg.RELAY),
                                      "relay_coalesced": (0, xg.RELAY_COALESCED)}


def test_busiest_link_bytes_of_the_pairwise_plans(xg):
    """bench.busiest_link_bytes (the link bound beside every BASELINE cell) on configs[3]'s pairwise
    m9 at 8 GPUs: 224 XOR rounds of 16 MiB on one link each direct, a quarter of that relayed
    (the figures of profiles/r05/link_load.txt and tests/test_relay.py); m1's single all-to-all step
    spreads its bytes over every link; the median link rate comes from the per-link sweep"""
    import bench
    P, A, d = 256, 32, 4 << 20
    rl = xg.aggregator_list(P, A)
    s9 = xg.Schedule(9, P, A, d, 200000000, rl, ntimes=1)
    assert bench.busiest_link_bytes(xg, s9, 8, 0, -1) == 3584 << 20
    assert bench.busiest_link_bytes(xg, s9, 8, 0, xg.RELAY) == 896 << 20
    s1 = xg.Schedule(1, P, A, d, 200000000, rl, ntimes=1)
    assert bench.busiest_link_bytes(xg, s1, 8, 0, -1) == 512 << 20
    assert bench.link_rate({"xgmi": {"links": {"GBps": [[None, 40.0, 50.0], [45.0, None, 60.0], [55.0, 52.0, None]]}}}) == 52.0
    assert bench.link_rate({"xgmi": None}) is None


def _line(outs):
    return json.loads([l for l in outs[0][0].splitlines() if l.startswith("{")][0])


@pytest.mark.parametrize("delays,chosen", [
    ("2:30", "direct"),                 # relay runs take 30 ms, the other forms ~0: direct kept
    ("-1:60,1:60,0:60,2:10,3:40", "relay"),  # relay 10 ms against 40-60 ms for every other form
    ("-1:60,1:60,0:60,2:30,3:10", "relay_coalesced"),
])
def test_headline_form_choice_weighs_the_relay_form(tmp_path, delays, chosen):
    """a workload whose pairwise rounds the relay form reroutes (P16 A8 -d 1 MiB, m9, 3 GPUs): the N > 1
    line's per-method choice times both relay forms beside direct and both packed forms, FORM_REPS times
    each (fake run times: XG_FAKE_FORM_DELAY), and keeps direct unless a form's median beats it by
    more than the spread"""
    argv = ["--gpus", "3", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-ktime", "--procs", "16",
            "--aggs", "8", "--comm-size", "3", "--methods", "9"]
    rcs, outs = _run_job(3, argv, tmp_path, {"XG_FAKE_FORM_DELAY": delays})
    assert rcs == [0, 0, 0], [o[1][-1500:] for o in outs]
    tune = _line(outs)["pack_autotune_ms_per_run"]["9"]
    assert "relay_ms" in tune and set(tune["stats"]) == {"direct", "packed_one_sided", "packed_two_sided", "relay",
                                                         "relay_coalesced"}
    assert tune["chosen"] == chosen, tune


def test_choose_form_rule():
    """choose_form: direct is kept unless another form's median beats it by more than the spread of
    either; among those that do, the lowest median; without direct, the lowest median"""
    import bench
    ms = lambda *v: [x / 1e3 for x in v]
    # relay's median 2 ms faster, both spreads 1 ms: relay
    c, st, margin = bench.choose_form({"direct": ms(10, 10.5, 11), "relay": ms(8, 8.5, 9)})
    assert c == "relay" and st["relay"]["median_ms"] == 8.5 and margin == pytest.approx(2 / 8.5, abs=1e-4)
    # 0.5 ms faster with a 1 ms spread: direct kept, a negative margin records the faster median
    c, st, margin = bench.choose_form({"direct": ms(10, 10.5, 11), "relay": ms(9.5, 10, 10.2)})
    assert c == "direct" and margin < 0
    # a noisy candidate (spread 5 ms) 3 ms ahead: direct kept
    c, _st, _m = bench.choose_form({"direct": ms(10, 10, 10), "packed_two_sided": ms(4, 7, 9)})
    assert c == "direct"
    # two qualifying forms: the lower median
    c, _st, _m = bench.choose_form({"direct": ms(10, 10, 10), "relay": ms(6, 6, 6), "packed_one_sided": ms(5, 5, 5)})
    assert c == "packed_one_sided"
    # direct failed verification: the lowest median of the rest
    c, _st, margin = bench.choose_form({"relay": ms(6, 6, 7), "packed_two_sided": ms(5, 9, 9)})
    assert c == "relay" and margin == pytest.approx(0.5)
    assert bench.choose_form({}) == (None, {}, None)


def test_cell_estimate_from_the_link_rate():
    """a BASELINE cell's least run time: every form's verified run + FORM_REPS timed runs, each its
    busiest-link bytes at the measured per-link rate; no rate, no estimate (the cell runs)"""
    import bench
    links = {"direct": (50 * 10 ** 9, 0), "relay": (25 * 10 ** 9, 0)}
    assert bench.cell_estimate_s(links, 50.0) == pytest.approx((1 + bench.FORM_REPS) * 1.5)
    assert bench.cell_estimate_s(links, None) == 0.0


@pytest.mark.parametrize("tier", [1, 2])
def test_bench_baseline_configs_drop_the_staging_that_does_not_fit(tmp_path, xg, tier):
    """GPU 1 of a 4-GPU job can hold configs[3]'s full-size regions with the staging of tier `tier`'s
    forms but not of the tier above (injected limit between the two; tier 1: every form but the
    coalesced relay form, tier 2: direct alone): the pairwise cells run the forms that fit, on every
    GPU alike, and say which forms were left out and why"""
    import bench
    P, A, d, c = 256, 32, 4 << 20, 200000000
    rl = xg.aggregator_list(P, A)
    sums = [[0] * xg.NBUF for _ in bench.CELL_TIERS]
    for m in (1, 2, 9, 10):
        s = xg.Schedule(m, P, A, d, c, rl, ntimes=1)
        for fname, f in bench.CELL_FORMS:
            rb = s.devplan(4, 1, f[0], 0, f[1]).region_bytes
            for k, names in enumerate(bench.CELL_TIERS):
                if fname in names:
                    sums[k] = [max(x, y) for x, y in zip(sums[k], rb)]
    lo, hi = sum(sums[tier]), sum(sums[tier - 1])
    assert lo < hi
    argv = ["--gpus", "4", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--methods", "1",
            "--baseline-configs", "on", "--no-ktime"]
    rcs, outs = _run_job(4, argv, tmp_path, {"XG_FAKE_REGIONS_FAIL": "%d:1" % ((lo + hi) // 2)})
    assert rcs == [0] * 4, [o[1][-1500:] for o in outs]
    cells = _line(outs)["baseline_configs_8gpu"]["cells"]
    for m in (9, 10):
        cell = cells["configs[3] m%d" % m]
        assert isinstance(cell, dict) and cell["verified"], cell
        ran = set(cell.get("forms", {"direct": 0}))
        assert ran == {"direct", "relay", "relay_coalesced"} & set(bench.CELL_TIERS[tier]), cell
        assert set(cell["forms_not_run"]) == {"relay", "relay_coalesced"} - ran, cell
    # the reduced -d configuration's regions fit whole (nothing relayed there: no relay form at all)
    assert "forms_not_run" not in cells["configs[3] at -d 4 KiB m9"]


def test_heartbeat_names_the_phase(capfd):
    """rank 0's heartbeat: the current phase on stderr every HEARTBEAT_S seconds, so a quiet phase
    (minutes of the reference at the BASELINE cells) shows progress"""
    import bench
    bench.phase("cpu baseline at the BASELINE 8-GPU configurations")
    stop = bench.start_heartbeat(0.2)
    time.sleep(0.7)
    stop.set()
    err = capfd.readouterr().err
    assert err.count("bench: cpu baseline at the BASELINE 8-GPU configurations (") >= 2, err


def test_reference_pinning_per_run(monkeypatch):
    """the reference's configs[1] baseline runs unpinned, its 256-rank BASELINE cells pinned to the
    quota's CPUs (when a quota sits below the mask); XG_REF_PIN=0 / 1 forces either"""
    import bench
    monkeypatch.setattr(bench, "host_cpus", lambda: (2, "test quota"))
    monkeypatch.delenv("XG_REF_PIN", raising=False)
    mask = sorted(os.sched_getaffinity(0))
    assert bench.reference_cpus(pin=False) is None
    assert bench.reference_cpus(pin=True) == (mask[:2] if len(mask) > 2 else None)
    monkeypatch.setenv("XG_REF_PIN", "0")
    assert bench.reference_cpus(pin=True) is None
    monkeypatch.setenv("XG_REF_PIN", "1")
    assert bench.reference_cpus(pin=False) == (mask[:2] if len(mask) > 2 else None)
