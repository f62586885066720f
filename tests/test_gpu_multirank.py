"""Real multi-rank jobs on the box's one MI355X: G processes, one RCCL communicator of G ranks.

Until round 5 the multi-rank path (ncclCommInitRank with nranks > 1, enqueue_step's groups to
real peers, xg_barrier / xg_allreduce_max across processes) had never executed on a device: RCCL
refuses two ranks on one GPU ("Duplicate GPU detected", profiles/r04/two_ranks/).  With
XG_SHARE_GPU=1 every rank names a host of its own (NCCL_HOSTID, runtime/ctx.hip), so RCCL accepts
the job and pairs the ranks over its socket transport on loopback instead of xGMI: the calls, the
groups, RCCL's pairing and the collectives are the real ones, the transport and its rates are not
the node's.  Every received slot is compared with the checksum the REFERENCE's receive buffer had
(tests/golden/, captured under MPICH by oracle/pmpi_capture.c).

Reference: the MPI_Issend / MPI_Irecv / MPI_Waitall exchange (mpi_test.c:1771-1816), MPI_Sendrecv
(:551-563), MPI_Alltoallw (:627, :912), MPI_Barrier / MPI_Reduce (:2184); pt2pt_test
(mpi_sendrecv_test.c:15-74).
"""
import json
import os
import re
import signal
import subprocess
import sys

import pytest

from conftest import REPO, baseline_configs, golden_configs

pytestmark = pytest.mark.gpu

WORKER = os.path.join(REPO, "tests", "multirank_worker.py")
BIN = os.path.join(REPO, "mpi-asynchronous-communication-test_amd", "bin")
DIRECT, ONE_SIDED, TWO_SIDED, RELAY, COALESCED = [0, -1], [1 << 30, 1], [1 << 30, 0], [0, 2], [0, 3]


def _env(tmp_path, **kw):
    env = dict(os.environ, XG_SHARE_GPU="1", NCCL_DEBUG=os.environ.get("NCCL_DEBUG", "WARN"),
               XG_MR_DIR=str(tmp_path), GPU_MAX_HW_QUEUES="1")     # the box exports 4: see runtime/ctx.hip
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "XG_RDZV_KEY"):
        env.pop(k, None)
    env.update({k: str(v) for k, v in kw.items()})
    return env


def _wait_all(procs, timeout):
    """wait for every process of the job (their output goes to files: a rank -- or its RCCL proxy
    thread logging a warning -- blocked on a full pipe nobody reads would stall every rank in
    RCCL); past `timeout` s end each one's session (its exact process group) and fail with what
    each rank printed last.  procs: [(Popen, stdout path, stderr path)] -> [(stdout, stderr)]"""
    import time
    t0 = time.time()
    try:
        for p, _o, _e in procs:
            p.wait(timeout=max(1.0, timeout - (time.time() - t0)))
    except subprocess.TimeoutExpired:
        for p, _o, _e in procs:
            if p.poll() is None:
                os.killpg(p.pid, signal.SIGKILL)
        for p, _o, _e in procs:
            p.wait()
        tails = ["rank %d: ...%s | stderr ...%s" % (r, open(o).read()[-300:], open(e).read()[-600:])
                 for r, (p, o, e) in enumerate(procs)]
        pytest.fail("multi-rank job still running after %d s\n%s" % (timeout, "\n".join(tails)))
    return [(open(o).read(), open(e).read()) for _p, o, e in procs]


def _spawn(cmd, env, cwd, tag, tmp_path):
    o, e = str(tmp_path / ("%s.out" % tag)), str(tmp_path / ("%s.err" % tag))
    with open(o, "w") as fo, open(e, "w") as fe:
        p = subprocess.Popen(cmd, env=env, cwd=cwd, stdout=fo, stderr=fe, text=True, start_new_session=True)
    return p, o, e


def _job(tmp_path, G, cases, timeout=120):
    """G worker processes over one RCCL communicator; -> rank 0's result lines"""
    import pathlib
    import tempfile
    tmp_path = pathlib.Path(tempfile.mkdtemp(prefix="job", dir=str(tmp_path)))   # its own RCCL id file
    procs = [_spawn([sys.executable, "-u", WORKER, json.dumps(cases)],
                    _env(tmp_path, RANK=r, WORLD_SIZE=G, LOCAL_RANK=r, XG_MR_DEADLINE=timeout - 10), None,
                    "rank%d" % r, tmp_path)
             for r in range(G)]
    outs = _wait_all(procs, timeout)
    failed = ["rank %d exit %d: %s" % (r, p.returncode, " | ".join(err.strip().splitlines()[-3:]))
              for r, ((p, _o, _e), (out, err)) in enumerate(zip(procs, outs)) if p.returncode]
    assert not failed, "\n".join(failed)
    lines = [json.loads(x) for x in outs[0][0].splitlines() if x.startswith("{")]
    assert lines and lines[-1] == {"done": True}, outs[0]
    return lines[:-1]


def _assert_exact(rows, expect_runs):
    assert len(rows) == expect_runs, [r for r in rows][:3]
    bad = [r for r in rows if "error" in r or r["wrong"] or r["slots"] != r["want"] or r["slots"] == 0]
    assert not bad, bad[:5]


GOLDEN = golden_configs()


@pytest.mark.parametrize("half", [0, 1])
def test_golden_configs_as_two_rank_jobs(tmp_path, half):
    """the 13 reference captures (README config, unaligned d, every placement type, -c 1..7,
    -k up to 3, A = 1, A = P, barrier types, -p 2/4, -d 0), every method 1-20, as 2-rank jobs in
    the direct and both packed forms"""
    from conftest import load_golden
    names = GOLDEN[half::2]
    cases = [{"golden": n, "forms": [DIRECT, TWO_SIDED, ONE_SIDED]} for n in names]
    runs = sum(len(load_golden(n)[0]["method_list"]) * 3 for n in names)
    _assert_exact(_job(tmp_path, 2, cases), runs)


@pytest.mark.parametrize("G", [3, 8])
def test_golden_configs_as_g_rank_jobs(tmp_path, G):
    """the same captures as 3-rank (a block map with a ragged last GPU; direct and two-sided) and
    8-rank jobs (the driver's node size; direct)"""
    from conftest import load_golden
    forms = [DIRECT, TWO_SIDED] if G < 8 else [DIRECT]
    cases = [{"golden": n, "forms": forms} for n in GOLDEN]
    runs = sum(len(load_golden(n)[0]["method_list"]) * len(forms) for n in GOLDEN)
    _assert_exact(_job(tmp_path, G, cases, timeout=140), runs)


def test_baseline_shapes_as_eight_rank_job(tmp_path):
    """the reference captured at the BASELINE.json shapes (configs[1] and configs[2] at full size,
    configs[3]'s P256 A32 at -d 64 KiB, configs[4]'s P256 A64 at -d 4 KiB for -c 1 and 8) as one
    8-rank job -- the configurations the driver's 8-GPU run executes, on its rank count"""
    from conftest import load_baseline
    names = [n for n in baseline_configs() if not n.startswith("cfg4") or n.endswith(("_c1", "_c8"))]
    assert len(names) == 5
    cases = [{"golden": "baseline/" + n, "forms": [DIRECT]} for n in names]
    runs = sum(len(load_baseline(n)[0]["method_list"]) for n in names)
    _assert_exact(_job(tmp_path, 8, cases, timeout=140), runs)


@pytest.mark.parametrize("cfg", ["cfg1_p32_a14_d1m", "cfg2_p64_a16_d256k"])
def test_bench_workloads_as_two_and_four_rank_jobs(tmp_path, cfg):
    """the bench's own N = 2 / 4 workloads (configs[1]) and configs[2]'s shape, both packed forms
    too (and the relay form at configs[1], 4 ranks), against the reference's checksums"""
    from conftest import load_baseline
    meta = load_baseline(cfg)[0]
    methods = meta["method_list"]
    for G in (2, 4):
        # configs[1]'s 1 MiB segments: at 4 ranks the relay form reroutes m9 / m10's XOR rounds
        forms = [DIRECT, ONE_SIDED, TWO_SIDED] + ([RELAY] if G > 2 and meta["d"] >= 1 << 20 else [])
        rows = _job(tmp_path, G, [{"golden": "baseline/" + cfg, "forms": forms}])
        _assert_exact(rows, len(forms) * len(methods))


@pytest.mark.parametrize("G", [4, 8])
def test_relay_form_as_multi_rank_job(tmp_path, G):
    """the relay forms (XG_RELAY, XG_RELAY_COALESCED) between real ranks: pairwise m9 / m10 (each XOR
    round relayed over every other GPU in two RCCL groups) and m12 / m1 (their permutation steps
    relayed, the rest direct) at P16 A8 -d 1 MiB, and at 8 ranks configs[3]'s P256 A32 at -d 1 MiB
    (lists of 4 MiB per round: the coalesced form packs 4 pieces per call) -- every slot byte-checked
    on the device, sampled slots against the oracle's closed form; an -d of (1 << 20) + 3 puts every
    piece of a relayed message at an odd address"""
    forms = [DIRECT, RELAY, COALESCED]
    cases = [{"shape": [16, 8, 1 << 20, 3], "methods": [9, 10, 12, 1], "forms": forms},
             {"shape": [16, 8, (1 << 20) + 3, 3], "methods": [9, 10, 12], "forms": forms},
             {"shape": [32, 16, (1 << 20) + 3, 3], "methods": [9, 11, 12], "forms": [COALESCED]}]
    if G == 8:
        cases.append({"shape": [256, 32, 1 << 20, 200000000], "methods": [9, 10], "forms": forms})
    rows = _job(tmp_path, G, cases, timeout=140)
    _assert_exact(rows, sum(len(c["methods"]) * len(c["forms"]) for c in cases))


@pytest.mark.parametrize("c", [1, 8])
def test_relay_form_config4_as_eight_rank_job(tmp_path, c):
    """configs[4]'s own plans (P256 A64) in the relay form between 8 real ranks, at -d 1 MiB (the
    smallest -d the relay form engages at: XG_RELAY_MIN_BYTES) and -c 1 / 8: m11 / m12, whose steps
    the relay form rewrites (252 of 256 and 256 of 256 at the stated size, profiles/r05/link_load.txt),
    and m7, which it leaves direct.  The N = 8 BASELINE phase times exactly these plans; every slot
    is byte-checked on the device and sampled slots equal the oracle's closed form.
    The coalesced relay form (XG_RELAY_COALESCED) runs the same relayed steps, and m7's steps in its
    weighted two-hop split.
    Reference: many_to_all_half_sync / all_to_many_half_sync2 (mpi_test.c:942-997, :999-1053)."""
    cases = [{"shape": [256, 64, 1 << 20, c], "methods": [11, 12, 7], "forms": [DIRECT, RELAY, COALESCED]}]
    rows = _job(tmp_path, 8, cases, timeout=140)
    _assert_exact(rows, 9)
    for form in (RELAY, COALESCED):
        relayed = {r["method"]: r["relayed_steps"] for r in rows if r["form"] == form}
        assert relayed[11] > 0 and relayed[12] > 0, (form, relayed)
        # m7: no uniform cut helps; the coalesced form's weighted two-hop split reroutes its steps
        assert (relayed[7] > 0) == (form == COALESCED), (form, relayed)
    assert all(r["relayed_steps"] == 0 for r in rows if r["form"] == DIRECT)


def _cli(args, tmp_path, G, timeout=120, exe="test"):
    env = _env(tmp_path, XG_GPUS=G, XG_RDZV_DIR=tmp_path)
    (tmp_path / "cwd").mkdir(exist_ok=True)
    job = _spawn([os.path.join(BIN, exe)] + [str(a) for a in args], env, str(tmp_path / "cwd"), exe, tmp_path)
    (out, err), = _wait_all([job], timeout)
    assert job[0].returncode == 0, err[-3000:]
    return out


def _masked(out):
    return [re.sub(r"[0-9]+\.[0-9]+", "T", x) for x in out.splitlines()]


@pytest.mark.parametrize("G", [2, 8])
def test_cli_readme_config_as_multi_rank_job(tmp_path, G):
    """bin/test --gpus G (the drop-in CLI spawning its own G processes) on the README configuration,
    every method 1-20 byte-verified on the device, and the report identical in form to the one-
    process run's"""
    args = ["--procs", 32, "-a", 14, "-d", 2048, "-c", 3, "-m", 0, "-i", 1, "-k", 2, "--verify"]
    out = _cli(args, tmp_path, G)
    assert out.count("verify = OK") == 20 and "FAILED" not in out, out[-2000:]
    (tmp_path / "one").mkdir()
    one = _cli(args, tmp_path / "one", 1)
    assert _masked(out) == _masked(one)


@pytest.mark.parametrize("form", [2, 3])
def test_cli_relay_forms_as_four_rank_job(tmp_path, form):
    """bin/test --gpus 4 --pack-form 2 / 3 (the relay and coalesced relay forms, through the drop-in
    CLI) at an odd -d past 1 MiB, where they reroute steps: every method 1-20 byte-verified on the
    device, the report identical in form to the one-process run's"""
    args = ["--procs", 12, "-a", 5, "-d", (1 << 20) + 3, "-c", 3, "-m", 0, "-i", 1, "-k", 1, "--verify",
            "--pack-form", form]
    out = _cli(args, tmp_path, 4)
    assert out.count("verify = OK") == 20 and "FAILED" not in out, out[-2000:]
    (tmp_path / "one").mkdir()
    one = _cli(args, tmp_path / "one", 1)
    assert _masked(out) == _masked(one)


def test_pt2pt_as_two_rank_job(tmp_path):
    """bin/pt2pt_test as two processes (the reference's pt2pt_test runs under mpiexec -n 2): rank
    1's Issend to rank 0 as an RCCL send between two communicator ranks; the output masked equals
    the reference's own 2-process output (tests/golden/pt2pt), one sendrecv_results.csv row per -k"""
    from conftest import GOLDEN as GDIR
    out = _cli(["-d", 4096, "-k", 3, "-i", 5], tmp_path, 2, exe="pt2pt_test")
    mask = lambda t: re.sub(r"\d+(\.\d+)?", "#", t)
    golden = open(os.path.join(GDIR, "pt2pt", "report_n2.txt")).read().splitlines()
    assert sorted(mask(out).splitlines()) == sorted(golden), out
    rows = open(str(tmp_path / "cwd" / "sendrecv_results.csv")).read().splitlines()
    assert len(rows) == 3 and all(float(r) > 0 for r in rows)


def test_bench_line_from_a_real_two_rank_job(tmp_path):
    """bench.py --gpus 2 with both ranks on this GPU: the whole N > 1 line -- per-method form choice
    with its margin, the per-launch roofline pass, the RCCL ceiling, the pt2pt sweep, the per-link
    sweep, RCCL's version, each phase's wall time -- from a real 2-rank RCCL job, labelled as not
    xGMI (the transport is RCCL's sockets)"""
    env = _env(tmp_path)
    job = _spawn([sys.executable, "-u", os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
                  "--no-cpu-baseline", "--baseline-configs", "off"], env, str(tmp_path), "bench", tmp_path)
    (out, err), = _wait_all([job], 130)
    assert job[0].returncode == 0, err[-3000:]
    line = json.loads([x for x in out.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["value"] > 0 and "not xGMI" in line["transport"]
    assert line["rccl_version"] >= 22700 and line["roofline"]["launches"] > 0
    assert all(t["chosen"] and t["margin"] is not None for t in line["pack_autotune_ms_per_run"].values())
    x = line["xgmi"]
    assert x["peak"] > 0 and x["ceiling_error"] is None and x["sweep_error"] is None and len(x["sweep"]) == 8
    assert x["links"]["rounds"] == 1 and x["links"]["GBps"][0][1] > 0 and x["links"]["GBps"][1][0] > 0
    assert set(line["phase_wall_s"]) >= {"timed steps", "xGMI per-link sweep"}


def test_bench_line_under_torchrun_launch_form(tmp_path):
    """the driver's own N > 1 command form -- python -m torch.distributed.run --nnodes=1
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port P bench.py --gpus 2 ... -- with both
    ranks on this GPU: rank 0 runs the reference's CPU baseline before it touches the GPU and writes
    the RCCL id, rank 1 waits for it (its watchdog allowing for rank 0's CPU phase), and rank 0 prints
    the one line (the launcher imports torch in its agent process only; no rank does)"""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = _env(tmp_path)
    job = _spawn([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                  "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(REPO, "bench.py"),
                  "--gpus", "2", "--steps", "3", "--warmup", "1", "--baseline-configs", "off", "--cpu-reps", "2"],
                 env, str(tmp_path), "torchrun", tmp_path)
    (out, err), = _wait_all([job], 140)
    assert job[0].returncode == 0, err[-3000:]
    lines = [x for x in out.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["value"] > 0 and "not xGMI" in line["transport"]
    assert line["cpu_baseline"]["kind"] in ("reference", "port") and line["xgmi"]["links"]["rounds"] == 1
    assert "cpu baseline" in line["phase_wall_s"]
