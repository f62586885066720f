"""bin/test on the GPU: stdout of every method equals the reference's stdout with
numbers masked (tests/golden/<cfg>/report_m<N>.txt), results.csv has the
reference's columns, and --verify confirms every byte on the device."""
import os
import re
import subprocess

import pytest

from conftest import GOLDEN, load_golden

pytestmark = pytest.mark.gpu


def _mask(text):
    return re.sub(r"\d+(\.\d+)?", "#", text)


@pytest.mark.parametrize("cfg", ["readme_p32_a14", "p16_a5_d1000_c3", "p16_a5_c4_b2", "p8_a3_d0_c3"])
def test_cli_report_matches_reference(pkg, cfg, tmp_path):
    meta, _, _ = load_golden(cfg)
    exe = os.path.join(os.path.dirname(pkg.__file__), "bin", "test")
    for m in meta["method_list"]:
        args = [exe, "--procs", str(meta["P"])] + meta["args"].split() + ["-m", str(m)]
        out = subprocess.run(args, capture_output=True, text=True, timeout=120, cwd=str(tmp_path))
        assert out.returncode == 0, out.stderr[-2000:]
        golden = open(os.path.join(GOLDEN, cfg, "report_m%d.txt" % m)).read()
        assert _mask(out.stdout) == golden, (cfg, m, out.stdout[:500])
        if m == 13:   # save_all_timing files: same names, shapes and rank column as the reference's
            for fn, (nrows, ncols, ranks) in meta["m13_timing_files"].items():
                rows = [r.split(",") for r in open(str(tmp_path / fn)).read().splitlines()]
                assert len(rows) == nrows and all(len(r) == ncols for r in rows), fn
                assert [int(r[0]) for r in rows] == ranks
    rows = open(str(tmp_path / "results.csv")).read().splitlines()
    assert rows[0].count(",") == 14 and len(rows) == 1 + len(meta["method_list"]) * meta["iters"]


def test_cli_verify_all_methods(pkg, tmp_path):
    exe = os.path.join(os.path.dirname(pkg.__file__), "bin", "test")
    out = subprocess.run([exe, "--procs", "20", "-a", "6", "-d", "4000", "-c", "3", "-m", "0", "-i", "2", "-k", "2",
                          "--verify", "--fingerprint", "strong"],
                         capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert out.returncode == 0, out.stderr[-2000:]
    verdicts = re.findall(r"verify = (\w+)", out.stdout)
    assert len(verdicts) == 40 and set(verdicts) == {"OK"}, out.stdout[-3000:]


def test_cli_refuses_reference_deadlock(pkg, tmp_path):
    """m6 at P32 A14 c3 with rendezvous-size segments hangs in the reference; here it is refused."""
    exe = os.path.join(os.path.dirname(pkg.__file__), "bin", "test")
    out = subprocess.run([exe, "--procs", "32", "-a", "14", "-d", "65536", "-c", "3", "-m", "6"],
                         capture_output=True, text=True, timeout=120, cwd=str(tmp_path))
    assert out.returncode == 0 and "deadlocks" in out.stderr


@pytest.mark.parametrize("cfg", ["cfg1_p32_a14_d1m", "cfg2_p64_a16_d256k", "cfg3_p256_a32_d64k", "cfg4_p256_a64_d4k_c3"])
def test_cli_report_matches_reference_at_baseline_shapes(pkg, cfg, tmp_path):
    """bin/test at the BASELINE.json shapes (one GPU hosts every rank): the report of every
    captured method equals the reference's with numbers masked, with --verify confirming every
    byte; a method the reference hung on (configs[1] m6) is refused and named on stderr."""
    from conftest import BASELINE, load_baseline
    meta, _, _ = load_baseline(cfg)
    exe = os.path.join(os.path.dirname(pkg.__file__), "bin", "test")
    for m in sorted(int(x) for x in meta["methods"]):
        args = [exe, "--procs", str(meta["P"])] + meta["args"].split() + ["-m", str(m)]
        out = subprocess.run(args + ["--verify"], capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
        assert out.returncode == 0, (cfg, m, out.stderr[-2000:])
        if meta["methods"][str(m)]["status"] == "timeout":
            assert "deadlocks" in out.stderr and "max total time" not in out.stdout, (cfg, m)
            continue
        golden = open(os.path.join(BASELINE, cfg, "report_m%d.txt" % m)).read()
        verified = [ln for ln in out.stdout.splitlines() if "verify = " in ln]
        body = "\n".join(ln for ln in out.stdout.splitlines() if "verify = " not in ln) + "\n"
        assert _mask(body) == golden, (cfg, m, out.stdout[:500])
        assert len(verified) == meta["iters"] and all("verify = OK" in ln for ln in verified), (cfg, m, verified)
