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


@pytest.mark.parametrize("cfg", ["readme_p32_a14", "p16_a5_d1000_c3"])
def test_cli_report_matches_reference(pkg, cfg, tmp_path):
    meta, _, _ = load_golden(cfg)
    exe = os.path.join(os.path.dirname(pkg.__file__), "bin", "test")
    for m in range(1, 13):
        args = [exe, "--procs", str(meta["P"])] + meta["args"].split() + ["-m", str(m)]
        out = subprocess.run(args, capture_output=True, text=True, timeout=120, cwd=str(tmp_path))
        assert out.returncode == 0, out.stderr[-2000:]
        golden = open(os.path.join(GOLDEN, cfg, "report_m%d.txt" % m)).read()
        assert _mask(out.stdout) == golden, (cfg, m, out.stdout[:500])
    rows = open(str(tmp_path / "results.csv")).read().splitlines()
    assert rows[0].count(",") == 14 and len(rows) == 1 + 12 * meta["iters"]


def test_cli_verify_all_methods(pkg, tmp_path):
    exe = os.path.join(os.path.dirname(pkg.__file__), "bin", "test")
    out = subprocess.run([exe, "--procs", "20", "-a", "6", "-d", "4000", "-c", "3", "-m", "0", "-i", "2", "-k", "2",
                          "--verify", "--fingerprint", "strong"],
                         capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert out.returncode == 0, out.stderr[-2000:]
    verdicts = re.findall(r"verify = (\w+)", out.stdout)
    assert len(verdicts) == 24 and set(verdicts) == {"OK"}, out.stdout[-3000:]


def test_cli_refuses_reference_deadlock(pkg, tmp_path):
    """m6 at P32 A14 c3 with rendezvous-size segments hangs in the reference; here it is refused."""
    exe = os.path.join(os.path.dirname(pkg.__file__), "bin", "test")
    out = subprocess.run([exe, "--procs", "32", "-a", "14", "-d", "65536", "-c", "3", "-m", "6"],
                         capture_output=True, text=True, timeout=120, cwd=str(tmp_path))
    assert out.returncode == 0 and "deadlocks" in out.stderr
