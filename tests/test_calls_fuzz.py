"""xg_calls_match under AddressSanitizer + UndefinedBehaviorSanitizer: tests/calls_fuzz.c built
with calls.c as one standalone executable (CPU only), random valid and broken G-GPU jobs."""
import os
import shutil
import subprocess

import pytest

from conftest import REPO


@pytest.mark.skipif(not shutil.which("gcc"), reason="gcc not found")
def test_calls_match_fuzz_under_sanitizers(tmp_path):
    exe = str(tmp_path / "calls_fuzz")
    src = os.path.join(REPO, "mpi-asynchronous-communication-test_amd", "csrc", "host", "calls.c")
    subprocess.run(["gcc", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-std=c99",
                    "-D_POSIX_C_SOURCE=200809L", "-Wall", "-Wextra", "-I", os.path.join(REPO, "include"), "-o", exe,
                    os.path.join(REPO, "tests", "calls_fuzz.c"), src], check=True)
    p = subprocess.run([exe, "3000"], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1"))
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    assert "ok after 3000 jobs" in p.stdout


@pytest.mark.skipif(not shutil.which("gcc"), reason="gcc not found")
def test_devplan_builders_fuzz_under_sanitizers(tmp_path):
    """every plan form of random shapes built and pairing-proven under ASan + UBSan (leaks on):
    tests/devplan_fuzz.c with all host sources"""
    exe = str(tmp_path / "devplan_fuzz")
    host = os.path.join(REPO, "mpi-asynchronous-communication-test_amd", "csrc", "host")
    srcs = [os.path.join(host, f) for f in ("programs.c", "sched.c", "devplan.c", "report.c", "hazard.c", "solo.c",
                                            "calls.c", "pieces.c")]
    subprocess.run(["gcc", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-std=c99",
                    "-D_POSIX_C_SOURCE=200809L", "-Wall", "-Wextra", "-I", os.path.join(REPO, "include"), "-I", host,
                    "-o", exe, os.path.join(REPO, "tests", "devplan_fuzz.c")] + srcs + ["-lm"], check=True)
    p = subprocess.run([exe, "150"], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1"))
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    assert "ok after 150 jobs" in p.stdout, p.stdout
