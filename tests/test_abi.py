"""The C-ABI libraries load without a GPU and export every function include/*.h declares."""
import ctypes
import os
import re

from conftest import REPO

PKG = os.path.join(REPO, "mpi-asynchronous-communication-test_amd")


def declared(header):
    src = open(os.path.join(REPO, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return set(re.findall(r"\b(xg_[a-z0-9_]+)\s*\(", src))


def test_host_library_exports_xg_sched_h(xg):
    lib = ctypes.CDLL(os.path.join(PKG, "lib", "libxghost.so"))
    names = declared("xg_sched.h")
    assert len(names) > 20
    missing = [n for n in sorted(names) if not hasattr(lib, n)]
    assert not missing, missing


def test_device_library_exports_xg_h(xg):
    xg.device()            # loads libxg.so; no HIP call is made
    lib = ctypes.CDLL(os.path.join(PKG, "lib", "libxg.so"))
    names = declared("xg.h")
    assert len(names) > 20
    missing = [n for n in sorted(names) if not hasattr(lib, n)]
    assert not missing, missing


def test_product_does_not_reference_oracle():
    """The product path never imports/links the checker."""
    for root, _dirs, files in os.walk(PKG):
        for f in files:
            if f.endswith((".py", ".c", ".h", ".hip", "Makefile")):
                txt = open(os.path.join(root, f), errors="ignore").read()
                assert "xg_oracle" not in txt and "oracle/" not in txt, f


def test_device_library_refuses_a_foreign_rocm_runtime():
    """A process that imported torch first holds torch's bundled libamdhip64.so.7 / librccl.so.1
    (the same sonames as /opt/rocm's): xg.device() refuses to load libxg.so there rather than
    bind it to another runtime (the full GPU suite hung in RCCL that way, profiles/r04/torch_runtime/).
    In a fresh process nothing foreign is mapped and it loads."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r); %s import __graft_entry__ as G; xg = G.load_package().xg\n"
            "try:\n    xg.device(); print('loaded', xg.foreign_rocm_runtime())\n"
            "except xg.XGError as e:\n    print('refused', e)\n")
    for pre, want in (("", "loaded []"), ("import torch;", "refused")):
        out = subprocess.run([sys.executable, "-c", code % (REPO, pre)], capture_output=True, text=True, timeout=300)
        assert out.returncode == 0 and out.stdout.startswith(want), (pre, out.stdout, out.stderr[-1000:])


def _foreign_hip(tmp_path):
    """a copy of /opt/rocm's libamdhip64.so.7 outside the ROCm install: what the loader binds first
    when LD_LIBRARY_PATH points at a directory holding one (torch's wheel bundles its own)"""
    import shutil
    d = tmp_path / "foreign"
    d.mkdir()
    shutil.copy("/opt/rocm/lib/libamdhip64.so.7", str(d))
    return dict(os.environ, LD_LIBRARY_PATH=str(d))


def test_cli_refuses_a_foreign_rocm_runtime(tmp_path):
    """bin/test and bin/pt2pt_test link libxg.so directly: with another libamdhip64.so.7 first on
    the search path they would run on it; xg_init refuses before any HIP call (xg_foreign_runtime)"""
    import subprocess
    env = _foreign_hip(tmp_path)
    exe = os.path.join(PKG, "bin", "test")
    out = subprocess.run([exe, "-m", "1", "-a", "2", "-d", "64", "--procs", "4"], capture_output=True, text=True,
                         timeout=60, env=env, cwd=str(tmp_path))
    assert out.returncode == 1 and "foreign ROCm runtime" in out.stderr, out.stderr[-2000:]
    assert "max total time" not in out.stdout
    pt = subprocess.run([os.path.join(PKG, "bin", "pt2pt_test"), "-d", "64", "-k", "1", "-i", "1"],
                        capture_output=True, text=True, timeout=60, env=dict(env, XG_PT2PT_SELF="1"), cwd=str(tmp_path))
    assert pt.returncode == 1 and "foreign ROCm runtime" in pt.stderr, pt.stderr[-2000:]


def test_bench_refuses_a_foreign_rocm_runtime(tmp_path):
    """bench.py (N = 1, no launcher) on a foreign runtime: libxg.so is refused after loading, the
    line says why (value null) and the process exits 1 -- nothing is measured on another runtime"""
    import json
    import subprocess
    import sys
    env = _foreign_hip(tmp_path)
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "1", "--warmup", "0",
                          "--no-cpu-baseline"], capture_output=True, text=True, timeout=120, env=env, cwd=str(tmp_path))
    assert out.returncode == 1, (out.stdout[-2000:], out.stderr[-2000:])
    line = json.loads([x for x in out.stdout.splitlines() if x.startswith("{")][-1])
    assert line["value"] is None and "outside /opt/rocm" in line["error"], line


def test_build_records_its_rocm_library_directory():
    """a ROCm installed elsewhere (distro packages, a conda env) that libxg.so was built
    and linked against is not foreign -- the Makefile records its library directory, in libxg.so
    (XG_ROCM_LIBDIR, xg_foreign_runtime) and in lib/rocm_libdir (xg.py's check before loading)"""
    libdir = os.path.realpath("/opt/rocm/lib")
    assert open(os.path.join(PKG, "lib", "rocm_libdir")).read().strip() == libdir
    assert libdir.encode() in open(os.path.join(PKG, "lib", "libxg.so"), "rb").read()
