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
