"""Host -> kernel -> host round trip of the armed engine's doorbell, by where the ring
word lives (tools/lib/libxgtools.so xgt_doorbell_rtt): host-pinned memory (kind 0,
today's doorbell) vs device memory written by the host through its mapping (1 fine-
grained, 2 uncached).  Each kind runs in its own child process (a device ring that the
host cannot map must not take the parent down)."""
import ctypes as C
import os
import subprocess
import sys

LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "mpi-asynchronous-communication-test_amd", "tools", "lib", "libxgtools.so")

if len(sys.argv) > 1:
    kind = int(sys.argv[1])
    lib = C.CDLL(LIB)
    lib.xgt_doorbell_rtt.argtypes = [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_double)]
    us = C.c_double()
    rc = lib.xgt_doorbell_rtt(0, kind, 2000, C.byref(us))
    print("kind %d rc %d round trip %.2f us" % (kind, rc, us.value if rc == 0 else -1), flush=True)
    sys.exit(0)
for kind in (0, 1, 2, 0):
    p = subprocess.run([sys.executable, __file__, str(kind)], capture_output=True, text=True, timeout=60)
    print(p.stdout.strip() or "kind %d: exit %d %s" % (kind, p.returncode, p.stderr.strip()[-300:]), flush=True)
