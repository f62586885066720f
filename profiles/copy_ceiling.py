"""HBM ceilings on contiguous buffers (tools/lib/libxgtools.so, not the product library):
grid-stride 16-B copy, the exchange's copy_kernel_g<4> and copy_kernel_b<4, sc1> over
32 KiB pieces, read-only and write-only streams.  usage: python3 profiles/copy_ceiling.py"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = C.CDLL(os.path.join(HERE, "mpi-asynchronous-communication-test_amd", "tools", "lib", "libxgtools.so"))
lib.xgt_copy_ceiling.argtypes = [C.c_int, C.c_int64, C.c_int, C.c_int, C.POINTER(C.c_double)]
names = {0: "grid-stride copy", 1: "copy_kernel_g<4>", 2: "copy_kernel_b<4,sc1>", 3: "read-only", 4: "write-only"}
for nb in (448 << 20, 1 << 30, 4 << 30):
    for kind in range(5):
        g = C.c_double()
        assert lib.xgt_copy_ceiling(0, nb, kind, 20, C.byref(g)) == 0
        print("bytes=%d %-22s %.1f GB/s" % (nb, names[kind], g.value), flush=True)
