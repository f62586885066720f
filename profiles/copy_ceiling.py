"""HBM ceilings on contiguous buffers (tools/lib/libxgtools.so, not the product library):
grid-stride 16-B copy, the exchange's copy_kernel_g<4> and copy_kernel_b<4, sc1> over
32 KiB pieces, read-only and write-only streams.  usage: python3 profiles/copy_ceiling.py"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = C.CDLL(os.path.join(HERE, "mpi-asynchronous-communication-test_amd", "tools", "lib", "libxgtools.so"))
lib.xgt_copy_ceiling.argtypes = [C.c_int, C.c_int64, C.c_int, C.c_int, C.POINTER(C.c_double)]
names = {0: "grid-stride copy", 1: "copy_kernel_g<4> 32K", 2: "copy_kernel_b<4,sc1>", 3: "read-only", 4: "write-only",
         5: "hipMemcpy DtoD", 6: "grid-stride copy nt", 7: "copy_kernel_g<4> 256K", 8: "copy_kernel_g<4> 64K",
         9: "copy_kernel_g<4,nt> 32K", 10: "read-only nt", 11: "write-only nt", 12: "grid-stride nt-load",
         13: "grid-stride nt-store", 14: "copy_kernel_g<8,nt> 32K", 15: "copy_kernel_g<2,nt> 32K",
         16: "m2a gather 32M stride", 17: "m2a gather skewed", 18: "c2 pack g<4> 16K", 19: "c2 pack p<4> x512",
         20: "c2 pack p<2> x512", 21: "c2 pack p<8> x256", 22: "c2 pack w<8> 8K", 23: "m2a gather w<8,nt> 8K",
         24: "m2a gather w<4,nt> 4K", 25: "m2a gather w<16,nt> 16K", 26: "c2 pack2 g<4> 16K", 27: "c2 pack2 w<8> 8K",
         28: "m2a g<4,nt> 64K", 29: "m2a g<8,nt> 32K", 30: "m2a g<4,nt> 128K", 31: "m2a g<4,nt> 16K",
         32: "m2a bb ld nt st nt", 33: "m2a bb ld nt st nt|sc1", 34: "m2a bb nt|sc0|sc1 both",
         35: "m2a bb ld nt st sc0|sc1", 36: "m2a bb ld plain st nt", 37: "m2a bb ld nt st plain",
         38: "contig bb ld nt st nt|sc1", 39: "m2a bb nt|sc1 both"}
kinds = [int(k) for k in os.environ.get("KINDS", "0,1,2,3,4,5,6,7,8,9").split(",")]
sizes = [int(x) << 20 for x in os.environ.get("SIZES_MIB", "448,1024,4096").split(",")]
for nb in sizes:
    for kind in kinds:
        g = C.c_double()
        assert lib.xgt_copy_ceiling(0, nb, kind, 20, C.byref(g)) == 0
        print("bytes=%d %-22s %.1f GB/s" % (nb, names[kind], g.value), flush=True)
