import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as G
xg = G.load_package().xg
ctx = xg.Context(0, 1, device=0)
for nb in (448 << 20, 1 << 30, 4 << 30):
    for kind in (0, 1, 2, 3, 4, 5, 6):
        print("bytes=%d kind=%d  %.1f GB/s" % (nb, kind, ctx.copy_ceiling(nb, kind, 20)), flush=True)
ctx.close()
