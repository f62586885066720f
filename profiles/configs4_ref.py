#!/usr/bin/env python3
"""configs[4] host-MPI baseline cells: the reference ./test (oracle/_ref/test) under MPICH,
mpiexec -n 256, m7 / m11 / m12 at -c 1..8, at a REDUCED -d (configs[4]'s 64 MiB is 1 TiB per
direction: no host holds it).  256 busy-polling MPI processes on the host's CPU share are
oversubscribed -- each cell gets a time limit, runs in its own process group (killed whole
when it runs over: an orphaned rank would hold the box) and reports "did not finish" then.
Prints a heartbeat line while a cell runs.  Cells already in <out> are skipped.
usage: configs4_ref.py <out.txt> <d> <limit_s> [cells, e.g. 12:5,7:6]"""
import os
import re
import signal
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out, d, lim = sys.argv[1], int(sys.argv[2]), float(sys.argv[3])
cells = ([tuple(map(int, c.split(":"))) for c in sys.argv[4].split(",")] if len(sys.argv) > 4
         else [(m, c) for c in range(1, 9) for m in (7, 11, 12)])
done = set()
if os.path.exists(out):
    for line in open(out):
        g = re.match(r"m(\d+) c(\d+) d(\d+):", line)
        if g and int(g.group(3)) == d:
            done.add((int(g.group(1)), int(g.group(2))))
else:
    sys.path.insert(0, REPO)
    import bench
    with open(out, "w") as f:
        f.write("# host CPUs: %s; mpiexec -n 256 -launcher fork, -a 64 -d %d -i 1 -k 1, limit %.0f s per cell\n"
                % (bench.host_cpus(), d, lim))
for m, c in cells:
    if (m, c) in done:
        continue
    cmd = ["/opt/conda/bin/mpiexec", "-launcher", "fork", "-n", "256", os.path.join(REPO, "oracle", "_ref", "test"),
           "-a", "64", "-d", str(d), "-c", str(c), "-m", str(m), "-i", "1", "-k", "1"]
    t0 = time.time()
    with open("/tmp/c4ref_cell.txt", "w") as fo:
        p = subprocess.Popen(cmd, stdout=fo, stderr=subprocess.STDOUT, cwd="/tmp", start_new_session=True)
        while p.poll() is None and time.time() - t0 < lim:
            time.sleep(1)
            if int(time.time() - t0) % 20 == 0:
                print("  m%d c%d running %.0f s" % (m, c, time.time() - t0), flush=True)
        if p.poll() is None:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()
    wall = time.time() - t0
    txt = open("/tmp/c4ref_cell.txt").read()
    g = re.search(r"\| (.*) max total time = ([0-9.]+)", txt)
    line = ("m%d c%d d%d: | %s max total time = %s  (wall %.1f s)" % (m, c, d, g.group(1), g.group(2), wall) if g
            else "m%d c%d d%d: did not finish in %.0f s" % (m, c, d, lim))
    with open(out, "a") as f:
        f.write(line + "\n")
    print(line, flush=True)
print("done")
