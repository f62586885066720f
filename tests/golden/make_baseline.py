#!/usr/bin/env python3
"""Capture the REAL reference at the BASELINE.json configuration shapes (tests/golden/baseline/).

Container-only, like make_golden.py (needs /root/reference + the image's MPICH): runs
oracle/_ref/test_capture (the reference objects + oracle/pmpi_capture.c) under mpiexec at

  cfg1_p32_a14_d1m     configs[1] at full size: -a 14 -d 1 MiB, m1-12, -i 2 -k 2
  cfg2_p64_a16_d256k   configs[2] at full size: -a 16 -d 256 KiB, m1-12
  cfg3_p256_a32_d64k   configs[3]'s shape at -d 64 KiB (4 MiB is 64 GiB per direction, more
                       than this host's RAM): m1, m2, m9, m10, -k 2
  cfg4_p256_a64_d4k_cN configs[4]'s shape at -d 4 KiB (64 MiB is 1 TiB per direction), -c N for
                       N = 1..8, m7, m11, m12, -k 2 (so the never-reset comm_size across -k,
                       mpi_test.c:965-967 / :1023-1025 / :1079-1081, is in the capture)

P = 256 traces are too large to keep whole (m9 at P256 makes 2 x 256 calls per rank per
repetition), so each config directory holds (a method listed in EXPECT_HANG is one the step compiler
proves deadlocked under MPI semantics at that shape -- m6 at configs[1]'s 1 MiB segments, past
MPICH's eager limit: it runs with a 90 s limit and is recorded as "timeout" if the reference
indeed never finishes, and fails the generator if it does finish):

  meta.json          the make_golden.py fields, plus
                     trace_sha1[m]  = per-rank sha1 of the rank's token string (iter 0) -- the
                                      whole trace of every rank, compared by digest
                     trace_sample_ranks = the ranks whose full token strings are kept
                     data_from      = the directory holding the checksum tables (the -c sweep
                                      delivers the same bytes at every -c, so cfg4_*_c2..c8
                                      point at c1 after the generator checked they are equal)
  trace_sample.txt.gz  "m<N> r<rank>: tok ..." for the sampled ranks (diagnostics)
  data_a2m.csv.gz / data_m2a.csv.gz  iter,src,dst,len,chk -- every captured received segment
  report_m<N>.txt    the reference's stdout with every number masked

usage: make_baseline.py [config names]   (default: all; existing directories are regenerated)
"""
import gzip
import hashlib
import json
import os
import shutil
import signal
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as MG   # noqa: E402  (parse_cap, mask_numbers, direction sets)

OUT = os.path.join(HERE, "baseline")

ALL12 = list(range(1, 13))
EXPECT_HANG = {("cfg1_p32_a14_d1m", 6)}
BASELINE = {
    "cfg1_p32_a14_d1m": (32, "-a 14 -d 1048576 -i 2 -k 2", ALL12),
    "cfg2_p64_a16_d256k": (64, "-a 16 -d 262144 -i 1 -k 1", ALL12),
    "cfg3_p256_a32_d64k": (256, "-a 32 -d 65536 -i 1 -k 2", [1, 2, 9, 10]),
}
for _c in range(1, 9):
    BASELINE["cfg4_p256_a64_d4k_c%d" % _c] = (256, "-a 64 -d 4096 -c %d -i 1 -k 2" % _c, [7, 11, 12])


def sample_ranks(P, aggs):
    """rank 0, 1, P-1, the first / middle / last aggregator, and every (P/8)-th rank"""
    s = {0, 1, P - 1, aggs[0], aggs[len(aggs) // 2], aggs[-1]}
    s |= set(range(0, P, max(1, P // 8)))
    return sorted(s)


def run_one(P, args, method, workdir, limit=900):
    """the reference under mpiexec, its own process group, killed whole past `limit` seconds"""
    for fn in os.listdir(workdir):
        os.unlink(os.path.join(workdir, fn))
    env = dict(os.environ, XG_CAPTURE_DIR=workdir)
    cmd = [MG.MPIEXEC, "-launcher", "fork", "-n", str(P), MG.CAPTURE] + args.split() + ["-m", str(method)]
    t0 = time.time()
    with open(os.path.join(workdir, "stdout.txt"), "w") as fo, open(os.path.join(workdir, "stderr.txt"), "w") as fe:
        p = subprocess.Popen(cmd, stdout=fo, stderr=fe, cwd=workdir, env=env, start_new_session=True)
        while p.poll() is None and time.time() - t0 < limit:
            time.sleep(0.5)
        if p.poll() is None:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()
            raise RuntimeError("reference did not finish in %d s: %s" % (limit, cmd))
    if p.returncode != 0:
        raise RuntimeError("reference failed: %s\n%s" % (cmd, open(os.path.join(workdir, "stderr.txt")).read()[-2000:]))
    stdout = open(os.path.join(workdir, "stdout.txt")).read()
    caps = [MG.parse_cap(os.path.join(workdir, "cap_%d.txt" % r), r) for r in range(P)]
    return stdout, caps, time.time() - t0


def gen_config(name, P, args, methods, work):
    outdir = os.path.join(OUT, name)
    if os.path.isdir(outdir):
        shutil.rmtree(outdir)
    os.makedirs(outdir)
    opts = dict(zip(args.split()[0::2], args.split()[1::2]))
    d = int(opts["-d"])
    iters = int(opts.get("-i", 1))
    meta = {"P": P, "args": args, "d": d, "iters": iters, "ntimes": int(opts.get("-k", 1)),
            "c": int(opts.get("-c", 200000000)), "A": int(opts["-a"]),
            "type": int(opts.get("-t", 1)), "proc_node": int(opts.get("-p", 1)),
            "methods": {}, "trace_sha1": {}, "wall_s": {}}
    tables = {"a2m": {}, "m2a": {}}
    samples = []
    for m in methods:
        if (name, m) in EXPECT_HANG:
            try:
                run_one(P, args, m, work, limit=90)
            except RuntimeError as e:
                if "did not finish" not in str(e):
                    raise
                meta["methods"][str(m)] = {"status": "timeout", "limit_s": 90}
                print(name, "m%d did not finish in 90 s, as predicted" % m, flush=True)
                continue
            raise RuntimeError("%s m%d finished although the step compiler predicts a deadlock" % (name, m))
        stdout, caps, wall = run_one(P, args, m, work)
        meta["wall_s"][str(m)] = round(wall, 1)
        hdr = stdout.splitlines()
        if "aggregators" not in meta:
            meta["header"] = hdr[0]
            meta["aggregators"] = [int(x) for x in hdr[1].split("=")[1].split(",") if x.strip()]
            meta["trace_sample_ranks"] = sample_ranks(P, meta["aggregators"])
        with open(os.path.join(outdir, "report_m%d.txt" % m), "w") as fp:
            fp.write(MG.mask_numbers(stdout))
        direction = "a2m" if m in MG.A2M_METHODS else "m2a"
        aggs = meta["aggregators"]
        aggidx = {g: i for i, g in enumerate(aggs)}
        table = tables[direction]
        digests, missing, layout_ok = [], 0, True
        for r in range(P):
            runs = caps[r]
            assert len(runs) == iters, (name, m, r, len(runs))
            toks = " ".join(runs[0]["tokens"])
            digests.append(hashlib.sha1(toks.encode()).hexdigest())
            if r in meta["trace_sample_ranks"]:
                samples.append("m%d r%d: %s" % (m, r, toks))
            for it, run in enumerate(runs):
                bases = set()
                for src, cnt, addr in run["recv"]:
                    if cnt:
                        bases.add(addr - (src if direction == "a2m" else aggidx[src]) * d)
                layout_ok &= len(bases) <= 1
                seen = {}
                for src, cnt, _addr, chk in run["data"]:
                    key = (it, src, r)
                    if key in seen:
                        assert seen[key] == (cnt, chk), ("reps differ", name, m, key)
                        continue
                    seen[key] = (cnt, chk)
                    if key in table:
                        assert table[key] == (cnt, chk), ("methods differ", name, m, key)
                    else:
                        table[key] = (cnt, chk)
                if direction == "a2m" and r in aggidx:
                    exp = {(it, s, r) for s in range(P)}
                elif direction == "m2a":
                    exp = {(it, g, r) for g in aggs}
                else:
                    exp = set()
                missing += len(exp - set(seen))
        meta["trace_sha1"][str(m)] = digests
        meta["methods"][str(m)] = {"status": "ok", "direction": direction, "uncaptured_pairs": missing,
                                   "layout_ok": layout_ok}
        print(name, "m%d ok (%.1f s, %d uncaptured)" % (m, wall, missing), flush=True)
    # the -c sweep moves the same bytes at every -c: keep one copy of the tables
    meta["data_from"] = name
    first = name[:-1] + "1" if name.startswith("cfg4_") else None
    if first and first != name and os.path.exists(os.path.join(OUT, first, "data_a2m.csv.gz")):
        same = all(_read_table(os.path.join(OUT, first, "data_%s.csv.gz" % dr)) == tables[dr]
                   for dr in ("a2m", "m2a"))
        assert same, (name, "bytes differ from", first)
        meta["data_from"] = first
    if meta["data_from"] == name:
        for direction, table in tables.items():
            with gzip.open(os.path.join(outdir, "data_%s.csv.gz" % direction), "wt") as fp:
                fp.write("iter,src,dst,len,chk\n")
                for (it, src, dst), (cnt, chk) in sorted(table.items()):
                    fp.write("%d,%d,%d,%d,%s\n" % (it, src, dst, cnt, chk))
    with gzip.open(os.path.join(outdir, "trace_sample.txt.gz"), "wt") as fp:
        fp.write("\n".join(samples) + "\n")
    with open(os.path.join(outdir, "meta.json"), "w") as fp:
        json.dump(meta, fp, indent=0, sort_keys=True)


def _read_table(path):
    out = {}
    for row in gzip.open(path, "rt").read().split("\n")[1:]:
        if row:
            it, src, dst, cnt, chk = row.split(",")
            out[(int(it), int(src), int(dst))] = (int(cnt), chk)
    return out


def main(selected=None):
    subprocess.run(["make", "-C", os.path.join(MG.REPO, "oracle")], check=True, capture_output=True)
    os.makedirs(OUT, exist_ok=True)
    work = tempfile.mkdtemp(prefix="xg_baseline_")
    try:
        for name, (P, args, methods) in BASELINE.items():
            if selected and name not in selected:
                continue
            gen_config(name, P, args, methods, work)
    finally:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main(set(sys.argv[1:]) or None)
