#!/usr/bin/env python3
"""Generate tests/golden/ fixtures by running the REAL reference benchmark.

Container-only (needs /root/reference + the image's MPICH).  Builds
oracle/_ref/test_capture (reference objects + oracle/pmpi_capture.c) with
oracle/Makefile, runs it under mpiexec for every config x method 1..12, and
reduces the per-rank capture files to small fixtures:

  <cfg>/meta.json        command line, P, A, d, c, k, i, t, p, aggregator list
                         (parsed from the reference's own header, mpi_test.c:2171-2177)
  <cfg>/data_a2m.csv.gz  iter,src,dst,len,chk  - every segment an aggregator received
  <cfg>/data_m2a.csv.gz  iter,src,dst,len,chk  - every segment a rank received
  <cfg>/trace.txt.gz     "m<N> r<rank>: tok tok ..."  per-rank MPI call trace of method N
                         (iter 0).  Tokens: B barrier, s<peer>:<cnt> send post,
                         r<peer>:<cnt> recv post, w<idx list> completion point, A alltoallw.
  <cfg>/report_m<N>.txt  the reference's stdout for -m N with every number masked '#'
  <cfg>/data_tam.csv.gz  m15/m16 (TAM): every message each rank received, in completion order
                         (method,iter,rank,k,src,count,chk) -- the final slots are filled by memcpy
  methods 1..20; tokens on a communicator other than MPI_COMM_WORLD carry @<comm>#<tag>;
  MPI_Isend is 'i'; counts are in the call's datatype (MPI_INT for TAM's size messages).
  usage.txt              the reference's `-h` text (stderr), argv0 replaced by {argv0}

Each method's captured data is checked against the direction table while
writing (all methods of one direction must deliver identical bytes); the
aggregator self-pairs that m3/m4/m6 move with memcpy (mpi_test.c:1473,
:1646, :1714) are invisible to PMPI and are listed in meta.json instead.
"""
import gzip
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
MPIEXEC = "/opt/conda/bin/mpiexec"
CAPTURE = os.path.join(REPO, "oracle", "_ref", "test_capture")

A2M_METHODS = {1, 3, 6, 7, 8, 9, 12, 13, 17, 18, 19, 20}
M2A_METHODS = {2, 4, 5, 10, 11, 14}
METHODS = [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20]
TAM = {15: "a2m", 16: "m2a"}     # all_to_many_tam / many_to_all_tam (collective_write, lustre_driver_test.c)

# name: (P, args)
CONFIGS = {
    "readme_p32_a14": (32, "-a 14 -p 1 -d 2048 -c 3 -i 2 -k 2"),
    "p16_a5_d1000_c3": (16, "-a 5 -d 1000 -c 3 -i 2 -k 2"),
    "p12_a5_d4096": (12, "-a 5 -d 4096 -i 2 -k 2"),
    "p16_a4_t2_c5": (16, "-a 4 -d 512 -c 5 -t 2 -i 1 -k 2"),
    "p8_a8_t0_c2": (8, "-a 8 -d 256 -c 2 -t 0 -i 1 -k 1"),
    "p64_a16_d256": (64, "-a 16 -d 256 -i 1 -k 1"),
    "p24_a7_t3_c1": (24, "-a 7 -d 64 -c 1 -t 3 -p 4 -i 1 -k 2"),
    "p32_a1_c4": (32, "-a 1 -d 128 -c 4 -i 1 -k 1"),
    "p8_a3_d1m_c2": (8, "-a 3 -d 1048576 -c 2 -i 1 -k 2"),
    "p20_a6_c7": (20, "-a 6 -d 24 -c 7 -i 1 -k 3"),
    "p16_a5_c3_b1": (16, "-a 5 -d 96 -c 3 -b 1 -p 4 -i 1 -k 2"),
    "p16_a5_c4_b2": (16, "-a 5 -d 96 -c 4 -b 2 -p 2 -i 1 -k 2"),
    "p8_a3_d0_c3": (8, "-a 3 -d 0 -c 3 -p 2 -i 1 -k 2"),        # empty segments (every message 0 bytes)
}


def idx_list(idxs):
    idxs = sorted(idxs)
    out, i = [], 0
    while i < len(idxs):
        j = i
        while j + 1 < len(idxs) and idxs[j + 1] == idxs[j] + 1:
            j += 1
        out.append(str(idxs[i]) if i == j else "%d-%d" % (idxs[i], idxs[j]))
        i = j + 1
    return ",".join(out)


def tok(kind, rank, peer, cnt, tag, comm, path, line):
    """s/i/r<peer>:<cnt>; on MPI_COMM_WORLD the tag is rank+peer except in TAM (+100*iter), where
    the token carries #<tag>; on any other communicator it carries @<comm>#<tag>."""
    if comm == 0:
        if tag == rank + peer:
            return "%s%d:%d" % (kind, peer, cnt)
        return "%s%d:%d#%d" % (kind, peer, cnt, tag)
    return "%s%d:%d@%d#%d" % (kind, peer, cnt, comm, tag)


def parse_cap(path, rank):
    """-> list of method runs; each {'tokens': [...], 'recv': [(src,cnt,addr)], 'data': [(src,cnt,addr,chk)]}"""
    runs, cur = [], None
    expect_idx = 0
    for line in open(path):
        f = line.split()
        if not f:
            continue
        if cur is None:
            cur = {"tokens": [], "recv": [], "data": []}
            expect_idx = 0
        k = f[0]
        if k == "B":
            cur["tokens"].append("B")
        elif k == "S":
            idx, peer, cnt, tag, comm = map(int, f[1:6])
            assert idx == expect_idx, (path, line)
            expect_idx += 1
            cur["tokens"].append(tok("i" if f[6] == "i" else "s", rank, peer, cnt, tag, comm, path, line))
        elif k == "R":
            idx, peer, cnt, tag, comm = map(int, f[1:6])
            assert idx == expect_idx, (path, line)
            expect_idx += 1
            cur["tokens"].append(tok("r", rank, peer, cnt, tag, comm, path, line))
            if comm == 0:
                cur["recv"].append((peer, cnt, 0 if f[6] == "(nil)" else int(f[6], 16)))
        elif k == "W":
            cur["tokens"].append("w" + idx_list(map(int, f[1:])))
        elif k == "A":
            cur["tokens"].append("A")
        elif k == "D":
            cur["data"].append((int(f[1]), int(f[2]), int(f[3], 16), f[4]))
        elif k == "E":
            runs.append(cur)
            cur = None
        else:
            raise ValueError(line)
    assert cur is None or not cur["tokens"], "trailing events in " + path
    return runs


def mask_numbers(text):
    return re.sub(r"\d+(\.\d+)?", "#", text)


def run_one(P, args, method, workdir):
    for fn in os.listdir(workdir):
        os.unlink(os.path.join(workdir, fn))
    env = dict(os.environ, XG_CAPTURE_DIR=workdir)
    cmd = [MPIEXEC, "-n", str(P), CAPTURE] + args.split() + ["-m", str(method)]
    try:
        out = subprocess.run(cmd, cwd=workdir, env=env, capture_output=True, text=True, timeout=300)
    except subprocess.TimeoutExpired:
        return None, None
    if out.returncode != 0:
        raise RuntimeError("reference failed: %s\n%s" % (cmd, out.stderr[-2000:]))
    caps = [parse_cap(os.path.join(workdir, "cap_%d.txt" % r), r) for r in range(P)]
    return out.stdout, caps


def main(selected=None):
    subprocess.run(["make", "-C", os.path.join(REPO, "oracle")], check=True, capture_output=True)
    # usage text (mpi_test.c:41-69), printed by `./test -h`; argv0 normalised to {argv0}
    ref = os.path.join(REPO, "oracle", "_ref", "test")
    u = subprocess.run([MPIEXEC, "-n", "1", ref, "-h"], capture_output=True, text=True, timeout=60)
    with open(os.path.join(HERE, "usage.txt"), "w") as fp:
        fp.write(u.stderr.replace(ref, "{argv0}"))
    work = tempfile.mkdtemp(prefix="xg_golden_")
    try:
        if not selected or "pt2pt" in selected:
            gen_pt2pt(work)
        for name, (P, args) in CONFIGS.items():
            if selected and name not in selected:
                continue
            gen_config(name, P, args, work)
    finally:
        shutil.rmtree(work, ignore_errors=True)


def gen_pt2pt(work):
    """pt2pt_test (mpi_sendrecv_test.c): masked stdout at 2 processes (the measured case) and
    1 process (only the status line, :25-27), and the CSV shape (one row per -k)."""
    ref = os.path.join(REPO, "oracle", "_ref", "pt2pt_test")
    outdir = os.path.join(HERE, "pt2pt")
    os.makedirs(outdir, exist_ok=True)
    meta = {"args": "-d 4096 -k 3 -i 5"}
    for n in (1, 2):
        csv_path = os.path.join(work, "sendrecv_results.csv")
        if os.path.exists(csv_path):
            os.unlink(csv_path)
        out = subprocess.run([MPIEXEC, "-launcher", "fork", "-n", str(n), ref] + meta["args"].split(),
                             capture_output=True, text=True, timeout=120, cwd=work)
        assert out.returncode == 0, out.stderr
        with open(os.path.join(outdir, "report_n%d.txt" % n), "w") as fp:
            fp.write(mask_numbers(out.stdout))
        meta["csv_rows_n%d" % n] = len(open(csv_path).read().splitlines()) if os.path.exists(csv_path) else None
    with open(os.path.join(outdir, "meta.json"), "w") as fp:
        json.dump(meta, fp, indent=1, sort_keys=True)
    print("pt2pt", meta, flush=True)


def gen_config(name, P, args, work):
    outdir = os.path.join(HERE, name)
    os.makedirs(outdir, exist_ok=True)
    opts = dict(zip(args.split()[0::2], args.split()[1::2]))
    d = int(opts["-d"])
    iters = int(opts.get("-i", 1))
    meta = {"P": P, "args": args, "d": d, "iters": iters, "ntimes": int(opts.get("-k", 1)),
            "c": int(opts.get("-c", 200000000)), "A": int(opts["-a"]),
            "type": int(opts.get("-t", 1)), "proc_node": int(opts.get("-p", 1)),
            "methods": {}}
    tables = {"a2m": {}, "m2a": {}}
    traces = []
    tam_rows = []
    for m in METHODS:
        stdout, caps = run_one(P, args, m, work)
        if caps is None:
            meta["methods"][str(m)] = {"status": "timeout"}
            print(name, "m%d TIMEOUT" % m, flush=True)
            continue
        if m == 13:   # save_all_timing (mpi_test.c:2008-2066): file names and shapes
            shapes = {}
            for fn in sorted(os.listdir(work)):
                if fn.endswith(".csv") and fn != "results.csv":
                    rows = [r.split(",") for r in open(os.path.join(work, fn)).read().splitlines()]
                    shapes[fn] = [len(rows), len(rows[0]) if rows else 0, [int(r[0]) for r in rows]]
            meta["m13_timing_files"] = shapes
        hdr = stdout.splitlines()
        if "aggregators" not in meta:
            meta["header"] = hdr[0]
            meta["aggregators"] = [int(x) for x in hdr[1].split("=")[1].split(",") if x.strip()]
        with open(os.path.join(outdir, "report_m%d.txt" % m), "w") as fp:
            fp.write(mask_numbers(stdout))
        if m in TAM:
            # every final slot is written by memcpy (invisible to PMPI): keep each rank's received
            # messages (intermediate aggregation buffers) in completion order instead
            for r in range(P):
                for it, run in enumerate(caps[r]):
                    if it == 0:
                        traces.append("m%d r%d: %s" % (m, r, " ".join(run["tokens"])))
                    for k, (src, cnt, _addr, chk) in enumerate(run["data"]):
                        tam_rows.append("%d,%d,%d,%d,%d,%d,%s" % (m, it, r, k, src, cnt, chk))
            meta["methods"][str(m)] = {"status": "ok", "direction": TAM[m], "uncaptured_pairs": [],
                                       "layout_ok": True, "tam": True}
            print(name, "m%d ok (TAM: %d received messages)" % (m, sum(1 for x in tam_rows if x.startswith("%d," % m))),
                  flush=True)
            continue
        direction = "a2m" if m in A2M_METHODS else "m2a"
        aggs = meta["aggregators"]
        aggidx = {g: i for i, g in enumerate(aggs)}
        table = tables[direction]
        missing = []
        layout_ok = True
        for r in range(P):
            runs = caps[r]
            assert len(runs) == iters, (name, m, r, len(runs))
            for it, run in enumerate(runs):
                if it == 0:
                    traces.append("m%d r%d: %s" % (m, r, " ".join(run["tokens"])))
                # receiver layout position (slot index) must be a fixed offset from the address
                bases = set()
                for src, cnt, addr in run["recv"]:
                    if cnt == 0:
                        continue
                    slot = src if direction == "a2m" else aggidx[src]
                    bases.add(addr - slot * d)
                if len(bases) > 1:
                    layout_ok = False
                seen = {}
                for src, cnt, addr, chk in run["data"]:
                    key = (it, src, r)
                    if key in seen:
                        assert seen[key] == (cnt, chk), ("reps differ", name, m, key)
                        continue
                    seen[key] = (cnt, chk)
                    if key in table:
                        assert table[key] == (cnt, chk), ("methods differ", name, m, key, table[key], (cnt, chk))
                    else:
                        table[key] = (cnt, chk)
                # expected pairs for this direction
                if direction == "a2m" and r in aggidx:
                    exp = {(it, s, r) for s in range(P)}
                elif direction == "m2a":
                    exp = {(it, g, r) for g in aggs}
                else:
                    exp = set()
                miss = sorted(exp - set(seen))
                missing += [list(k) for k in miss]
        meta["methods"][str(m)] = {"status": "ok", "direction": direction,
                                   "uncaptured_pairs": missing, "layout_ok": layout_ok}
        print(name, "m%d ok (%d uncaptured)" % (m, len(missing)), flush=True)
    for direction, table in tables.items():
        with gzip.open(os.path.join(outdir, "data_%s.csv.gz" % direction), "wt") as fp:
            fp.write("iter,src,dst,len,chk\n")
            for (it, src, dst), (cnt, chk) in sorted(table.items()):
                fp.write("%d,%d,%d,%d,%s\n" % (it, src, dst, cnt, chk))
    with gzip.open(os.path.join(outdir, "data_tam.csv.gz"), "wt") as fp:
        fp.write("method,iter,rank,k,src,count,chk\n" + "".join(x + "\n" for x in tam_rows))
    with gzip.open(os.path.join(outdir, "trace.txt.gz"), "wt") as fp:
        fp.write("\n".join(traces) + "\n")
    with open(os.path.join(outdir, "meta.json"), "w") as fp:
        json.dump(meta, fp, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(set(sys.argv[1:]) or None)
