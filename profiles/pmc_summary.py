#!/usr/bin/env python3
"""Reduce rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE in separate runs) of
`python3 bench.py --no-cpu-baseline --steps 5 --warmup 1` to HBM bytes per
copy_kernel launch, with the gfx950 correction of MI355X_MICROARCH.md (HBM):
FETCH_SIZE reports 1/2 of the bytes of a wide (16 B/lane) coalesced stream,
so read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE is exact (x1024).

usage: pmc_summary.py <fetch_dir> <write_dir> <out.json> [source tag]
"""
import csv
import json
import sys


def per_kernel(path, counter):
    acc = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        acc.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main(fdir, wdir, out, source=""):
    f = per_kernel(fdir + "/run_counter_collection.csv", "FETCH_SIZE")
    w = per_kernel(wdir + "/run_counter_collection.csv", "WRITE_SIZE")
    res = {"method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes; "
                     "read = 2*FETCH_SIZE*1024 (gfx950 wide-stream correction), write = WRITE_SIZE*1024",
           "source": source, "kernels": {}}
    for k in sorted(set(f) | set(w)):
        rd = 2 * f.get(k, 0.0) * 1024
        wr = w.get(k, 0.0) * 1024
        res["kernels"][k] = {"fetch_size_kb": f.get(k), "write_size_kb": w.get(k),
                             "hbm_read_bytes": rd, "hbm_write_bytes": wr, "hbm_bytes": rd + wr}
        if "copy_kernel" in k and (rd + wr) > res.get("hbm_bytes_per_launch", 0):
            res["hbm_bytes_per_launch"] = int(rd + wr)
            res["copy_kernel"] = k
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:5])
