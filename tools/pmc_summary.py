#!/usr/bin/env python3
"""Per-kernel HBM traffic from two rocprofv3 PMC passes of bench.py.

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d <fetch_dir> -o run -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d <write_dir> -o run -- python3 bench.py ...
    python tools/pmc_summary.py <fetch_dir> <write_dir> --L 32 --beta 16 --chains 1 -o profiles/r01_pmc_traffic.json

FETCH_SIZE and WRITE_SIZE are in KiB per dispatch.  On gfx950 FETCH_SIZE
reports half of the bytes of wide streaming reads (MI355X_MICROARCH.md, HBM
section), so hbm_bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.  The two
counters come from separate passes (they do not fit one TCC pass), so the
per-launch means are combined, not individual dispatches.
"""
import argparse
import collections
import csv
import glob
import json
import os
import re


def short(name: str) -> str:
    n = name.split("(")[0].replace("void ", "").replace("dwh::", "").strip()
    return re.sub(r"\s+", "", n)


def read(dirname: str, counter: str):
    files = glob.glob(os.path.join(dirname, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {dirname}")
    agg = collections.defaultdict(list)
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                if row["Counter_Name"] == counter:
                    agg[short(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    return agg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--L", type=int, required=True)
    ap.add_argument("--beta", type=float, required=True)
    ap.add_argument("--chains", type=int, default=1)
    ap.add_argument("-o", "--out", required=True)
    a = ap.parse_args()
    fetch = read(a.fetch_dir, "FETCH_SIZE")
    write = read(a.write_dir, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) & set(write)):
        fk = sum(fetch[k]) / len(fetch[k])
        wk = sum(write[k]) / len(write[k])
        kernels[k] = {"launches_fetch_pass": len(fetch[k]), "launches_write_pass": len(write[k]),
                      "fetch_size_kib": fk, "write_size_kib": wk,
                      "hbm_read_bytes": 2.0 * fk * 1024.0, "hbm_write_bytes": wk * 1024.0,
                      "hbm_bytes_per_launch": 2.0 * fk * 1024.0 + wk * 1024.0}
    rec = {"workload": {"L": a.L, "beta": a.beta, "chains": a.chains},
           "correction": "hbm = 2*FETCH_SIZE + WRITE_SIZE (KiB -> bytes); gfx950 FETCH_SIZE halves wide reads",
           "kernels": kernels}
    with open(a.out, "w") as f:
        json.dump(rec, f, indent=1)
    for k, v in kernels.items():
        print(f"{k:40s} {v['hbm_bytes_per_launch'] / 1e6:10.1f} MB/launch")


if __name__ == "__main__":
    main()
