#!/usr/bin/env python3
"""Per-dispatch SQ counter table of one leapfrog step from a rocprofv3 --pmc pass
(tools/pmc_sq.sh): wave cycles split into parked (SQ_WAIT_ANY: s_waitcnt /
barrier), issue-stalled (SQ_WAIT_INST_ANY) and active (SQ_ACTIVE_INST_ANY),
each as % of SQ_WAVE_CYCLES; MFMA busy cycles; GRBM_GUI_ACTIVE.

Usage: python tools/pmc_stage.py <pmc_dir> [--marker k_cr_pair_force] [--which -2]
"""
import argparse
import collections
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("--marker", default="k_cr_pair_force", help="a kernel launched once per leapfrog step")
    ap.add_argument("--which", type=int, default=-2, help="which marker occurrence starts the step")
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.pmc_dir, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {a.pmc_dir}")
    disp = collections.OrderedDict()
    for fn in files:
        with open(fn) as f:
            for r in csv.DictReader(f):
                d = disp.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"], "grid": r["Grid_Size"]})
                d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ids = sorted(disp)
    marks = [i for i in ids if a.marker in disp[i]["name"]]
    if len(marks) < 2:
        raise SystemExit("fewer than two step markers")
    i0, i1 = marks[a.which - 1], marks[a.which]
    print("kernel                          grid   waves   wavecyc  wait%  inst%   act% mfmaBusy      gui")
    for i in ids:
        if not (i0 <= i < i1):
            continue
        d = disp[i]
        name = d["name"].split("(")[0].replace("void ", "").replace("dwh::", "")
        wc = d.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        print(f"{name[:28]:28s} {d['grid']:>8s} {d.get('SQ_WAVES', 0):7.0f} {wc:9.3g} "
              f"{100 * d.get('SQ_WAIT_ANY', 0) / wc:6.1f} {100 * d.get('SQ_WAIT_INST_ANY', 0) / wc:6.1f} "
              f"{100 * d.get('SQ_ACTIVE_INST_ANY', 0) / wc:6.1f} {d.get('SQ_VALU_MFMA_BUSY_CYCLES', 0):8.3g} "
              f"{d.get('GRBM_GUI_ACTIVE', 0):8.3g}")


if __name__ == "__main__":
    main()
