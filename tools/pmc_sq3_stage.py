#!/usr/bin/env python3
"""Instruction classes and the issue split of every dispatch of one leapfrog
step, from the round-5 counter passes (tools/pmc_sq3.sh: groups A-D, each its
own run of the same bench; dispatches aligned by position inside the step,
the step = the dispatches from one k_cr_pair_force to the next).

Per dispatch: instructions per wave (VALU, of them f64 ADD/MUL/FMA and MFMA;
VMEM reads, SALU, SMEM, LDS) and the wave-cycle split (SQ counters in
quad-cycles, shares of SQ_WAVE_CYCLES): active instruction issue (ANY, and of
it VALU / VMEM / scalar / LDS / misc), issue-stalled (SQ_WAIT_INST_ANY: the
wave has an instruction but its pipe / dependency is not ready — for an f64
MFMA stream that is the DP pipe busy with another wave's MFMA or the
accumulator chain), parked (SQ_WAIT_ANY: s_waitcnt / barrier).

Usage: python tools/pmc_sq3_stage.py <dir with sq3_A..D> [--json out.json]
"""
import argparse
import collections
import csv
import glob
import json
import os


def load(d):
    disp = collections.OrderedDict()
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as f:
            for r in csv.DictReader(f):
                e = disp.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"], "grid": int(r["Grid_Size"])})
                e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ds = [disp[k] for k in sorted(disp)]
    marks = [i for i, x in enumerate(ds) if "k_cr_pair_force" in x["name"]]
    i0, i1 = marks[-2], marks[-1]
    return ds[i0:i1]


def short(n):
    return n.split("(")[0].replace("void ", "").replace("dwh::", "").replace(" ", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    groups = {g: load(os.path.join(a.root, f"sq3_{g}")) for g in "ABCD" if os.path.isdir(os.path.join(a.root, f"sq3_{g}"))}
    n = min(len(v) for v in groups.values())
    rows = []
    for i in range(n):
        names = {short(v[i]["name"]) for v in groups.values()}
        if len(names) != 1:
            raise SystemExit(f"dispatch {i}: passes disagree {names}")
        r = {"kernel": names.pop(), "grid": groups["A"][i]["grid"]}
        for v in groups.values():
            for k, x in v[i].items():
                if k.startswith("SQ_") and k != "SQ_WAVE_CYCLES":
                    r[k] = x
        r["SQ_WAVE_CYCLES"] = groups["A"][i].get("SQ_WAVE_CYCLES", 0.0)
        rows.append(r)
    hdr = ("kernel", "waves", "valu/w", "f64add", "f64mul", "f64fma", "mfma/w", "vmem/w", "salu/w", "smem/w",
           "lds/w", "act%", "valu%", "vmem%", "sca%", "lds%", "stall%", "park%")
    print(("{:24s}" + "{:>8s}" * (len(hdr) - 1)).format(*hdr))
    out = []
    for r in rows:
        w = r.get("SQ_WAVES", 1.0) or 1.0
        wc = r["SQ_WAVE_CYCLES"] or 1.0
        pw = lambda k: r.get(k, 0.0) / w
        pc = lambda k: 100.0 * r.get(k, 0.0) / wc
        rec = {"kernel": r["kernel"], "grid": r["grid"], "waves": w,
               "per_wave": {k: pw(k) for k in ("SQ_INSTS_VALU", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                                               "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MFMA_F64", "SQ_INSTS_MFMA",
                                               "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SALU",
                                               "SQ_INSTS_SMEM", "SQ_INSTS_LDS")},
               "cycle_share_pct": {k: pc(k) for k in ("SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_VMEM",
                                                      "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_MISC",
                                                      "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY")},
               "wave_cycles_quad": wc, "mfma_busy_cycles": r.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)}
        out.append(rec)
        print(("{:24s}" + "{:8.0f}" + "{:8.1f}" * 9 + "{:8.1f}" * 7).format(
            r["kernel"][:24], w, pw("SQ_INSTS_VALU"), pw("SQ_INSTS_VALU_ADD_F64"), pw("SQ_INSTS_VALU_MUL_F64"),
            pw("SQ_INSTS_VALU_FMA_F64"), pw("SQ_INSTS_VALU_MFMA_F64"), pw("SQ_INSTS_VMEM_RD"), pw("SQ_INSTS_SALU"),
            pw("SQ_INSTS_SMEM"), pw("SQ_INSTS_LDS"), pc("SQ_ACTIVE_INST_ANY"), pc("SQ_ACTIVE_INST_VALU"),
            pc("SQ_ACTIVE_INST_VMEM"), pc("SQ_ACTIVE_INST_SCA"), pc("SQ_ACTIVE_INST_LDS"), pc("SQ_WAIT_INST_ANY"),
            pc("SQ_WAIT_ANY")))
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"source": os.path.relpath(a.root), "units": "instructions per wave; shares of SQ_WAVE_CYCLES (quad-cycles)",
                       "dispatches": out}, f, indent=1)


if __name__ == "__main__":
    main()
