#!/usr/bin/env python3
"""MFMA utilisation of the CR kernel families from a rocprofv3 SQ pass
(tools/pmc_sq.sh: SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE, ...) and the
f64 MFMA peak micro's pass (tools/micro/mfma_f64_peak.hip under the same
counters), written as the JSON bench.py reads for `roofline.mfma_busy_frac`
and `roofline.hw_frac`.

SQ_VALU_MFMA_BUSY_CYCLES counts 64 cycles per v_mfma_f64_16x16x4_f64
(calibrated on the peak micro: 2^31 for 2^25 MFMAs), so per launch
  executed MFMA flops = busy * 2048 / 64,
and against a launch's duration d (the bench's HIP events, not the profiled
run's): busy fraction of the chip's 1024 SIMDs = busy / (d * 2.4 GHz * 1024)
= executed flops / d / 78.6 TFLOP/s.  Per-dispatch averages are taken over
the last `--steps` complete leapfrog steps of the profiled bench (a step =
the dispatches from one k_cr_pair_force to the next).

Usage: python tools/pmc_mfma.py <sq_dir> [--peak <peak_pmc_dir>] [--peak-log <mfma_f64_peak.txt>]
                                [--L 32 --beta 16 --chains 1] -o out.json
"""
import argparse
import collections
import csv
import glob
import json
import os
import re


def dispatches(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    disp = collections.OrderedDict()
    for fn in files:
        with open(fn) as f:
            for r in csv.DictReader(f):
                e = disp.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"], "grid": int(r["Grid_Size"])})
                e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [disp[k] for k in sorted(disp)]


def family(name):
    n = name.split("(")[0].replace("void ", "").replace("dwh::", "").strip()
    return re.sub(r"\s+", "", n)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("sq_dir")
    ap.add_argument("--peak", default=None)
    ap.add_argument("--peak-log", default=None)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--marker", default="k_cr_pair_force")
    ap.add_argument("--L", type=int, default=32)
    ap.add_argument("--beta", type=float, default=16.0)
    ap.add_argument("--chains", type=int, default=1)
    ap.add_argument("-o", "--out", required=True)
    a = ap.parse_args()
    ds = dispatches(a.sq_dir)
    marks = [i for i, d in enumerate(ds) if a.marker in d["name"]]
    if len(marks) < a.steps + 1:
        raise SystemExit(f"{len(marks)} step markers, need {a.steps + 1}")
    i0, i1 = marks[-a.steps - 1], marks[-1]
    agg = collections.OrderedDict()
    for d in ds[i0:i1]:
        k = agg.setdefault(family(d["name"]), {"launches": 0, "busy": 0.0, "gui": 0.0, "wave_cycles": 0.0,
                                              "wait": 0.0, "wait_inst": 0.0, "active": 0.0})
        k["launches"] += 1
        k["busy"] += d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        k["gui"] += d.get("GRBM_GUI_ACTIVE", 0.0)
        k["wave_cycles"] += d.get("SQ_WAVE_CYCLES", 0.0)
        k["wait"] += d.get("SQ_WAIT_ANY", 0.0)
        k["wait_inst"] += d.get("SQ_WAIT_INST_ANY", 0.0)
        k["active"] += d.get("SQ_ACTIVE_INST_ANY", 0.0)
    kernels = {}
    for name, k in agg.items():
        n = k["launches"]
        wc = k["wave_cycles"] or 1.0
        kernels[name] = {
            "launches_per_step": n / a.steps,
            "mfma_busy_cycles_per_launch": k["busy"] / n,
            "mfma_exec_flops_per_launch": k["busy"] / n * 2048.0 / 64.0,
            # busy over the profiled dispatch's own GPU-active cycles (GRBM_GUI_ACTIVE / 8 XCDs);
            # profiled dispatches run serialised and longer than in the timed run
            "busy_frac_profiled": k["busy"] / (k["gui"] / 8.0 * 1024.0) if k["gui"] else None,
            "wave_parked_frac": k["wait"] / wc, "wave_issue_stall_frac": k["wait_inst"] / wc,
            "wave_active_frac": k["active"] / wc,
        }
    out = {"workload": {"L": a.L, "beta": a.beta, "chains": a.chains},
           "source": os.path.relpath(a.sq_dir), "steps": a.steps,
           "counter": "SQ_VALU_MFMA_BUSY_CYCLES (64 cycles per v_mfma_f64_16x16x4_f64)",
           "kernels": kernels}
    if a.peak:
        pk = [d for d in dispatches(a.peak) if "k_peak" in d["name"]]
        rows = []
        for d in pk:
            rows.append({"grid": d["grid"], "busy_frac_profiled": d["SQ_VALU_MFMA_BUSY_CYCLES"] /
                         (d["GRBM_GUI_ACTIVE"] / 8.0 * 1024.0)})
        out["peak_micro"] = {"kernel": "tools/micro/mfma_f64_peak.hip k_peak", "dispatches": rows}
    if a.peak_log:
        best = None
        for line in open(a.peak_log):
            m = re.search(r"blocks/CU=(\d+)\s+([\d.]+) TFLOP/s.*?([\d.]+) cycles/MFMA/wave, clock ([\d.]+) GHz", line)
            if m:
                rec = {"blocks_per_cu": int(m.group(1)), "tflops": float(m.group(2)),
                       "cycles_per_mfma_per_wave": float(m.group(3)), "clock_ghz": float(m.group(4))}
                out.setdefault("peak_runs", []).append(rec)
                if best is None or rec["tflops"] > best["tflops"]:
                    best = rec
        if best:
            out["attainable_tflops"] = best["tflops"]
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    for name, k in kernels.items():
        print(f"{name[:40]:40s} {k['launches_per_step']:5.1f}/step  busy/launch {k['mfma_busy_cycles_per_launch']:.4g}"
              f"  exec GF/launch {k['mfma_exec_flops_per_launch'] / 1e9:.4g}  busy_frac_profiled "
              f"{(k['busy_frac_profiled'] or 0):.3f}")
    if "attainable_tflops" in out:
        print("attainable f64 MFMA:", out["attainable_tflops"], "TFLOP/s")


if __name__ == "__main__":
    main()
