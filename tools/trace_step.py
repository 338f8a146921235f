"""Per-launch timeline of one leapfrog step from a rocprofv3 kernel trace.

Usage: python tools/trace_step.py <run_kernel_trace.csv> [--marker k_cr_fill] [--which -2]
Prints each launch between two consecutive markers (duration, gap to the
previous launch, grid) and per-kernel totals for the step.
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="k_cr_pair_force", help="a kernel launched once per leapfrog step")
    ap.add_argument("--which", type=int, default=-2, help="which marker occurrence starts the step")
    ap.add_argument("--quiet", action="store_true")
    a = ap.parse_args()
    tr = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(tr) if a.marker in r["Kernel_Name"]]
    i0, i1 = idx[a.which - 1], idx[a.which]
    prev = None
    tot = collections.defaultdict(float)
    for r in tr[i0:i1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        tot[name] += (e - s) / 1000
        if not a.quiet:
            gap = (s - prev) / 1000 if prev else 0.0
            print(f"{name:34s} dur={(e - s) / 1000:7.1f}us gap={gap:6.1f}us grid={r['Grid_Size_X']}x{r['Grid_Size_Y']}")
        prev = e
    span = (int(tr[i1]["Start_Timestamp"]) - int(tr[i0]["Start_Timestamp"])) / 1000
    print(f"step span {span:.1f} us")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
        print(f"  {k:34s} {v:8.1f} us  {100 * v / span:5.1f}%")


if __name__ == "__main__":
    main()
