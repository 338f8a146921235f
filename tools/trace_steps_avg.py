"""Mean duration of every launch position of a leapfrog step over all steps
of a rocprofv3 kernel trace (the steps between consecutive k_cr_pair_force
launches with the most common launch count), for stage-by-stage A/B.

Usage: python tools/trace_steps_avg.py <run_kernel_trace.csv> [--marker k_cr_pair_force]
"""
import argparse
import collections
import csv
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="k_cr_pair_force")
    a = ap.parse_args()
    tr = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(tr) if a.marker in r["Kernel_Name"]]
    steps = [tr[i0:i1] for i0, i1 in zip(idx, idx[1:])]
    names = lambda st: tuple(r["Kernel_Name"].split("(")[0].replace("void ", "") for r in st)
    common = collections.Counter(names(st) for st in steps).most_common(1)[0][0]
    sel = [st for st in steps if names(st) == common]
    print(f"{len(sel)} steps of {len(common)} launches (of {len(steps)})")
    tot = 0.0
    for j, nm in enumerate(common):
        d = [(int(st[j]["End_Timestamp"]) - int(st[j]["Start_Timestamp"])) / 1000 for st in sel]
        g = [(int(st[j]["Start_Timestamp"]) - int(st[j - 1]["End_Timestamp"])) / 1000 for st in sel] if j else [0.0]
        tot += statistics.median(d)
        print(f"{j:2d} {nm:30s} grid={sel[0][j]['Grid_Size_X']:>7s} med {statistics.median(d):6.2f} us  "
              f"mean {statistics.mean(d):6.2f}  gap {statistics.median(g):5.2f}")
    span = [(int(st[-1]["End_Timestamp"]) - int(st[0]["Start_Timestamp"])) / 1000 for st in sel]
    print(f"sum of medians {tot:.1f} us, median step span {statistics.median(span):.1f} us (profiler gaps included)")


if __name__ == "__main__":
    main()
