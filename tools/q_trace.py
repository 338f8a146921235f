#!/usr/bin/env python3
"""Per-step timeline of the quaternion reduction from a rocprofv3 kernel trace
(--kernel-trace --output-format csv): for each k_q_* kernel the mean duration
over 8 bins of the site steps of the first reduction in the trace, and the
mean gap between a kernel's end and the next one's start.
Usage: python tools/q_trace.py run_kernel_trace.csv"""
import csv
import re
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ev = []
    for r in rows:
        m = re.search(r"(k_q_\w+)", r["Kernel_Name"])
        if m:
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1)))
    ev.sort()
    # the first reduction: from the first k_q_rs to the first k_q_rot
    end = next((i for i, e in enumerate(ev) if e[2] == "k_q_rot"), len(ev))
    ev = ev[:end]
    names = sorted({e[2] for e in ev})
    per = defaultdict(list)
    gaps = []
    for i, (s, e, nm) in enumerate(ev):
        per[nm].append(e - s)
        if i + 1 < len(ev):
            gaps.append(ev[i + 1][0] - e)
    nb = 8
    print("kernel".ljust(12), " ".join(f"bin{b}".rjust(7) for b in range(nb)), "   mean  total_ms")
    for nm in names:
        d = per[nm]
        L = len(d)
        bins = [d[b * L // nb:(b + 1) * L // nb] for b in range(nb)]
        print(nm.ljust(12), " ".join(f"{(sum(x) / len(x) / 1e3 if x else 0):7.2f}" for x in bins),
              f"{sum(d) / L / 1e3:7.2f} {sum(d) / 1e6:8.3f}")
    if gaps:
        print(f"gaps: mean {sum(gaps) / len(gaps) / 1e3:.2f} us over {len(gaps)}; wall {(ev[-1][1] - ev[0][0]) / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
