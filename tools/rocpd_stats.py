"""Per-kernel statistics (calls, total, average, min, max in ns) from a
rocprofv3 rocpd SQLite database (rocprofv3 7.x writes results.db by default):
python tools/rocpd_stats.py results.db [out.csv]"""
import csv
import sqlite3
import sys


def stats(db_path):
    db = sqlite3.connect(db_path)
    rows = db.execute(
        "select s.display_name, d.end - d.start from rocpd_kernel_dispatch d "
        "join rocpd_info_kernel_symbol s on s.id = d.kernel_id").fetchall()
    agg = {}
    for name, dur in rows:
        a = agg.setdefault(name, [0, 0, float("inf"), 0])
        a[0] += 1
        a[1] += dur
        a[2] = min(a[2], dur)
        a[3] = max(a[3], dur)
    out = [(n, a[0], a[1], a[1] / a[0], a[2], a[3]) for n, a in agg.items()]
    out.sort(key=lambda r: -r[2])
    return out


def main():
    out = stats(sys.argv[1])
    tot = sum(r[2] for r in out)
    for n, c, t, av, mn, mx in out[:30]:
        print(f"{n[:60]:60s} {c:7d} {t / 1e6:9.2f} ms {av / 1e3:8.2f} us {100 * t / tot:5.1f}%")
    print(f"total {tot / 1e6:.2f} ms")
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs"])
            w.writerows(out)


if __name__ == "__main__":
    main()
