"""Per-call kernel totals of a rocprofv3 kernel_stats.csv:
python tools/kstats_top.py <csv> <calls> [top]."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
calls = int(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 20
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total per call {tot / calls / 1e6:.2f} ms")
for r in rows[:top]:
    nm = r["Name"].replace("dwh::(anonymous namespace)::", "").split("(")[0][:44]
    print(f"  {nm:44s} {int(r['Calls']) // calls:6d} {float(r['TotalDurationNs']) / calls / 1e6:8.2f} ms/call "
          f"{float(r['AverageNs']) / 1e3:9.1f} us avg")
