"""Summarise a rocprofv3 kernel_stats.csv: per-kernel total ms, calls, avg us, share (short names)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot/1e6:.1f} ms ({tot/1e6/steps:.1f} ms/step over {steps:g} steps)")
for r in rows[: int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    n = r["Name"].replace("(anonymous namespace)::", "")
    short = n.split("(")[0][:70] if not n.startswith(("Cijk", "Custom")) else n[:40] + "..." + n.split("_MT")[1][:14]
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.1f} us "
          f"{float(r['Percentage']):5.1f}%  {short}")
