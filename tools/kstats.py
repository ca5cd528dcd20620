"""Print a rocprofv3 kernel_stats.csv compactly: python tools/kstats.py <csv> [top]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
for r in rows[:top]:
    print("%-70s %6s calls %10.1f us avg %9.3f ms tot %6s %%" % (
        r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6, r["Percentage"][:5]))
