"""Print a rocprofv3 kernel_stats.csv as a short table: name, calls, total ms, avg us."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
for r in rows[:n]:
    name = r["Name"].split("(")[0].replace("void ", "")[:60]
    print(f"{name:60s} {r['Calls']:>5} {int(r['TotalDurationNs']) / 1e6:9.2f} ms  avg {float(r['AverageNs']) / 1e3:9.1f} us")
