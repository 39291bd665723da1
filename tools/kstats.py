"""Top kernels of a rocprofv3 --stats kernel_stats.csv: calls, average and total ms."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:n]:
    name = r["Name"].replace("void ", "").split("(")[0][:70]
    print(f"{name:72s} {int(r['Calls']):5d} {float(r['AverageNs']) / 1e6:10.3f} ms avg {float(r['TotalDurationNs']) / 1e6:10.1f} ms tot")
