"""Sum rocprofv3 counter-collection CSVs per kernel-name substring (dev tool)."""
import csv, glob, sys
pat = sys.argv[1]
for f in sorted(glob.glob(sys.argv[2] + "/**/*counter_collection.csv", recursive=True)):
    agg = {}
    n = set()
    for r in csv.DictReader(open(f)):
        if pat not in r["Kernel_Name"]:
            continue
        n.add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
        agg[r["Counter_Name"]] = agg.get(r["Counter_Name"], 0) + float(r["Counter_Value"])
    print(f, "dispatches", len(n), {k: "%.3g" % v for k, v in sorted(agg.items())})
