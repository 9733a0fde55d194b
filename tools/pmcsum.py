"""Average PMC counters per kernel from rocprofv3 counter_collection.csv files (dev tool)."""
import collections
import csv
import glob
import sys

for f in sys.argv[1:]:
    for path in glob.glob(f):
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for x in csv.DictReader(open(path)):
            agg[x["Kernel_Name"][:48]][x["Counter_Name"]].append(float(x["Counter_Value"]))
        print("##", path)
        for k, v in agg.items():
            if "grid_lane" in k or "select" in k or "p2plane" in k or len(sys.argv) > 99:
                print(f"  {k:48s}", {c: f"{sum(vals) / len(vals):.3g}" for c, vals in sorted(v.items())})
