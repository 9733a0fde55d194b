"""Print a rocprofv3 kernel_stats.csv compactly (dev tool)."""
import csv
import sys

for x in list(csv.DictReader(open(sys.argv[1])))[:int(sys.argv[2]) if len(sys.argv) > 2 else 15]:
    print(f"{x['Name'][:60]:60s} {x['Calls']:>5s} {float(x['AverageNs'])/1e3:9.1f} us {float(x['Percentage']):6.2f}%")
