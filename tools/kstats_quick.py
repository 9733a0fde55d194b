"""Summarise a rocprofv3 kernel trace (dev tool): per-kernel totals and the
last iteration's kernel sequence with the idle gaps between kernels."""
import csv
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
r = list(csv.reader(open(f"{d}/run_kernel_stats.csv")))
for row in r[1:]:
    print(f"{row[0][:60]:60s} {row[1]:>5s} {int(row[2]) / 1e3:10.1f} {float(row[3]) / 1e3:8.2f}")
t = sorted(csv.DictReader(open(f"{d}/run_kernel_trace.csv")), key=lambda x: int(x["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
t0 = None
for x in t[-n:]:
    s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
    print(f"  {x['Kernel_Name'][:45]:45s} gap {(s - (t0 or s)) / 1e3:6.1f} dur {(e - s) / 1e3:6.1f}")
    t0 = e
ks = [x for x in t if "grid_lane" in x["Kernel_Name"]]
print("match per launch:", [round((int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3, 1) for x in ks][:40])
