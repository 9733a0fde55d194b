"""Summarise bench JSON lines in gpurun_out (dev tool)."""
import glob
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
for f in sorted(glob.glob(os.path.join(d, "bench_*.json"))):
    try:
        j = json.load(open(f))
    except Exception as e:  # noqa: BLE001
        print(os.path.basename(f), "unreadable", e)
        continue
    r = j["roofline"]
    print(f"{os.path.basename(f):24s} {j['ms_per_step']:8.4f} ms/it  {j['value']:.3g} {j['unit']}  "
          f"match {r['avg_launch_ms']*1e3:7.1f} us  {r['achieved']:7.1f} GB/s  "
          f"pairs/launch {j['compute_roofline']['pairs_evaluated_per_launch']:.3g}")
