"""Summarise rocprofv3 kernel traces (development tool).

python tools/trace_summary.py gpurun_out/var/*/   -> per kernel-name position in the last
iteration: duration (us), plus the mean over the last `--last` occurrences.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not f:
        return []
    rows = list(csv.DictReader(open(f[0])))
    seq = [(r["Kernel_Name"].split("(")[0].replace("void ", "")[:48], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3,
            int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    seq.sort(key=lambda x: x[2])
    return seq


def main():
    for d in sys.argv[1:]:
        seq = load(d)
        if not seq:
            continue
        # one iteration = from the last match launch to the end
        idx = [i for i, s in enumerate(seq) if "match" in s[0] or "grid_" in s[0]]
        starts = idx[-3:]
        print(f"== {d}")
        per = defaultdict(list)
        for a, b in zip(starts, starts[1:] + [len(seq)]):
            for j, s in enumerate(seq[a:b]):
                per[(j, s[0])].append(s[1])
        for (j, name), v in sorted(per.items()):
            print(f"  {j:2d} {name:48s} {sum(v) / len(v):9.2f} us")
        a = starts[-2]
        b = starts[-1]
        print(f"  iteration wall (match start to next match start): {(seq[b][2] - seq[a][2]) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
