"""Steady-state anatomy of the device loop from a rocprofv3 kernel trace
(development tool): the last N iterations (delimited by the step launch),
per-kernel average duration, the average gap in front of each kernel, and
the iteration period.  Usage: python tools/trace_iter.py run_kernel_trace.csv [N]"""
import csv
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"pmx::(\w+)", name)
    if m:
        return m.group(1)
    return name.split("(")[0][-40:]


def main(path, n_last=20):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    steps = [i for i, r in enumerate(rows) if r[2] in ("loop_step_kernel", "finalize_step_kernel")]
    if len(steps) < n_last + 1:
        print("not enough loop iterations", len(steps))
        return
    # iterations made only of loop kernels (+ the batch flag copy), the
    # steady ones: period below `cut` us
    loopk = {"grid_lane_kernel", "counter_sum_kernel", "select_all_kernel", "p2plane_partial_kernel",
             "finalize_kernel", "loop_step_kernel", "__amd_rocclr_copyBuffer", "p2point_pass1_kernel",
             "p2point_pass2_kernel", "p2point_means_kernel", "grid_tile_kernel", "finalize_step_kernel",
             "p2plane_select_kernel"}
    cut = float(sys.argv[3]) if len(sys.argv) > 3 else 150.0
    its = []
    for a, b in zip(steps[:-1], steps[1:]):
        ks = {rows[i][2] for i in range(a + 1, b + 1)}
        per = (rows[b][1] - rows[a][1]) / 1e3
        if (ks <= loopk or os.environ.get("TRACE_ALL")) and per < cut:
            its.append((a, b, per))
    its = its[-n_last:]
    dur = defaultdict(list)
    gap = defaultdict(list)
    for a, b, _ in its:
        for i in range(a + 1, b + 1):
            s, e, k = rows[i]
            dur[k].append((e - s) / 1e3)
            gap[k].append((s - rows[i - 1][1]) / 1e3)
    n_last = len(its)
    period = sum(x[2] for x in its) / max(n_last, 1)
    print(f"iteration period {period:.2f} us over {n_last} steady iterations (period < {cut} us)")
    tot = 0.0
    for k in dur:
        c = len(dur[k]) / n_last
        d = sum(dur[k]) / len(dur[k])
        g = sum(gap[k]) / len(gap[k])
        tot += c * (d + g)
        print(f"  {k:28s} x{c:4.2f}  dur {d:7.2f} us  gap-before {g:6.2f} us")
    print(f"  (sum of dur + gaps per iteration {tot:.2f} us)")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20)
