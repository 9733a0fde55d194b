"""Per-iteration anatomy of one whole ICP from a rocprofv3 kernel trace
(development tool): the ICP that starts at the n-th cold tile match
(grid_tile_kernel), iterations delimited by loop_step_kernel; per iteration
the kernels (duration us) and the period.
Usage: python tools/whole_icp_trace.py run_kernel_trace.csv [nth_tile=2] [iters=40]"""
import csv
import re
import sys


def short(name):
    m = re.search(r"pmx::(\w+)", name)
    return m.group(1) if m else name.split("(")[0][-24:]


def main(path, nth=2, iters=40):
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
                  for r in csv.DictReader(open(path)))
    tiles = [i for i, r in enumerate(rows) if r[2] == "grid_tile_kernel"]
    i0 = tiles[nth]
    it, prev_end, t_start = 0, rows[i0][0], rows[i0][0]
    cur = []
    agg = {}
    for s, e, n in rows[i0:]:
        cur.append((n, (e - s) / 1e3, (s - prev_end) / 1e3))
        prev_end = e
        agg[n] = agg.get(n, 0.0) + (e - s) / 1e3
        if n == "loop_step_kernel":
            tot = (e - t_start) / 1e3
            print(f"it {it:2d} {tot:7.1f} us: " + " ".join(f"{k[:10]}={d:.1f}" + (f"(+{g:.0f})" if g > 2 else "")
                                                         for k, d, g in cur))
            t_start, cur = e, []
            it += 1
            if it >= iters:
                break
    print("span", (prev_end - rows[i0][0]) / 1e3, "us")
    for k, v in sorted(agg.items(), key=lambda x: -x[1]):
        print(f"  {k:28s} {v:8.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2, int(sys.argv[3]) if len(sys.argv) > 3 else 40)
