"""Per-phase kernel time and HBM traffic of one bench.py command (dev tool).

usage: python tools/pmc_phases.py TRACE_DIR FETCH_DIR WRITE_DIR W K "COMMAND" > out.json

bench.py (with --no-cpu-baseline) ends, on the context stream (device loop,
one ICP object), with pass A = prepare + W warmup + K timed iterations (the
timed region) and pass B = prepare + W + K iterations with HIP events around
every match launch (the live roofline measurement); nothing is dispatched
after pass B.  Every iteration launches the match kernel once, so the last
2 (W + K) match dispatches are the two passes.  This tool averages the kernel
trace durations and the PMC counters (separate rocprofv3 --pmc runs of the
same command, dispatches aligned by their order) over:
  timed      pass A, iterations W .. W+K-1 (what ms_per_step covers)
  roofline   pass B, iterations W .. W+K-1 (what bench.py's live events time)
  cold       pass A, iteration 0 (the first match at the initial pose)
  all        every launch of the command
gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts half
the bytes of 16-B-per-lane reads, so fetch_bytes = 2 x FETCH_SIZE (KiB);
WRITE_SIZE is exact.
"""
import collections
import csv
import glob
import json
import sys

# (the match of a new reading's first iteration is the tile kernel's cold form)
KERNELS = {"match": ("grid_lane_kernel", "grid_tile_kernel"), "p2plane": "p2plane_partial_kernel", "tail": "loop_tail_kernel",
           "step": "loop_step_kernel", "counter_sum": "counter_sum_kernel", "select": "select_all_kernel",
           "finalize": "finalize_kernel"}


def rows(d, pattern):
    out = []
    for path in sorted(glob.glob(f"{d}/**/{pattern}", recursive=True)):
        out += list(csv.DictReader(open(path)))
    return out


def series(rs, sub, key):
    subs = sub if isinstance(sub, tuple) else (sub,)
    v = [(int(x["Dispatch_Id"]), x) for x in rs if any(t in x["Kernel_Name"] for t in subs)]
    v.sort(key=lambda t: t[0])
    return [key(x) for _, x in v]


def main():
    tdir, fdir, wdir, W, K, cmd = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5]), sys.argv[6]
    tr = rows(tdir, "*kernel_trace.csv")
    fe = [x for x in rows(fdir, "*counter_collection.csv") if x["Counter_Name"] == "FETCH_SIZE"]
    wr = [x for x in rows(wdir, "*counter_collection.csv") if x["Counter_Name"] == "WRITE_SIZE"]
    n = len(series(tr, KERNELS["match"], lambda x: 0))
    a0 = n - 2 * (W + K)  # (pass A's first match)
    phases = {"timed": (a0 + W, a0 + W + K), "roofline": (n - K, n), "cold": (a0, a0 + 1)}
    out = {"command": cmd, "warmup": W, "steps": K,
           "unit": "ns per launch; bytes per launch (fetch = 2 x FETCH_SIZE, gfx950 correction; write exact)",
           "phases": {k: f"match dispatches [{a}, {b})" for k, (a, b) in phases.items()}}
    for name, sub in KERNELS.items():
        dur = series(tr, sub, lambda x: int(x["End_Timestamp"]) - int(x["Start_Timestamp"]))
        if not dur:
            continue
        f = series(fe, sub, lambda x: 2.0 * 1024.0 * float(x["Counter_Value"]))
        w = series(wr, sub, lambda x: 1024.0 * float(x["Counter_Value"]))
        per_it = len(dur) / max(len(series(tr, KERNELS["match"], lambda x: 0)), 1)
        res = {"launches": len(dur), "launches_per_match": per_it}

        def avg(a, lo, hi):
            # (slices counted from the end: the device warm-up before the
            # passes is time-based, so the runs differ in their first launches)
            lo_e, hi_e = lo - len(dur), hi - len(dur)
            s = a[lo_e:hi_e if hi_e < 0 else None] if len(a) >= -lo_e else []
            return sum(s) / len(s) if s else None

        def summarize(lo, hi):
            d = avg(dur, lo, hi)
            ff = avg(f, lo, hi)
            ww = avg(w, lo, hi)
            return {"avg_ns": d, "fetch_bytes_per_launch": ff, "write_bytes_per_launch": ww,
                    "hbm_bytes_per_launch": (ff + ww) if ff is not None and ww is not None else None,
                    "launches_averaged": len(dur[lo:hi])}

        res["all"] = {"avg_ns": sum(dur) / len(dur), "launches_averaged": len(dur)}
        if per_it == 1.0:  # one launch per iteration: phase slices are meaningful
            for ph, (a, b) in phases.items():
                res[ph] = summarize(a, b)
        out[name] = res
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
