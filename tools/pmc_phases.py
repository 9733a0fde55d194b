"""Per-phase kernel time and HBM traffic of one bench.py command (dev tool).

usage: python tools/pmc_phases.py TRACE_DIR FETCH_DIR WRITE_DIR W K "COMMAND" > out.json
       (FETCH_DIR / WRITE_DIR may be "-": durations only)

bench.py (with --no-cpu-baseline) ends, on the context stream (device loop,
one ICP object), with pass A = prepare + W warmup + K timed iterations (the
timed region) and pass B = prepare + W + K iterations with HIP events around
every match (the live roofline measurement); nothing is dispatched after
pass B.  Every iteration runs one match: the tile kernel (cold form, a new
reading's first iteration) or the per-lane kernel (a match of several
launches — the round-4 certify / search split, since removed — is summed),
so the last 2 (W + K) matches are the two passes (with tile dispatch, C5,
the tile kernel's warm form and the per-lane kernel it leaves the match to
are launched back to back every iteration: the adjacent pair is one match); each phase also lists the
durations it averages ("launch_ns").  This tool averages the kernel trace
durations and the PMC counters (separate rocprofv3 --pmc runs of the same
command, dispatches aligned by their order from the end) over:
  timed      pass A, iterations W .. W+K-1 (what ms_per_step covers)
  roofline   pass B, iterations W .. W+K-1 (what bench.py's live events time)
  cold       pass A, iteration 0 (the first match at the initial pose)
  all        every launch of the command
and lists every kernel dispatched in pass A's timed iterations W .. W+K-2
(complete iterations: from one match to the next) with its count and mean
duration ("timed_kernels": the rocprof stats restricted to the timed region).
gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts half
the bytes of 16-B-per-lane reads, so fetch_bytes = 2 x FETCH_SIZE (KiB);
WRITE_SIZE is exact.
"""
import collections
import csv
import glob
import json
import sys

# a match opens with one of these; the search kernel belongs to the certify
# kernel before it
MATCH_OPEN = ("grid_lane_kernel", "grid_tile_kernel", "grid_certify_kernel")
MATCH_MORE = ("grid_search_kernel",)
KERNELS = {"p2plane": "p2plane_partial_kernel", "tail": "loop_tail_kernel", "step": "loop_step_kernel",
           "finalize_step": "finalize_step_kernel", "p2point": "p2point_pass1_kernel",
           "counter_sum": "counter_sum_kernel", "select": "select_all_kernel", "finalize": "finalize_kernel"}


def rows(d, pattern):
    if d == "-":
        return []
    out = []
    for path in sorted(glob.glob(f"{d}/**/{pattern}", recursive=True)):
        out += list(csv.DictReader(open(path)))
    return out


def has(name, subs):
    return any(t in name for t in subs)


def series(rs, sub, key):
    subs = sub if isinstance(sub, tuple) else (sub,)
    v = [(int(x["Dispatch_Id"]), x) for x in rs if has(x["Kernel_Name"], subs)]
    v.sort(key=lambda t: t[0])
    return [key(x) for _, x in v]


def match_series(rs, key):
    """Per match: (first dispatch id, summed key) in dispatch order."""
    v = sorted(((int(x["Dispatch_Id"]), x) for x in rs if has(x["Kernel_Name"], MATCH_OPEN + MATCH_MORE)),
               key=lambda t: t[0])
    out = []
    last = None  # (dispatch id, kernel name) of the previous match kernel
    for d, x in v:
        name = x["Kernel_Name"]
        # (tile dispatch, C5: every iteration launches the tile kernel's warm
        # form and then the per-lane kernel, one of which returns at once —
        # the adjacent pair is one match)
        pair = last is not None and "grid_lane_kernel" in name and "grid_tile_kernel" in last[1] and d == last[0] + 1
        if (has(name, MATCH_OPEN) and not pair) or not out:
            out.append([d, key(x)])
        else:
            out[-1][1] += key(x)
        last = (d, name)
    return out


def fetch_key(x):
    return 2.0 * 1024.0 * float(x["Counter_Value"])


def write_key(x):
    return 1024.0 * float(x["Counter_Value"])


def dur_key(x):
    return int(x["End_Timestamp"]) - int(x["Start_Timestamp"])


def summarize(dur, f, w, lo, hi):
    def avg(a):
        # (slices counted from the end: the device warm-up before the passes
        # is time-based, so the runs differ in their first launches)
        lo_e, hi_e = lo - len(dur), hi - len(dur)
        s = a[lo_e:hi_e if hi_e < 0 else None] if len(a) >= -lo_e else []
        return sum(s) / len(s) if s else None

    d, ff, ww = avg(dur), avg(f), avg(w)
    return {"avg_ns": d, "fetch_bytes_per_launch": ff, "write_bytes_per_launch": ww,
            "hbm_bytes_per_launch": (ff + ww) if ff is not None and ww is not None else None,
            "launches_averaged": len(dur[lo:hi])}


def main():
    tdir, fdir, wdir, W, K, cmd = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5]), sys.argv[6]
    tr = rows(tdir, "*kernel_trace.csv")
    fe = [x for x in rows(fdir, "*counter_collection.csv") if x["Counter_Name"] == "FETCH_SIZE"]
    wr = [x for x in rows(wdir, "*counter_collection.csv") if x["Counter_Name"] == "WRITE_SIZE"]
    mt = match_series(tr, dur_key)
    n = len(mt)
    a0 = n - 2 * (W + K)  # (pass A's first match)
    phases = {"timed": (a0 + W, a0 + W + K), "roofline": (n - K, n), "cold": (a0, a0 + 1)}
    out = {"command": cmd, "warmup": W, "steps": K,
           "unit": "ns per launch; bytes per launch (fetch = 2 x FETCH_SIZE, gfx950 correction; write exact)",
           "phases": {k: f"matches [{a}, {b}) of {n}" for k, (a, b) in phases.items()},
           "match_kernels": "one match = " + " | ".join(MATCH_OPEN[:2]) + " | " + MATCH_OPEN[2] + " + " +
                            MATCH_MORE[0] + " (durations and bytes summed per match)"}

    # the match, one entry per iteration
    dur = [v for _, v in mt]
    f = [v for _, v in match_series(fe, fetch_key)]
    w = [v for _, v in match_series(wr, write_key)]
    res = {"launches": n, "all": {"avg_ns": sum(dur) / max(n, 1), "launches_averaged": n}}
    for ph, (a, b) in phases.items():
        res[ph] = summarize(dur, f, w, a, b)
        res[ph]["launch_ns"] = dur[a:b] if a >= 0 else []  # (the averaged launches themselves)
    out["match"] = res

    for name, sub in KERNELS.items():
        d = series(tr, sub, dur_key)
        if not d:
            continue
        per_it = len(d) / max(n, 1)
        r = {"launches": len(d), "launches_per_match": per_it, "all": {"avg_ns": sum(d) / len(d),
                                                                         "launches_averaged": len(d)}}
        if per_it == 1.0:  # one launch per iteration: phase slices are meaningful
            for ph, (a, b) in phases.items():
                r[ph] = summarize(d, series(fe, sub, fetch_key), series(wr, sub, write_key), a, b)
        out[name] = r

    # every kernel of pass A's complete timed iterations
    if a0 >= 0 and K >= 2:
        lo_id, hi_id = mt[a0 + W][0], mt[a0 + W + K - 1][0]
        acc = collections.defaultdict(list)
        for x in tr:
            if lo_id <= int(x["Dispatch_Id"]) < hi_id:
                acc[x["Kernel_Name"]].append(dur_key(x))
        its = K - 1
        tk = {name: {"count": len(v), "per_iteration": len(v) / its, "avg_ns": sum(v) / len(v),
                     "ns_per_iteration": sum(v) / its} for name, v in acc.items()}
        out["timed_kernels"] = {"iterations": its, "dispatch_ids": [lo_id, hi_id],
                                "busy_ns_per_iteration": sum(t["ns_per_iteration"] for t in tk.values()),
                                "kernels": dict(sorted(tk.items(), key=lambda t: -t[1]["ns_per_iteration"]))}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
