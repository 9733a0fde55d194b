"""Benchmark: ICP iterations/s and matched-pairs/s on the BASELINE.json workload.

    python bench.py [--gpus N --steps K --warmup W] [--config c3] [--matcher brute]

A "step" is one ICP iteration of the hot path — fused transform + k-NN
match, outlier weighting, normal equations, the host 6x6 solve and the
checker — over the synthetic cloud of the configuration.
Default workload = BASELINE config 3: 1M -> 1M float, k = 1, TrimmedDist
ratio 0.85, point-to-plane, one GPU.  With N GPUs (torchrun, one process per
GPU) every rank holds its own 1M-point reading shard against the replicated
1M reference (weak scaling) and each iteration all-reduces the quantile
histograms and the normal equations over RCCL.

Timing: W untimed iterations, then exactly K iterations between a barrier +
device synchronisation on both sides; the max over ranks is reported.  The
defaults (K = 40, W = 0) time one whole ICP of 40 iterations from the initial
pose — the same work the CPU baseline times.  The
clouds are resident in HBM before the timed region.  The match kernel's
device time is measured with HIP events on the context stream (pmx_timing_*).
The CPU baseline (rank 0, N = 1 only) is the oracle's libnabo-style kd-tree
restatement of the reference CPU path on the same inputs (a bounded number of
iterations), timed on this host.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (N per rank, M, dtype, knn, filters, minimizer)
    "c2": (100_000, 100_000, np.float32, 1, [("TrimmedDistOutlierFilter", {"ratio": 0.85})], "PointToPlaneErrorMinimizer"),
    "c3": (1_000_000, 1_000_000, np.float32, 1, [("TrimmedDistOutlierFilter", {"ratio": 0.85})], "PointToPlaneErrorMinimizer"),
    "c4": (1_000_000, 1_000_000, np.float32, 4, [("MaxDistOutlierFilter", {"maxDist": 0.05})], "PointToPlaneErrorMinimizer"),
    "c5": (10_000_000, 1_000_000, np.float64, 1, [], "PointToPointErrorMinimizer"),
}
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E (MI355X_MICROARCH.md)
FP32_VALU_TFLOPS = 157.3   # MI355X FP32 vector peak (spec)
FP64_VALU_TFLOPS = 78.6


def chain_yaml(knn, filters, minimizer, search_type, maxit, differential=None):
    lines = ["matcher:", "  KDTreeMatcher:", f"    knn: {knn}", "    epsilon: 0", f"    searchType: {search_type}",
             "outlierFilters:"]
    for name, p in filters:
        lines.append(f"  - {name}:")
        lines += [f"      {k}: {v}" for k, v in p.items()]
    lines += ["errorMinimizer:", f"  {minimizer}", "transformationCheckers:", "  - CounterTransformationChecker:",
              f"      maxIterationCount: {maxit}"]
    if differential:
        lines.append("  - DifferentialTransformationChecker:")
        lines += [f"      {k}: {v}" for k, v in differential.items()]
    lines += ["inspector:", "  NullInspector", "logger:", "  NullLogger"]
    return "\n".join(lines) + "\n"


# parity runs: Counter 40 + Differential, equal iteration counts required
PARITY_DIFF = {"minDiffRotErr": 0.001, "minDiffTransErr": 0.01, "smoothLength": 4}


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(cfg_name, reading, reference, normals, knn, filters, minimizer, iters, threads, one_thread_iters):
    """The oracle (C restatement of the reference CPU path: libnabo-style
    kd-tree, nth_element quantile, -O3) on the same inputs, timed on this host.
    Runs (all cores): the timing chain (Counter `iters`, the workload's chain),
    the parity chain (+ Differential), and the timing chain with T-precision
    accumulation of the minimiser sums (the reference's Eigen arithmetic);
    then a bounded 1-thread sample (the reference's default: no OpenMP,
    CMakeLists.txt:160)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py as O

    nrm = normals if minimizer.startswith("PointToPlane") else None
    n = reading.shape[0]

    def run(th, maxit, diff, acc):
        cfg = O.make_cfg(knn=knn, filters=tuple(filters), minimizer=minimizer, counter_max=maxit, threads=th,
                         method="kdtree", differential=diff, acc_mode=acc)
        t0 = time.perf_counter()
        rc, T, st, _ = O.icp(cfg, reading, reference, normals=nrm)
        return rc, T, st, time.perf_counter() - t0

    rc, T, st, wall = run(threads, iters, None, 0)
    if rc != 0:
        return None, None
    loop = st.loop_seconds
    out = {"value": n * knn * st.iterations / loop, "unit": "matched-pairs/s", "cores": threads,
           "kind": "port", "iters_per_s": st.iterations / loop,
           "host_cpu": cpu_model(), "host_nproc": os.cpu_count(),
           "sample": f"{cfg_name} inputs ({n}->{reference.shape[0]}), the whole timing chain ({st.iterations} ICP "
                     f"iterations from the initial pose), oracle restatement of the reference CPU path "
                     f"(libnabo-style kd-tree with the incremental box bound, nth_element quantile, gcc -O3), "
                     f"{threads} threads, loop {loop:.2f} s (setup+loop {wall:.2f} s)"}
    runs = {"counter": {"T": T, "iterations": int(st.iterations), "kept": int(st.kept)}}
    rcd, Td, std, _ = run(threads, iters, PARITY_DIFF, 0)
    if rcd == 0:
        runs["differential"] = {"T": Td, "iterations": int(std.iterations), "kept": int(std.kept)}
    rcT, TT, stT, _ = run(threads, iters, None, 1)
    if rcT == 0:
        runs["counter_Tsums"] = {"T": TT, "iterations": int(stT.iterations), "kept": int(stT.kept)}
    rc1, T1, st1, _ = run(1, one_thread_iters, None, 0)
    if rc1 == 0:
        out["single_thread"] = {"value": n * knn * st1.iterations / st1.loop_seconds, "unit": "matched-pairs/s",
                                "cores": 1, "iters_per_s": st1.iterations / st1.loop_seconds,
                                "sample": f"first {st1.iterations} ICP iterations (the cold, most expensive ones), "
                                          f"1 thread, loop {st1.loop_seconds:.2f} s"}
    return out, runs


def parity_entry(Tg, sg, ref, tol, chain):
    frob = float(np.linalg.norm(np.asarray(Tg, np.float64) - np.asarray(ref["T"], np.float64)))
    return {"frob": frob, "tolerance": tol,
            "pass": bool(frob <= tol and int(sg.iterations) == ref["iterations"] and int(sg.kept) == ref["kept"]),
            "iterations_gpu": int(sg.iterations), "iterations_cpu": ref["iterations"],
            "kept_gpu": int(sg.kept), "kept_cpu": ref["kept"], "chain": chain}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # default: one whole ICP of 40 iterations from the initial pose, as the
    # CPU baseline runs it (SURVEY.md §8(d) timing runs)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=0)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--matcher", default="grid", choices=["brute", "grid"],
                    help="KDTreeMatcher searchType 0 (brute force) or 1 (spatial grid)")
    ap.add_argument("--cpu-iters", type=int, default=40)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--cpu-one-thread-iters", type=int, default=2,
                    help="ICP iterations of the bounded single-thread CPU sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist", action="store_true",
                    help="use the torchrun/RCCL multi-rank path even at world size 1 (rehearsal on one GPU)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1 or args.dist
    if dist:
        # torch is imported BEFORE libpmx is loaded: torch bundles its own HIP
        # runtime and RCCL (same SONAMEs), and loading it after libpmx would put
        # two HIP runtimes in the process.  In this order libpmx binds to the
        # already-loaded ones.
        import torch
        import torch.distributed as tdist

        # (gloo prints its connection banner on fd 1: keep stdout for the one
        # JSON line by pointing fd 1 at stderr while the group is created)
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            tdist.init_process_group("gloo", init_method="env://")  # control plane only
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    from libpointmatcher_amd import _capi
    from libpointmatcher_amd.icp import ICP
    from libpointmatcher_amd.synth import reading_cloud, reference_cloud

    N, M, dtype, knn, filters, minimizer = CONFIGS[args.config]
    reference, normals = reference_cloud(M, dtype)
    # each rank's shard of the global reading (weak scaling: N per rank)
    if dist:
        full = reading_cloud(N * world, dtype)
        reading = np.ascontiguousarray(full[rank * N:(rank + 1) * N])
        del full
    else:
        reading = reading_cloud(N, dtype)

    search_type = 0 if args.matcher == "brute" else 1
    total_it = args.warmup + args.steps + 10
    icp = ICP(dtype, device=local_rank)
    icp.load_yaml(chain_yaml(knn, filters, minimizer, search_type, total_it))
    if dist:
        import torch

        uid = bytearray(_capi.Context.unique_id() if rank == 0 else bytes(128))
        t = torch.tensor(list(uid), dtype=torch.uint8)
        tdist.broadcast(t, src=0)
        icp.comm_init(bytes(t.tolist()), world, rank)

    nrm_in = normals if minimizer.startswith("PointToPlane") else None
    # setup (reported separately): reference upload + grid
    # build (Matcher::init), reading upload + slot order, ICP.cpp:265-347.
    # The first prepare also creates the device context (HIP runtime, code
    # objects, RCCL communicator): reported as first_prepare_ms; setup_ms is
    # the per-compute cost, a second prepare on the live context.
    t_s = time.perf_counter()
    icp.prepare(reading, reference, nrm_in)
    first_prepare_s = time.perf_counter() - t_s
    t_s = time.perf_counter()
    icp.prepare(reading, reference, nrm_in)
    setup_s = time.perf_counter() - t_s
    if args.warmup > 0:
        icp.iterate(args.warmup)

    def barrier():
        if dist:
            tdist.barrier()

    barrier()
    t0 = time.perf_counter()
    icp.iterate(args.steps)   # each iteration ends with the system copy-back: device is synchronised
    t1 = time.perf_counter()
    barrier()
    elapsed = t1 - t0
    st = icp.stats()
    # Roofline pass: the same ICP again (prepare resets the pose and the
    # match history), now with HIP events around every match launch on the
    # context stream.  The events are kept out of the timed region above: each
    # record is a marker packet that adds ~6 us of idle GPU time per record
    # pair to the iteration (measured in the kernel trace).  The first
    # iteration's match is a cold search at the initial pose (no previous
    # k-lists to certify): with --warmup > 0 it is timed on its own.
    icp.prepare(reading, reference, nrm_in)
    cold_launch_ms = None
    if args.warmup > 0:
        icp.timing(True)
        icp.iterate(1)
        cold_ms, cold_n = icp.timing_read()
        cold_launch_ms = cold_ms / max(cold_n, 1)
        icp.iterate(args.warmup - 1)
    icp.timing(True)
    icp.iterate(args.steps)
    match_ms, launches = icp.timing_read()
    icp.timing(False)
    if dist:
        import torch

        e = torch.tensor([elapsed], dtype=torch.float64)
        tdist.all_reduce(e, op=tdist.ReduceOp.MAX)
        elapsed = float(e.item())

    pairs = N * world * knn * args.steps
    avg_match_s = match_ms * 1e-3 / max(launches, 1)
    esz = np.dtype(dtype).itemsize
    # algorithmic bytes of one match launch: the reading shard (4 T per point),
    # the reference (4 T per point) and the k (dist, id) outputs per query
    alg_bytes = N * 4 * esz + M * 4 * esz + N * knn * (esz + 4)
    # pair evaluations per match launch: N*M for brute force, the measured
    # PointCountTouched per iteration for the grid search
    pairs_eval = N * M if args.matcher == "brute" else st.point_count_touched / max(st.iterations, 1)
    flops = 8.0 * pairs_eval  # 3 sub + 3 mul + 2 add per pair
    if args.matcher == "grid":
        # the grid adds the order / id / cell-range traffic: ids (4 B) of every
        # reference point and the visit order (4 B) of every query
        alg_bytes_extra = N * 4 + M * 4
    else:
        alg_bytes_extra = 0
    alg_bytes += alg_bytes_extra
    achieved_gbs = alg_bytes / avg_match_s / 1e9
    # HBM traffic of the match kernel from the committed PMC passes of this
    # exact command (profiles/r01/pmc_c3_traffic.json: rocprofv3 FETCH_SIZE x2
    # (gfx950 correction) + WRITE_SIZE, per launch); null for other configs
    traffic, traffic_src = None, None
    if args.config == "c3" and args.matcher == "grid" and world == 1:
        # the PMC passes of this exact driver command (tools/pmc_phases.py:
        # FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE per launch, averaged
        # over the launches of the timed steps)
        src = os.path.join("profiles", "r02", "pmc_c3_driver.json")
        try:
            with open(os.path.join(ROOT, src)) as f:
                pm = json.load(f)
            traffic = pm["match"]["timed"]["hbm_bytes_per_launch"]
            traffic_src = src
        except (OSError, KeyError, TypeError, ValueError):
            pass
    peak_tf = FP32_VALU_TFLOPS if esz == 4 else FP64_VALU_TFLOPS
    metric = "ICP iterations/sec + matched-pairs/sec, 1M→1M pts, k=1, point-to-plane"
    try:
        with open(os.path.join(ROOT, "BASELINE.json")) as f:
            metric = json.load(f)["metric"]
    except Exception:
        pass
    result = {
        "metric": metric,
        "value": pairs / elapsed,
        "unit": "matched-pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32" if esz == 4 else "f64",
        "data": "synthetic (box+sphere surface, seeds 1/2, sigma 0.01, SURVEY.md §8(d))",
        "config": {"workload": f"BASELINE {args.config}: {N * world}->{M} {'float' if esz == 4 else 'double'}, "
                               f"k={knn}, {', '.join(f[0] for f in filters) or 'no outlier filter'}, {minimizer}",
                   "matcher": f"KDTreeMatcher searchType={search_type} ({args.matcher}, exact)",
                   "reading_per_gpu": N, "reference": M, "parallelism": f"reading sharded x{world}, RCCL all-reduce"},
        "icp_iterations_per_s": args.steps / elapsed,
        "kept_pairs_last_iter": st.kept,
        "roofline": {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved_gbs / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_unit": "HBM bytes per launch (PMC)", "traffic_source": traffic_src,
                     "kernel": "match (k-NN + fused transform)", "avg_launch_ms": avg_match_s * 1e3,
                     "algorithmic_bytes_per_launch": alg_bytes,
                     "cold_launch_ms": cold_launch_ms,
                     "note": "steady-state launches certify most k-lists from the previous iteration "
                             "(exact temporal reuse, DESIGN.md §5); with --warmup 0 (default) the timed steps are "
                             "the whole 40-iteration ICP from the initial pose, cold first iterations included; "
                             "cold_launch_ms (warmup > 0) is the first iteration's full search"},
        "compute_roofline": {"bound": "valu", "achieved": flops / avg_match_s / 1e12, "peak": peak_tf,
                             "unit": "TFLOP/s", "frac": flops / avg_match_s / 1e12 / peak_tf,
                             "pairs_evaluated_per_launch": pairs_eval,
                             "note": "brute-force match is VALU-bound (8 FLOP/pair); the HBM fraction is small by construction"},
    }
    if args.matcher == "grid":
        result["compute_roofline"]["note"] = ("grid search: FLOP counts only the pairs actually evaluated; the kernel "
                                              "is gather-latency-bound, neither VALU- nor HBM-bandwidth-bound")
    result["setup_ms"] = setup_s * 1e3
    result["first_prepare_ms"] = first_prepare_s * 1e3
    result["setup_note"] = ("ICP::compute setup before the first iteration, on a live device context: reference "
                            "filters + mean + centring (host, T-sequential), Matcher::init (reference upload, grid "
                            "levels built on the device), reading upload + Morton slot order (device sort); "
                            "first_prepare_ms adds the context creation (HIP runtime, code objects)")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = args.cpu_threads or min(16, os.cpu_count() or 1)
        # GPU side of the parity checks: whole ICPs from the initial pose
        # with the timing chain and with the parity chain (same inputs)
        gpu = {}
        for name, diff in (("counter", None), ("differential", PARITY_DIFF)):
            icp.load_yaml(chain_yaml(knn, filters, minimizer, search_type, args.cpu_iters, diff))
            gpu[name] = (icp.compute(reading, reference, nrm_in), icp.stats())
        cb, runs = cpu_baseline(args.config, reading, reference, normals, knn, filters, minimizer,
                                args.cpu_iters, threads, args.cpu_one_thread_iters)
        result["cpu_baseline"] = cb
        if runs is not None:
            tol = 1e-5 if esz == 4 else 1e-12
            par = {"counter": parity_entry(*gpu["counter"], runs["counter"], tol,
                                           f"the workload's chain, Counter {args.cpu_iters}")}
            if "differential" in runs:
                par["differential"] = parity_entry(*gpu["differential"], runs["differential"], tol,
                                                   f"+ DifferentialTransformationChecker {PARITY_DIFF}")
            par["pass"] = all(v["pass"] for v in par.values() if isinstance(v, dict))
            if "counter_Tsums" in runs:
                TT = np.asarray(runs["counter_Tsums"]["T"], np.float64)
                par["accumulation_gap"] = {
                    "frob_cpu_f64sums_vs_cpu_Tsums": float(np.linalg.norm(np.asarray(runs["counter"]["T"],
                                                                                     np.float64) - TT)),
                    "frob_gpu_vs_cpu_Tsums": float(np.linalg.norm(np.asarray(gpu["counter"][0], np.float64) - TT)),
                    "note": "GPU and oracle sum the normal equations in fp64 from T products; the reference sums "
                            "in T (Eigen GEMM): the size of that deliberate difference here (Counter chain)"}
            result["parity"] = par
    else:
        result["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(result), flush=True)
    icp.close()
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
