"""Benchmark: ICP iterations/s and matched-pairs/s on the BASELINE.json workload.

    python bench.py [--gpus N --steps K --warmup W] [--config c3] [--matcher brute] [--scaling strong|weak]

A "step" is one ICP iteration of the hot path — fused transform + k-NN
match, outlier weighting, normal equations, the 6x6 solve and the checker —
over the synthetic cloud of the configuration.  Default
workload = BASELINE config 3: 1M -> 1M float, k = 1, TrimmedDist ratio 0.85,
point-to-plane.  With N GPUs (torchrun, one process per GPU) the GLOBAL
1M-point reading is split into N contiguous shards against the replicated 1M
reference (strong scaling, the north_star "1M->1M at 1/2/4/8 MI355X"; weak:
--scaling weak, 1M per rank), and each iteration exchanges the quantile
window segments (all-gather) and the normal equations (all-reduce) over RCCL.

Timing: W untimed iterations, then exactly K iterations between a barrier +
device synchronisation on both sides; the max over ranks is reported.  The
clouds are resident in HBM before the timed region.  The match kernel's
device time is measured with HIP events on the context stream (pmx_timing_*).
Every run also times one whole ICP from the initial pose (`whole_icp`: 40
iterations of the same chain, the work the CPU baseline times, cold first
match included).  The CPU baseline (rank 0, N = 1 only) is the oracle's
libnabo-style kd-tree restatement of the reference CPU path on the same
inputs, built -march=native on this host, on every core the job may use and
on one thread.
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
    # (not a BASELINE config: C3 with the reference's default VarTrimmedDist, to time its device sort + partial_sum)
    "c3v": (1_000_000, 1_000_000, np.float32, 1,
            [("VarTrimmedDistOutlierFilter", {"minRatio": 0.05, "maxRatio": 0.99, "lambda": 2.35})],
            "PointToPlaneErrorMinimizer"),
}
BASELINE_CONFIGS = ("c2", "c3", "c4", "c5")
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


def usable_cores():
    """CPUs this process may run on: the affinity mask, capped by a cgroup
    CPU quota and by OMP_NUM_THREADS when the launcher set one (the GPU box
    shares its host: os.cpu_count() reports the whole machine)."""
    n = len(os.sched_getaffinity(0))
    info = {"affinity": n, "host_nproc": os.cpu_count()}
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            info["cgroup_quota"] = float(q) / float(per)
            n = min(n, max(1, int(float(q) / float(per))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        info["omp_num_threads"] = int(omp)
        n = min(n, int(omp))
    return n, info


def native_oracle():
    """The oracle built -march=native on this host (the reference's build,
    CMakeLists.txt:70 -O3; the prebuilt oracle/build is x86-64-v3).  Returns
    (library path or None, ISA note)."""
    import subprocess
    out = os.path.join(ROOT, "oracle", "build_native", "libpmo.so")
    src = os.path.join(ROOT, "oracle", "pmo.c")
    try:
        os.makedirs(os.path.dirname(out), exist_ok=True)
        subprocess.run(["gcc", "-O3", "-march=native", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-fopenmp",
                        "-shared", "-o", out, src, "-lm"], check=True, capture_output=True, timeout=120)
        return out, "gcc -O3 -march=native"
    except Exception as e:  # (no compiler on the host: the prebuilt library)
        return None, f"gcc -O3 -march=x86-64-v3 (prebuilt; native build failed: {type(e).__name__})"


def cpu_baseline(cfg_name, reading, reference, normals, knn, filters, minimizer, iters, threads, one_thread_cap_s):
    """The oracle (C restatement of the reference CPU path: libnabo-style
    kd-tree, nth_element quantile, -O3 -march=native) on the same inputs,
    timed on this host.  Runs (all usable cores): the timing chain (Counter
    `iters`, the workload's chain), the parity chain (+ Differential), and the
    timing chain with T-precision accumulation of the minimiser sums (the
    reference's Eigen arithmetic); then the timing chain on one thread (the
    reference's default: no OpenMP, CMakeLists.txt:160), over all `iters`
    iterations unless that would exceed one_thread_cap_s."""
    lib, isa = native_oracle()
    if lib:
        os.environ["PMO_LIB"] = lib
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

    print(f"[bench] cpu baseline: {threads} threads ({isa})", file=sys.stderr, flush=True)
    rc, T, st, wall = run(threads, iters, None, 0)
    if rc != 0:
        return None, None
    loop = st.loop_seconds
    cores, cinfo = usable_cores()
    out = {"value": n * knn * st.iterations / loop, "unit": "matched-pairs/s", "cores": threads,
           "kind": "port", "iters_per_s": st.iterations / loop, "ms_per_iteration": 1e3 * loop / st.iterations,
           "build": isa, "host_cpu": cpu_model(), "host_cores": cinfo,
           "sample": f"{cfg_name} inputs ({n}->{reference.shape[0]}), the whole timing chain ({st.iterations} ICP "
                     f"iterations from the initial pose), oracle restatement of the reference CPU path "
                     f"(libnabo-style kd-tree with the incremental box bound, nth_element quantile, {isa}), "
                     f"{threads} threads (every core this job may use), loop {loop:.2f} s (setup+loop {wall:.2f} s)"}
    runs = {"counter": {"T": T, "iterations": int(st.iterations), "kept": int(st.kept)}}
    rcd, Td, std, _ = run(threads, iters, PARITY_DIFF, 0)
    if rcd == 0:
        runs["differential"] = {"T": Td, "iterations": int(std.iterations), "kept": int(std.kept)}
    rcT, TT, stT, _ = run(threads, iters, None, 1)
    if rcT == 0:
        runs["counter_Tsums"] = {"T": TT, "iterations": int(stT.iterations), "kept": int(stT.kept)}
    # one thread: every iteration of the chain when the estimate (the
    # all-core loop times its thread count) fits the cap, else the first ones
    est = loop * threads
    it1 = iters if est <= one_thread_cap_s else max(2, int(iters * one_thread_cap_s / est))
    print(f"[bench] cpu baseline: 1 thread, {it1} iterations (estimate {est * it1 / iters:.0f} s)", file=sys.stderr,
          flush=True)
    rc1, T1, st1, _ = run(1, it1, None, 0)
    if rc1 == 0:
        out["single_thread"] = {"value": n * knn * st1.iterations / st1.loop_seconds, "unit": "matched-pairs/s",
                                "cores": 1, "iters_per_s": st1.iterations / st1.loop_seconds,
                                "ms_per_iteration": 1e3 * st1.loop_seconds / st1.iterations,
                                "sample": f"{'the whole timing chain' if it1 == iters else 'the first'} "
                                          f"({st1.iterations} ICP iterations from the initial pose), 1 thread, "
                                          f"{isa}, loop {st1.loop_seconds:.2f} s"}
    return out, runs


def parity_entry(Tg, sg, ref, tol, chain):
    frob = float(np.linalg.norm(np.asarray(Tg, np.float64) - np.asarray(ref["T"], np.float64)))
    return {"frob": frob, "tolerance": tol,
            "pass": bool(frob <= tol and int(sg.iterations) == ref["iterations"] and int(sg.kept) == ref["kept"]),
            "iterations_gpu": int(sg.iterations), "iterations_cpu": ref["iterations"],
            "kept_gpu": int(sg.kept), "kept_cpu": ref["kept"], "chain": chain}


def shard_range(n, world, rank):
    """Contiguous reading shard of a rank (the multi-rank tests' convention)."""
    base, rem = divmod(n, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=0)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--matcher", default="grid", choices=["brute", "grid"],
                    help="KDTreeMatcher searchType 0 (brute force) or 1 (spatial grid)")
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                    help="strong: the configuration's global reading split over the ranks (default); "
                         "weak: the configuration's reading on every rank")
    ap.add_argument("--cpu-iters", type=int, default=40)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--cpu-one-thread-cap", type=float, default=100.0,
                    help="seconds the 1-thread CPU sample may take (fewer iterations beyond)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--device-warmup", type=float, default=0.3,
                    help="seconds of untimed whole ICPs before the measured regions (GPU clock ramp)")
    ap.add_argument("--dist", action="store_true",
                    help="use the torchrun/RCCL multi-rank path even at world size 1 (rehearsal on one GPU)")
    ap.add_argument("--emulate-ranks", type=int, default=1,
                    help="per-rank cost model on one process: run only shard 0 of the global reading split G ways "
                         "(the work one rank of a G-GPU strong-scaling run does; with --dist its collectives are "
                         "issued at world size 1).  A projection input, not a multi-GPU measurement")
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

    N_cfg, M, dtype, knn, filters, minimizer = CONFIGS[args.config]
    reference, normals = reference_cloud(M, dtype)
    strong = args.scaling == "strong"
    N_global = N_cfg if strong else N_cfg * world
    if dist or args.emulate_ranks > 1:
        full = reading_cloud(N_global, dtype)
        G = world if world > 1 else max(1, args.emulate_ranks)
        lo, hi = shard_range(N_global, G, rank)
        reading = np.ascontiguousarray(full[lo:hi])
        del full
    else:
        reading = reading_cloud(N_global, dtype)
    N = reading.shape[0]  # this rank's shard
    # (the per-rank cost model counts the shard's own pairs)
    N_work = N if (args.emulate_ranks > 1 and world == 1) else N_global

    search_type = 0 if args.matcher == "brute" else 1
    total_it = args.warmup + args.steps + 10
    icp = ICP(dtype, device=local_rank)
    icp.load_yaml(chain_yaml(knn, filters, minimizer, search_type, total_it))
    if dist:
        import torch

        uid = bytearray(_capi.Context.unique_id() if rank == 0 else bytes(128))
        t = torch.tensor(list(uid), dtype=torch.uint8)
        tdist.broadcast(t, src=0)
        # (RCCL prints its version banner on fd 1 at communicator creation:
        # stdout stays the one JSON line)
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            icp.comm_init(bytes(t.tolist()), world, rank)
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)

    def barrier():
        if dist:
            tdist.barrier()

    def max_over_ranks(v):
        if not dist:
            return v
        import torch

        e = torch.tensor([v], dtype=torch.float64)
        tdist.all_reduce(e, op=tdist.ReduceOp.MAX)
        return float(e.item())

    nrm_in = normals if minimizer.startswith("PointToPlane") else None
    # setup (reported separately): reference upload + grid
    # build (Matcher::init), reading upload + slot order, ICP.cpp:265-347.
    # The first prepare also creates the device context (HIP runtime, code
    # objects, RCCL communicator): reported as first_prepare_ms; setup_ms is
    # the per-compute cost, measured after the device warm-up below.
    t_s = time.perf_counter()
    icp.prepare(reading, reference, nrm_in)
    first_prepare_s = time.perf_counter() - t_s

    # ---- device warm-up (untimed): whole ICPs of the timing chain for at
    # least --device-warmup seconds, so the GPU runs at its working clocks
    # when the measured regions start (a fresh process, or a GPU left idle by
    # the host-side work, otherwise pays the clock ramp inside them: the same
    # 20-iteration driver command measured 0.079 and 0.179 ms/iteration)
    whole_yaml = chain_yaml(knn, filters, minimizer, search_type, args.cpu_iters)
    icp.load_yaml(whole_yaml)
    w_end = time.perf_counter() + args.device_warmup
    n_warm = 0
    while True:
        icp.prepare(reading, reference, nrm_in)
        icp.iterate(args.cpu_iters)
        n_warm += 1
        # (every rank runs the same number: the sharded ICP exchanges collectives)
        if max_over_ranks(1.0 if time.perf_counter() >= w_end else 0.0) > 0.0:
            break
    # setup: the per-compute cost on the live, warm context — the best of
    # three prepares after the device warm-up, with its reference / reading
    # parts from that prepare's statistics
    setup_s, setup_parts = None, None
    for _ in range(3):
        barrier()
        t_s = time.perf_counter()
        icp.prepare(reading, reference, nrm_in)
        dt = max_over_ranks(time.perf_counter() - t_s)
        if setup_s is None or dt < setup_s:
            pst = icp.stats()
            setup_s = dt
            setup_parts = {"reference_ms": 1e3 * pst.reference_preprocessing_duration,
                           "reading_ms": 1e3 * pst.reading_preprocessing_duration}

    # ---- one whole ICP from the initial pose (the representative workload:
    # what every new scan pays, and what the CPU baseline times): the timing
    # chain of the CPU baseline (Counter cpu_iters), prepare untimed
    icp.prepare(reading, reference, nrm_in)
    barrier()
    w0 = time.perf_counter()
    icp.iterate(args.cpu_iters)
    w1 = time.perf_counter()
    barrier()
    whole_s = max_over_ranks(w1 - w0)
    wst = icp.stats()
    hits, misses = icp.select_stats()
    # the same ICP once more, one iteration per call with HIP events around
    # each match: the cold first match and the matches of the first iterations
    icp.prepare(reading, reference, nrm_in)
    first_match_us = []
    for _ in range(min(8, args.cpu_iters)):
        icp.timing(True)
        icp.iterate(1)
        ms, nl = icp.timing_read()
        first_match_us.append(round(1e3 * ms / max(nl, 1), 2))
    icp.timing(False)
    whole = {"iterations": int(wst.iterations), "ms": 1e3 * whole_s,
             "ms_per_iteration": 1e3 * whole_s / max(int(wst.iterations), 1),
             "matched_pairs_per_s": N_work * knn * int(wst.iterations) / whole_s,
             "cold_match_ms": first_match_us[0] * 1e-3 if first_match_us else None,
             "first_matches_us": first_match_us,
             "window_hits": int(hits), "window_misses": int(misses),
             "chain": f"the workload's chain, CounterTransformationChecker {args.cpu_iters}, from the initial pose "
                      f"(prepare untimed, then {args.cpu_iters} iterations timed as the CPU baseline's loop); "
                      f"first_matches_us: device time of each of the first matches (separate run, HIP events)",
             "device_warmup": f"{n_warm} untimed whole ICPs ({args.device_warmup:.2f} s) before every measured region"}

    # ---- ICPSequence (before the driver region: the last dispatches of the
    # command are the timed pass and the roofline pass, tools/pmc_phases.py)
    seq_ms, seq_note = None, None
    if not dist:
        # ICPSequence (ICP.cpp:455-609): the map set once, then each scan pays
        # only the reading side (upload, slot order) and its iterations
        from libpointmatcher_amd.icp import ICPSequence

        seq = ICPSequence(dtype, device=local_rank)
        seq.load_yaml(chain_yaml(knn, filters, minimizer, search_type, args.cpu_iters))
        seq.set_map(reference, nrm_in)
        seq.compute(reading)  # (warm)
        scans = []
        for _ in range(3):
            t_q = time.perf_counter()
            seq.prepare(reading)
            t_p = time.perf_counter()
            seq.iterate(args.cpu_iters)
            t_e = time.perf_counter()
            scans.append((1e3 * (t_p - t_q), 1e3 * (t_e - t_q)))
        seq.close()
        seq_ms = min(x[1] for x in scans)
        seq_note = (f"ICPSequence: map set once; per scan the reading-side setup "
                    f"({min(x[0] for x in scans):.2f} ms) + {args.cpu_iters} iterations from the initial pose; best of 3")

    # ---- the driver's region: W untimed iterations, then exactly K timed
    icp.load_yaml(chain_yaml(knn, filters, minimizer, search_type, total_it))
    icp.prepare(reading, reference, nrm_in)
    if args.warmup > 0:
        icp.iterate(args.warmup)

    cs0 = icp.comm_stats() if dist else None
    barrier()
    t0 = time.perf_counter()
    icp.iterate(args.steps)   # each batch ends with the status copy-back: device is synchronised
    t1 = time.perf_counter()
    barrier()
    elapsed = max_over_ranks(t1 - t0)
    st = icp.stats()
    # per-iteration evidence of the timed iterations (pmx_loop_diag): the grid
    # level each match ran on, the quantile window verdict, the pairs
    # evaluated and the full searches (the rest certified by temporal reuse)
    dg = icp.loop_diag(0, args.warmup + args.steps)[args.warmup:]
    diag = {"levels": [int(x) for x in dg[:, 0]], "window": [int(x) for x in dg[:, 1]],
            "pairs_evaluated": [int(x) for x in dg[:, 2]], "full_searches": [int(x) for x in dg[:, 3]],
            "note": "timed iterations only: grid level index of each match (0 = the finest; DESIGN.md §3), "
                    "window 1 = quantile resolved in the match's key window, 0 = radix passes, -1 = no window"}
    # collectives and host synchronisations of the timed iterations (sharded
    # runs: stall-and-replay)
    comm = ({k: v - cs0[k] for k, v in icp.comm_stats().items()} if dist else None)
    # Roofline pass: the same ICP again (prepare resets the pose and the
    # match history), now with HIP events around every match launch on the
    # context stream.  The events are kept out of the timed region above: each
    # record is a marker packet that adds idle GPU time to the iteration.
    icp.prepare(reading, reference, nrm_in)
    if args.warmup > 0:
        icp.iterate(args.warmup)
    icp.timing(True)
    icp.iterate(args.steps)
    match_ms, launches = icp.timing_read()
    icp.timing(False)

    pairs = N_work * knn * args.steps
    avg_match_s = match_ms * 1e-3 / max(launches, 1)
    esz = np.dtype(dtype).itemsize
    # algorithmic bytes of one match launch: the reading shard (4 T per point),
    # the reference (4 T per point) and the k (dist, id) outputs per query
    alg_bytes = N * 4 * esz + M * 4 * esz + N * knn * (esz + 4)
    alg_bytes_survey = alg_bytes  # N*16 + M*16 + N*k*8 (fp32; doubled for fp64 but the ids)
    # pair evaluations per match launch: N*M for brute force, the measured
    # PointCountTouched per iteration for the grid search
    # (the timed iterations' own pairs, from the per-iteration record)
    pairs_eval = N * M if args.matcher == "brute" else float(dg[:, 2].mean())
    flops = 8.0 * pairs_eval  # 3 sub + 3 mul + 2 add per pair
    if args.matcher == "grid":
        # the grid adds the order / id / cell-range traffic: ids (4 B) of every
        # reference point and the visit order (4 B) of every query
        alg_bytes += N * 4 + M * 4
    achieved_gbs = alg_bytes_survey / avg_match_s / 1e9
    achieved_grid_gbs = alg_bytes / avg_match_s / 1e9
    # HBM traffic of the match kernel from the committed PMC passes of this
    # exact command (tools/pmc_phases.py: FETCH_SIZE x2 (gfx950 correction) +
    # WRITE_SIZE per launch, averaged over the launches of the timed steps);
    # null for other configurations
    traffic, traffic_src = None, None
    if args.matcher == "grid" and world == 1:
        for src in (os.path.join("profiles", "r06", f"pmc_{args.config}_driver.json"),
                    os.path.join("profiles", "r05", f"pmc_{args.config}_driver.json"),
                    os.path.join("profiles", "r04", f"pmc_{args.config}_driver.json"),
                    os.path.join("profiles", "r03", f"pmc_{args.config}_driver.json")):
            try:
                with open(os.path.join(ROOT, src)) as f:
                    pm = json.load(f)
                traffic = pm["match"]["timed"]["hbm_bytes_per_launch"]
                traffic_src = src
                break
            except (OSError, KeyError, TypeError, ValueError):
                pass
    peak_tf = FP32_VALU_TFLOPS if esz == 4 else FP64_VALU_TFLOPS
    metric = "ICP iterations/sec + matched-pairs/sec, 1M→1M pts, k=1, point-to-plane"
    try:
        with open(os.path.join(ROOT, "BASELINE.json")) as f:
            metric = json.load(f)["metric"]
    except Exception:
        pass
    if args.emulate_ranks > 1 and world == 1:
        par = (f"per-rank cost model: shard 0 of {args.emulate_ranks} of the {N_global} reading on one GPU "
               f"({'RCCL collectives issued at world size 1' if dist else 'no communicator'}); value is this shard's "
               f"rate, not a multi-GPU measurement")
    elif dist:
        par = (f"reading sharded x{world} ({'strong: ' + str(N_global) + ' global' if strong else 'weak: ' + str(N_cfg) + ' per rank'}), "
               f"reference replicated; RCCL per iteration: quantile window all-gather (+ radix histogram all-reduces "
               f"on a window miss) and the normal-equation all-reduce")
    else:
        par = "one GPU, no communicator"
    result = {
        "metric": metric,
        "value": pairs / elapsed,
        "unit": "matched-pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "f32" if esz == 4 else "f64",
        "data": "synthetic (box+sphere surface, seeds 1/2, sigma 0.01, SURVEY.md §8(d))",
        "config": {"workload": f"{'BASELINE ' + args.config if args.config in BASELINE_CONFIGS else args.config + ' (not a BASELINE config: C3 with VarTrimmedDist)'}: {N_global}->{M} {'float' if esz == 4 else 'double'}, "
                               f"k={knn}, {', '.join(f[0] for f in filters) or 'no outlier filter'}, {minimizer}",
                   "matcher": f"KDTreeMatcher searchType={search_type} ({args.matcher}, exact)",
                   "reading_global": N_global, "reading_per_gpu": N, "reference": M, "parallelism": par},
        "icp_iterations_per_s": args.steps / elapsed,
        "comm_timed": comm,
        "kept_pairs_last_iter": st.kept,
        "timed_iterations": diag,
        "whole_icp": whole,
        "roofline": {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved_gbs / HBM_PEAK_GBS, "traffic": traffic,
                     "achieved_with_grid_bytes": achieved_grid_gbs, "frac_with_grid_bytes": achieved_grid_gbs / HBM_PEAK_GBS,
                     "grid_bytes_per_launch": alg_bytes,
                     "traffic_unit": "bytes per launch past L2 (PMC FETCH_SIZE x2 + WRITE_SIZE)",
                     "traffic_source": traffic_src,
                     "kernel": "match (k-NN + fused transform)", "avg_launch_ms": avg_match_s * 1e3,
                     "launches": (f"the {args.steps} matches of a repeat of the timed region (prepare, {args.warmup} "
                                  f"untimed, then {args.steps} iterations; HIP events recorded by each match's own "
                                  f"dispatch on the context stream, hipExtLaunchKernelGGL start / stop: grid_lane_kernel; "
                                  f"tools/pmc_phases.py 'roofline' phase = the same launches in the rocprof trace)"),
                     "algorithmic_bytes_per_launch": alg_bytes_survey,
                     "algorithmic_bytes_rule": "SURVEY.md §8(d): N*4T + M*4T + N*k*(T + 4 id) per launch; "
                                               "grid_bytes_per_launch adds the grid's order (4 B / query) and "
                                               "id (4 B / reference point) arrays",
                     "note": "steady-state launches certify most k-lists from the previous iteration (exact temporal "
                             "reuse, DESIGN.md §5); the ~70 MB C3 working set fits the 256 MB Infinity Cache, so "
                             "PMC FETCH_SIZE counts L2-miss bytes (MALL hits included) and 8 TB/s HBM is not the "
                             "binding ceiling of this gather-latency-bound kernel; whole_icp.first_matches_us has "
                             "the cold (initial-pose) matches"},
        "compute_roofline": {"bound": "valu", "achieved": flops / avg_match_s / 1e12, "peak": peak_tf,
                             "unit": "TFLOP/s", "frac": flops / avg_match_s / 1e12 / peak_tf,
                             "pairs_evaluated_per_launch": pairs_eval,
                             "note": "brute-force match is VALU-bound (8 FLOP/pair); the HBM fraction is small by construction"},
    }
    if args.matcher == "grid":
        result["compute_roofline"]["note"] = ("grid search: FLOP counts only the pairs actually evaluated; the kernel "
                                              "is gather-latency-bound, neither VALU- nor HBM-bandwidth-bound")
    result["setup_ms"] = setup_s * 1e3
    if seq_ms is not None:
        result["sequence_scan_ms"] = seq_ms
        result["sequence_scan_note"] = seq_note
    result["setup_parts"] = setup_parts
    result["first_prepare_ms"] = first_prepare_s * 1e3
    result["setup_note"] = ("ICP::compute setup before the first iteration, on a live device context (best of three "
                            "prepares after the device warm-up): reference mean (host thread, T-sequential) + "
                            "upload + centring, Matcher::init (the cold grid level; the finer ones on a side stream, "
                            "awaited by the second match), reading upload (overlapping the level build) + Morton slot "
                            "order (device sort); first_prepare_ms adds the context creation (HIP runtime, code objects)")
    if rank == 0 and world == 1 and args.emulate_ranks == 1 and not args.no_cpu_baseline:
        threads = args.cpu_threads or usable_cores()[0]
        # GPU side of the parity checks: whole ICPs from the initial pose
        # with the timing chain and with the parity chain (same inputs)
        gpu = {}
        for name, diff in (("counter", None), ("differential", PARITY_DIFF)):
            icp.load_yaml(chain_yaml(knn, filters, minimizer, search_type, args.cpu_iters, diff))
            gpu[name] = (icp.compute(reading, reference, nrm_in), icp.stats())
        cb, runs = cpu_baseline(args.config, reading, reference, normals, knn, filters, minimizer,
                                args.cpu_iters, threads, args.cpu_one_thread_cap)
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
            if cb:
                result["whole_icp"]["vs_cpu_all_cores"] = whole["matched_pairs_per_s"] / cb["value"]
    else:
        result["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(result), flush=True)
    icp.close()
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
