"""The product's multi-rank path, executed: two ranks on the one MI355X.

Each rank is its own process with its own pmx_ctx on device 0 and the
reading's contiguous shard.  RCCL cannot put two ranks on one
GPU, so the ranks exchange over the host-staged collectives of the C ABI
(pmx_comm_init_host) with torch.distributed gloo as the transport: the same
library code, kernels and exchange steps as the RCCL path — only the
transport under coll_allreduce / coll_allgather differs.  The RCCL transport
itself is exercised at one rank (a communicator issues every collective at
any nranks) by test_rccl_one_rank_is_bit_identical.

Bars (against the single-process oracle on the WHOLE reading):
  * the TrimmedDist limit (radix select with histogram all-reduce) bit-equal;
  * the point-to-plane system equal to fp64 reassociation (1e-12 relative);
  * VarTrimmedDist (distance all-gather) kept count exact;
  * whole ICPs through the host chain (device loop, quantile window exchanged
    as all-gathered segments): final T within 1e-5 (f32) / 1e-12 (f64) with
    equal iteration counts and kept pairs, every rank the same T;
  * the sharded window resolves quantiles (hits > 0) and equals the radix
    path (option spec_select=0) bit for bit;
  * a window hit costs an iteration two collectives (pmx_comm_stats).
Reference semantics: OutlierFilter.cpp:63-103, Matches.cpp:60-87,
OutlierFiltersImpl.cpp:132-223, PointToPlane.cpp:171-243, ICP.cpp:317-449.
"""
import multiprocessing as mp
import os
import socket
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(__file__))
from helpers import chain_yaml  # noqa: E402

pytestmark = pytest.mark.gpu

DIFF = dict(minDiffRotErr=0.001, minDiffTransErr=0.01, smoothLength=4)
TOL = {"float32": 1e-5, "float64": 1e-12}
N_RD, N_REF = 60000, 50000
VT = dict(minRatio=0.05, maxRatio=0.99, **{"lambda": 2.35})


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def shard_range(n, world, rank):
    base, rem = divmod(n, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def _clouds(dtype):
    from libpointmatcher_amd.synth import reading_cloud, reference_cloud

    ref, nrm = reference_cloud(N_REF, dtype)
    return reading_cloud(N_RD, dtype), ref, nrm


P2PLANE, P2POINT = "PointToPlaneErrorMinimizer", "PointToPointErrorMinimizer"
# whole-ICP cases: (tag, knn, outlier filters, minimizer, Counter max, Differential, reference normals)
ICP_RUNS = [
    ("trim", 1, (("TrimmedDistOutlierFilter", {"ratio": 0.85}),), P2PLANE, 30, DIFF, True),
    ("vt", 1, (("VarTrimmedDistOutlierFilter", VT),), P2PLANE, 20, DIFF, True),
    ("med", 1, (("MedianDistOutlierFilter", {"factor": 3.0}), ("MaxDistOutlierFilter", {"maxDist": 0.5})), P2PLANE,
     20, None, True),
    ("p2pt", 1, (), P2POINT, 10, None, False),
    ("robust", 1, (("RobustOutlierFilter", {"robustFct": "cauchy", "scaleEstimator": "mad", "tuning": 1}),),
     P2POINT, 15, DIFF, False),
    # the sharded benchmark chains: C4 (k = 4, MaxDist, point-to-plane) and
    # C5 (empty chain, point-to-point, 40 iterations)
    ("c4", 4, (("MaxDistOutlierFilter", {"maxDist": 0.05}),), P2PLANE, 20, DIFF, True),
    ("c5", 1, (), P2POINT, 40, None, False),
]


def _worker(rank, world, port, outdir, env):
    os.environ.update(env)
    # torch first: its bundled HIP runtime is then the one libpmx binds to (bench.py)
    import torch  # noqa: F401
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # MR_LOOP_ONLY: the device loop and the window ICP chains only (the
    # forced-miss replay run)
    loop_only = os.environ.get("MR_LOOP_ONLY") == "1"
    try:
        from libpointmatcher_amd import _capi
        from libpointmatcher_amd.icp import ICP

        comm = _capi.gloo_host_comm()
        res = {}
        for dn in ("float32", "float64"):
            dtype = np.dtype(dn)
            rd, ref, nrm = _clouds(dtype)
            lo, hi = shard_range(rd.shape[0], world, rank)
            shard = np.ascontiguousarray(rd[lo:hi])
            I = np.eye(4, dtype=dtype)
            # per-module calls through the C ABI
            ctx = _capi.Context(0, dtype)
            ctx.comm_init_host(comm)
            assert ctx.comm_size() == (world, rank, 2)
            ctx.set_reference(ref, nrm)
            ctx.set_reading(shard)
            if not loop_only:
                ctx.match(I, knn=1)
                ctx.outlier("TrimmedDistOutlierFilter", 0, ratio=0.85)
                A, b, st = ctx.p2plane_system()
                res[f"{dn}_trim"] = np.concatenate([A.ravel(), b, [st.limit, st.kept, st.n_total]])
                ctx.match(I, knn=1)
                ctx.outlier("VarTrimmedDistOutlierFilter", 0, **VT)
                A, b, st = ctx.p2plane_system()
                res[f"{dn}_vt"] = np.concatenate([A.ravel(), b, [st.limit, st.kept]])
                # RobustOutlierFilter: MAD (two sharded selects) and std (all-reduced moments)
                for tag, fct, mode in (("rmad", "cauchy", _capi.RS_MAD), ("rstd", "welsch", _capi.RS_STD)):
                    ctx.match(I, knn=2)
                    ctx.outlier_robust(0, fct, 0.8, np.inf, mode, 0.0)
                    A, b, st = ctx.p2plane_system()
                    res[f"{dn}_{tag}"] = np.concatenate([A.ravel(), b, [ctx.robust_scale(0), st.kept, st.sum_w]])
                ctx.set_reading(shard)
            # the device loop on the context: quantile window exchanged as segments
            ctx.loop_begin(filters=[("TrimmedDistOutlierFilter", 0.85)], checkers=[("CounterTransformationChecker", 25)])
            ar0, ag0 = ctx.comm_stats()
            sy0 = ctx.comm_loop_stats()
            cb0 = dict(comm.calls)
            ls = ctx.loop_run(25)
            hits, misses = ctx.loop_select_stats()
            ar1, ag1 = ctx.comm_stats()
            sy1 = ctx.comm_loop_stats()
            res[f"{dn}_loop"] = np.concatenate([np.asarray(ls.T_iter[:16]), [ls.iterations, ls.last.kept, hits,
                                                                              misses]])
            # the collectives of the loop: native counter, and the transport's own count
            res[f"{dn}_coll"] = np.array([ar1 - ar0, ag1 - ag0, comm.calls["allreduce"] - cb0["allreduce"],
                                          comm.calls["allgather"] - cb0["allgather"], ls.iterations, hits, misses])
            # how the loop synchronised: verdict reads, blind iterations, stalls replayed
            res[f"{dn}_sync"] = np.array([b - a for a, b in zip(sy0, sy1)])
            ctx.close()
            # whole ICPs through the host chain (pmx_icp_comm_init_host)
            for tag, knn, filters, minimizer, maxit, diff, with_n in ICP_RUNS:
                if loop_only and tag not in ("trim", "med"):
                    continue
                icp = ICP(dtype)
                icp.comm_init_host(comm)
                icp.load_yaml(chain_yaml(knn=knn, filters=filters, minimizer=minimizer, maxit=maxit,
                                         differential=diff))
                T = icp.compute(shard, ref, nrm if with_n else None)
                s = icp.stats()
                res[f"{dn}_icp_{tag}"] = np.concatenate([T.astype(np.float64).ravel(), [s.iterations, s.kept]])
                icp.close()
        assert not comm.errors, comm.errors
        np.savez(os.path.join(outdir, f"rank{rank}.npz"), **res)
    finally:
        dist.destroy_process_group()


def _run_two_ranks(tmp, env):
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(i, 2, port, str(tmp), env)) for i in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(540)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.exitcode is None:
            p.kill()
    assert codes == [0, 0], codes
    return [dict(np.load(tmp / f"rank{i}.npz")) for i in range(2)]


@pytest.fixture(scope="module")
def two_ranks(tmp_path_factory):
    return _run_two_ranks(tmp_path_factory.mktemp("mr_gpu"), {})


@pytest.fixture(scope="module")
def two_ranks_radix(tmp_path_factory):
    # the same runs with the quantile window off: every limit from the radix
    # passes with their histogram all-reduce
    return _run_two_ranks(tmp_path_factory.mktemp("mr_gpu_radix"), {"PMX_OPTS": "spec_select=0"})


@pytest.mark.timeout(900)
@pytest.mark.parametrize("dn", ["float32", "float64"])
def test_sharded_modules_vs_oracle(two_ranks, oracle, dn):
    r = two_ranks
    dtype = np.dtype(dn)
    rd, ref, nrm = _clouds(dtype)
    for key in (f"{dn}_trim", f"{dn}_vt"):
        np.testing.assert_array_equal(r[0][key], r[1][key])  # every rank holds the same system and limit
    d, ids, _ = oracle.knn(ref, rd, k=1)
    # TrimmedDist: the global quantile, bit-equal
    rc, q = oracle.quantile(d, 0.85)
    assert rc == 0
    got = r[0][f"{dn}_trim"]
    assert dtype.type(got[-3]) == q
    rc, w = oracle.outlier_chain([("TrimmedDistOutlierFilter", {"ratio": 0.85})], d)
    rc, A, b, st = oracle.p2plane_system(rd, ref, nrm, d, ids, w)
    assert int(got[-2]) == st.kept and int(got[-1]) == N_RD
    full = np.concatenate([A.ravel(), b])
    np.testing.assert_allclose(got[:42], full, rtol=1e-12, atol=1e-12 * np.abs(full).max())
    # VarTrimmedDist: the distances all-gathered, the same optimised ratio
    rc, w = oracle.outlier_chain([("VarTrimmedDistOutlierFilter", VT)], d)
    assert rc == 0
    assert int(r[0][f"{dn}_vt"][-1]) == int((w != 0).sum())
    # RobustOutlierFilter over the shards: the global scale (MAD bit-equal, std
    # to fp64 reassociation), the weighted system (full A) to the weights' tolerance
    d2, ids2, _ = oracle.knn(ref, rd, k=2)
    for tag, fct, scale in (("rmad", "cauchy", "mad"), ("rstd", "welsch", "std")):
        np.testing.assert_array_equal(r[0][f"{dn}_{tag}"], r[1][f"{dn}_{tag}"])
        rb = oracle.make_robust({"robustFct": fct, "scaleEstimator": scale, "tuning": 0.8})
        rc, w = oracle.robust_weights(rb, d2, ids2)
        assert rc == 0
        rc, A, b, st = oracle.p2plane_system(rd, ref, nrm, d2, ids2, w)
        got = r[0][f"{dn}_{tag}"]
        if scale == "mad":
            assert got[-3] == rb.scale
        else:
            np.testing.assert_allclose(got[-3], rb.scale, rtol=4e-7 if dn == "float32" else 1e-13)
        assert int(got[-2]) == st.kept
        full = np.concatenate([A.ravel(), b])
        tol = 1e-6 if dn == "float32" else 1e-11  # (device exp vs libm: the weights to ~1 ulp)
        np.testing.assert_allclose(got[:42], full, rtol=tol, atol=tol * np.abs(full).max())


@pytest.mark.timeout(900)
@pytest.mark.parametrize("dn", ["float32", "float64"])
def test_sharded_icp_vs_oracle(two_ranks, oracle, dn):
    r = two_ranks
    dtype = np.dtype(dn)
    rd, ref, nrm = _clouds(dtype)
    from test_gpu_configs import THREADS

    for tag, knn, filters, minimizer, maxit, diff, with_n in ICP_RUNS:
        a, b2 = r[0][f"{dn}_icp_{tag}"], r[1][f"{dn}_icp_{tag}"]
        np.testing.assert_array_equal(a, b2)  # every rank ends with the same transform
        cfg = oracle.make_cfg(knn=knn, filters=filters, minimizer=minimizer, counter_max=maxit, differential=diff,
                              threads=THREADS)
        rc, To, so, _ = oracle.icp(cfg, rd, ref, normals=nrm if with_n else None)
        assert rc == 0
        T = a[:16].reshape(4, 4)
        frob = np.linalg.norm(T - To.astype(np.float64))
        print(f"{dn} {tag}: iterations {int(a[16])}/{so.iterations} kept {int(a[17])}/{so.kept} |dT|={frob:.3g}")
        assert int(a[16]) == so.iterations
        assert int(a[17]) == so.kept
        assert frob <= TOL[dn]


@pytest.mark.timeout(900)
@pytest.mark.parametrize("dn", ["float32", "float64"])
def test_sharded_window_equals_radix(two_ranks, two_ranks_radix, dn):
    w, x = two_ranks[0][f"{dn}_loop"], two_ranks_radix[0][f"{dn}_loop"]
    np.testing.assert_array_equal(two_ranks[0][f"{dn}_loop"], two_ranks[1][f"{dn}_loop"])
    assert w[18] > 0, "the exchanged window never resolved a quantile"
    assert x[18] == 0
    np.testing.assert_array_equal(w[:18], x[:18])  # T_iter, iterations, kept: bit-identical
    for k in [k for k in two_ranks[0] if "_icp_" in k]:
        np.testing.assert_array_equal(two_ranks[0][k], two_ranks_radix[0][k])


@pytest.mark.timeout(900)
@pytest.mark.parametrize("dn", ["float32", "float64"])
def test_sharded_hit_iterations_two_collectives(two_ranks, two_ranks_radix, dn):
    """A window hit costs a sharded iteration two collectives (the segments'
    all-gather, the system's all-reduce); a miss adds the radix passes'
    histogram all-reduces.  Counted natively (pmx_comm_stats) and by the
    transport itself."""
    passes = 3 if dn == "float32" else 6
    for r in (two_ranks[0], two_ranks[1]):
        ar, ag, cb_ar, cb_ag, iters, hits, misses = (int(v) for v in r[f"{dn}_coll"])
        syncs, blind, stalls = (int(v) for v in r[f"{dn}_sync"])
        print(f"{dn}: {iters} iterations, {hits} hits / {misses} misses: {ar} all-reduces, {ag} all-gathers; "
              f"{syncs} verdict syncs, {blind} blind iterations, {stalls} stalls")
        assert (ar, ag) == (cb_ar, cb_ag)  # every collective the library counts reached the transport
        assert hits > 0 and hits + misses <= ag
        # per enqueued iteration: one all-gather + the system's all-reduce, the
        # passes on a miss, and a stalled iteration's replayed system
        assert ar == ag + passes * misses + stalls
        assert ag <= iters + 1 + 2 * 4 * stalls  # (a stall wastes at most the two batches in flight)
        # the verdict is read back only while the window settles: after the
        # first (known) miss and every later miss, until two hits in a row
        assert syncs <= 3 * misses + 2
        assert blind >= hits - 2 * (misses + 1)
        assert blind > 0
        assert syncs + blind <= ag
    # the radix path: every iteration runs the passes
    ar, ag, _, _, iters, hits, _ = (int(v) for v in two_ranks_radix[0][f"{dn}_coll"])
    assert hits == 0 and ag == 0 and ar % (1 + passes) == 0 and ar // (1 + passes) >= iters


@pytest.mark.parametrize("dn", ["float32", "float64"])
def test_rccl_one_rank_is_bit_identical(oracle, dn, monkeypatch):
    """A communicator issues every collective (RCCL all-reduce / all-gather of
    the histograms, window segments, distances and systems) even at one rank;
    the result must equal the unsharded run bit for bit.  (The unsharded loop
    runs the module chain here: its fused iteration sums in another order.)"""
    from libpointmatcher_amd import _capi


    dtype = np.dtype(dn)
    rd, ref, nrm = _clouds(dtype)
    out = []
    for comm in ("none", "rccl", "host"):
        ctx = _capi.Context(0, dtype)
        if comm == "rccl":
            ctx.comm_init(_capi.Context.unique_id(), 1, 0)
            assert ctx.comm_size() == (1, 0, 1)
        elif comm == "host":
            hc = _capi.HostComm(1, 0, lambda a, op: None, lambda a: a)
            ctx.comm_init_host(hc)
        ctx.set_reference(ref, nrm)
        ctx.set_reading(rd)
        ctx.match(np.eye(4, dtype=dtype), knn=1)
        ctx.outlier("VarTrimmedDistOutlierFilter", 0, **VT)
        A, b, st = ctx.p2plane_system()
        ctx.loop_begin(filters=[("TrimmedDistOutlierFilter", 0.85)], checkers=[("CounterTransformationChecker", 20)])
        ls = ctx.loop_run(20)
        hits, _ = ctx.loop_select_stats()
        out.append((A, b, st.kept, np.asarray(ls.T_iter[:16]), ls.last.kept, hits))
        ctx.close()
    for o in out[1:]:
        np.testing.assert_array_equal(o[0], out[0][0])
        np.testing.assert_array_equal(o[1], out[0][1])
        assert o[2] == out[0][2] and o[4] == out[0][4]
        np.testing.assert_array_equal(o[3], out[0][3])
        assert o[5] > 0


@pytest.fixture(scope="module")
def two_ranks_forced_miss(tmp_path_factory):
    # misses forced at loop iterations 10 and 17 (past the settling
    # iterations: enqueued blind, so they stall the device loop and replay)
    return _run_two_ranks(tmp_path_factory.mktemp("mr_gpu_miss"), {"PMX_OPTS": "force_miss=10:17",
                                                                   "MR_LOOP_ONLY": "1"})


@pytest.mark.timeout(900)
@pytest.mark.parametrize("dn", ["float32", "float64"])
def test_sharded_stall_replay_bit_identical(two_ranks, two_ranks_forced_miss, dn):
    """A window miss in an iteration enqueued without reading its verdict
    stalls the device loop; the host replays it at the batch check (its radix
    passes with their histogram all-reduces, then the rest).  Forced misses
    mid-batch must leave every result bit-identical to the run without them
    (which itself equals the oracle, test_sharded_icp_vs_oracle)."""
    f, r = two_ranks_forced_miss, two_ranks
    np.testing.assert_array_equal(f[0][f"{dn}_loop"], f[1][f"{dn}_loop"])
    np.testing.assert_array_equal(f[0][f"{dn}_loop"][:18], r[0][f"{dn}_loop"][:18])  # T_iter, iterations, kept
    syncs, blind, stalls = (int(v) for v in f[0][f"{dn}_sync"])
    print(f"{dn}: forced misses -> {stalls} stalls, {syncs} verdict syncs, {blind} blind iterations")
    assert stalls >= 1
    for tag in ("trim", "med"):
        np.testing.assert_array_equal(f[0][f"{dn}_icp_{tag}"], r[0][f"{dn}_icp_{tag}"])
        np.testing.assert_array_equal(f[1][f"{dn}_icp_{tag}"], r[1][f"{dn}_icp_{tag}"])


# ---- the BASELINE C3 size, sharded (1M -> 1M float, two ranks of 500 K) ----
def _worker_c3(rank, world, port, outdir):
    import torch  # noqa: F401
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from libpointmatcher_amd import _capi
        from libpointmatcher_amd.icp import ICP
        from libpointmatcher_amd.synth import reading_cloud, reference_cloud

        comm = _capi.gloo_host_comm()
        ref, nrm = reference_cloud(1_000_000, np.float32)
        rd = reading_cloud(1_000_000, np.float32)
        lo, hi = shard_range(rd.shape[0], world, rank)
        icp = ICP(np.float32)
        icp.comm_init_host(comm)
        icp.load_yaml(chain_yaml(maxit=40))
        T = icp.compute(np.ascontiguousarray(rd[lo:hi]), ref, nrm)
        s = icp.stats()
        icp.close()
        assert not comm.errors, comm.errors
        np.savez(os.path.join(outdir, f"c3_rank{rank}.npz"), T=T.astype(np.float64), it=s.iterations, kept=s.kept)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(900)
def test_sharded_c3_size_vs_oracle(tmp_path, oracle):
    """The BASELINE C3 workload (1M -> 1M float, TrimmedDist 0.85,
    point-to-plane, Counter 40) through the host chain on two ranks of 500 K
    reading points each: every rank's final T within 1e-5 of the
    single-process oracle on the whole reading, the same iteration count and
    kept pairs (the kept count is global: every rank reads the all-reduced
    system)."""
    from libpointmatcher_amd.synth import reading_cloud, reference_cloud

    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker_c3, args=(i, 2, port, str(tmp_path))) for i in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(600)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.exitcode is None:
            p.kill()
    assert codes == [0, 0], codes
    r = [dict(np.load(tmp_path / f"c3_rank{i}.npz")) for i in range(2)]
    np.testing.assert_array_equal(r[0]["T"], r[1]["T"])
    ref, nrm = reference_cloud(1_000_000, np.float32)
    rd = reading_cloud(1_000_000, np.float32)
    cfg = oracle.make_cfg(counter_max=40, threads=8)
    rc, To, so, _ = oracle.icp(cfg, rd, ref, normals=nrm)
    assert rc == 0
    assert np.linalg.norm(r[0]["T"] - To) <= TOL["float32"]
    assert int(r[0]["it"]) == 40
    assert int(r[0]["kept"]) == 850001


# ---- the BASELINE multi-GPU configurations at their own sizes, sharded ----
# (the north_star's 8-GPU configs C4 and C5 on two ranks of one MI355X over
# the host-staged transport; the same library path as RCCL)
BIG_CASES = {
    # tag: (reading N, reference M, dtype, knn, filters, minimizer, Counter max, Differential, traced)
    "c4": (1_000_000, 1_000_000, "float32", 4, (("MaxDistOutlierFilter", {"maxDist": 0.05}),), P2PLANE, 20, DIFF,
           False),
    "c5": (10_000_000, 1_000_000, "float64", 1, (), P2POINT, 5, None, False),
    "c5x40": (2_000_000, 1_000_000, "float64", 1, (), P2POINT, 40, None, True),
}


def _worker_big(rank, world, port, outdir, tag):
    import torch  # noqa: F401
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from libpointmatcher_amd import _capi
        from libpointmatcher_amd.icp import ICP
        from libpointmatcher_amd.synth import reading_cloud, reference_cloud

        n, m, dn, knn, filters, minimizer, maxit, diff, traced = BIG_CASES[tag]
        dtype = np.dtype(dn)
        comm = _capi.gloo_host_comm()
        ref, nrm = reference_cloud(m, dtype)
        rd = reading_cloud(n, dtype)
        lo, hi = shard_range(n, world, rank)
        shard = np.ascontiguousarray(rd[lo:hi])
        del rd
        icp = ICP(dtype)
        icp.comm_init_host(comm)
        if traced:
            icp.keep_trace(True)
        icp.load_yaml(chain_yaml(knn=knn, filters=filters, minimizer=minimizer, maxit=maxit, differential=diff))
        T = icp.compute(shard, ref, nrm if minimizer == P2PLANE else None)
        s = icp.stats()
        tr = np.asarray(icp.trace(), np.float64) if traced else np.zeros((0, 4, 4))
        icp.close()
        assert not comm.errors, comm.errors
        np.savez(os.path.join(outdir, f"{tag}_rank{rank}.npz"), T=T.astype(np.float64), it=s.iterations, kept=s.kept,
                 trace=tr)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(1200)
@pytest.mark.parametrize("tag", ["c4", "c5", "c5x40"])
def test_sharded_baseline_configs_vs_oracle(tmp_path, oracle, tag):
    """BASELINE C4 (1M -> 1M float, k = 4, MaxDist 0.05, point-to-plane,
    Counter 20 + Differential) and C5 (10M -> 1M double, empty chain,
    point-to-point, 5 iterations; and its chain for 40 traced iterations on
    2M -> 1M) through the host chain on two ranks, each with half of the
    reading: every rank the same T, within 1e-5 (float) / 1e-12 (double) of
    the single-process oracle on the whole reading (every T_iter of the
    trace for c5x40), with equal iteration counts and kept pairs.
    Reference: MatchersImpl.cpp:85-101, ErrorMinimizers/PointToPoint.cpp:61-101,
    PointToPlane.cpp:171-243, ICP.cpp:317-449."""
    from libpointmatcher_amd.synth import reading_cloud, reference_cloud
    from test_gpu_configs import THREADS

    n, m, dn, knn, filters, minimizer, maxit, diff, traced = BIG_CASES[tag]
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker_big, args=(i, 2, port, str(tmp_path), tag)) for i in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(900)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.exitcode is None:
            p.kill()
    assert codes == [0, 0], codes
    r = [dict(np.load(tmp_path / f"{tag}_rank{i}.npz")) for i in range(2)]
    np.testing.assert_array_equal(r[0]["T"], r[1]["T"])
    np.testing.assert_array_equal(r[0]["trace"], r[1]["trace"])
    dtype = np.dtype(dn)
    ref, nrm = reference_cloud(m, dtype)
    rd = reading_cloud(n, dtype)
    cfg = oracle.make_cfg(knn=knn, filters=filters, minimizer=minimizer, counter_max=maxit, differential=diff,
                          threads=THREADS)
    rc, To, so, to = oracle.icp(cfg, rd, ref, normals=nrm if minimizer == P2PLANE else None, trace=traced)
    assert rc == 0
    frob = np.linalg.norm(r[0]["T"] - To.astype(np.float64))
    print(f"{tag} sharded x2: iterations {int(r[0]['it'])}/{so.iterations} kept {int(r[0]['kept'])}/{so.kept} "
          f"|dT|_F = {frob:.3g}")
    assert int(r[0]["it"]) == so.iterations
    assert int(r[0]["kept"]) == so.kept
    assert frob <= TOL[dn]
    if traced:
        assert len(r[0]["trace"]) == so.iterations == maxit
        worst = max(np.linalg.norm(a - np.asarray(b, np.float64)) for a, b in zip(r[0]["trace"], to))
        print(f"{tag}: worst iteration |dT|_F = {worst:.3g}")
        assert worst <= TOL[dn]
