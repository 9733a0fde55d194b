"""World-size-2 (gloo, CPU) tests of the multi-GPU protocol.

The multi-GPU path (pmx_capi.hip) shards the reading over the
ranks, replicates the reference, and per ICP iteration
  1. all-reduces each 2048-bin radix-select histogram between the `hist` and
     `pick` kernels (pmx_select.hip), so the TrimmedDist quantile
     (Matches.cpp:60-87) is the exact order statistic of the GLOBAL match set;
  2. all-reduces the packed fp64 normal equations (PointToPlane.cpp:171-243),
     then every rank runs the same host solve.
These tests run that protocol with gloo collectives in two processes, on the
oracle's per-shard arithmetic, and check it against the single-process oracle:
the quantile bit-exactly, the system to fp64 reassociation, and the whole ICP
to the north-star tolerance.  The device side of the same protocol is covered
on one GPU by tests/test_gpu_*.py (the histogram and system all-reduce are the
only cross-rank steps).
"""
import os
import socket
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(__file__))
import oracle_py as O  # noqa: E402
from helpers import hom, pca_normals  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def shard_range(n, world, rank):
    """Contiguous reading shard of rank (bench.py / pmx_set_reading convention)."""
    base, rem = divmod(n, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


# ---------------------------------------------------------------------------
# numpy restatement of the device select protocol (pmx_select.hip digit_of,
# select_hist_kernel, select_pick_kernel), with the histogram all-reduce
# ---------------------------------------------------------------------------
def _digits(bits):
    return [(21, 11), (10, 11), (0, 10)] if bits == 32 else \
        [(53, 11), (42, 11), (31, 11), (20, 11), (10, 10), (0, 10)]


def sharded_select(d_local, ratio, allreduce):
    dt = d_local.dtype
    bits = 32 if dt == np.float32 else 64
    ut = np.uint32 if bits == 32 else np.uint64
    inf_key = ut(0x7F800000) if bits == 32 else ut(0x7FF0000000000000)
    keys = np.ascontiguousarray(d_local).ravel().view(ut)
    keys = keys[keys < inf_key]
    prefix = 0
    rank = 0
    for p, (shift, nb_bits) in enumerate(_digits(bits)):
        nb = 1 << nb_bits
        sel = keys if p == 0 else keys[(keys >> ut(shift + nb_bits)) == ut(prefix)]
        hist = np.bincount(((sel >> ut(shift)) & ut(nb - 1)).astype(np.int64), minlength=nb).astype(np.int64)
        hist = allreduce(hist)
        if p == 0:
            count = int(hist.sum())
            if count == 0:
                return None
            q = dt.type(ratio)
            if q == 1:
                rank = count - 1
            else:
                rank = min(int(dt.type(count) * q), count - 1)
        cum = np.cumsum(hist)
        digit = int(np.searchsorted(cum, rank, side="right"))
        rank -= int(cum[digit - 1]) if digit > 0 else 0
        prefix = (prefix << nb_bits) | digit
    return np.array([prefix], dtype=ut).view(dt)[0]


def _gloo_allreduce(a):
    import torch
    import torch.distributed as dist

    t = torch.from_numpy(np.ascontiguousarray(a))
    dist.all_reduce(t)
    return t.numpy()


def _single_allreduce(a):
    return a


# ---------------------------------------------------------------------------
# sharded ICP: the oracle's per-shard kernels + the two all-reduces
# ---------------------------------------------------------------------------
def sharded_icp(reading, ref, normals, ratio, iters, world, rank, allreduce):
    dt = ref.dtype
    rows = ref.shape[1]
    D = rows - 1
    lo, hi = shard_range(reading.shape[0], world, rank)
    shard = np.ascontiguousarray(reading[lo:hi])
    # reference centring (ICP.cpp:291-299): sequential sum in T as the oracle
    mean = np.zeros(D, dt)
    for r in range(D):
        s = dt.type(0)
        for v in ref[:, r]:
            s = dt.type(s + v)
        mean[r] = dt.type(s / dt.type(ref.shape[0]))
    refc = ref.copy()
    refc[:, :D] -= mean
    T_ref = np.eye(rows, dtype=dt)
    T_ref[:D, D] = mean
    T_md = np.eye(rows, dtype=dt)
    T_md[:D, D] = -mean
    rd0 = O.transform(T_md, shard)
    T_iter = np.eye(rows, dtype=dt)
    for _ in range(iters):
        step = O.transform(T_iter, rd0)
        d, ids, _ = O.knn(refc, step, k=1, method="brute")
        limit = sharded_select(d, ratio, allreduce)
        w = ((d <= limit) & np.isfinite(d)).astype(dt)
        _, A, b, _ = O.p2plane_system(step, refc, normals, d, ids, w)
        packed = allreduce(np.concatenate([A.ravel(), b]))
        n = A.shape[0]
        rc, dT = O.p2plane_solve(packed[: n * n].reshape(n, n), packed[n * n:], rows, dt)
        assert rc == 0
        T_iter = (dT.astype(np.float64) @ T_iter.astype(np.float64)).astype(dt)
    return (T_ref.astype(np.float64) @ T_iter.astype(np.float64) @ T_md.astype(np.float64)).astype(dt)


def _problem(dtype, n=3000, seed=7):
    rng = np.random.default_rng(seed)
    # a curved open surface (well-conditioned for point-to-plane)
    u = rng.uniform(-1, 1, (n, 2))
    ref3 = np.column_stack([u[:, 0], u[:, 1], 0.3 * np.sin(2 * u[:, 0]) + 0.2 * u[:, 1] ** 2])
    ref = hom(ref3, dtype)
    nrm = pca_normals(ref3).astype(dtype)
    th = 0.05
    R = np.array([[np.cos(th), -np.sin(th), 0], [np.sin(th), np.cos(th), 0], [0, 0, 1]])
    rd3 = (ref3[rng.permutation(n)[: n * 2 // 3]] - 0.02) @ R.T + rng.normal(0, 0.003, (n * 2 // 3, 3))
    return hom(rd3, dtype), ref, nrm


def _worker(rank, world, port, outdir, dtype_name):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dtype = np.dtype(dtype_name)
        rng = np.random.default_rng(11)
        res = {}
        # 1. sharded quantiles over distributions with ties, inf and a tail
        base = rng.exponential(1.0, 20001).astype(dtype)
        base[rng.integers(0, base.size, 500)] = np.inf
        base[:3000] = base[3000:6000]  # exact ties
        for j, ratio in enumerate([0.0, 0.1, 0.5, 0.85, 0.999, 1.0]):
            lo, hi = shard_range(base.size, world, rank)
            res[f"q{j}"] = np.array([sharded_select(base[lo:hi], ratio, _gloo_allreduce)])
        # 2. sharded normal equations
        reading, ref, nrm = _problem(dtype)
        lo, hi = shard_range(reading.shape[0], world, rank)
        d, ids, _ = O.knn(ref, reading[lo:hi], k=1, method="brute")
        w = np.ones_like(d)
        _, A, b, _ = O.p2plane_system(reading[lo:hi], ref, nrm, d, ids, w)
        res["Ab"] = _gloo_allreduce(np.concatenate([A.ravel(), b]))
        # 3. the sharded ICP loop
        res["T"] = sharded_icp(reading, ref, nrm, 0.85, 6, world, rank, _gloo_allreduce)
        np.savez(os.path.join(outdir, f"rank{rank}.npz"), **res)
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module", params=["float32", "float64"])
def two_rank_results(request, tmp_path_factory):
    # plain multiprocessing: the parent never imports torch, so torch's bundled
    # HIP runtime is not loaded next to the /opt/rocm one libpmx links
    import multiprocessing as mp

    O.build()
    out = tmp_path_factory.mktemp("mr_" + request.param)
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(i, 2, port, str(out), request.param)) for i in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    r = [dict(np.load(out / f"rank{i}.npz")) for i in range(2)]
    return np.dtype(request.param), r


def test_shard_ranges_cover():
    for n in [0, 1, 5, 1000, 1001]:
        for world in [1, 2, 3, 8]:
            rs = [shard_range(n, world, r) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_single_process_select_equals_oracle(dtype):
    rng = np.random.default_rng(3)
    for _ in range(5):
        d = rng.lognormal(0, 2, rng.integers(1, 4000)).astype(dtype)
        d[rng.random(d.size) < 0.05] = np.inf
        if not np.isfinite(d).any():
            continue
        for ratio in [0.0, 0.3, 0.85, 1.0]:
            rc, q = O.quantile(d, ratio)
            assert rc == 0
            assert sharded_select(d, ratio, _single_allreduce) == q


def test_two_rank_quantile_bit_exact(two_rank_results):
    dtype, r = two_rank_results
    rng = np.random.default_rng(11)
    base = rng.exponential(1.0, 20001).astype(dtype)
    base[rng.integers(0, base.size, 500)] = np.inf
    base[:3000] = base[3000:6000]
    for j, ratio in enumerate([0.0, 0.1, 0.5, 0.85, 0.999, 1.0]):
        rc, q = O.quantile(base, ratio)
        assert rc == 0
        assert r[0][f"q{j}"][0] == q and r[1][f"q{j}"][0] == q, (ratio, r[0][f"q{j}"], q)


def test_two_rank_system_allreduce(two_rank_results):
    dtype, r = two_rank_results
    reading, ref, nrm = _problem(dtype)
    d, ids, _ = O.knn(ref, reading, k=1, method="brute")
    _, A, b, _ = O.p2plane_system(reading, ref, nrm, d, ids, np.ones_like(d))
    full = np.concatenate([A.ravel(), b])
    np.testing.assert_array_equal(r[0]["Ab"], r[1]["Ab"])  # every rank solves the same system
    np.testing.assert_allclose(r[0]["Ab"], full, rtol=1e-12, atol=1e-12 * np.abs(full).max())


def test_two_rank_icp_matches_single_process(two_rank_results):
    dtype, r = two_rank_results
    reading, ref, nrm = _problem(dtype)
    tol = 1e-5 if dtype == np.float32 else 1e-12
    np.testing.assert_array_equal(r[0]["T"], r[1]["T"])
    T1 = sharded_icp(reading, ref, nrm, 0.85, 6, 1, 0, _single_allreduce)
    cfg = O.make_cfg(knn=1, method="brute", counter_max=6, filters=(("TrimmedDistOutlierFilter", {"ratio": 0.85}),))
    rc, To, _, _ = O.icp(cfg, reading, ref, normals=nrm)
    assert rc == 0
    assert np.linalg.norm(T1.astype(np.float64) - To) <= tol  # the protocol model is the oracle at N=1
    assert np.linalg.norm(r[0]["T"].astype(np.float64) - To) <= tol


def test_set_default_sharded_raises():
    """setDefault() (ICP.cpp:99-113) puts RandomSampling on the reading and
    SamplingSurfaceNormal (samplingMethod 0) on the reference: both draw from
    the process's rand() state, so a sharded ICP refuses the chain with
    ConfigurationError before any device work.
    Runs without a GPU: the check precedes the device context."""
    from libpointmatcher_amd import _capi
    from libpointmatcher_amd.icp import ICP, ConfigurationError
    comm = _capi.HostComm(2, 0, lambda a, op: None, lambda a: np.concatenate([a, a]))
    icp = ICP(np.float32)
    icp.set_default()
    icp.comm_init_host(comm)
    pts = hom(np.random.default_rng(0).normal(size=(64, 3)).astype(np.float32))
    with pytest.raises(ConfigurationError, match="rand"):
        icp.compute(pts, pts)
    icp.close()
