"""Exact grid search (searchType 1/2) == brute force (searchType 0) == oracle,
bit for bit, on the geometries where a shell search can go wrong: queries
outside the reference bounding box, planar / 2-D data (degenerate z extent),
duplicated points (ties), non-finite reference points, a radius, large k,
and surface data at the benchmark density.
"""
import numpy as np
import pytest

from libpointmatcher_amd import _capi as P
from libpointmatcher_amd.synth import random_cloud, reading_cloud, reference_cloud

pytestmark = pytest.mark.gpu

# every test runs against each grid search form: the per-lane kernel (default),
# coarse / fine levels, no temporal reuse, and the wave-cooperative tile kernel
# (with a box budget that sends most lanes to the per-lane fallback); the
# forms are context options (PMX_OPTS, README "Options")
MODES = {"lane": "", "lane_coarse": "grid_levels=32", "lane_noreuse": "grid_reuse=0", "lane_fine": "grid_levels=1",
         "tile": "grid_mode=tile", "tile_fallback": "grid_mode=tile,tile_max=16"}


@pytest.fixture(autouse=True, params=sorted(MODES))
def grid_mode(request, monkeypatch):
    monkeypatch.setenv("PMX_OPTS", MODES[request.param])
    return request.param


def match(ref, rd, T, k, search, max_dist=np.inf, dtype=np.float32):
    ctx = P.Context(0, dtype)
    ctx.set_search(search)
    ctx.set_reference(ref)
    ctx.set_reading(rd)
    ctx.match(T, knn=k, max_dist=max_dist)
    d, i = ctx.get_matches()
    ctx.close()
    return d, i


def same(a, b):
    return np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def check(oracle, ref, rd, T, k, max_dist=np.inf, dtype=np.float32):
    g = match(ref, rd, T, k, 1, max_dist, dtype)
    b = match(ref, rd, T, k, 0, max_dist, dtype)
    o = oracle.knn(ref, oracle.transform(T, rd), k=k, max_dist=max_dist, method="kdtree")[:2]
    assert same(g, b), "grid != brute"
    assert same(g, o), "grid != oracle"


@pytest.mark.parametrize("k", [1, 3, 9])
def test_surface_density(oracle, k):
    ref, _ = reference_cloud(200_000)
    rd = reading_cloud(50_000)
    check(oracle, ref, rd, np.eye(4, dtype=np.float32), k)


def test_queries_outside_bbox(oracle):
    ref = random_cloud(20_000, seed=1)
    rd = random_cloud(5_000, seed=2, scale=4.0)  # most queries far outside [-1, 1]^3
    for k in (1, 4):
        check(oracle, ref, rd, np.eye(4, dtype=np.float32), k)


def test_planar_and_2d(oracle):
    rng = np.random.default_rng(3)
    ref = np.hstack([rng.uniform(-5, 5, (30_000, 2)), np.zeros((30_000, 1)), np.ones((30_000, 1))]).astype(np.float32)
    rd = np.hstack([rng.uniform(-6, 6, (8_000, 2)), rng.normal(0, 0.5, (8_000, 1)), np.ones((8_000, 1))]).astype(np.float32)
    check(oracle, ref, rd, np.eye(4, dtype=np.float32), 1)
    check(oracle, ref, rd, np.eye(4, dtype=np.float32), 5)
    ref2 = random_cloud(20_000, rows=3, seed=4)
    rd2 = random_cloud(5_000, rows=3, seed=5, scale=1.5)
    check(oracle, ref2, rd2, np.eye(3, dtype=np.float32), 2)


def test_ties_duplicates_and_nonfinite(oracle):
    base = random_cloud(5_000, seed=6)
    ref = np.concatenate([base, base, base[:1000]])
    ref[17, 0] = np.inf
    ref[99, 1] = np.nan
    rd = base[::2].copy()
    for k in (1, 3):
        check(oracle, ref, rd, np.eye(4, dtype=np.float32), k)


def test_radius_and_double(oracle):
    ref = random_cloud(30_000, seed=7, dtype=np.float64)
    rd = random_cloud(10_000, seed=8, dtype=np.float64, scale=1.2)
    check(oracle, ref, rd, np.eye(4), 1, max_dist=0.02, dtype=np.float64)
    check(oracle, ref, rd, np.eye(4), 4, max_dist=0.05, dtype=np.float64)


def test_transformed_reading(oracle):
    # the slot order is chosen from the initial pose; a large step transform
    # scrambles the locality of each wave's queries (bigger LDS boxes, more
    # fallbacks) but never the result
    ref, _ = reference_cloud(100_000)
    rd = reading_cloud(40_000)
    th = 0.7
    T = np.eye(4, dtype=np.float32)
    T[:3, :3] = [[np.cos(th), 0, np.sin(th)], [0, 1, 0], [-np.sin(th), 0, np.cos(th)]]
    T[:3, 3] = [0.3, -0.2, 0.1]
    for k in (1, 4):
        check(oracle, ref, rd, T, k)


def test_tiny_reference(oracle):
    for M in (1, 2, 7):
        ref = random_cloud(M, seed=9)
        rd = random_cloud(300, seed=10, scale=3.0)
        check(oracle, ref, rd, np.eye(4, dtype=np.float32), min(2, M))


def test_adaptive_levels_stay_exact(oracle, grid_mode):
    # misaligned steps push the matcher to coarser grid levels, aligned ones
    # back to the finest: every match in between must equal the oracle's
    if grid_mode != "lane":
        pytest.skip("level adaptation is exercised once, with the default kernel")
    from libpointmatcher_amd.synth import t_gt

    ref, nrm = reference_cloud(100_000)
    rd = reading_cloud(30_000)
    ctx = P.Context(0, np.float32)
    ctx.set_search(1)
    ctx.set_reference(ref, nrm)
    ctx.set_reading(rd)
    th = 0.5
    Tbad = np.eye(4, dtype=np.float32)
    Tbad[:3, :3] = [[np.cos(th), -np.sin(th), 0], [np.sin(th), np.cos(th), 0], [0, 0, 1]]
    Tgood = t_gt().astype(np.float32)
    seen = []
    for T in [Tbad, Tbad, Tbad, Tgood, Tgood, Tgood, Tbad, Tgood]:
        ctx.match(T, knn=2)
        ctx.outlier("TrimmedDistOutlierFilter", 0, ratio=0.85)
        _, _, st = ctx.p2plane_system()
        seen.append(st.visited)
        d, i = ctx.get_matches()
        od, oi, _ = oracle.knn(ref, oracle.transform(T, rd), k=2, method="kdtree")
        assert np.array_equal(d, od) and np.array_equal(i, oi)
    ctx.close()
    assert len(set(seen)) > 2  # the level (and so the pair count) did change


def test_grid_visits_far_fewer_pairs():
    ref, nrm = reference_cloud(200_000)
    rd = reading_cloud(100_000)
    stats = []
    for search in (0, 1):
        ctx = P.Context(0, np.float32)
        ctx.set_search(search)
        ctx.set_reference(ref, nrm)
        ctx.set_reading(rd)
        ctx.match(np.eye(4, dtype=np.float32), knn=1)
        ctx.outlier("TrimmedDistOutlierFilter", 0, ratio=0.85)
        A, b, st = ctx.p2plane_system()
        stats.append((st.visited, A.copy(), b.copy()))
        ctx.close()
    assert stats[0][0] == 200_000 * 100_000
    assert stats[1][0] < stats[0][0] / 100  # tile kernel: ~750 pairs per query here
    assert np.array_equal(stats[0][1], stats[1][1]) and np.array_equal(stats[0][2], stats[1][2])


@pytest.mark.parametrize("k", [1, 3, 4, 9])
def test_temporal_reuse_stays_exact(oracle, grid_mode, k):
    # consecutive matches of one reading may reuse the previous k-lists when
    # the certificate holds (pmx_grid.hip temporal reuse): small steps (the
    # converging ICP case), a repeated pose, a large jump (nothing certifies),
    # a radius, and a new reading of the same size (stale lists never reused)
    from libpointmatcher_amd.synth import t_gt

    ref, nrm = reference_cloud(100_000)
    rd = reading_cloud(20_000)
    ctx = P.Context(0, np.float32)
    ctx.set_search(1)
    ctx.set_reference(ref, nrm)
    ctx.set_reading(rd)
    Tg = t_gt().astype(np.float32)
    th = 0.4
    Tjump = np.eye(4, dtype=np.float32)
    Tjump[:3, :3] = [[np.cos(th), 0, np.sin(th)], [0, 1, 0], [-np.sin(th), 0, np.cos(th)]]
    steps = [(np.eye(4, dtype=np.float32), np.inf), (Tg, np.inf), (Tg, np.inf), (Tg, np.inf), (Tg, np.inf),
             (Tjump, np.inf), (Tg, 0.05), (Tg, 0.05), (Tg, np.inf)]
    visits = []
    for T, md in steps:
        ctx.match(T, knn=k, max_dist=md)
        d, i = ctx.get_matches()
        od, oi, _ = oracle.knn(ref, oracle.transform(T, rd), k=k, max_dist=md, method="kdtree")
        assert np.array_equal(d, od) and np.array_equal(i, oi)
        ctx.outlier("NullOutlierFilter", 0)
        _, _, st = ctx.p2plane_system()
        visits.append(st.visited)
    rd2 = reading_cloud(20_000)[::-1].copy()  # same size, other order: stale positions
    ctx.set_reading(rd2)
    ctx.match(Tg, knn=k)
    d, i = ctx.get_matches()
    od, oi, _ = oracle.knn(ref, oracle.transform(Tg, rd2), k=k, method="kdtree")
    assert np.array_equal(d, od) and np.array_equal(i, oi)
    ctx.close()
    if grid_mode in ("lane", "lane_coarse", "lane_fine"):
        # the repeated pose was certified from the previous match (k pairs per
        # query) (the adaptive level may move during the first repeats: a
        # level change restarts the reuse chain)
        assert min(visits[2:5]) <= 1.1 * 20_000 * k < visits[0]


@pytest.mark.parametrize("k", [1, 3])
def test_neighbour_records_equal_gathers(oracle, grid_mode, monkeypatch, k):
    # the k = 1 neighbour records (pmx_grid.hip write_nbr: the certificate's
    # neighbour and the point-to-plane reduction's point and normal read in
    # slot order) give the same matches and the same normal equations, bit
    # for bit, as the gathers by id (option nbr_cache=0), through reuse,
    # a jump, a radius and a new reading
    from libpointmatcher_amd.synth import t_gt

    ref, nrm = reference_cloud(100_000)
    rd = reading_cloud(20_000)
    Tg = t_gt().astype(np.float32)
    Tj = Tg.copy()
    Tj[:3, 3] += 0.02
    steps = [(np.eye(4, dtype=np.float32), np.inf), (Tg, np.inf), (Tg, np.inf), (Tj, np.inf), (Tj, 0.05),
             (Tg, np.inf)]
    runs = []
    for on in ("1", "0"):
        monkeypatch.setenv("PMX_OPTS", ",".join(o for o in (MODES[grid_mode], "nbr_cache=" + on) if o))
        ctx = P.Context(0, np.float32)
        ctx.set_search(1)
        ctx.set_reference(ref, nrm)
        out = []
        for r in (rd, reading_cloud(20_000)[::-1].copy()):
            ctx.set_reading(r)
            for T, md in steps:
                ctx.match(T, knn=k, max_dist=md)
                d, i = ctx.get_matches()
                ctx.outlier("TrimmedDistOutlierFilter", 0, ratio=0.85)
                A, b, st = ctx.p2plane_system()
                out.append((d, i, A, b, st.kept))
        ctx.close()
        runs.append(out)
    for (d1, i1, A1, b1, k1), (d0, i0, A0, b0, k0) in zip(*runs):
        assert np.array_equal(d1, d0) and np.array_equal(i1, i0)
        assert np.array_equal(A1, A0) and np.array_equal(b1, b0) and k1 == k0
    od, oi, _ = oracle.knn(ref, oracle.transform(Tg, rd), k=k, method="kdtree")
    assert np.array_equal(runs[0][len(steps) - 1][0], od) and np.array_equal(runs[0][len(steps) - 1][1], oi)


def test_reference_without_normals_after_one_with(oracle, grid_mode):
    # a context that held a reference with normals (kept buffers) then a
    # larger one without: nothing stale is gathered
    ref1, nrm1 = reference_cloud(30_000)
    ref2, _ = reference_cloud(120_000)
    rd = reading_cloud(20_000)
    T = np.eye(4, dtype=np.float32)
    ctx = P.Context(0, np.float32)
    ctx.set_search(1)
    ctx.set_reference(ref1, nrm1)
    ctx.set_reading(rd)
    ctx.match(T, knn=1)
    ctx.set_reference(ref2)
    ctx.set_reading(rd)
    for _ in range(2):
        ctx.match(T, knn=1)
        d, i = ctx.get_matches()
        od, oi, _ = oracle.knn(ref2, oracle.transform(T, rd), k=1, method="kdtree")
        assert np.array_equal(d, od) and np.array_equal(i, oi)
    ctx.close()
