"""k-NN for k > 16 (KDTreeMatcher knn: any k >= 1; pmx_knn_wide.hip): the
wave-per-query search over the grid and over the whole reference (brute
force) against the oracle's kd-tree, bit for bit (distances and ids, ties by
original index), on the geometries of test_gpu_grid.py: surface density,
queries outside the reference box, 2-D data, duplicated and non-finite
points, a search radius, fewer reference points than k.  Then whole ICPs with
knn = 32 through the device loop and the host chain against the oracle ICP
(MatchersImpl.cpp:85-101, ICP.cpp:317-449).
"""
import numpy as np
import pytest

from libpointmatcher_amd import _capi as P
from libpointmatcher_amd.synth import random_cloud, reading_cloud, reference_cloud

pytestmark = pytest.mark.gpu


def match(ref, rd, T, k, search, max_dist=np.inf, dtype=np.float32):
    ctx = P.Context(0, dtype)
    ctx.set_search(search)
    ctx.set_reference(ref)
    ctx.set_reading(rd)
    ctx.match(T, knn=k, max_dist=max_dist)
    d, i = ctx.get_matches()
    ctx.close()
    return d, i


def check(oracle, ref, rd, T, k, max_dist=np.inf, dtype=np.float32):
    o = oracle.knn(ref, oracle.transform(T, rd), k=k, max_dist=max_dist, method="kdtree")[:2]
    for search in (1, 0):  # grid, brute force
        g = match(ref, rd, T, k, search, max_dist, dtype)
        np.testing.assert_array_equal(g[1], o[1], err_msg=f"ids, search {search}, k {k}")
        np.testing.assert_array_equal(g[0], o[0], err_msg=f"dists, search {search}, k {k}")


@pytest.mark.parametrize("k", [17, 32, 64, 100, 256, 512, 1024, 1500])
def test_surface_density(oracle, k):
    ref, _ = reference_cloud(40_000)
    rd = reading_cloud(3_000)
    check(oracle, ref, rd, np.eye(4, dtype=np.float32), k)


@pytest.mark.parametrize("k", [20, 64, 129])
def test_double_and_radius(oracle, k):
    ref = random_cloud(20_000, seed=7, dtype=np.float64)
    rd = random_cloud(2_000, seed=8, dtype=np.float64, scale=1.2)
    check(oracle, ref, rd, np.eye(4), k, dtype=np.float64)
    check(oracle, ref, rd, np.eye(4), k, max_dist=0.1, dtype=np.float64)


def test_outside_bbox_2d_ties_nonfinite(oracle):
    ref = random_cloud(10_000, seed=1)
    rd = random_cloud(1_500, seed=2, scale=4.0)
    check(oracle, ref, rd, np.eye(4, dtype=np.float32), 40)
    ref2 = random_cloud(8_000, rows=3, seed=4)
    rd2 = random_cloud(1_500, rows=3, seed=5, scale=1.5)
    check(oracle, ref2, rd2, np.eye(3, dtype=np.float32), 33)
    base = random_cloud(3_000, seed=6)
    ref3 = np.concatenate([base, base, base[:500]])
    ref3[17, 0] = np.inf
    ref3[99, 1] = np.nan
    check(oracle, ref3, base[::3].copy(), np.eye(4, dtype=np.float32), 48)


def test_fewer_points_than_k(oracle):
    for M in (1, 7, 40):
        ref = random_cloud(M, seed=9)
        rd = random_cloud(300, seed=10, scale=3.0)
        check(oracle, ref, rd, np.eye(4, dtype=np.float32), 64)
    # chunked lists (k > 1024): the reference runs out inside the first and the second chunk
    for M in (700, 1800):
        ref = random_cloud(M, seed=11)
        rd = random_cloud(200, seed=12, scale=2.0)
        check(oracle, ref, rd, np.eye(4, dtype=np.float32), 2100)
    # ... and with a radius that ends the list early
    ref = random_cloud(5_000, seed=13, dtype=np.float64)
    rd = random_cloud(300, seed=14, dtype=np.float64)
    check(oracle, ref, rd, np.eye(4), 1300, max_dist=0.3, dtype=np.float64)


def test_transformed_reading(oracle):
    ref, _ = reference_cloud(60_000)
    rd = reading_cloud(4_000)
    th = 0.5
    T = np.eye(4, dtype=np.float32)
    T[:3, :3] = [[np.cos(th), 0, np.sin(th)], [0, 1, 0], [-np.sin(th), 0, np.cos(th)]]
    T[:3, 3] = [0.3, -0.2, 0.1]
    check(oracle, ref, rd, T, 24)


def test_knn_bounds():
    ctx = P.Context(0, np.float32)
    ctx.set_reference(random_cloud(100, seed=1))
    ctx.set_reading(random_cloud(10, seed=2))
    with pytest.raises(P.InvalidParameter):
        ctx.match(np.eye(4, dtype=np.float32), knn=0)
    ctx.close()


@pytest.mark.parametrize("dn,knn", [("float32", 32), ("float64", 32), ("float32", 512)])
def test_icp_knn32_vs_oracle(oracle, dn, knn):
    """Whole ICP with knn = 32 and 512 (TrimmedDist over the N x k distances,
    point-to-plane over every kept pair): the host chain (device loop) against
    the oracle ICP, equal iterations, T within 1e-5 (f32) / 1e-12 (f64).
    (knn = 512 on smaller clouds: the oracle's kd-tree inserts into a
    512-entry list.)"""
    from helpers import chain_yaml
    from libpointmatcher_amd.icp import ICP

    dtype = np.dtype(dn)
    ref, nrm = reference_cloud(30_000 if knn <= 64 else 12_000, dtype)
    rd = reading_cloud(6_000 if knn <= 64 else 1_200, dtype)
    diff = dict(minDiffRotErr=0.001, minDiffTransErr=0.01, smoothLength=4)
    icp = ICP(dtype)
    icp.load_yaml(chain_yaml(knn=knn, filters=(("TrimmedDistOutlierFilter", {"ratio": 0.8}),), maxit=20,
                             differential=diff))
    T = icp.compute(rd, ref, nrm)
    s = icp.stats()
    icp.close()
    cfg = oracle.make_cfg(knn=knn, filters=(("TrimmedDistOutlierFilter", {"ratio": 0.8}),), counter_max=20,
                          differential=diff, threads=8)
    rc, To, so, _ = oracle.icp(cfg, rd, ref, normals=nrm)
    assert rc == 0
    frob = np.linalg.norm(T.astype(np.float64) - To.astype(np.float64))
    print(f"{dn}: iterations {s.iterations}/{so.iterations} kept {s.kept}/{so.kept} |dT|={frob:.3g}")
    assert s.iterations == so.iterations
    assert s.kept == so.kept
    assert frob <= (1e-5 if dn == "float32" else 1e-12)
