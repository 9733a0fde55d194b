"""KDTreeVarDistMatcher (MatchersImpl.cpp:106-150): a search radius per
reading point, libnabo's knn with maxRadii.  The k nearest within a radius are
the prefix of the k nearest, so the oracle is its exact k-NN (maxDist inf)
with the entries beyond each query's radius (squared in T, as libnabo does)
set to (inf, -1).  Bar: ids identical, distances bitwise identical, for the
brute force and the grid search, full and temporal-reuse matches, f32/f64.
Through the ICP: the matcher loads from YAML with the reading's
"maxSearchDist" descriptor; with all radii equal to a KDTreeMatcher's maxDist
the two chains give the same transform bit for bit, and the device loop
equals the per-module calls.
"""
import numpy as np
import pytest

from libpointmatcher_amd import _capi as P
from libpointmatcher_amd.icp import ICP
from libpointmatcher_amd.synth import random_cloud, reading_cloud, reference_cloud

pytestmark = pytest.mark.gpu


def _T(ang, tr, dtype):
    c, s = np.cos(ang), np.sin(ang)
    T = np.eye(4)
    T[:2, :2] = [[c, -s], [s, c]]
    T[:3, 3] = [tr, -tr / 2, tr / 3]
    return T.astype(dtype)


def _oracle_masked(oracle, ref, step, k, radii):
    od, oi, _ = oracle.knn(ref, step, k=k, method="brute")
    r2 = (radii * radii).astype(radii.dtype)  # (squared in T)
    cut = ~(od <= r2[:, None])
    od = od.copy()
    oi = oi.copy()
    od[cut] = np.inf
    oi[cut] = -1
    return od, oi


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("search", [0, 1])
@pytest.mark.parametrize("k", [1, 3])
def test_vardist_match_vs_oracle(oracle, dtype, search, k):
    ref = random_cloud(20000, seed=31, dtype=dtype)
    rd = random_cloud(12000, seed=32, dtype=dtype, scale=1.2)
    rng = np.random.default_rng(33)
    radii = rng.uniform(0.0, 0.08, rd.shape[0]).astype(dtype)
    radii[::97] = np.inf  # (unbounded points)
    ctx = P.Context(0, dtype)
    ctx.set_search(search)
    ctx.set_reference(ref)
    ctx.set_reading(rd)
    ctx.set_reading_radii(radii)
    for it in range(4):  # the first match is full, the next may certify from the previous one
        T = _T(0.01 / (it + 1), 0.01 / (it + 1), dtype)
        ctx.match(T, knn=k, max_dist=0.5)  # (maxDist is ignored while radii are set)
        d, i = ctx.get_matches()
        od, oi = _oracle_masked(oracle, ref, oracle.transform(T, rd), k, radii)
        assert np.array_equal(i, oi)
        assert np.array_equal(d.view(np.uint32 if dtype == np.float32 else np.uint64),
                              od.view(np.uint32 if dtype == np.float32 else np.uint64))
        assert (i == -1).any() and (i >= 0).any()
    # cleared: the matcher's maxDist again
    ctx.set_reading_radii(None)
    ctx.match(np.eye(4, dtype=dtype), knn=k, max_dist=0.03)
    d, i = ctx.get_matches()
    od, oi, _ = oracle.knn(ref, rd, k=k, max_dist=0.03, method="brute")
    assert np.array_equal(i, oi) and np.array_equal(d, od)
    ctx.close()


def _yaml(matcher):
    return (f"matcher:\n  {matcher}\n"
            "outlierFilters:\n  - TrimmedDistOutlierFilter:\n      ratio: 0.8\n"
            "errorMinimizer:\n  PointToPlaneErrorMinimizer\n"
            "transformationCheckers:\n  - CounterTransformationChecker:\n      maxIterationCount: 25\n"
            "inspector:\n  NullInspector\nlogger:\n  NullLogger\n")


def test_vardist_icp_equals_kdtree_with_uniform_radii(monkeypatch):
    ref, nrm = reference_cloud(40000, np.float32)
    rd = reading_cloud(30000, np.float32)
    out = {}
    for loop in ("1", "0"):
        monkeypatch.setenv("PMX_DEVICE_LOOP", loop)
        a = ICP(np.float32)
        a.load_yaml(_yaml("KDTreeMatcher:\n    knn: 2\n    maxDist: 0.2"))
        Ta = a.compute(rd, ref, nrm)
        b = ICP(np.float32)
        b.load_yaml(_yaml("KDTreeVarDistMatcher:\n    knn: 2\n    maxDistField: maxSearchDist"))
        b.add_descriptor("reading", "maxSearchDist", np.full(rd.shape[0], 0.2, np.float32))
        Tb = b.compute(rd, ref, nrm)
        assert a.stats().iterations == b.stats().iterations
        assert np.array_equal(Ta, Tb)
        # per-point radii: the device loop and the per-module calls agree
        c = ICP(np.float32)
        c.load_yaml(_yaml("KDTreeVarDistMatcher:\n    knn: 2"))
        c.add_descriptor("reading", "maxSearchDist",
                         np.random.default_rng(5).uniform(0.02, 0.3, rd.shape[0]).astype(np.float32))
        out[loop] = (c.compute(rd, ref, nrm), c.stats().iterations, c.stats().kept)
    assert out["1"][1:] == out["0"][1:]
    assert np.array_equal(out["1"][0], out["0"][0])


def test_vardist_missing_descriptor_raises():
    ref, nrm = reference_cloud(5000, np.float32)
    rd = reading_cloud(4000, np.float32)
    c = ICP(np.float32)
    c.load_yaml(_yaml("KDTreeVarDistMatcher:\n    knn: 1\n    maxDistField: radius"))
    with pytest.raises(Exception, match="radius"):
        c.compute(rd, ref, nrm)
