"""SurfaceNormalDataPointsFilter on the GPU (pmx_surface_normals, pmx_normals.hip)
against the CPU oracle (oracle/pmo_impl.inc), and through the ICP chain.

Bar: the self k-NN bit-identical (matched ids), eigenvalues / densities / mean
distances within float rounding of the oracle (same T arithmetic, same
double Jacobi), normals and eigenvectors equal under the shared sign
convention (the reference's EigenSolver sign is implementation-defined [ext];
the point-to-plane minimiser does not depend on it), degenerate points and
smoothNormals as the reference (SurfaceNormal.cpp:208-236, 256-283).  End to
end: the reference's validT3d known answer (utest/utest.cpp:352-356) with the
reference cloud's normals computed by the filter instead of read from the CSV.
"""
import numpy as np
import pytest

from helpers import hom, validate3d
from libpointmatcher_amd import _capi
from libpointmatcher_amd.icp import ICP
from libpointmatcher_amd.synth import reference_cloud

pytestmark = pytest.mark.gpu

TOL = {np.float32: 2e-5, np.float64: 1e-12}


def compare(g, o, dtype):
    tol = TOL[dtype]
    assert g["degenerate"] == o["degenerate"]
    assert np.array_equal(g["matched_ids"], o["matched_ids"])
    scale = np.maximum(np.abs(o["eig_values"]).max(axis=1, keepdims=True), 1e-30)
    assert np.max(np.abs(g["eig_values"] - o["eig_values"]) / scale) <= tol
    np.testing.assert_allclose(g["normals"], o["normals"], rtol=0, atol=50 * tol)
    np.testing.assert_allclose(g["eig_vectors"], o["eig_vectors"], rtol=0, atol=50 * tol)
    np.testing.assert_allclose(g["densities"], o["densities"], rtol=10 * tol)
    np.testing.assert_allclose(g["mean_dists"], o["mean_dists"], rtol=10 * tol)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("k", [3, 5, 10, 16, 32])
def test_surface_normals_equal_oracle(oracle, dtype, k):
    ref, nrm = reference_cloud(30000, dtype)
    g = _capi.surface_normals(ref, knn=k)
    o = oracle.surface_normals(ref, k=k)
    compare(g, o, dtype)
    if k >= 5:  # the box / sphere surface: PCA normals follow the analytic ones away from edges
        assert np.median(np.abs(np.sum(g["normals"] * nrm, axis=1))) > 0.999


def test_surface_normals_radius_2d_degenerate_smooth(oracle):
    ref, _ = reference_cloud(20000, np.float32)
    compare(_capi.surface_normals(ref, knn=8, max_dist=0.05), oracle.surface_normals(ref, k=8, max_dist=0.05),
            np.float32)
    # 2-D clouds (rows = 3): 2x2 covariance, 2-D normals
    rng = np.random.default_rng(7)
    t = rng.uniform(0, 2 * np.pi, 5000)
    ring = hom(np.column_stack([np.cos(t), np.sin(t)]) * (1 + rng.normal(0, 0.01, (5000, 1))), np.float32)
    compare(_capi.surface_normals(ring, knn=6), oracle.surface_normals(ring, k=6), np.float32)
    # collinear points: every covariance fails the rank test
    s = np.linspace(0, 1, 300)
    line = hom(np.column_stack([s, 2 * s, -s]), np.float32)
    g = _capi.surface_normals(line, knn=5)
    assert g["degenerate"] == 300 and np.all(g["normals"] == 0)
    compare(g, oracle.surface_normals(line, k=5), np.float32)
    # smoothNormals (sequential, in place)
    g = _capi.surface_normals(ref, knn=6, smooth=True)
    o = oracle.surface_normals(ref, k=6, smooth=True)
    np.testing.assert_allclose(g["normals"], o["normals"], rtol=0, atol=1e-4)


def test_surface_normals_wide_knn_and_bounds(oracle):
    """knn past the per-lane lists (the wave-per-query self-match): 64 and
    100 neighbours (SurfaceNormal.h:68 bounds knn only from below)."""
    ref, _ = reference_cloud(8000, np.float64)
    for k in (64, 100):
        compare(_capi.surface_normals(ref, knn=k), oracle.surface_normals(ref, k=k), np.float64)
    with pytest.raises(_capi.InvalidParameter):
        _capi.surface_normals(ref, knn=0)


CHAIN = """
referenceDataPointsFilters:
  - SurfaceNormalDataPointsFilter:
      knn: {knn}
      keepDensities: 1
matcher:
  KDTreeMatcher:
    knn: 1
outlierFilters:
  - TrimmedDistOutlierFilter:
      ratio: 0.85
errorMinimizer:
  PointToPlaneErrorMinimizer
transformationCheckers:
  - CounterTransformationChecker:
      maxIterationCount: 40
  - DifferentialTransformationChecker:
      minDiffRotErr: 0.001
      minDiffTransErr: 0.01
      smoothLength: 4
inspector:
  NullInspector
logger:
  NullLogger
"""


@pytest.mark.parametrize("mode", ["loop", "modules"])
def test_validT3d_with_gpu_normals(monkeypatch, golden, mode):
    # utest/utest.cpp:352-356: car_cloud401 -> car_cloud400, point-to-plane,
    # tolerance 0.1 (utest.h:81-82); the reference normals come from the
    # SurfaceNormal filter in the reference chain (the CSV's own normals unused)
    monkeypatch.setenv("PMX_DEVICE_LOOP", "1" if mode == "loop" else "0")
    g, kat = golden
    icp = ICP(np.float32)
    icp.load_yaml(CHAIN.format(knn=7))
    T = icp.compute(hom(g["car401"], np.float32), hom(g["car400"], np.float32), None)
    ok, dt, da = validate3d(T, np.array(kat["validT3d"]), kat["tol3d"])
    assert ok, (dt, da)
