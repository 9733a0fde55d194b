"""SamplingSurfaceNormalDataPointsFilter on the GPU (pmx_ssn.hip) against the
oracle restatement (oracle/pmo_impl.inc), and the reference's icp_data
regression configurations run unchanged through the GPU chain.

Parity bar (same deterministic rules on both sides: median-split ties by
point index, a leaf's points in index order, Jacobi eigen pairs): the kept
point set and the features / descriptors bit-exact, normals / eigen pairs /
densities to 1e-6 (f32) / 1e-12 (f64) relative (double-precision Jacobi and
libm pow on two implementations).  samplingMethod 0 draws from the process's
rand() state: both sides are seeded with the same srand.
Reference: SamplingSurfaceNormal.cpp:80-342, utils/utils.h:86-156,
utest/utest.cpp:81-160 (icp_data: median relative displacement < 3 %).
"""
import ctypes

import numpy as np
import pytest
import yaml

from helpers import hom, rel_displacement
from libpointmatcher_amd import _capi
from libpointmatcher_amd.icp import ICP
from libpointmatcher_amd.synth import reference_cloud

pytestmark = pytest.mark.gpu

_libc = ctypes.CDLL(None)
TOL = {np.float32: 1e-6, np.float64: 1e-12}


def _cloud(dtype, D, n, seed=3):
    if D == 3:
        ref, _ = reference_cloud(n, dtype)
        return ref
    rng = np.random.default_rng(seed)
    t = rng.uniform(0, 2 * np.pi, n)
    r = 1 + 0.2 * np.sin(5 * t) + rng.normal(0, 0.01, n)
    return np.stack([r * np.cos(t), r * np.sin(t), np.ones(n)], 1).astype(dtype)


def _compare(g, o, dtype, flags):
    assert len(g["features"]) == len(o["features"])
    assert g["unfit"] == o["unfit"]
    np.testing.assert_array_equal(g["features"], o["features"])
    np.testing.assert_array_equal(g["descriptors"], o["descriptors"])
    tol = TOL[dtype]
    if flags & _capi.SSN_NORMALS:
        np.testing.assert_allclose(g["normals"], o["normals"], rtol=tol, atol=tol)
    if flags & _capi.SSN_EIGVALUES:
        sc = max(1.0, float(np.abs(o["eig_values"]).max()) if len(o["eig_values"]) else 1.0)
        np.testing.assert_allclose(g["eig_values"], o["eig_values"], rtol=tol, atol=tol * sc)
    if flags & _capi.SSN_EIGVECTORS:
        np.testing.assert_allclose(g["eig_vectors"], o["eig_vectors"], rtol=tol, atol=tol)
    if flags & _capi.SSN_DENSITIES:
        np.testing.assert_allclose(g["densities"], o["densities"], rtol=tol)


ALL = _capi.SSN_NORMALS | _capi.SSN_DENSITIES | _capi.SSN_EIGVALUES | _capi.SSN_EIGVECTORS


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("D", [3, 2])
@pytest.mark.parametrize("method,knn,flags", [
    (1, 7, ALL | _capi.SSN_AVERAGE),
    (1, 10, _capi.SSN_NORMALS),
    (1, 3, ALL),
    (0, 7, ALL),
    (0, 16, _capi.SSN_NORMALS | _capi.SSN_DENSITIES),
])
def test_ssn_equals_oracle(oracle, dtype, D, method, knn, flags):
    pts = _cloud(dtype, D, 30001)
    rng = np.random.default_rng(9)
    desc = rng.normal(0, 1, (pts.shape[0], 4)).astype(dtype)
    _libc.srand(1234)
    g = _capi.sampling_surface_normals(pts, desc, knn=knn, sampling_method=method, ratio=0.6, flags=flags)
    _libc.srand(1234)
    o = oracle.sampling_surface_normals(pts, desc, knn=knn, method=method, ratio=0.6, flags=flags)
    assert len(o["features"]) > 0
    _compare(g, o, dtype, flags)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_ssn_drops_large_boxes_and_ties(oracle, dtype):
    # a grid with many equal coordinates (median-split ties) and a few far
    # outliers whose leaves exceed maxBoxDim
    g1 = np.stack(np.meshgrid(np.arange(40), np.arange(30), np.arange(3), indexing="ij"), -1).reshape(-1, 3) * 0.1
    far = np.array([[100.0, 0, 0], [0, 100.0, 0], [0, 0, 100.0], [50.0, 50.0, 50.0]])
    pts = hom(np.concatenate([g1, far]), dtype)
    for method in (0, 1):
        _libc.srand(7)
        g = _capi.sampling_surface_normals(pts, None, knn=5, sampling_method=method, ratio=0.5, max_box_dim=1.0,
                                           flags=ALL)
        _libc.srand(7)
        o = oracle.sampling_surface_normals(pts, None, knn=5, method=method, ratio=0.5, max_box=1.0, flags=ALL)
        assert o["unfit"] > 0
        _compare(g, o, dtype, ALL)


def test_ssn_planar_rank_and_small_clouds(oracle):
    # planar 2-D-degenerate leaves pass the rank test (rank 2 + 1 >= 3);
    # collinear leaves fail it (unfit); tiny clouds are one leaf
    rng = np.random.default_rng(4)
    plane = hom(np.column_stack([rng.uniform(0, 1, (500, 2)), np.zeros(500)]), np.float32)
    line = hom(np.column_stack([rng.uniform(0, 1, 300), np.zeros(300), np.zeros(300)]), np.float32)
    for pts in (plane, line, plane[:5], plane[:1]):
        g = _capi.sampling_surface_normals(pts, None, knn=7, sampling_method=1, flags=ALL)
        o = oracle.sampling_surface_normals(pts, None, knn=7, method=1, flags=ALL)
        _compare(g, o, np.float32, ALL)
    assert oracle.sampling_surface_normals(line, None, knn=7, method=1, flags=ALL)["unfit"] == 300


# ---------------------------------------------------------------------------
# icp_data: the reference's regression configurations, unchanged
# ---------------------------------------------------------------------------
SUPPORTED = ["SamplingSurfaceNormalDataPointsFilter1", "SamplingSurfaceNormalDataPointsFilter2",
             "SamplingSurfaceNormalDataPointsFilter3", "defaultBoundingBoxDataPointsFilter",
             "defaultDistanceLimitDataPointsFilter", "defaultFixStepSamplingDataPointsFilter",
             "defaultIdentityDataPointsFilter",
             "defaultMaxDistDataPointsFilter", "defaultPointToPlaneMinDistDataPointsFilter",
             "defaultPointToPointMinDistDataPointsFilter"]


@pytest.mark.parametrize("name", SUPPORTED)
def test_icp_data_config_unchanged(golden, name):
    """utest.cpp:81-160: icp(data = cloud.00001, ref = cloud.00000) with the
    config file as is; the median displacement against the stored *.ref_trans
    is below 3 % of the median transformed coordinate."""
    g, kat = golden
    text = kat["icp_data_configs"][name]
    icp = ICP(np.float32)
    icp.load_yaml(text)
    _libc.srand(1)
    T = icp.compute(hom(g["vtk1"], np.float32), hom(g["vtk0"], np.float32), None)
    refT = np.array(kat["icp_data_ref_trans"][name])
    err = rel_displacement(T, refT, g["vtk1"])
    print(f"{name}: rel err {err:.4f}, iterations {icp.stats().iterations}")
    assert err < kat["icp_data_rel_tol"]


def test_icp_data_identity_config_equals_oracle(golden, oracle):
    """defaultIdentityDataPointsFilter.yaml (deterministic: samplingMethod 1,
    no rand()): the GPU chain with the config unchanged against the oracle
    ICP on the oracle-filtered reference — same iterations, |dT|_F <= 1e-5."""
    g, kat = golden
    text = kat["icp_data_configs"]["defaultIdentityDataPointsFilter"]
    icp = ICP(np.float32)
    icp.load_yaml(text)
    rd, ref = hom(g["vtk1"], np.float32), hom(g["vtk0"], np.float32)
    Tg = icp.compute(rd, ref, None)
    sg = icp.stats()
    cfg = yaml.safe_load(text)["referenceDataPointsFilters"][0]["SamplingSurfaceNormalDataPointsFilter"]
    o = oracle.sampling_surface_normals(ref, None, knn=cfg["knn"], method=cfg["samplingMethod"],
                                        ratio=cfg["ratio"], flags=oracle.SSN_NORMALS)
    c = oracle.make_cfg(filters=(("TrimmedDistOutlierFilter", {"ratio": 0.75}),), counter_max=40,
                        differential=dict(minDiffRotErr=0.001, minDiffTransErr=0.01, smoothLength=4), threads=8)
    rc, To, so, _ = oracle.icp(c, rd, o["features"], normals=o["normals"])
    assert rc == 0
    assert sg.iterations == so.iterations
    assert np.linalg.norm(Tg - To) <= 1e-5
