"""VoxelGridDataPointsFilter on the GPU (pmx_voxel.hip) against the oracle's
restatement of the reference walk (oracle/pmo_impl.inc pmo_voxel_grid), and the
reference's own ICP cases (utest/ui/DataFilters.cpp:612-669).

Bar: bit-exact features and descriptors — the voxel of a point is the same
unsigned arithmetic on the same T values, a voxel's sum runs in point order
in T on both sides (the stable sort keeps the order), the kept points come in
index order.  Covered: f32/f64, 2-D and 3-D, useCentroid on/off (off: the
reference's row-shifted voxel centres), averageExistingDescriptors on/off,
descriptors, dense voxels (thousands of points) and one point per voxel.
"""
import numpy as np
import pytest

from helpers import chain_yaml, hom, validate2d, validate3d
from libpointmatcher_amd import _capi
from libpointmatcher_amd.icp import ICP

pytestmark = pytest.mark.gpu

DIFF = dict(minDiffRotErr=0.001, minDiffTransErr=0.01, smoothLength=4)


def _cloud(n, rows, dtype, seed, scale=3.0):
    rng = np.random.default_rng(seed)
    p = rng.normal(0, scale, (n, rows - 1))
    return np.hstack([p, np.ones((n, 1))]).astype(dtype)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("rows", [4, 3])
@pytest.mark.parametrize("centroid,avg", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("vs", [(0.5, 0.5, 0.5), (0.05, 0.1, 0.2), (20.0, 20.0, 20.0), (1e-3, 1e-3, 1e-3)])
def test_voxel_grid_equals_oracle(oracle, dtype, rows, centroid, avg, vs):
    if rows == 4 and vs[0] < 0.01:
        pytest.skip("more than 2^32 voxels: test_voxel_grid_too_many_voxels")
    pts = _cloud(40000, rows, dtype, seed=rows)
    desc = np.random.default_rng(5).normal(size=(pts.shape[0], 3)).astype(dtype)
    gf, gd = _capi.voxel_grid(pts, desc, vs, centroid, avg)
    of, od = oracle.voxel_grid(pts, desc, vs, centroid, avg)
    assert gf.shape == of.shape and gd.shape == od.shape
    assert np.array_equal(gf, of) and np.array_equal(gd, od)
    assert 0 < len(gf) <= len(pts)


def test_voxel_grid_too_many_voxels():
    # the reference's unsigned voxel count wraps past 2^32 and indexes out of
    # its vector (undefined); here the reference's allocation error is raised
    with pytest.raises(_capi.InvalidParameter, match="voxel"):
        _capi.voxel_grid(_cloud(1000, 4, np.float32, 9), None, (1e-3, 1e-3, 1e-3))


def test_voxel_grid_no_descriptors_and_tiny(oracle):
    for pts in (_cloud(1, 4, np.float32, 1), _cloud(7, 4, np.float32, 2), _cloud(3000, 3, np.float32, 3)):
        gf, gd = _capi.voxel_grid(pts, None, (0.3, 0.3, 0.3))
        of, od = oracle.voxel_grid(pts, None, (0.3, 0.3, 0.3))
        assert np.array_equal(gf, of) and gd.shape == (len(gf), 0)


def _reading_voxel(yaml, vs, centroid=True, avg=True):
    return ("readingDataPointsFilters:\n  - VoxelGridDataPointsFilter:\n"
            f"      vSizeX: {vs}\n      vSizeY: {vs}\n      vSizeZ: {vs}\n"
            f"      useCentroid: {int(centroid)}\n      averageExistingDescriptors: {int(avg)}\n" + yaml)


def test_reference_ui_cases(golden):
    """DataFilters.cpp:633-668: vSize 0.02 on the 2-D boxes (validT2d), 1 on
    the car clouds (validT3d); the reference's loops over useCentroid /
    averageExistingDescriptors set both to true on every pass."""
    g, kat = golden
    icp = ICP(np.float32)
    icp.load_yaml(_reading_voxel(chain_yaml(minimizer="PointToPointErrorMinimizer", differential=DIFF), 0.02,
                                 True, True))
    T = icp.compute(hom(g["box2"], np.float32), hom(g["box1"], np.float32), None)
    ok, dt, da = validate2d(T, np.array(kat["validT2d"]), kat["tol2d"])
    assert ok, (dt, da)
    icp = ICP(np.float32)
    icp.load_yaml(_reading_voxel(chain_yaml(differential=DIFF), 1, True, True))
    T = icp.compute(hom(g["car401"], np.float32), hom(g["car400"], np.float32), g["car400_normals"])
    ok, dt, da = validate3d(T, np.array(kat["validT3d"]), kat["tol3d"])
    assert ok, (dt, da)


def test_chain_equals_prefiltered_reading(golden, oracle):
    """the ICP with the voxel reading filter gives the bit-identical transform
    of the ICP without it on the oracle-filtered reading"""
    g, kat = golden
    rd, ref = hom(g["car401"], np.float32), hom(g["car400"], np.float32)
    a = ICP(np.float32)
    a.load_yaml(_reading_voxel(chain_yaml(differential=DIFF), 0.3))
    Ta = a.compute(rd, ref, g["car400_normals"])
    pre, _ = oracle.voxel_grid(rd, None, (0.3, 0.3, 0.3))
    b = ICP(np.float32)
    b.load_yaml(chain_yaml(differential=DIFF))
    Tb = b.compute(pre, ref, g["car400_normals"])
    assert np.array_equal(Ta, Tb)
