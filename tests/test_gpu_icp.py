"""End-to-end parity of the GPU ICP chain (host C++ chain over the C ABI)
against the CPU oracle, and the reference's known answers through the GPU.

Bar (BASELINE.json north star): final transform within 1e-5 (float) /
1e-12 (double) Frobenius norm of the CPU path on identical inputs, with equal
iteration counts.
"""
import numpy as np
import pytest

from helpers import chain_yaml, hom, pca_normals, planar_grid, rel_displacement, validate2d, validate3d
from libpointmatcher_amd.icp import ICP
from libpointmatcher_amd.synth import reading_cloud, reference_cloud

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["loop", "modules"])
def icp_mode(request, monkeypatch):
    """Every chain runs twice: as the device-resident loop (the default when
    every module has a device form) and through the per-module calls."""
    monkeypatch.setenv("PMX_DEVICE_LOOP", "1" if request.param == "loop" else "0")
    return request.param

DIFF = dict(minDiffRotErr=0.001, minDiffTransErr=0.01, smoothLength=4)


def run_both(oracle, reading, reference, normals, dtype, knn=1, maxdist=np.inf, filters=(("TrimmedDistOutlierFilter", {"ratio": 0.85}),),
             minimizer="PointToPlaneErrorMinimizer", maxit=40, differential=None, threads=8):
    icp = ICP(dtype)
    icp.load_yaml(chain_yaml(knn=knn, maxdist="inf" if np.isinf(maxdist) else maxdist, filters=filters,
                             minimizer=minimizer, maxit=maxit, differential=differential))
    icp.keep_trace(True)
    Tg = icp.compute(reading, reference, normals)
    sg = icp.stats()
    trg = icp.trace()
    cfg = oracle.make_cfg(knn=knn, max_dist=maxdist, filters=tuple(filters), minimizer=minimizer, counter_max=maxit,
                          differential=differential, threads=threads)
    rc, To, so, tro = oracle.icp(cfg, reading.astype(dtype), reference.astype(dtype),
                                 normals=None if normals is None else normals.astype(dtype), trace=True)
    assert rc == 0
    return Tg, sg, trg, To, so, tro


TOL = {np.float32: 1e-5, np.float64: 1e-12}


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_p2plane_trimmed_synthetic(oracle, dtype):
    ref, nrm = reference_cloud(60000, dtype)
    rd = reading_cloud(50000, dtype)
    Tg, sg, trg, To, so, tro = run_both(oracle, rd, ref, nrm, dtype, maxit=30)
    assert sg.iterations == so.iterations == 30
    assert np.linalg.norm(Tg - To) <= TOL[dtype], np.linalg.norm(Tg - To)
    assert sg.kept == so.kept
    # per-iteration agreement of T_iter
    assert np.abs(trg - tro).max() <= 10 * TOL[dtype]


def test_c2_100k_with_differential(oracle):
    # BASELINE config 2 size, Differential checker: equal iteration counts
    ref, nrm = reference_cloud(100_000, np.float32)
    rd = reading_cloud(100_000, np.float32)
    Tg, sg, trg, To, so, tro = run_both(oracle, rd, ref, nrm, np.float32, differential=DIFF, threads=16)
    assert sg.iterations == so.iterations
    assert np.linalg.norm(Tg - To) <= 1e-5


def test_k4_maxdist_p2plane(oracle):
    ref, nrm = reference_cloud(40000, np.float32)
    rd = reading_cloud(30000, np.float32)
    Tg, sg, trg, To, so, tro = run_both(oracle, rd, ref, nrm, np.float32, knn=4,
                                        filters=[("MaxDistOutlierFilter", {"maxDist": 0.05})], maxit=20)
    assert np.linalg.norm(Tg - To) <= 1e-5
    assert sg.kept == so.kept


def test_p2point_double_no_filter(oracle):
    # config-5 shape (double, empty chain, point-to-point) at test size
    ref, nrm = reference_cloud(40000, np.float64)
    rd = reading_cloud(60000, np.float64)
    Tg, sg, trg, To, so, tro = run_both(oracle, rd, ref, None, np.float64, filters=[],
                                        minimizer="PointToPointErrorMinimizer", maxit=20)
    assert np.linalg.norm(Tg - To) <= 1e-12


@pytest.mark.parametrize("filters", [
    [("VarTrimmedDistOutlierFilter", {"minRatio": 0.6, "maxRatio": 0.8, "lambda": 0.9})],
    [("MedianDistOutlierFilter", {"factor": 3.0}), ("MaxDistOutlierFilter", {"maxDist": 0.1})],
    [("NullOutlierFilter", {})],
])
def test_other_outlier_chains(oracle, filters):
    ref, nrm = reference_cloud(30000, np.float32)
    rd = reading_cloud(25000, np.float32)
    Tg, sg, trg, To, so, tro = run_both(oracle, rd, ref, nrm, np.float32, filters=filters, maxit=15)
    assert np.linalg.norm(Tg - To) <= 1e-5


# ------------------------------------------------ reference KATs on the GPU --
@pytest.mark.parametrize("minimizer", ["PointToPointErrorMinimizer", "PointToPlaneErrorMinimizer"])
def test_kat_validT3d_gpu(oracle, golden, minimizer):
    g, kat = golden
    Tg, sg, trg, To, so, tro = run_both(oracle, hom(g["car401"]), hom(g["car400"]), g["car400_normals"], np.float32,
                                        minimizer=minimizer, differential=DIFF)
    ok, dt, da = validate3d(Tg, np.array(kat["validT3d"]), kat["tol3d"])
    assert ok, (dt, da)
    assert sg.iterations == so.iterations and np.linalg.norm(Tg - To) <= 1e-5


def test_kat_validT2d_gpu(oracle, golden):
    g, kat = golden
    Tg, sg, trg, To, so, tro = run_both(oracle, hom(g["box2"]), hom(g["box1"]), None, np.float32,
                                        minimizer="PointToPointErrorMinimizer", differential=DIFF)
    ok, dt, da = validate2d(Tg, np.array(kat["validT2d"]), kat["tol2d"])
    assert ok, (dt, da)
    assert np.linalg.norm(Tg - To) <= 1e-5


def test_kat_icp_singular_gpu(oracle):
    pts0, pts1 = planar_grid()
    nrm = np.tile(np.array([[0, 0, 1]], np.float32), (pts1.shape[0], 1))
    Tg, sg, trg, To, so, tro = run_both(oracle, pts0, pts1, nrm, np.float32,
                                        filters=[("TrimmedDistOutlierFilter", {"ratio": 1.0})], differential=DIFF)
    exp = np.eye(4)
    exp[2, 3] = 1
    assert np.linalg.norm(Tg - exp) <= 1e-5 * min(np.linalg.norm(Tg), np.linalg.norm(exp))


def test_kat_icp_identity_gpu(oracle, golden):
    g, _ = golden
    pts = g["vtk0"]
    nrm = pca_normals(pts.astype(np.float64)).astype(np.float32)
    icp = ICP(np.float32)
    icp.load_yaml(chain_yaml(filters=[("TrimmedDistOutlierFilter", {"ratio": 1.0})], differential=DIFF))
    T = icp.compute(hom(pts), hom(pts), nrm)
    assert np.linalg.norm(T - np.eye(4)) <= 1e-4 * 2.0


def test_regression_ref_trans_gpu(oracle, golden):
    g, kat = golden
    refT = np.array(kat["icp_data_ref_trans"]["defaultPointToPointMinDistDataPointsFilter"])
    Tg, sg, trg, To, so, tro = run_both(oracle, hom(g["vtk1"]), hom(g["vtk0"]), None, np.float32,
                                        filters=[("TrimmedDistOutlierFilter", {"ratio": 0.75})],
                                        minimizer="PointToPointErrorMinimizer", maxit=150, differential=DIFF)
    assert rel_displacement(Tg, refT, g["vtk1"]) < kat["icp_data_rel_tol"]
    assert np.linalg.norm(Tg - To) <= 1e-5


def test_convergence_error_propagates():
    # all matches beyond the radius: every weight 0 -> "no point to minimize"
    ref, nrm = reference_cloud(5000, np.float32)
    rd = reading_cloud(3000, np.float32)
    rd[:, :3] += 100.0
    icp = ICP(np.float32)
    icp.load_yaml(chain_yaml(maxdist=0.01, filters=[]))
    from libpointmatcher_amd._capi import ConvergenceError
    with pytest.raises(ConvergenceError, match="no point to minimize"):
        icp.compute(rd, ref, nrm)
    icp.load_yaml(chain_yaml(maxdist=0.01))
    with pytest.raises(ConvergenceError, match="no outlier to filter"):
        icp.compute(rd, ref, nrm)


def test_prepare_iterate_finish_equals_compute(oracle):
    ref, nrm = reference_cloud(20000, np.float32)
    rd = reading_cloud(20000, np.float32)
    a = ICP(np.float32)
    a.load_yaml(chain_yaml(maxit=12))
    T1 = a.compute(rd, ref, nrm)
    b = ICP(np.float32)
    b.load_yaml(chain_yaml(maxit=12))
    b.prepare(rd, ref, nrm)
    done = b.iterate(5)
    assert not done
    done = b.iterate(100)
    assert done
    T2 = b.finish()
    assert np.array_equal(T1, T2)
