"""RobustOutlierFilter on the GPU (pmx_robust.hip scale estimators, the
weighted reductions of pmx_reduce.hip) against the oracle
(oracle/pmo_impl.inc pmo_robust_weights, pinned by tests/test_robust_oracle.py).

Bar: the scale bit-exact for mad / berg (order statistics) and to 1 ulp for
std (fp64 sums in another order); weights to rtol 1e-6 (f32) / 1e-12 (f64)
(device exp / pow / sqrt vs libm); the weighted normal equations to the same
relative bound; ErrorElements counts exact.  The reference's regression
configuration defaultRobustOutlierFilter.yaml runs unchanged through the GPU
chain (utest.cpp:81-160 3 % rule) and follows the oracle ICP iteration for
iteration.
Reference: OutlierFiltersImpl.cpp:394-598, Matches.cpp:88-129,
PointToPoint.cpp:61-101, PointToPlane.cpp:171-243.
"""
import numpy as np
import pytest

from helpers import hom, rel_displacement
from libpointmatcher_amd import _capi as P
from libpointmatcher_amd.icp import ICP
from libpointmatcher_amd.synth import reading_cloud, reference_cloud

pytestmark = pytest.mark.gpu

TOL = {np.float32: 1e-6, np.float64: 1e-12}
FCTS = ["cauchy", "welsch", "sc", "gm", "tukey", "huber", "L1", "student"]
SCALES = ["mad", "std", "berg", "none"]


def _T(dtype, ang=0.02, tr=0.01):
    c, s = np.cos(ang), np.sin(ang)
    T = np.eye(4)
    T[:2, :2] = [[c, -s], [s, c]]
    T[:3, 3] = [tr, -tr, tr / 2]
    return T.astype(dtype)


def _gpu_mode(r_it, scale, nb):
    """the host class's schedule (libpointmatcher_amd RobustOF::compute)"""
    rec = r_it <= nb or nb == 0
    if scale == "mad":
        return P.RS_MAD if rec else P.RS_KEEP
    if scale == "std":
        return P.RS_STD if rec else P.RS_KEEP
    if scale == "berg":
        return P.RS_KEEP if not rec else (P.RS_BERG_FIRST if r_it == 1 else P.RS_BERG_NEXT)
    return P.RS_NONE


def _setup(dtype, k, max_dist=np.inf, n=12000, m=16000):
    ref, nrm = reference_cloud(m, dtype)
    rd = reading_cloud(n, dtype)
    ctx = P.Context(0, dtype)
    ctx.set_reference(ref, nrm)
    ctx.set_reading(rd)
    return ctx, ref, nrm, rd


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("scale", SCALES)
@pytest.mark.parametrize("fct", FCTS)
def test_robust_weights_and_scale(oracle, dtype, scale, fct):
    k = 3
    ctx, ref, nrm, rd = _setup(dtype, k)
    tol = TOL[dtype]
    nb, approx = (2, 2.5) if fct in ("cauchy", "huber") else (0, np.inf)
    p = {"robustFct": fct, "scaleEstimator": scale, "tuning": 0.8, "nbIterationForScale": nb,
         "approximation": approx}
    r = oracle.make_robust(p)
    tg = 0.8 if scale == "berg" else 0.0
    tuning = 0.8
    if scale == "berg":
        tuning = {"cauchy": 4.3040, "tukey": 7.0589, "huber": 2.0138}.get(fct, 0.8)
    for it in range(1, 4):  # three iterations of the schedule at moving poses
        T = _T(dtype, ang=0.02 / it, tr=0.01 / it)
        ctx.match(T, knn=k)
        ctx.outlier_robust(0, fct, tuning, approx, _gpu_mode(it, scale, nb), tg)
        w = ctx.get_weights()
        s = ctx.robust_scale(0)
        d, i = ctx.get_matches()
        rc, ow = oracle.robust_weights(r, d, i)
        assert rc == 0
        if scale == "std":
            np.testing.assert_allclose(s, r.scale, rtol=4e-7 if dtype == np.float32 else 1e-13)
        else:
            assert s == r.scale
        np.testing.assert_allclose(w, ow, rtol=tol, atol=tol)
        assert np.array_equal(w == 0, ow == 0) or scale == "std"
    ctx.close()


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("minimizer", ["p2plane", "p2point"])
@pytest.mark.parametrize("chain", ["robust", "trimmed+robust", "robust+maxdist", "p2pl_distance"])
def test_weighted_systems(oracle, dtype, minimizer, chain):
    k = 4
    ctx, ref, nrm, rd = _setup(dtype, k, n=15000, m=20000)
    T = _T(dtype, ang=0.01, tr=0.008)
    ctx.match(T, knn=k, max_dist=0.12)
    p = {"robustFct": "cauchy", "scaleEstimator": "mad", "tuning": 1.0}
    p2pl = chain == "p2pl_distance"
    if p2pl:
        p["distanceType"] = "point2plane"
    r = oracle.make_robust(p)
    d, i = ctx.get_matches()
    step = oracle.transform(T, rd)
    if chain == "trimmed+robust":
        ctx.outlier("TrimmedDistOutlierFilter", 0, ratio=0.8)
        ctx.outlier_robust(1, "cauchy", 1.0, np.inf, P.RS_MAD, 0.0)
        _, w0 = oracle.outlier_chain([("TrimmedDistOutlierFilter", {"ratio": 0.8})], d)
        _, w1 = oracle.robust_weights(r, d, i)
        ow = w0 * w1
    elif chain == "robust+maxdist":
        ctx.outlier_robust(0, "cauchy", 1.0, np.inf, P.RS_MAD, 0.0)
        ctx.outlier("MaxDistOutlierFilter", 1, maxDist=0.06)
        _, w0 = oracle.robust_weights(r, d, i)
        _, w1 = oracle.outlier_chain([("MaxDistOutlierFilter", {"maxDist": 0.06})], d)
        ow = w0 * w1
    else:
        ctx.outlier_robust(0, "cauchy", 1.0, np.inf, P.RS_MAD, 0.0, point2plane=p2pl)
        _, ow = oracle.robust_weights(r, d, i, step=step, ref=ref, normals=nrm[:, :3] if nrm.shape[1] > 3 else nrm)
    tol = TOL[dtype]
    w = ctx.get_weights()
    np.testing.assert_allclose(w, ow, rtol=tol, atol=tol)
    if minimizer == "p2plane":
        A, b, st = ctx.p2plane_system()
        rc, oA, ob, ost = oracle.p2plane_system(step, ref, nrm, d, i, w)
        assert rc == 0
        np.testing.assert_allclose(A, oA, rtol=1e-9, atol=1e-9 * np.abs(oA).max())
        np.testing.assert_allclose(b, ob, rtol=1e-9, atol=1e-9 * np.abs(ob).max())
    else:
        mp, mq, m, st = ctx.p2point_system()
        rc, dT, ost = oracle.p2point(step, ref, d, i, w)
        assert rc == 0
        keep = np.isfinite(d) & (w != 0)
        ww = np.where(keep, w, 0).astype(np.float64)
        sw = ww.sum()
        pm = (step[:, None, :3].astype(np.float64) * ww[..., None]).sum((0, 1)) / sw
        q = ref[np.where(i >= 0, i, 0), :3].astype(np.float64)
        qm = (q * ww[..., None]).sum((0, 1)) / sw
        np.testing.assert_allclose(mp, pm, rtol=1e-5 if dtype == np.float32 else 1e-11, atol=1e-6)
        np.testing.assert_allclose(mq, qm, rtol=1e-5 if dtype == np.float32 else 1e-11, atol=1e-6)
        np.testing.assert_allclose(st.sum_w, ost.sum_w, rtol=1e-9)
    assert st.kept == ost.kept and st.nonzero_weights == ost.nonzero_weights
    assert st.rejected_matches == ost.rejected_matches and st.rejected_points == ost.rejected_points
    np.testing.assert_allclose(st.sum_w, ost.sum_w, rtol=1e-9)
    ctx.close()


def test_icp_data_robust_config_unchanged(golden):
    g, kat = golden
    text = kat["icp_data_configs"]["defaultRobustOutlierFilter"]
    icp = ICP(np.float32)
    icp.load_yaml(text)
    T = icp.compute(hom(g["vtk1"], np.float32), hom(g["vtk0"], np.float32), None)
    refT = np.array(kat["icp_data_ref_trans"]["defaultRobustOutlierFilter"])
    err = rel_displacement(T, refT, g["vtk1"])
    print(f"defaultRobustOutlierFilter: rel err {err:.4f}, iterations {icp.stats().iterations}")
    assert err < kat["icp_data_rel_tol"]


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_icp_robust_equals_oracle(golden, oracle, dtype):
    """the same chain through the GPU ICP and the oracle ICP: same iteration
    count, |dT|_F <= 1e-5 (f32) / 1e-12 (f64), the north_star bar (cauchy
    weights in T; the sums' order differs)"""
    g, kat = golden
    text = kat["icp_data_configs"]["defaultRobustOutlierFilter"]
    icp = ICP(dtype)
    icp.load_yaml(text)
    rd, ref = hom(g["vtk1"], dtype), hom(g["vtk0"], dtype)
    Tg = icp.compute(rd, ref, None)
    c = oracle.make_cfg(knn=10, filters=(("RobustOutlierFilter", {"robustFct": "cauchy", "scaleEstimator": "mad",
                                                                    "tuning": 1}),),
                        minimizer="PointToPointErrorMinimizer", counter_max=40,
                        differential=dict(minDiffRotErr=0.001, minDiffTransErr=0.01, smoothLength=4), threads=8)
    rc, To, so, _ = oracle.icp(c, rd, ref)
    assert rc == 0
    frob = np.linalg.norm(Tg.astype(np.float64) - To.astype(np.float64))
    print(f"robust {np.dtype(dtype).name}: iterations {icp.stats().iterations}/{so.iterations} |dT|={frob:.3g}")
    assert icp.stats().iterations == so.iterations
    assert frob <= (1e-5 if dtype == np.float32 else 1e-12)


ROBUST_LOOP_CASES = [
    # (robust params, minimizer, with normals)
    ({"robustFct": "cauchy", "scaleEstimator": "mad", "tuning": 1}, "PointToPointErrorMinimizer", False),
    ({"robustFct": "huber", "scaleEstimator": "berg", "tuning": 0.05}, "PointToPointErrorMinimizer", False),
    ({"robustFct": "welsch", "scaleEstimator": "std", "tuning": 1.5, "nbIterationForScale": 3},
     "PointToPlaneErrorMinimizer", True),
    ({"robustFct": "tukey", "scaleEstimator": "mad", "tuning": 4, "distanceType": "point2plane",
      "nbIterationForScale": 5}, "PointToPlaneErrorMinimizer", True),
]


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("case", range(len(ROBUST_LOOP_CASES)))
def test_robust_device_loop_equals_modules(monkeypatch, oracle, dtype, case):
    """RobustOutlierFilter chains on the device loop (pmx_loop_*: the scale
    schedule from the loop's iteration index, the weighted reductions and the
    full-A step on the device) against the per-module calls (PMX_DEVICE_LOOP=0)
    and the oracle ICP: same iteration count, |dT|_F within 1e-5 / 1e-12."""
    from helpers import chain_yaml

    params, minimizer, with_n = ROBUST_LOOP_CASES[case]
    ref, nrm = reference_cloud(40_000, dtype)
    rd = reading_cloud(20_000, dtype)
    diff = dict(minDiffRotErr=0.001, minDiffTransErr=0.01, smoothLength=4)
    filters = (("RobustOutlierFilter", params),)
    yaml = chain_yaml(knn=2, filters=filters, minimizer=minimizer, maxit=25, differential=diff)
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("PMX_DEVICE_LOOP", mode)
        icp = ICP(dtype)
        icp.load_yaml(yaml)
        T = icp.compute(rd, ref, nrm if with_n else None)
        out[mode] = (T, icp.stats())
        icp.close()
    (Tl, sl), (Tm, sm) = out["1"], out["0"]
    cfg = oracle.make_cfg(knn=2, filters=filters, minimizer=minimizer, counter_max=25, differential=diff, threads=8)
    rc, To, so, _ = oracle.icp(cfg, rd, ref, normals=nrm if with_n else None)
    assert rc == 0
    tol = 1e-5 if dtype == np.float32 else 1e-12
    fl = np.linalg.norm(Tl.astype(np.float64) - To.astype(np.float64))
    fm = np.linalg.norm(Tm.astype(np.float64) - To.astype(np.float64))
    print(f"{np.dtype(dtype).name} {params['robustFct']}/{params['scaleEstimator']}: iterations loop {sl.iterations} "
          f"modules {sm.iterations} oracle {so.iterations}; |dT| loop {fl:.3g} modules {fm:.3g}")
    assert sl.iterations == sm.iterations == so.iterations
    assert sl.kept == sm.kept
    assert fl <= tol and fm <= tol


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("params", [
    {"robustFct": "huber", "scaleEstimator": "berg", "tuning": 0.05},
    {"robustFct": "cauchy", "scaleEstimator": "mad", "tuning": 1, "nbIterationForScale": 3},
])
def test_robust_second_compute_vs_oracle(monkeypatch, oracle, dtype, params):
    """RobustOutlierFilter keeps its iteration count across compute() calls
    (OutlierFiltersImpl.cpp:500-540: berg's first-call scale, the
    nbIterationForScale schedule).  A second compute on the same ICP object
    starts past the first call's iterations.  Both calls of the device loop
    (scale mode per loop iteration from the host module's count) and of the
    per-module path against the oracle ICP with ONE filter object kept across
    its two calls (pmo_icp_keep): same iterations, T within 1e-5 / 1e-12."""
    from helpers import chain_yaml

    ref, _ = reference_cloud(40_000, dtype)
    rd = reading_cloud(20_000, dtype)
    rd2 = reading_cloud(15_000, dtype)
    maxit = 12
    filters = (("RobustOutlierFilter", params),)
    yaml = chain_yaml(knn=2, filters=filters, minimizer="PointToPointErrorMinimizer", maxit=maxit)
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("PMX_DEVICE_LOOP", mode)
        icp = ICP(dtype)
        icp.load_yaml(yaml)
        res = []
        for r in (rd, rd2):
            T = icp.compute(r, ref, None)
            s = icp.stats()
            res.append((T.astype(np.float64), s.iterations, s.kept))
        icp.close()
        out[mode] = res
    cfg = oracle.make_cfg(knn=2, filters=filters, minimizer="PointToPointErrorMinimizer", counter_max=maxit,
                          threads=8)
    ores = []
    for r in (rd, rd2):
        rc, To, so, _ = oracle.icp(cfg, r, ref, keep_robust=True)
        assert rc == 0
        ores.append((To.astype(np.float64), so.iterations))
    # the filter object saw both calls' iterations (its counter starts at 1)
    assert cfg.robust.iteration == 1 + ores[0][1] + ores[1][1]
    tol = 1e-5 if dtype == np.float32 else 1e-12
    for call in range(2):
        (Tl, il, kl), (Tm, im, km), (To, io) = out["1"][call], out["0"][call], ores[call]
        fl, fm = np.linalg.norm(Tl - To), np.linalg.norm(Tm - To)
        print(f"{params['scaleEstimator']} call {call + 1}: iterations {il}/{im}/{io} kept {kl}/{km} "
              f"|dT| loop {fl:.3g} modules {fm:.3g}")
        assert il == im == io and kl == km
        assert fl <= tol and fm <= tol
    # the second call differs from a fresh filter's (the schedule carried over)
    cfg2 = oracle.make_cfg(knn=2, filters=filters, minimizer="PointToPointErrorMinimizer", counter_max=maxit,
                           threads=8)
    rc, Tf, _, _ = oracle.icp(cfg2, rd2, ref)
    assert rc == 0
    print(f"fresh filter vs kept on call 2: |dT| {np.linalg.norm(Tf.astype(np.float64) - ores[1][0]):.3g}")
