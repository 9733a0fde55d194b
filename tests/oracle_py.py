"""ctypes wrapper around the CPU oracle (oracle/build/libpmo.so).

TEST INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py as the checker.  The product package
(libpointmatcher_amd) never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# (PMO_LIB: another build of the same source, e.g. bench.py's -march=native one)
LIB = os.environ.get("PMO_LIB") or os.path.join(ROOT, "oracle", "build", "libpmo.so")

# error codes (oracle/pmo.h)
OK, E_NO_POINTS, E_EMPTY_QUANTILE, E_BAD_PARAM, E_TRANSFORMATION, E_NAN = 0, -1, -2, -3, -4, -5
OF = {"NullOutlierFilter": 0, "MaxDistOutlierFilter": 1, "MinDistOutlierFilter": 2,
      "MedianDistOutlierFilter": 3, "TrimmedDistOutlierFilter": 4, "VarTrimmedDistOutlierFilter": 5,
      "RobustOutlierFilter": 6}
OF_PARAMS = {0: [], 1: [("maxDist", 1.0)], 2: [("minDist", 1.0)], 3: [("factor", 3.0)],
             4: [("ratio", 0.85)], 5: [("minRatio", 0.05), ("maxRatio", 0.99), ("lambda", 2.35)], 6: []}
ROBUST_FCT = {"cauchy": 0, "welsch": 1, "sc": 2, "gm": 3, "tukey": 4, "huber": 5, "L1": 6, "student": 7}
ROBUST_SCALE = {"none": 0, "mad": 1, "std": 2, "berg": 3}


class Robust(C.Structure):
    """pmo_robust: RobustOutlierFilter parameters + state (zero state = a new filter)."""
    _fields_ = [("fct", C.c_int), ("scale_est", C.c_int), ("nb_iter", C.c_int), ("point2plane", C.c_int),
                ("tuning", C.c_double), ("approximation", C.c_double), ("iteration", C.c_int),
                ("k", C.c_double), ("target", C.c_double), ("scale", C.c_double)]


def make_robust(p):
    r = Robust()
    r.fct = ROBUST_FCT[p.get("robustFct", "cauchy")]
    r.scale_est = ROBUST_SCALE[p.get("scaleEstimator", "mad")]
    r.nb_iter = int(p.get("nbIterationForScale", 0))
    r.point2plane = 1 if p.get("distanceType", "point2point") == "point2plane" else 0
    r.tuning = float(p.get("tuning", 1.0))
    r.approximation = float(p.get("approximation", np.inf))
    return r


def robust_weights(r, dists, ids, step=None, ref=None, normals=None):
    """One RobustOutlierFilter::compute on (N, k) matches; r (Robust) is updated."""
    d = np.ascontiguousarray(dists)
    N, k = d.shape
    ids = np.ascontiguousarray(ids, dtype=np.int32)
    w = np.empty_like(d)
    rows = step.shape[1] if step is not None else 4
    f = getattr(lib(), "pmo_robust_weights_" + _sfx(d.dtype))
    rc = f(C.byref(r), _p(d), _p(ids), k, C.c_int64(N), _p(step), rows, _p(ref),
           _p(np.ascontiguousarray(normals, dtype=d.dtype) if normals is not None else None), _p(w))
    return rc, w
MIN = {"PointToPlaneErrorMinimizer": 0, "PointToPointErrorMinimizer": 1}


class Cfg(C.Structure):
    _fields_ = [("knn", C.c_int), ("maxDist", C.c_double), ("knn_method", C.c_int),
                ("knn_threads", C.c_int), ("n_filters", C.c_int),
                ("filter_type", C.c_int * 8), ("filter_p", (C.c_double * 3) * 8),
                ("minimizer", C.c_int), ("acc_mode", C.c_int), ("counter_max", C.c_int),
                ("diff_enabled", C.c_int), ("diff_rot", C.c_double), ("diff_trans", C.c_double),
                ("diff_smooth", C.c_int), ("robust", Robust)]


class Stats(C.Structure):
    _fields_ = [("iterations", C.c_int64), ("kept", C.c_int64), ("nonzero_weights", C.c_int64),
                ("rejected_matches", C.c_int64), ("rejected_points", C.c_int64),
                ("touched", C.c_int64), ("sum_w", C.c_double), ("point_used_ratio", C.c_double),
                ("weighted_point_used_ratio", C.c_double), ("max_iter_reached", C.c_int),
                ("error", C.c_int), ("last_limit", C.c_double), ("loop_seconds", C.c_double)]

    def asdict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = C.CDLL(LIB)
    return _lib


def _sfx(dtype):
    return "f32" if np.dtype(dtype) == np.float32 else "f64"


def _p(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def knn(ref, query, k=1, max_dist=np.inf, method="kdtree", threads=1):
    """ref, query: (n, rows) arrays (rows = D+1).  Returns dists (N,k), ids (N,k), touched."""
    dt = ref.dtype
    ref = np.ascontiguousarray(ref)
    query = np.ascontiguousarray(query, dtype=dt)
    N, rows = query.shape
    dists = np.empty((N, k), dt)
    ids = np.empty((N, k), np.int32)
    f = getattr(lib(), "pmo_knn_" + _sfx(dt))
    f.restype = C.c_int64
    scal = C.c_float if dt == np.float32 else C.c_double
    touched = f(_p(ref), rows, C.c_int64(ref.shape[0]), _p(query), C.c_int64(N), k,
                scal(max_dist), 1 if method == "kdtree" else 0, threads, _p(dists), _p(ids))
    return dists, ids, touched


def quantile(dists, q):
    d = np.ascontiguousarray(dists).ravel()
    out = np.zeros(1, d.dtype)
    f = getattr(lib(), "pmo_quantile_" + _sfx(d.dtype))
    scal = C.c_float if d.dtype == np.float32 else C.c_double
    rc = f(_p(d), C.c_int64(d.size), scal(q), _p(out))
    return rc, out[0]


def outlier_chain(filters, dists):
    """filters: list of (name, {param: value}); dists (N,k)."""
    d = np.ascontiguousarray(dists)
    N, k = d.shape
    types, params = _filters(filters)
    w = np.empty_like(d)
    f = getattr(lib(), "pmo_outlier_chain_" + _sfx(d.dtype))
    rc = f(len(filters), _p(types), _p(params), _p(d), k, C.c_int64(N), _p(w))
    return rc, w


def vartrimmed_ratio(dists, min_ratio, max_ratio, lam):
    d = np.ascontiguousarray(dists).ravel()
    out = np.zeros(1, d.dtype)
    scal = C.c_float if d.dtype == np.float32 else C.c_double
    f = getattr(lib(), "pmo_vartrimmed_ratio_" + _sfx(d.dtype))
    rc = f(_p(d), C.c_int64(d.size), scal(min_ratio), scal(max_ratio), scal(lam), _p(out))
    return rc, out[0]


def transform(T, pts):
    pts = np.ascontiguousarray(pts)
    T = np.ascontiguousarray(T, dtype=pts.dtype)
    out = np.empty_like(pts)
    getattr(lib(), "pmo_transform_" + _sfx(pts.dtype))(_p(T), pts.shape[1], _p(pts),
                                                         C.c_int64(pts.shape[0]), _p(out))
    return out


def p2plane_system(reading_t, ref, normals, dists, ids, w, acc_mode=0):
    rows = reading_t.shape[1]
    n = 6 if rows == 4 else 3
    A = np.zeros(n * n)
    b = np.zeros(n)
    st = Stats()
    N, k = dists.shape
    rc = getattr(lib(), "pmo_p2plane_system_" + _sfx(reading_t.dtype))(
        rows, _p(reading_t), _p(ref), _p(np.ascontiguousarray(normals)), _p(dists), _p(ids), _p(w),
        k, C.c_int64(N), acc_mode, _p(A), _p(b), C.byref(st))
    return rc, A.reshape(n, n), b, st


def p2plane_solve(A, b, rows, dtype):
    dT = np.zeros((rows, rows), dtype)
    A = np.ascontiguousarray(A, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    rc = getattr(lib(), "pmo_p2plane_solve_" + _sfx(dtype))(rows, _p(A), _p(b), _p(dT))
    return rc, dT


def p2point(reading_t, ref, dists, ids, w, acc_mode=0):
    rows = reading_t.shape[1]
    N, k = dists.shape
    dT = np.zeros((rows, rows), reading_t.dtype)
    st = Stats()
    rc = getattr(lib(), "pmo_p2point_" + _sfx(reading_t.dtype))(
        rows, _p(reading_t), _p(ref), _p(dists), _p(ids), _p(w), k, C.c_int64(N), acc_mode,
        _p(dT), C.byref(st))
    return rc, dT, st


def _filters(filters):
    types = np.zeros(8, np.int32)
    params = np.zeros((8, 3), np.float64)
    for i, (name, p) in enumerate(filters):
        t = OF[name]
        types[i] = t
        for j, (pn, default) in enumerate(OF_PARAMS[t]):
            params[i, j] = float(p.get(pn, default))
    return types, params


def make_cfg(knn=1, max_dist=np.inf, method="kdtree", threads=1, filters=(("TrimmedDistOutlierFilter", {"ratio": 0.85}),),
             minimizer="PointToPlaneErrorMinimizer", counter_max=40, differential=None, acc_mode=0):
    cfg = Cfg()
    cfg.knn = knn
    cfg.maxDist = max_dist
    cfg.knn_method = 1 if method == "kdtree" else 0
    cfg.knn_threads = threads
    cfg.n_filters = len(filters)
    types, params = _filters(filters)
    for name, p in filters:
        if name == "RobustOutlierFilter":
            cfg.robust = make_robust(p)
    for i in range(8):
        cfg.filter_type[i] = int(types[i])
        for j in range(3):
            cfg.filter_p[i][j] = float(params[i, j])
    cfg.minimizer = MIN[minimizer]
    cfg.acc_mode = acc_mode
    cfg.counter_max = counter_max if counter_max is not None else -1
    if differential:
        cfg.diff_enabled = 1
        cfg.diff_rot = differential.get("minDiffRotErr", 0.001)
        cfg.diff_trans = differential.get("minDiffTransErr", 0.001)
        cfg.diff_smooth = int(differential.get("smoothLength", 3))
    return cfg


def icp(cfg, reading, reference, normals=None, T_init=None, trace=False, keep_robust=False):
    """reading, reference: (n, rows) arrays incl. homogeneous row.  Returns (rc, T, stats, trace).
    keep_robust: cfg.robust is one RobustOutlierFilter object kept across calls
    (pmo_icp_keep: its iteration count and scale are updated in cfg)."""
    dt = reference.dtype
    reading = np.ascontiguousarray(reading, dtype=dt)
    reference = np.ascontiguousarray(reference)
    rows = reading.shape[1]
    if T_init is None:
        T_init = np.eye(rows, dtype=dt)
    T_init = np.ascontiguousarray(T_init, dtype=dt)
    T_out = np.zeros((rows, rows), dt)
    st = Stats()
    maxit = max(cfg.counter_max, 1) if cfg.counter_max >= 0 else 4096
    tr = np.zeros((maxit, rows, rows), dt) if trace else None
    nrm = np.ascontiguousarray(normals, dtype=dt) if normals is not None else None
    rc = getattr(lib(), ("pmo_icp_keep_" if keep_robust else "pmo_icp_") + _sfx(dt))(
        C.byref(cfg), _p(reading), rows, C.c_int64(reading.shape[0]), _p(reference),
        C.c_int64(reference.shape[0]), _p(nrm), _p(T_init), _p(T_out), C.byref(st), _p(tr))
    if trace:
        tr = tr[: st.iterations]
    return rc, T_out, st, tr


def surface_normals(pts, k=5, max_dist=np.inf, threads=8, smooth=False):
    """SurfaceNormalDataPointsFilter restated (oracle/pmo_impl.inc).  pts: (n, rows).
    Returns a dict of point-major arrays and the degenerate count."""
    dt = pts.dtype
    pts = np.ascontiguousarray(pts)
    n, rows = pts.shape
    D = rows - 1
    out = {"normals": np.empty((n, D), dt), "densities": np.empty(n, dt), "eig_values": np.empty((n, D), dt),
           "eig_vectors": np.empty((n, D * D), dt), "matched_ids": np.empty((n, k), dt),
           "mean_dists": np.empty(n, dt)}
    deg = C.c_int64(0)
    f = getattr(lib(), "pmo_surface_normals_" + _sfx(dt))
    f.restype = C.c_int
    ct = C.c_float if dt == np.float32 else C.c_double
    rc = f(_p(pts), C.c_int(rows), C.c_int64(n), C.c_int(k), ct(max_dist), C.c_int(threads), C.c_int(int(smooth)),
           _p(out["normals"]), _p(out["densities"]), _p(out["eig_values"]), _p(out["eig_vectors"]),
           _p(out["matched_ids"]), _p(out["mean_dists"]), C.byref(deg))
    assert rc == OK, rc
    out["degenerate"] = deg.value
    return out


SSN_NORMALS, SSN_DENSITIES, SSN_EIGVALUES, SSN_EIGVECTORS, SSN_AVERAGE = 1, 2, 4, 8, 16


def sampling_surface_normals(pts, desc=None, knn=7, method=0, ratio=0.5, max_box=np.inf,
                             flags=SSN_NORMALS | SSN_AVERAGE):
    """SamplingSurfaceNormalDataPointsFilter restated (pmo_impl.inc).  pts (n, rows);
    desc (n, desc_dim) or None.  Returns a dict of the kept points' arrays."""
    pts = np.ascontiguousarray(pts)
    dt = pts.dtype
    n, rows = pts.shape
    D = rows - 1
    dd = 0 if desc is None else desc.shape[1]
    desc = None if desc is None else np.ascontiguousarray(desc, dtype=dt)
    out = {"features": np.zeros((n, rows), dt), "descriptors": np.zeros((n, dd), dt),
           "normals": np.zeros((n, D), dt), "densities": np.zeros(n, dt), "eig_values": np.zeros((n, D), dt),
           "eig_vectors": np.zeros((n, D * D), dt)}
    no = C.c_int64(0)
    unfit = C.c_int64(0)
    scal = C.c_float if dt == np.float32 else C.c_double
    f = getattr(lib(), "pmo_sampling_surface_normals_" + _sfx(dt))
    rc = f(_p(pts), rows, C.c_int64(n), _p(desc), dd, int(knn), int(method), scal(ratio), scal(max_box),
           C.c_uint(flags), _p(out["features"]), _p(out["descriptors"]), _p(out["normals"]), _p(out["densities"]),
           _p(out["eig_values"]), _p(out["eig_vectors"]), C.byref(no), C.byref(unfit))
    if rc != 0:
        raise RuntimeError(f"pmo_sampling_surface_normals failed ({rc})")
    m = no.value
    res = {k: v[:m] for k, v in out.items()}
    res["unfit"] = unfit.value
    return res


def voxel_grid(pts, desc=None, vsize=(1.0, 1.0, 1.0), use_centroid=True, average_desc=True):
    """VoxelGridDataPointsFilter restated (oracle/pmo_impl.inc).  Returns (features, descriptors)."""
    pts = np.ascontiguousarray(pts)
    dt = pts.dtype
    n, rows = pts.shape
    dd = 0 if desc is None else desc.shape[1]
    d = None if desc is None else np.ascontiguousarray(desc, dtype=dt)
    of = np.empty((n, rows), dt)
    od = np.empty((n, max(dd, 1)), dt)
    no = C.c_int64(0)
    vs = np.ascontiguousarray(vsize, dtype=np.float64)
    rc = getattr(lib(), "pmo_voxel_grid_" + _sfx(dt))(_p(pts), rows, C.c_int64(n), _p(d), dd, _p(vs),
                                                       1 if use_centroid else 0, 1 if average_desc else 0, _p(of),
                                                       _p(od), C.byref(no))
    if rc:
        raise ValueError(f"pmo_voxel_grid failed ({rc})")
    return of[:no.value], od[:no.value, :dd]
