"""ctypes binding of the C ABI in include/pmx.h (libpointmatcher_amd/lib/libpmx.so).

This is plumbing for Python callers (tests, bench, smoke): every call goes to
the HIP library.  There is no CPU fallback — if the library or a GPU is
missing, the calls raise.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIBDIR = os.path.join(HERE, "lib")
# PMX_LIB_VARIANT: a kernel-variant build under lib/<variant>/ (tuning
# experiments through this module only; the host chain links lib/libpmx.so)
LIBPMX = os.path.join(LIBDIR, os.environ.get("PMX_LIB_VARIANT", ""), "libpmx.so")
LIBPMX_ICP = os.path.join(LIBDIR, "libpmx_icp.so")

PMX_F32, PMX_F64 = 0, 1
PMX_OK = 0
PMX_E_NO_POINTS = -1
PMX_E_EMPTY_QUANTILE = -2
PMX_E_BAD_PARAM = -3
PMX_E_TRANSFORMATION = -4
PMX_E_CONVERGENCE = -5
PMX_E_HIP = -10
PMX_E_RCCL = -11
PMX_E_STATE = -12
PMX_E_NO_DEVICE = -13


class ConvergenceError(RuntimeError):
    """PointMatcher<T>::ConvergenceError (pointmatcher/PointMatcher.h:83-87)."""


class InvalidParameter(RuntimeError):
    """Parametrizable::InvalidParameter (pointmatcher/Parametrizable.h:101-104)."""


class TransformationError(RuntimeError):
    """TransformationError (pointmatcher/PointMatcher.h:148-151)."""


class PmxError(RuntimeError):
    pass


class Stats(C.Structure):
    _fields_ = [("kept", C.c_int64), ("nonzero_weights", C.c_int64),
                ("rejected_matches", C.c_int64), ("rejected_points", C.c_int64),
                ("sum_w", C.c_double), ("limit", C.c_double), ("n_total", C.c_int64),
                ("visited", C.c_int64), ("fallback_queries", C.c_int64)]

    def asdict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


# device-resident loop (pmx_loop_*)
FILTER_KIND = {"default": 0, "NullOutlierFilter": 1, "MaxDistOutlierFilter": 2, "MinDistOutlierFilter": 3,
               "MedianDistOutlierFilter": 4, "TrimmedDistOutlierFilter": 5, "VarTrimmedDistOutlierFilter": 6}
CHECK_KIND = {"CounterTransformationChecker": 0, "DifferentialTransformationChecker": 1,
              "BoundTransformationChecker": 2}


class LoopCfg(C.Structure):
    _fields_ = [("knn", C.c_int), ("max_dist", C.c_double), ("n_filters", C.c_int),
                ("filter_kind", C.c_int * 8), ("filter_p", (C.c_double * 3) * 8), ("minimizer", C.c_int),
                ("n_checkers", C.c_int), ("checker_kind", C.c_int * 8), ("checker_p", (C.c_double * 3) * 8),
                ("keep_trace", C.c_int),
                # PMX_FILTER_ROBUST (include/pmx.h)
                ("robust_fct", C.c_int), ("robust_estimator", C.c_int), ("robust_p2pl", C.c_int),
                ("robust_nb_iter_for_scale", C.c_int), ("robust_first_call", C.c_int),
                ("robust_tuning", C.c_double), ("robust_approx", C.c_double), ("robust_berg_target", C.c_double)]


class LoopStatus(C.Structure):
    _fields_ = [("iterations", C.c_int), ("done", C.c_int), ("reason", C.c_int), ("error", C.c_int),
                ("point_count_touched", C.c_int64), ("last", Stats), ("T_iter", C.c_double * 16),
                ("cond", (C.c_double * 2) * 8)]


# host-staged collectives (pmx_comm_init_host)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_int)
ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64)
COLL_F64, COLL_U32, COLL_U64 = 0, 1, 2
COLL_SUM, COLL_MAX = 0, 1
_COLL_CT = {COLL_F64: C.c_double, COLL_U32: C.c_uint32, COLL_U64: C.c_uint64}


class HostComm:
    """A transport for pmx_comm_init_host: allreduce(np_array, op) reduces the
    array in place over the ranks ("sum" / "max"), allgather(np_uint8_array)
    returns the nranks concatenated blocks.  The ctypes callbacks stay alive
    with this object (keep it referenced for the life of the context)."""

    def __init__(self, nranks, rank, allreduce, allgather):
        self.nranks, self.rank = nranks, rank
        self.errors = []
        self.calls = {"allreduce": 0, "allgather": 0}  # (callbacks made, every context on this transport)

        def _ar(user, buf, count, typ, op):
            self.calls["allreduce"] += 1
            try:
                a = np.ctypeslib.as_array(C.cast(buf, C.POINTER(_COLL_CT[typ])), shape=(count,))
                allreduce(a, "max" if op == COLL_MAX else "sum")
                return 0
            except Exception as e:  # (an exception must not cross the C frame)
                self.errors.append(repr(e))
                return 1

        def _ag(user, send, recv, nbytes):
            self.calls["allgather"] += 1
            try:
                a = np.ctypeslib.as_array(C.cast(send, C.POINTER(C.c_uint8)), shape=(nbytes,))
                out = np.ctypeslib.as_array(C.cast(recv, C.POINTER(C.c_uint8)), shape=(nbytes * nranks,))
                out[:] = allgather(a.copy())
                return 0
            except Exception as e:
                self.errors.append(repr(e))
                return 1

        self.ar = ALLREDUCE_FN(_ar)
        self.ag = ALLGATHER_FN(_ag)


def gloo_host_comm():
    """HostComm over the default torch.distributed process group (gloo on the
    CPU): the multi-rank test path on one GPU.  Integers travel as int64."""
    import torch
    import torch.distributed as dist

    def allreduce(a, op):
        t = torch.from_numpy(a.astype(np.float64) if a.dtype == np.float64 else a.astype(np.int64))
        dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
        a[:] = t.numpy().astype(a.dtype)

    def allgather(a):
        t = torch.from_numpy(a)
        outs = [torch.empty_like(t) for _ in range(dist.get_world_size())]
        dist.all_gather(outs, t)
        return torch.cat(outs).numpy()

    return HostComm(dist.get_world_size(), dist.get_rank(), allreduce, allgather)


_lib = None

EXPORTS = [
    "pmx_ctx_create", "pmx_ctx_destroy", "pmx_ctx_set_option", "pmx_last_error", "pmx_device_count", "pmx_version",
    "pmx_comm_unique_id", "pmx_comm_init", "pmx_comm_init_host", "pmx_comm_size", "pmx_comm_stats", "pmx_comm_loop_stats", "pmx_set_reference", "pmx_set_reference_centred", "pmx_set_reference_mean_centred", "pmx_set_reading", "pmx_set_search", "pmx_match",
    "pmx_outlier_default", "pmx_outlier_null", "pmx_outlier_maxdist", "pmx_outlier_mindist",
    "pmx_outlier_mediandist", "pmx_outlier_trimmed", "pmx_outlier_vartrimmed", "pmx_outlier_robust",
    "pmx_robust_scale", "pmx_set_reading_radii",
    "pmx_p2plane_system", "pmx_p2point_system", "pmx_get_matches", "pmx_get_weights", "pmx_vartrim_partial_sums",
    "pmx_get_shape", "pmx_grid_level_records", "pmx_timing_enable", "pmx_timing_read", "pmx_sync",
    "pmx_loop_begin", "pmx_loop_run", "pmx_loop_trace", "pmx_loop_select_stats", "pmx_loop_diag", "pmx_surface_normals",
    "pmx_sampling_surface_normals", "pmx_voxel_grid",
]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIBPMX):
            raise PmxError(f"{LIBPMX} not built (run __graft_entry__.build() or make -C libpointmatcher_amd)")
        l = C.CDLL(LIBPMX, mode=C.RTLD_GLOBAL)
        l.pmx_last_error.restype = C.c_char_p
        l.pmx_version.restype = C.c_char_p
        l.pmx_last_error.argtypes = [C.c_void_p]
        l.pmx_ctx_create.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_void_p)]
        l.pmx_ctx_destroy.argtypes = [C.c_void_p]
        l.pmx_ctx_set_option.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p]
        l.pmx_comm_unique_id.argtypes = [C.c_void_p]
        l.pmx_comm_init.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int]
        l.pmx_comm_init_host.argtypes = [C.c_void_p, C.c_int, C.c_int, ALLREDUCE_FN, ALLGATHER_FN, C.c_void_p]
        l.pmx_comm_size.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]
        l.pmx_comm_stats.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        l.pmx_comm_loop_stats.argtypes = [C.c_void_p] + [C.POINTER(C.c_uint64)] * 3
        l.pmx_set_reference.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int64, C.c_void_p]
        l.pmx_set_reference_centred.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int64, C.c_void_p, C.c_void_p]
        l.pmx_set_reference_mean_centred.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int64, C.c_void_p,
                                                     C.c_void_p]
        l.pmx_set_reading.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int64, C.c_void_p]
        l.pmx_set_search.argtypes = [C.c_void_p, C.c_int]
        l.pmx_match.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_double, C.c_double,
                                C.POINTER(C.c_uint64)]
        l.pmx_outlier_default.argtypes = [C.c_void_p]
        l.pmx_outlier_null.argtypes = [C.c_void_p, C.c_int]
        for f in ("maxdist", "mindist", "mediandist", "trimmed"):
            getattr(l, "pmx_outlier_" + f).argtypes = [C.c_void_p, C.c_int, C.c_double]
        l.pmx_outlier_vartrimmed.argtypes = [C.c_void_p, C.c_int, C.c_double, C.c_double, C.c_double]
        l.pmx_outlier_robust.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_double, C.c_double, C.c_int, C.c_double,
                                         C.c_int]
        l.pmx_robust_scale.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_double)]
        l.pmx_set_reading_radii.argtypes = [C.c_void_p, C.c_void_p]
        l.pmx_p2plane_system.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(Stats)]
        l.pmx_p2point_system.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                         C.POINTER(Stats)]
        l.pmx_get_matches.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        l.pmx_get_weights.argtypes = [C.c_void_p, C.c_void_p]
        l.pmx_vartrim_partial_sums.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.POINTER(C.c_int64)]
        l.pmx_get_shape.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int)]
        l.pmx_grid_level_records.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int64), C.c_void_p, C.c_void_p,
                                             C.c_void_p]
        l.pmx_timing_enable.argtypes = [C.c_void_p, C.c_int]
        l.pmx_timing_read.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_int64),
                                      C.POINTER(C.c_double)]
        l.pmx_sync.argtypes = [C.c_void_p]
        l.pmx_loop_begin.argtypes = [C.c_void_p, C.POINTER(LoopCfg), C.c_void_p]
        l.pmx_loop_run.argtypes = [C.c_void_p, C.c_int, C.POINTER(LoopStatus)]
        l.pmx_loop_trace.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p]
        l.pmx_loop_select_stats.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        l.pmx_loop_diag.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p]
        l.pmx_surface_normals.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int64, C.c_int, C.c_double,
                                          C.c_uint] + [C.c_void_p] * 6 + [C.POINTER(C.c_int64)]
        l.pmx_voxel_grid.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int64, C.c_void_p, C.c_int,
                                     C.POINTER(C.c_double), C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                     C.POINTER(C.c_int64)]
        l.pmx_sampling_surface_normals.argtypes = ([C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int64, C.c_void_p,
                                                    C.c_int, C.c_int, C.c_int, C.c_double, C.c_double, C.c_uint]
                                                   + [C.c_void_p] * 6 + [C.POINTER(C.c_int64)] * 2)
        _lib = l
    return _lib


def device_count():
    return lib().pmx_device_count()


PMX_SN_SMOOTH = 1


def surface_normals(points, knn=5, max_dist=np.inf, smooth=False, device=0):
    """SurfaceNormalDataPointsFilter (DataPointsFilters/SurfaceNormal.cpp:80-290) on
    the GPU (pmx_surface_normals).  points: (n, rows) float32/float64 with the
    homogeneous row last.  Returns a dict of point-major arrays: normals (n, D),
    densities (n,), eig_values (n, D), eig_vectors (n, D*D), matched_ids (n, knn),
    mean_dists (n,), and the degenerate count."""
    pts = np.ascontiguousarray(points)
    if pts.dtype not in (np.float32, np.float64):
        pts = pts.astype(np.float32)
    n, rows = pts.shape
    D = rows - 1
    dt = pts.dtype
    out = {"normals": np.empty((n, D), dt), "densities": np.empty(n, dt), "eig_values": np.empty((n, D), dt),
           "eig_vectors": np.empty((n, D * D), dt), "matched_ids": np.empty((n, knn), dt),
           "mean_dists": np.empty(n, dt)}
    deg = C.c_int64(0)
    l = lib()
    rc = l.pmx_surface_normals(int(device), PMX_F64 if dt == np.float64 else PMX_F32, _ptr(pts), rows, n, int(knn),
                               float(max_dist), PMX_SN_SMOOTH if smooth else 0, _ptr(out["normals"]),
                               _ptr(out["densities"]), _ptr(out["eig_values"]), _ptr(out["eig_vectors"]),
                               _ptr(out["matched_ids"]), _ptr(out["mean_dists"]), C.byref(deg))
    if rc != PMX_OK:
        raise_for(rc, l.pmx_last_error(None).decode())
    out["degenerate"] = deg.value
    return out


SSN_NORMALS, SSN_DENSITIES, SSN_EIGVALUES, SSN_EIGVECTORS, SSN_AVERAGE = 1, 2, 4, 8, 16
# RobustOutlierFilter functions / scale modes of one call (include/pmx.h PMX_RF_*, PMX_RS_*)
ROBUST_FCT = {"cauchy": 0, "welsch": 1, "sc": 2, "gm": 3, "tukey": 4, "huber": 5, "L1": 6, "student": 7}
RS_NONE, RS_MAD, RS_STD, RS_BERG_FIRST, RS_BERG_NEXT, RS_KEEP = range(6)


def sampling_surface_normals(points, descriptors=None, knn=7, sampling_method=0, ratio=0.5, max_box_dim=np.inf,
                             flags=SSN_NORMALS | SSN_AVERAGE, device=0):
    """SamplingSurfaceNormalDataPointsFilter (DataPointsFilters/SamplingSurfaceNormal.cpp:80-342)
    on the GPU (pmx_sampling_surface_normals).  points (n, rows) with the
    homogeneous row last; descriptors (n, desc_dim) or None.  Returns the kept
    points' features, descriptors, normals, densities, eig_values,
    eig_vectors (point-major) and the unfit count."""
    pts = np.ascontiguousarray(points)
    if pts.dtype not in (np.float32, np.float64):
        pts = pts.astype(np.float32)
    dt = pts.dtype
    n, rows = pts.shape
    D = rows - 1
    dd = 0 if descriptors is None else descriptors.shape[1]
    desc = None if descriptors is None else np.ascontiguousarray(descriptors, dtype=dt)
    out = {"features": np.empty((n, rows), dt), "descriptors": np.empty((n, dd), dt),
           "normals": np.empty((n, D), dt), "densities": np.empty(n, dt), "eig_values": np.empty((n, D), dt),
           "eig_vectors": np.empty((n, D * D), dt)}
    no, unfit = C.c_int64(0), C.c_int64(0)
    l = lib()
    rc = l.pmx_sampling_surface_normals(int(device), PMX_F64 if dt == np.float64 else PMX_F32, _ptr(pts), rows, n,
                                        _ptr(desc), dd, int(knn), int(sampling_method), float(ratio),
                                        float(max_box_dim), int(flags), _ptr(out["features"]),
                                        _ptr(out["descriptors"]) if dd else None, _ptr(out["normals"]),
                                        _ptr(out["densities"]), _ptr(out["eig_values"]), _ptr(out["eig_vectors"]),
                                        C.byref(no), C.byref(unfit))
    if rc != PMX_OK:
        raise_for(rc, l.pmx_last_error(None).decode())
    m = no.value
    res = {k: v[:m] for k, v in out.items()}
    res["unfit"] = unfit.value
    return res


def voxel_grid(points, descriptors=None, vsize=(1.0, 1.0, 1.0), use_centroid=True, average_descriptors=True,
               device=0):
    """VoxelGridDataPointsFilter (DataPointsFilters/VoxelGrid.cpp:60-343) on the
    GPU (pmx_voxel_grid).  points (n, rows) with the homogeneous row last;
    descriptors (n, desc_dim) or None.  Returns (features, descriptors) of
    the kept points, in index order."""
    pts = np.ascontiguousarray(points)
    if pts.dtype not in (np.float32, np.float64):
        pts = pts.astype(np.float32)
    dt = pts.dtype
    n, rows = pts.shape
    dd = 0 if descriptors is None else descriptors.shape[1]
    desc = None if descriptors is None else np.ascontiguousarray(descriptors, dtype=dt)
    of = np.empty((n, rows), dt)
    od = np.empty((n, dd), dt)
    vs = (C.c_double * 3)(*[float(v) for v in vsize])
    no = C.c_int64(0)
    l = lib()
    rc = l.pmx_voxel_grid(int(device), PMX_F64 if dt == np.float64 else PMX_F32, _ptr(pts), rows, n, _ptr(desc), dd,
                          vs, 1 if use_centroid else 0, 1 if average_descriptors else 0, _ptr(of),
                          _ptr(od) if dd else None, C.byref(no))
    if rc != PMX_OK:
        raise_for(rc, l.pmx_last_error(None).decode())
    return of[:no.value], od[:no.value]


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def raise_for(code, msg=""):
    if code == PMX_OK:
        return
    if code in (PMX_E_NO_POINTS, PMX_E_EMPTY_QUANTILE, PMX_E_CONVERGENCE):
        raise ConvergenceError(msg)
    if code == PMX_E_BAD_PARAM:
        raise InvalidParameter(msg)
    if code == PMX_E_TRANSFORMATION:
        raise TransformationError(msg)
    raise PmxError(f"pmx error {code}: {msg}")


class Context:
    """One device context (one ICP object / one rank)."""

    def __init__(self, device=0, dtype=np.float32):
        self.dtype = np.dtype(dtype)
        self._l = lib()
        h = C.c_void_p()
        rc = self._l.pmx_ctx_create(device, PMX_F64 if self.dtype == np.float64 else PMX_F32, C.byref(h))
        if rc != PMX_OK:
            raise PmxError(f"pmx_ctx_create failed ({rc}: {self._l.pmx_last_error(None).decode()}); "
                           f"visible HIP devices: {device_count()}")
        self.h = h
        self.rows = None
        self.knn = None
        self.N = 0

    def set_option(self, name, value):
        """One developer option (README "Options"; pmx_ctx_set_option)."""
        self._chk(self._l.pmx_ctx_set_option(self.h, str(name).encode(), str(value).encode()))

    def level_records(self, level, normals=True):
        """Grid level `level`'s records (pmx_grid_level_records): original
        reference ids, points (n, 4) and, with normals, normals (n, 4)."""
        n = C.c_int64(0)
        self._chk(self._l.pmx_grid_level_records(self.h, int(level), C.byref(n), None, None, None))
        ids = np.zeros(n.value, np.int32)
        pts = np.zeros((n.value, 4), self.dtype)
        nrm = np.zeros((n.value, 4), self.dtype) if normals else None
        self._chk(self._l.pmx_grid_level_records(self.h, int(level), C.byref(n), _ptr(ids), _ptr(pts),
                                                 _ptr(nrm) if normals else None))
        return ids, pts, nrm

    def close(self):
        if self.h:
            self._l.pmx_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc):
        if rc != PMX_OK:
            raise_for(rc, self._l.pmx_last_error(self.h).decode())

    def _arr(self, a):
        return np.ascontiguousarray(a, dtype=self.dtype)

    # --- multi-GPU
    @staticmethod
    def unique_id():
        buf = (C.c_char * 128)()
        rc = lib().pmx_comm_unique_id(buf)
        if rc != PMX_OK:
            raise PmxError(f"pmx_comm_unique_id failed ({rc})")
        return bytes(buf)

    def comm_init(self, uid: bytes, nranks: int, rank: int):
        buf = (C.c_char * 128).from_buffer_copy(uid)
        self._chk(self._l.pmx_comm_init(self.h, buf, nranks, rank))

    def comm_init_host(self, comm: HostComm):
        self._comm = comm  # (the callbacks must outlive the context)
        self._chk(self._l.pmx_comm_init_host(self.h, comm.nranks, comm.rank, comm.ar, comm.ag, None))

    def comm_size(self):
        n, r, k = C.c_int(), C.c_int(), C.c_int()
        self._chk(self._l.pmx_comm_size(self.h, C.byref(n), C.byref(r), C.byref(k)))
        return n.value, r.value, k.value

    def comm_stats(self):
        """(all-reduces, all-gathers) this context has issued (pmx_comm_stats)."""
        a, g = C.c_uint64(), C.c_uint64()
        self._chk(self._l.pmx_comm_stats(self.h, C.byref(a), C.byref(g)))
        return a.value, g.value

    def comm_loop_stats(self):
        """(verdict syncs, async iterations, stalls) of the sharded device loop (pmx_comm_loop_stats)."""
        v, a, st = C.c_uint64(), C.c_uint64(), C.c_uint64()
        self._chk(self._l.pmx_comm_loop_stats(self.h, C.byref(v), C.byref(a), C.byref(st)))
        return v.value, a.value, st.value

    # --- clouds
    def set_reference(self, feat, normals=None):
        feat = self._arr(feat)
        nrm = self._arr(normals) if normals is not None else None
        self.rows = feat.shape[1]
        self._ref_keep = (feat, nrm)
        self._chk(self._l.pmx_set_reference(self.h, _ptr(feat), feat.shape[1], feat.shape[0], _ptr(nrm)))

    def set_reading(self, feat, T0=None):
        feat = self._arr(feat)
        rows = feat.shape[1]
        T0 = self._arr(np.eye(rows) if T0 is None else T0)
        self.N = feat.shape[0]
        self._chk(self._l.pmx_set_reading(self.h, _ptr(feat), rows, feat.shape[0], _ptr(T0)))

    def set_reading_radii(self, radii):
        """KDTreeVarDistMatcher: one search radius per reading point (None clears)."""
        r = self._arr(radii) if radii is not None else None
        self._chk(self._l.pmx_set_reading_radii(self.h, _ptr(r) if r is not None else None))

    # --- per-iteration
    def set_search(self, search_type: int):
        """0 = brute force, 1/2 = exact grid search (KDTreeMatcher searchType)."""
        self._chk(self._l.pmx_set_search(self.h, int(search_type)))

    def match(self, T, knn=1, max_dist=np.inf, epsilon=0.0):
        T = self._arr(T)
        v = C.c_uint64(0)
        self._chk(self._l.pmx_match(self.h, _ptr(T), knn, float(max_dist), float(epsilon), C.byref(v)))
        self.knn = knn
        return v.value

    def outlier_default(self):
        self._chk(self._l.pmx_outlier_default(self.h))

    def outlier(self, name, pos=0, **p):
        l, h = self._l, self.h
        if name == "NullOutlierFilter":
            rc = l.pmx_outlier_null(h, pos)
        elif name == "MaxDistOutlierFilter":
            rc = l.pmx_outlier_maxdist(h, pos, float(p.get("maxDist", 1.0)))
        elif name == "MinDistOutlierFilter":
            rc = l.pmx_outlier_mindist(h, pos, float(p.get("minDist", 1.0)))
        elif name == "MedianDistOutlierFilter":
            rc = l.pmx_outlier_mediandist(h, pos, float(p.get("factor", 3.0)))
        elif name == "TrimmedDistOutlierFilter":
            rc = l.pmx_outlier_trimmed(h, pos, float(p.get("ratio", 0.85)))
        elif name == "VarTrimmedDistOutlierFilter":
            rc = l.pmx_outlier_vartrimmed(h, pos, float(p.get("minRatio", 0.05)),
                                          float(p.get("maxRatio", 0.99)), float(p.get("lambda", 2.35)))
        else:
            raise InvalidParameter(f"unknown outlier filter {name}")
        self._chk(rc)

    def outlier_robust(self, pos=0, fct="cauchy", tuning=1.0, approximation=np.inf, scale_mode=RS_MAD,
                       berg_target=0.0, point2plane=False):
        """One RobustOutlierFilter call with the scale mode given (the filter's
        iteration schedule is the caller's, as libpointmatcher_amd.icp does)."""
        self._chk(self._l.pmx_outlier_robust(self.h, pos, ROBUST_FCT[fct], float(tuning), float(approximation),
                                             int(scale_mode), float(berg_target), 1 if point2plane else 0))

    def robust_scale(self, pos=0):
        v = C.c_double()
        self._chk(self._l.pmx_robust_scale(self.h, pos, C.byref(v)))
        return v.value

    def p2plane_system(self):
        n = 6 if self.rows == 4 else 3
        A = np.zeros(n * n)
        b = np.zeros(n)
        st = Stats()
        self._chk(self._l.pmx_p2plane_system(self.h, _ptr(A), _ptr(b), C.byref(st)))
        return A.reshape(n, n), b, st

    def p2point_system(self):
        D = self.rows - 1
        mp = np.zeros(D)
        mq = np.zeros(D)
        m = np.zeros(D * D)
        st = Stats()
        self._chk(self._l.pmx_p2point_system(self.h, _ptr(mp), _ptr(mq), _ptr(m), C.byref(st)))
        return mp, mq, m.reshape(D, D), st

    def get_matches(self):
        d = np.empty((self.N, self.knn), self.dtype)
        i = np.empty((self.N, self.knn), np.int32)
        self._chk(self._l.pmx_get_matches(self.h, _ptr(d), _ptr(i)))
        return d, i

    def get_weights(self):
        w = np.empty((self.N, self.knn), self.dtype)
        self._chk(self._l.pmx_get_weights(self.h, _ptr(w)))
        return w

    def vartrim_partial_sums(self):
        """The last VarTrimmedDist filter's partial sums (diagnostic)."""
        n = C.c_int64(0)
        self._chk(self._l.pmx_vartrim_partial_sums(self.h, None, 0, C.byref(n)))
        out = np.empty(n.value, self.dtype)
        self._chk(self._l.pmx_vartrim_partial_sums(self.h, _ptr(out), out.size, C.byref(n)))
        return out

    # --- timing
    def timing(self, on=True):
        self._chk(self._l.pmx_timing_enable(self.h, 1 if on else 0))

    def timing_read(self):
        ms = C.c_double()
        n = C.c_int64()
        o = C.c_double()
        self._chk(self._l.pmx_timing_read(self.h, C.byref(ms), C.byref(n), C.byref(o)))
        return ms.value, n.value

    def sync(self):
        self._chk(self._l.pmx_sync(self.h))

    # --- device-resident loop
    def loop_begin(self, knn=1, max_dist=np.inf, filters=(), minimizer="PointToPlaneErrorMinimizer",
                   checkers=(), T0=None, keep_trace=False):
        """filters: [(name, params...)], checkers: [(name, params...)] in chain order
        (Counter: max; Differential: rot, trans, smoothLength; Bound: rot, trans)."""
        cfg = LoopCfg()
        cfg.knn = knn
        cfg.max_dist = float(max_dist)
        cfg.n_filters = len(filters)
        for i, (name, *p) in enumerate(filters):
            cfg.filter_kind[i] = FILTER_KIND[name]
            for j, v in enumerate(p):
                cfg.filter_p[i][j] = float(v)
        cfg.minimizer = 0 if minimizer.startswith("PointToPlane") else 1
        cfg.n_checkers = len(checkers)
        for i, (name, *p) in enumerate(checkers):
            cfg.checker_kind[i] = CHECK_KIND[name]
            for j, v in enumerate(p):
                cfg.checker_p[i][j] = float(v)
        cfg.keep_trace = 1 if keep_trace else 0
        T0 = self._arr(np.eye(self.rows) if T0 is None else T0)
        self._loop_keep = cfg
        self._chk(self._l.pmx_loop_begin(self.h, C.byref(cfg), _ptr(T0)))

    def loop_run(self, n):
        """Run up to n iterations; returns the status (raises the ICP's exception)."""
        st = LoopStatus()
        rc = self._l.pmx_loop_run(self.h, int(n), C.byref(st))
        self.last_loop_status = st
        self._chk(rc)
        return st

    def loop_select_stats(self):
        """(window hits, radix fallbacks) of the fused quantile window (pmx_spec.h)."""
        h, m = C.c_uint64(), C.c_uint64()
        self._chk(self._l.pmx_loop_select_stats(self.h, C.byref(h), C.byref(m)))
        return h.value, m.value

    def loop_diag(self, first, count):
        """Per-iteration diagnostics of the current loop (pmx_loop_diag): int64
        rows (grid level, window verdict 1/0/-1, pairs evaluated, full searches)."""
        out = np.zeros((count, 4), np.int64)
        self._chk(self._l.pmx_loop_diag(self.h, int(first), int(count), _ptr(out)))
        return out

    def loop_T(self, st):
        r = self.rows
        return np.array(st.T_iter[:r * r], dtype=self.dtype).reshape(r, r)

    def loop_trace(self, first, count):
        r = self.rows
        out = np.empty((count, r, r), self.dtype)
        self._chk(self._l.pmx_loop_trace(self.h, int(first), int(count), _ptr(out)))
        return out
