"""ctypes binding of the host ICP chain (include/pmx_icp.h, lib/libpmx_icp.so).

    icp = ICP(np.float32)
    icp.load_yaml(open("chain.yaml").read())     # or icp.set_default()
    T = icp.compute(reading, reference, ref_normals)

Clouds are (n, rows) arrays with the homogeneous row last (rows = D + 1) —
the memory layout of the reference's column-major (D+1) x n features.
Errors raise the Python mirrors of the reference exception types.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _capi
from ._capi import ConvergenceError, InvalidParameter, TransformationError

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "lib", os.environ.get("PMX_LIB_VARIANT", ""), "libpmx_icp.so")  # (variant: _capi.py)


class InvalidElement(RuntimeError):
    """InvalidElement (pointmatcher/Registrar.h:69-72): unknown module name."""


class InvalidModuleType(RuntimeError):
    """ICPChainBase::InvalidModuleType (pointmatcher/ICP.cpp:158-166)."""


class ConfigurationError(RuntimeError):
    """PointMatcherSupport::ConfigurationError / YAML syntax."""


_ERR = {-1: ConvergenceError, -3: InvalidParameter, -4: TransformationError, -5: InvalidElement,
        -6: InvalidModuleType, -7: ConfigurationError, -10: RuntimeError}


class IcpStats(C.Structure):
    _fields_ = [("iterations", C.c_int64), ("point_count_touched", C.c_int64),
                ("overlap_ratio", C.c_double), ("point_used_ratio", C.c_double), ("kept", C.c_int64),
                ("rejected_matches", C.c_int64), ("rejected_points", C.c_int64),
                ("convergence_duration", C.c_double), ("reference_preprocessing_duration", C.c_double),
                ("reading_preprocessing_duration", C.c_double), ("max_iterations_reached", C.c_int)]

    def asdict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


_lib = None


def lib():
    global _lib
    if _lib is None:
        _capi.lib()  # libpmx.so first (RTLD_GLOBAL)
        if not os.path.exists(LIB):
            raise _capi.PmxError(f"{LIB} not built")
        l = C.CDLL(LIB)
        l.pmx_icp_create.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_void_p)]
        l.pmx_icp_destroy.argtypes = [C.c_void_p]
        l.pmx_icp_last_error.argtypes = [C.c_void_p]
        l.pmx_icp_last_error.restype = C.c_char_p
        l.pmx_icp_set_default.argtypes = [C.c_void_p]
        l.pmx_icp_load_yaml.argtypes = [C.c_void_p, C.c_char_p]
        l.pmx_icp_comm_init.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int]
        l.pmx_icp_comm_init_host.argtypes = [C.c_void_p, C.c_int, C.c_int, _capi.ALLREDUCE_FN, _capi.ALLGATHER_FN,
                                             C.c_void_p]
        l.pmx_icp_keep_trace.argtypes = [C.c_void_p, C.c_int]
        l.pmx_icp_add_descriptor.argtypes = [C.c_void_p, C.c_int, C.c_char_p, C.c_int, C.c_void_p, C.c_int64]
        l.pmx_cloud_load.argtypes = [C.c_char_p, C.c_int, C.POINTER(C.c_void_p)]
        l.pmx_cloud_destroy.argtypes = [C.c_void_p]
        l.pmx_cloud_last_error.restype = C.c_char_p
        l.pmx_cloud_info.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int), C.POINTER(C.c_int),
                                     C.POINTER(C.c_int), C.POINTER(C.c_int)]
        l.pmx_cloud_label.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_char_p, C.c_int, C.POINTER(C.c_int)]
        l.pmx_cloud_data.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        l.pmx_icp_compute.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int64, C.c_void_p, C.c_int64,
                                      C.c_void_p, C.c_void_p, C.c_void_p]
        l.pmx_icp_prepare.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int64, C.c_void_p, C.c_int64,
                                      C.c_void_p, C.c_void_p]
        l.pmx_icp_iterate.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int)]
        l.pmx_icp_finish.argtypes = [C.c_void_p, C.c_void_p]
        l.pmx_icp_stats_get.argtypes = [C.c_void_p, C.POINTER(IcpStats)]
        l.pmx_icp_trace_get.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        l.pmx_icp_timing.argtypes = [C.c_void_p, C.c_int]
        l.pmx_icp_timing_read.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_int64)]
        l.pmx_icp_select_stats.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        l.pmx_icp_comm_stats.argtypes = [C.c_void_p] + [C.POINTER(C.c_uint64)] * 5
        l.pmx_icp_loop_diag.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p]
        l.pmx_icp_set_map.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int64, C.c_void_p, C.POINTER(C.c_int)]
        l.pmx_icp_clear_map.argtypes = [C.c_void_p]
        l.pmx_icp_has_map.argtypes = [C.c_void_p, C.POINTER(C.c_int)]
        l.pmx_icp_get_map.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.POINTER(C.c_int64), C.POINTER(C.c_int)]
        l.pmx_icp_sequence_prepare.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int64, C.c_void_p,
                                               C.POINTER(C.c_int)]
        l.pmx_icp_sequence_compute.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int64, C.c_void_p, C.c_void_p]
        _lib = l
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


class Cloud:
    """DataPoints loaded from a .csv / .vtk file (DataPoints::load, IO.cpp:374-389)."""

    def __init__(self, features, feature_labels, descriptors, descriptor_labels):
        self.features = features                  # (n, rows), homogeneous row last
        self.feature_labels = feature_labels      # [(name, span)]
        self.descriptors = descriptors            # (n, desc_dim)
        self.descriptor_labels = descriptor_labels

    def descriptor(self, name):
        off = 0
        for lab, span in self.descriptor_labels:
            if lab == name:
                return self.descriptors[:, off:off + span]
            off += span
        raise KeyError(name)

    def descriptor_exists(self, name):
        return any(lab == name for lab, _ in self.descriptor_labels)


def load_cloud(path, dtype=np.float32):
    l = lib()
    dt = np.dtype(dtype)
    h = C.c_void_p()
    rc = l.pmx_cloud_load(str(path).encode(), 1 if dt == np.float64 else 0, C.byref(h))
    if rc:
        raise _ERR.get(rc, RuntimeError)(l.pmx_cloud_last_error().decode())
    try:
        n, rows, dd, nfl, ndl = C.c_int64(), C.c_int(), C.c_int(), C.c_int(), C.c_int()
        l.pmx_cloud_info(h, C.byref(n), C.byref(rows), C.byref(dd), C.byref(nfl), C.byref(ndl))
        labels = []
        for which, cnt in ((0, nfl.value), (1, ndl.value)):
            ls = []
            for i in range(cnt):
                buf = C.create_string_buffer(256)
                span = C.c_int()
                l.pmx_cloud_label(h, which, i, buf, 256, C.byref(span))
                ls.append((buf.value.decode(), span.value))
            labels.append(ls)
        f = np.empty((n.value, rows.value), dt)
        d = np.empty((n.value, dd.value), dt)
        l.pmx_cloud_data(h, _p(f), _p(d) if dd.value else None)
        return Cloud(f, labels[0], d, labels[1])
    finally:
        l.pmx_cloud_destroy(h)


class ICP:
    """PointMatcher<T>::ICP on the MI355X path (one object per rank / thread)."""

    def __init__(self, dtype=np.float32, device=0):
        self.dtype = np.dtype(dtype)
        self._l = lib()
        h = C.c_void_p()
        rc = self._l.pmx_icp_create(1 if self.dtype == np.float64 else 0, device, C.byref(h))
        if rc:
            raise RuntimeError("pmx_icp_create failed")
        self.h = h
        self.rows = None

    def close(self):
        if getattr(self, "h", None):
            self._l.pmx_icp_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc):
        if rc:
            msg = self._l.pmx_icp_last_error(self.h).decode()
            raise _ERR.get(rc, RuntimeError)(msg)

    # --- configuration
    def set_default(self):
        self._chk(self._l.pmx_icp_set_default(self.h))

    def load_yaml(self, text: str):
        self._chk(self._l.pmx_icp_load_yaml(self.h, text.encode()))

    def comm_init(self, uid: bytes, nranks: int, rank: int):
        buf = (C.c_char * 128).from_buffer_copy(uid)
        self._chk(self._l.pmx_icp_comm_init(self.h, buf, nranks, rank))

    def comm_init_host(self, comm):
        """Multi-rank over a _capi.HostComm (e.g. _capi.gloo_host_comm())."""
        self._comm = comm  # (the callbacks must outlive the ICP object)
        self._chk(self._l.pmx_icp_comm_init_host(self.h, comm.nranks, comm.rank, comm.ar, comm.ag, None))

    def keep_trace(self, on=True):
        self._chk(self._l.pmx_icp_keep_trace(self.h, 1 if on else 0))

    def add_descriptor(self, cloud, name, values):
        """Stage a descriptor (n,) or (n, span) for the next compute / prepare;
        cloud: "reading" or "reference" (e.g. the reading's "maxSearchDist"
        of KDTreeVarDistMatcher)."""
        if cloud not in ("reading", "reference"):
            raise ValueError(f'cloud must be "reading" or "reference", not {cloud!r}')
        v = np.ascontiguousarray(values, dtype=self.dtype)
        span = 1 if v.ndim == 1 else v.shape[1]
        self._chk(self._l.pmx_icp_add_descriptor(self.h, 0 if cloud == "reading" else 1, name.encode(), span, _p(v),
                                                 v.shape[0]))

    # --- run
    def _args(self, reading, reference, normals, T_init):
        rd = np.ascontiguousarray(reading, dtype=self.dtype)
        ref = np.ascontiguousarray(reference, dtype=self.dtype)
        nrm = np.ascontiguousarray(normals, dtype=self.dtype) if normals is not None else None
        rows = rd.shape[1]
        if ref.shape[1] != rows:
            raise ValueError("reading and reference must have the same number of rows")
        Ti = np.ascontiguousarray(np.eye(rows) if T_init is None else T_init, dtype=self.dtype)
        self.rows = rows
        self._keep = (rd, ref, nrm, Ti)
        return rd, ref, nrm, Ti, rows

    def compute(self, reading, reference, normals=None, T_init=None):
        rd, ref, nrm, Ti, rows = self._args(reading, reference, normals, T_init)
        out = np.zeros((rows, rows), self.dtype)
        self._chk(self._l.pmx_icp_compute(self.h, _p(rd), rows, rd.shape[0], _p(ref), ref.shape[0], _p(nrm),
                                          _p(Ti), _p(out)))
        return out

    __call__ = compute

    def prepare(self, reading, reference, normals=None, T_init=None):
        rd, ref, nrm, Ti, rows = self._args(reading, reference, normals, T_init)
        self._chk(self._l.pmx_icp_prepare(self.h, _p(rd), rows, rd.shape[0], _p(ref), ref.shape[0], _p(nrm),
                                          _p(Ti)))

    def iterate(self, n=1):
        done = C.c_int(0)
        self._chk(self._l.pmx_icp_iterate(self.h, n, C.byref(done)))
        return bool(done.value)

    def finish(self):
        out = np.zeros((self.rows, self.rows), self.dtype)
        self._chk(self._l.pmx_icp_finish(self.h, _p(out)))
        return out

    # --- introspection
    def stats(self):
        s = IcpStats()
        self._l.pmx_icp_stats_get(self.h, C.byref(s))
        return s

    def trace(self, max_iters=100000):
        it = self.stats().iterations
        out = np.zeros((max(it, 1), self.rows, self.rows), self.dtype)
        n = self._l.pmx_icp_trace_get(self.h, _p(out), min(it, max_iters))
        return out[:n]

    def timing(self, on=True):
        self._chk(self._l.pmx_icp_timing(self.h, 1 if on else 0))

    def select_stats(self):
        """(window hits, window misses) of the device loop since the last prepare."""
        h, m = C.c_uint64(), C.c_uint64()
        self._chk(self._l.pmx_icp_select_stats(self.h, C.byref(h), C.byref(m)))
        return h.value, m.value

    def loop_diag(self, first, count):
        """Per-iteration diagnostics of the device loop since the last prepare
        (pmx_icp_loop_diag): int64 rows [grid level, window verdict (1 hit, 0
        radix passes, -1 no window), pairs evaluated, full searches]."""
        out = np.zeros((count, 4), np.int64)
        self._chk(self._l.pmx_icp_loop_diag(self.h, int(first), int(count), out.ctypes.data_as(C.c_void_p)))
        return out

    def comm_stats(self):
        """Multi-rank diagnostics since creation: {allreduces, allgathers, verdict_syncs,
        async_iterations, stalls} (pmx_icp_comm_stats)."""
        v = [C.c_uint64() for _ in range(5)]
        self._chk(self._l.pmx_icp_comm_stats(self.h, *[C.byref(x) for x in v]))
        keys = ("allreduces", "allgathers", "verdict_syncs", "async_iterations", "stalls")
        return dict(zip(keys, (x.value for x in v)))

    def timing_read(self):
        ms = C.c_double()
        n = C.c_int64()
        self._chk(self._l.pmx_icp_timing_read(self.h, C.byref(ms), C.byref(n)))
        return ms.value, n.value


class ICPSequence(ICP):
    """PointMatcher<T>::ICPSequence (PointMatcher.h:730-764, ICP.cpp:455-609):
    the map is centred, filtered and indexed once by set_map and stays on the
    device; compute(reading, T_init) matches each new reading against it."""

    def set_map(self, cloud, normals=None):
        """ICPSequence::setMap; False for an empty cloud (ignored)."""
        m = np.ascontiguousarray(cloud, dtype=self.dtype)
        nrm = np.ascontiguousarray(normals, dtype=self.dtype) if normals is not None else None
        ok = C.c_int(0)
        self._chk(self._l.pmx_icp_set_map(self.h, _p(m), m.shape[1], m.shape[0], _p(nrm), C.byref(ok)))
        return bool(ok.value)

    def clear_map(self):
        self._chk(self._l.pmx_icp_clear_map(self.h))

    def has_map(self):
        h = C.c_int(0)
        self._chk(self._l.pmx_icp_has_map(self.h, C.byref(h)))
        return bool(h.value)

    def get_map(self):
        """The prefiltered map in global coordinates (getPrefilteredMap), (n, rows)."""
        n = C.c_int64(0)
        rows = C.c_int(0)
        self._chk(self._l.pmx_icp_get_map(self.h, None, 0, C.byref(n), C.byref(rows)))
        out = np.zeros((n.value, rows.value), self.dtype)  # (sized by the library: the held map's rows)
        self._chk(self._l.pmx_icp_get_map(self.h, _p(out), out.size, C.byref(n), C.byref(rows)))
        return out

    def _rd(self, reading, T_init):
        rd = np.ascontiguousarray(reading, dtype=self.dtype)
        rows = rd.shape[1]
        Ti = np.ascontiguousarray(np.eye(rows) if T_init is None else T_init, dtype=self.dtype)
        self.rows = rows
        self._keep = (rd, Ti)
        return rd, Ti, rows

    def compute(self, reading, T_init=None):
        """ICPSequence::compute(cloudIn, T_refIn_dataIn); identity without a map."""
        rd, Ti, rows = self._rd(reading, T_init)
        out = np.zeros((rows, rows), self.dtype)
        self._chk(self._l.pmx_icp_sequence_compute(self.h, _p(rd), rows, rd.shape[0], _p(Ti), _p(out)))
        return out

    __call__ = compute

    def prepare(self, reading, T_init=None):
        """The first phase of compute (then iterate / finish); False without a map."""
        rd, Ti, rows = self._rd(reading, T_init)
        ok = C.c_int(0)
        self._chk(self._l.pmx_icp_sequence_prepare(self.h, _p(rd), rows, rd.shape[0], _p(Ti), C.byref(ok)))
        return bool(ok.value)

    def compute_with_reference(self, reading, reference, normals=None, T_init=None):
        """ICP::compute on this object (the map is re-indexed by the next sequence compute)."""
        return ICP.compute(self, reading, reference, normals, T_init)
