"""ICPSequence with a resident map (PointMatcher.h:730-764, ICP.cpp:455-609).

Ten scans registered one after the other against one map (set once: centred,
filtered and indexed on the device), each initialised with the previous
scan's result, as an odometry front end does.  Bars:
  * every scan's T equals a plain ICP::compute of the same reading against the
    map with the same T_init, bit for bit (the same centring: no reference
    filters, so the map mean equals the filtered reference's mean);
  * every scan's T equals the oracle ICP (1e-5 f32 / 1e-12 f64 Frobenius) with
    the same iteration count;
  * hasMap / getPrefilteredMap / clearMap (identity without a map) and a
    chain reload that re-indexes the held map (ICP.cpp:520-539).
"""
import numpy as np
import pytest

from helpers import chain_yaml
from libpointmatcher_amd.icp import ICP, ICPSequence
from libpointmatcher_amd.synth import reading_cloud, reference_cloud

pytestmark = pytest.mark.gpu

DIFF = dict(minDiffRotErr=0.001, minDiffTransErr=0.01, smoothLength=4)
FILTERS = (("TrimmedDistOutlierFilter", {"ratio": 0.85}),)
TOL = {"float32": 1e-5, "float64": 1e-12}


def _pose(i):
    """The sensor's drift at scan i: a small rotation about z and a translation."""
    a = 0.004 * i
    T = np.eye(4)
    T[:2, :2] = [[np.cos(a), -np.sin(a)], [np.sin(a), np.cos(a)]]
    T[:3, 3] = [0.01 * i, -0.005 * i, 0.002 * i]
    return T


def _scans(dtype, n=20_000, count=10):
    base = reading_cloud(n, np.float64)
    out = []
    for i in range(count):
        P = _pose(i)
        s = base.copy()
        s[:, :3] = base[:, :3] @ P[:3, :3].T + P[:3, 3]
        out.append(s.astype(dtype))
    return out


@pytest.mark.parametrize("dn", ["float32", "float64"])
def test_sequence_equals_per_scan_compute_and_oracle(oracle, dn):
    dtype = np.dtype(dn)
    ref, nrm = reference_cloud(80_000, dtype)
    yaml = chain_yaml(filters=FILTERS, maxit=30, differential=DIFF)
    seq = ICPSequence(dtype)
    seq.load_yaml(yaml)
    assert not seq.has_map()
    assert seq.set_map(ref, nrm)
    assert seq.has_map()
    icp = ICP(dtype)
    icp.load_yaml(yaml)
    cfg = oracle.make_cfg(filters=FILTERS, counter_max=30, differential=DIFF)
    T_prev = np.eye(4, dtype=dtype)
    for i, rd in enumerate(_scans(dtype)):
        T = seq.compute(rd, T_prev)
        it = seq.stats().iterations
        T_plain = icp.compute(rd, ref, nrm, T_init=T_prev)
        np.testing.assert_array_equal(T, T_plain, err_msg=f"scan {i}: sequence != per-scan compute")
        assert icp.stats().iterations == it
        rc, To, so, _ = oracle.icp(cfg, rd, ref, normals=nrm, T_init=T_prev)
        assert rc == 0
        frob = np.linalg.norm(T.astype(np.float64) - To.astype(np.float64))
        print(f"{dn} scan {i}: iterations {it}/{so.iterations} |dT|={frob:.3g}")
        assert it == so.iterations
        assert frob <= TOL[dn]
        T_prev = T
    seq.close()
    icp.close()


def test_map_accessors_and_reload():
    dtype = np.float32
    ref, nrm = reference_cloud(30_000, dtype)
    rd = reading_cloud(8_000, dtype)
    seq = ICPSequence(dtype)
    seq.load_yaml(chain_yaml(filters=FILTERS, maxit=20, differential=DIFF))
    np.testing.assert_array_equal(seq.compute(rd), np.eye(4, dtype=dtype))  # no map: identity
    assert not seq.set_map(ref[:0])  # an empty map is ignored
    assert not seq.has_map()
    assert seq.set_map(ref, nrm)
    g = seq.get_map()
    assert g.shape == ref.shape
    np.testing.assert_allclose(g, ref, atol=1e-5)  # centred and moved back (T arithmetic)
    T1 = seq.compute(rd)
    # a chain reload re-indexes the held map; a plain compute on the object
    # replaces the device's reference, the next sequence compute restores it
    seq.load_yaml(chain_yaml(filters=FILTERS, maxit=20, differential=DIFF))
    np.testing.assert_array_equal(seq.compute(rd), T1)
    seq.compute_with_reference(rd, ref[::2].copy(), nrm[::2].copy())
    np.testing.assert_array_equal(seq.compute(rd), T1)
    seq.clear_map()
    assert not seq.has_map()
    np.testing.assert_array_equal(seq.compute(rd), np.eye(4, dtype=dtype))
    seq.close()


def test_map_kept_when_set_map_fails_and_get_map_sized_by_library():
    """get_map sizes its buffer from the held map's rows (not from
    the last reading's), and a set_map whose reference filter throws leaves
    the previous map indexed (pm_icp.cpp setMap commits after Matcher::init)."""
    dtype = np.float32
    ref, nrm = reference_cloud(30_000, dtype)
    rd = reading_cloud(8_000, dtype)
    yaml = chain_yaml(filters=FILTERS, maxit=20, differential=DIFF)
    # DistanceLimit on z: valid for 3-D clouds (D = 3), throws for 2-D ones (DistanceLimit.cpp:68-70)
    yaml = ("referenceDataPointsFilters:\n  - DistanceLimitDataPointsFilter:\n      dim: 2\n      dist: 100\n"
            "      removeInside: 0\n" + yaml)
    seq = ICPSequence(dtype)
    seq.load_yaml(yaml)
    assert seq.set_map(ref, nrm)
    T1 = seq.compute(rd)
    assert not seq.set_map(np.zeros((0, 3), dtype))  # ignored
    with pytest.raises(Exception):
        seq.set_map(np.ascontiguousarray(ref[:, [0, 1, 3]]))  # a 2-D map: the filter throws
    assert seq.has_map()
    g = seq.get_map()
    assert g.shape == ref.shape
    np.testing.assert_array_equal(seq.compute(rd), T1)  # the previous map, still indexed
    # a 2-D ICP on the same object (3-row clouds) replaces the device reference
    # only (the chain without the reference filter, which would throw on 2-D)
    seq.load_yaml(chain_yaml(filters=FILTERS, maxit=20, differential=DIFF))
    T1 = seq.compute(rd)  # (the same filtered map: every point has z < 100)
    r2 = np.ascontiguousarray(ref[::3][:, [0, 1, 3]])
    seq.compute_with_reference(np.ascontiguousarray(rd[:, [0, 1, 3]]), r2, np.ascontiguousarray(nrm[::3][:, :2]))
    assert seq.get_map().shape == ref.shape
    np.testing.assert_array_equal(seq.compute(rd), T1)
    seq.close()
