"""The device-resident ICP loop (pmx_loop_*, pmx_loop.hip) against the
per-module path and the CPU oracle.

The loop moves the step solve, the T_iter update (ICP.cpp:419) and the
transformation checkers (TransformationCheckersImpl.cpp:45-225) onto the GPU.
Bar: the same iteration count and the final transform within 1e-5 (float) /
1e-12 (double) of the oracle and of the per-module path; errors raised with
the reference's exception type and message.
"""
import numpy as np
import pytest

from helpers import chain_yaml
from libpointmatcher_amd import _capi
from libpointmatcher_amd._capi import ConvergenceError
from libpointmatcher_amd.icp import ICP
from libpointmatcher_amd.synth import reading_cloud, reference_cloud

pytestmark = pytest.mark.gpu

TOL = {np.float32: 1e-5, np.float64: 1e-12}
DIFF = dict(minDiffRotErr=0.001, minDiffTransErr=0.01, smoothLength=4)


def run_mode(monkeypatch, mode, yaml, rd, ref, nrm, dtype):
    monkeypatch.setenv("PMX_DEVICE_LOOP", "1" if mode == "loop" else "0")
    icp = ICP(dtype)
    icp.load_yaml(yaml)
    icp.keep_trace(True)
    T = icp.compute(rd, ref, nrm)
    return T, icp.stats(), icp.trace()


@pytest.mark.parametrize("reuse", ["0", "1"])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("minimizer", ["PointToPlaneErrorMinimizer", "PointToPointErrorMinimizer"])
def test_loop_equals_modules(monkeypatch, oracle, dtype, minimizer, reuse):
    # reuse=1: the grid match may certify the previous iteration's k-lists
    # (LoopCtl.Tprev in loop mode, the host's previous step in module mode)
    monkeypatch.setenv("PMX_OPTS", "grid_reuse=" + reuse)
    ref, nrm = reference_cloud(50000, dtype)
    rd = reading_cloud(40000, dtype)
    yaml = chain_yaml(minimizer=minimizer, maxit=25, differential=DIFF)
    Tl, sl, trl = run_mode(monkeypatch, "loop", yaml, rd, ref, nrm, dtype)
    Tm, sm, trm = run_mode(monkeypatch, "modules", yaml, rd, ref, nrm, dtype)
    assert sl.iterations == sm.iterations
    assert len(trl) == len(trm) == sl.iterations
    assert np.linalg.norm(Tl - Tm) <= TOL[dtype]
    assert np.abs(trl - trm).max() <= 10 * TOL[dtype]
    # statistics mirrored from the device loop
    assert sl.kept == sm.kept
    assert sl.rejected_matches == sm.rejected_matches
    assert sl.max_iterations_reached == sm.max_iterations_reached
    # (pair evaluations: a diagnostic, not the reference's libnabo count; the
    # two modes may search some iterations from the LDS box and others with
    # the per-lane walk — the LDS box is launched on the host's knowledge of
    # the last match — so the counts agree only in magnitude)
    assert 0.5 * sm.point_count_touched <= sl.point_count_touched <= 2.0 * sm.point_count_touched
    cfg = oracle.make_cfg(minimizer=minimizer, counter_max=25, differential=DIFF, threads=8)
    rc, To, so, _ = oracle.icp(cfg, rd, ref, normals=nrm, trace=True)
    assert rc == 0 and so.iterations == sl.iterations
    assert np.linalg.norm(Tl - To) <= TOL[dtype]


def test_loop_2d(monkeypatch, oracle):
    rng = np.random.default_rng(5)
    t = rng.uniform(0, 2 * np.pi, 20000)
    ref = np.stack([np.cos(t) * (1 + 0.2 * np.sin(5 * t)), np.sin(t) * (1 + 0.2 * np.sin(5 * t)),
                    np.ones_like(t)], 1).astype(np.float32)
    c, s = np.cos(0.05), np.sin(0.05)
    R = np.array([[c, -s], [s, c]])
    rd = ref.copy()
    rd[:, :2] = (ref[:, :2].astype(np.float64) @ R.T + [0.02, -0.01]).astype(np.float32)
    yaml = chain_yaml(minimizer="PointToPointErrorMinimizer", maxit=30, differential=DIFF)
    Tl, sl, _ = run_mode(monkeypatch, "loop", yaml, rd, ref, None, np.float32)
    Tm, sm, _ = run_mode(monkeypatch, "modules", yaml, rd, ref, None, np.float32)
    assert sl.iterations == sm.iterations
    assert np.linalg.norm(Tl - Tm) <= 1e-5
    cfg = oracle.make_cfg(minimizer="PointToPointErrorMinimizer", counter_max=30, differential=DIFF, threads=8)
    rc, To, so, _ = oracle.icp(cfg, rd, ref, trace=False)
    assert rc == 0 and np.linalg.norm(Tl - To) <= 1e-5


@pytest.mark.parametrize("filters", [
    [("VarTrimmedDistOutlierFilter", {"minRatio": 0.6, "maxRatio": 0.8, "lambda": 0.9})],
    [("MedianDistOutlierFilter", {"factor": 3.0}), ("MaxDistOutlierFilter", {"maxDist": 0.1})],
    [("MinDistOutlierFilter", {"minDist": 0.0001}), ("TrimmedDistOutlierFilter", {"ratio": 0.7})],
    [],
])
def test_loop_filter_chains(monkeypatch, oracle, filters):
    ref, nrm = reference_cloud(30000, np.float32)
    rd = reading_cloud(25000, np.float32)
    yaml = chain_yaml(filters=filters, knn=2, maxit=15)
    Tl, sl, _ = run_mode(monkeypatch, "loop", yaml, rd, ref, nrm, np.float32)
    Tm, sm, _ = run_mode(monkeypatch, "modules", yaml, rd, ref, nrm, np.float32)
    assert sl.iterations == sm.iterations == 15
    assert np.linalg.norm(Tl - Tm) <= 1e-5
    cfg = oracle.make_cfg(knn=2, filters=tuple(filters), counter_max=15, threads=8)
    rc, To, so, _ = oracle.icp(cfg, rd, ref, normals=nrm)
    assert rc == 0 and np.linalg.norm(Tl - To) <= 1e-5


def test_bound_checker_raises_in_both_modes(monkeypatch):
    # BoundTransformationChecker (TransformationCheckersImpl.cpp:196-225): the
    # reading is shifted 0.05 away, the bound allows 0.01 of translation
    ref, nrm = reference_cloud(20000, np.float32)
    rd = reading_cloud(20000, np.float32)
    yaml = chain_yaml(maxit=30, bound={"maxRotationNorm": 1.0, "maxTranslationNorm": 0.01})
    msgs, iters = [], []
    for mode in ("loop", "modules"):
        monkeypatch.setenv("PMX_DEVICE_LOOP", "1" if mode == "loop" else "0")
        icp = ICP(np.float32)
        icp.load_yaml(yaml)
        with pytest.raises(ConvergenceError, match="limit out of bounds") as ei:
            icp.compute(rd, ref, nrm)
        msgs.append(str(ei.value))
        iters.append(icp.stats().iterations)
    assert iters[0] == iters[1]
    # same numbers, printed like the reference's ostream at T precision
    assert msgs[0].split("tr:")[0] == msgs[1].split("tr:")[0]


def test_loop_capi_direct():
    """pmx_loop_begin / run / trace through the C ABI: partial runs, the
    stop flag, the trace and the Counter's MaxNumIterationsReached."""
    ref, nrm = reference_cloud(20000, np.float32)
    rd = reading_cloud(20000, np.float32)
    ctx = _capi.Context(0, np.float32)
    ctx.set_reference(ref, nrm)
    ctx.set_reading(rd)
    ctx.loop_begin(knn=1, filters=[("TrimmedDistOutlierFilter", 0.85)],
                   checkers=[("CounterTransformationChecker", 10)], keep_trace=True)
    st = ctx.loop_run(3)
    assert st.iterations == 3 and not st.done
    st = ctx.loop_run(100)
    assert st.iterations == 10 and st.done and st.reason == 1
    assert st.cond[0][0] == 10.0
    tr = ctx.loop_trace(0, 10)
    assert np.array_equal(tr[-1], ctx.loop_T(st))
    st2 = ctx.loop_run(5)  # stopped: nothing more runs
    assert st2.iterations == 10
    assert np.abs(tr[:3] - ctx.loop_trace(0, 3)).max() == 0
    with pytest.raises(_capi.InvalidParameter):
        ctx.loop_trace(5, 6)  # beyond the completed iterations
    ctx.close()


def test_loop_no_points_error():
    ref, nrm = reference_cloud(5000, np.float32)
    rd = reading_cloud(3000, np.float32)
    rd[:, :3] += 100.0
    ctx = _capi.Context(0, np.float32)
    ctx.set_reference(ref, nrm)
    ctx.set_reading(rd)
    ctx.loop_begin(knn=1, max_dist=0.01, checkers=[("CounterTransformationChecker", 10)])
    with pytest.raises(ConvergenceError, match="no point to minimize"):
        ctx.loop_run(10)
    st = ctx.last_loop_status
    assert st.iterations == 0 and st.done and st.error == _capi.PMX_E_NO_POINTS
    ctx.loop_begin(knn=1, max_dist=0.01, filters=[("TrimmedDistOutlierFilter", 0.8)],
                   checkers=[("CounterTransformationChecker", 10)])
    with pytest.raises(ConvergenceError, match="no outlier to filter"):
        ctx.loop_run(10)
    ctx.close()


def test_loop_rejects_brute_force():
    ref, nrm = reference_cloud(2000, np.float32)
    ctx = _capi.Context(0, np.float32)
    ctx.set_search(0)
    ctx.set_reference(ref, nrm)
    ctx.set_reading(reading_cloud(1000, np.float32))
    with pytest.raises(_capi.InvalidParameter):
        ctx.loop_begin(knn=1, checkers=[("CounterTransformationChecker", 3)])
    ctx.close()


@pytest.mark.parametrize("knn,max_dist", [(1, np.inf), (3, np.inf), (1, 0.05)])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("filt", [("TrimmedDistOutlierFilter", 0.85), ("MedianDistOutlierFilter", 3.0),
                                  ("TrimmedDistOutlierFilter", 1.0)])
def test_quantile_window_is_exact(monkeypatch, dtype, filt, knn, max_dist):
    """The quantile resolved inside the match's key window (pmx_spec.h) is the
    radix select's: with and without the window the whole loop is bit-identical
    (the limit feeds the weights, the system and every later iteration) and the
    window resolves most converged iterations — also with k > 1 and with
    radius-limited matches (infinite distances excluded from the count).
    (Oracle parity of the loop with the window on, the default:
    test_loop_equals_modules / _filter_chains.)"""
    ref, nrm = reference_cloud(60000, dtype)
    rd = reading_cloud(50000, dtype)
    out = {}
    for on in ("1", "0"):
        monkeypatch.setenv("PMX_OPTS", "spec_select=" + on)
        ctx = _capi.Context(0, dtype)
        ctx.set_reference(ref, nrm)
        ctx.set_reading(rd)
        ctx.loop_begin(knn=knn, max_dist=max_dist, filters=[filt], checkers=[("CounterTransformationChecker", 30)],
                       keep_trace=True)
        st = ctx.loop_run(30)
        out[on] = (ctx.loop_trace(0, st.iterations), ctx.loop_select_stats(), st.last.kept, st.iterations)
        ctx.close()
    tr1, (hits, misses), kept1, it1 = out["1"]
    tr0, (h0, m0), kept0, it0 = out["0"]
    assert it1 == it0 == 30
    assert h0 == 0 and m0 == 0
    assert hits + misses == 30 and hits >= 15, (hits, misses)
    assert kept1 == kept0
    assert np.array_equal(tr1, tr0)
