"""Context options (README "Options", pmx_ctx_set_option / PMX_OPTS) and the
device-loop paths they switch between.

* An unknown option or a malformed value is an error, never ignored.
* The fused finalize + step launch (and the match's counter phase folded into
  it) leaves the same iterations as the unfused launches: T_iter of every
  iteration and the per-iteration diagnostics bit for bit (the same sums in
  the same order, the same step arithmetic).
* Coarser grid levels built on demand: with the finest level as the cold one
  only it exists after Matcher::init, its long walks make the device loop
  request coarser ones between batches (ensure_level), and the
  iterations equal the default run's bit for bit; the side-stream level
  builds give the same result as building every level on the context stream.
Reference semantics: ICP.cpp:371-430 (the loop), MatchersImpl.cpp:77-101.
"""
import numpy as np
import pytest

from libpointmatcher_amd import _capi as P
from libpointmatcher_amd.synth import reading_cloud, reference_cloud, t_gt

pytestmark = pytest.mark.gpu


def test_unknown_option_fails(monkeypatch):
    monkeypatch.setenv("PMX_OPTS", "no_such_option=1")
    with pytest.raises(P.PmxError):
        P.Context(0, np.float32)
    monkeypatch.setenv("PMX_OPTS", "grid_levels=2:x")
    with pytest.raises(P.PmxError):
        P.Context(0, np.float32)
    monkeypatch.setenv("PMX_OPTS", "grid_levels=2:8,coop_max=8")
    ctx = P.Context(0, np.float32)
    ctx.set_option("fuse_step", 0)
    with pytest.raises(Exception):
        ctx.set_option("fuse_step", "yes")
    with pytest.raises(Exception):
        ctx.set_option("bogus", 1)
    ctx.close()


def _loop(opts, ref, nrm, rd, T0, knn, filters, minimizer, iters, dtype=np.float32):
    ctx = P.Context(0, dtype)
    for k, v in opts.items():
        ctx.set_option(k, v)
    ctx.set_reference(ref, nrm)
    ctx.set_reading(rd)
    ctx.loop_begin(knn=knn, filters=filters, minimizer=minimizer,
                   checkers=[("CounterTransformationChecker", iters)], T0=T0, keep_trace=True)
    st = ctx.loop_run(iters)
    n = st.iterations
    tr = ctx.loop_trace(0, n)
    dg = ctx.loop_diag(0, n)
    ctx.close()
    return n, tr, dg


@pytest.mark.parametrize("chain", ["trimmed_p2plane", "maxdist_k4", "p2point"])
def test_fused_step_equals_unfused(chain):
    ref, nrm = reference_cloud(200_000)
    rd = reading_cloud(100_000)
    T0 = np.eye(4, dtype=np.float32)
    if chain == "trimmed_p2plane":
        args = (1, [("TrimmedDistOutlierFilter", 0.85)], "PointToPlaneErrorMinimizer")
    elif chain == "maxdist_k4":  # (no quantile window: the counter phase folds into the fused launch)
        args = (4, [("MaxDistOutlierFilter", 0.5)], "PointToPlaneErrorMinimizer")
    else:
        args = (1, [("TrimmedDistOutlierFilter", 0.9)], "PointToPointErrorMinimizer")
    base = _loop({}, ref, nrm, rd, T0, *args, iters=15)
    for opts in ({"step_counter": 0}, {"fuse_step": 0}):
        other = _loop(opts, ref, nrm, rd, T0, *args, iters=15)
        assert other[0] == base[0]
        assert np.array_equal(other[1], base[1]), f"{opts}: T_iter differs"
        assert np.array_equal(other[2], base[2]), f"{opts}: diagnostics differ"


def test_coarse_levels_on_demand():
    """Levels 0.25 / 2 / 8 points per cell with the finest as the cold one:
    Matcher::init builds only it; a 16-NN search there evaluates far more
    than 32 cells' worth of points per query (the level choice's measure), so
    the loop asks for the next coarser level, which the host builds between
    batches (ensure_level).  Any level answers exactly,
    so the iterations equal the default run's (its levels built at
    Matcher::init and on the side stream) bit for bit — and that run is pinned
    to the oracle by test_gpu_loop.py / test_gpu_configs.py."""
    ref, nrm = reference_cloud(200_000)
    rd = reading_cloud(100_000)
    T0 = t_gt().astype(np.float32)
    T0[:3, 3] += np.array([0.3, -0.2, 0.15], np.float32)
    args = (16, [("TrimmedDistOutlierFilter", 0.85)], "PointToPlaneErrorMinimizer")
    lazy = {"grid_levels": "0.25:2:8", "first_ppc": 0.25}
    n, tr, dg = _loop(lazy, ref, nrm, rd, T0, *args, iters=12)
    assert dg[:, 0].max() > 0, f"the loop never moved to a coarser level: {dg[:, 0]}"
    n2, tr2, _ = _loop(dict(lazy, side_levels=0), ref, nrm, rd, T0, *args, iters=12)
    n3, tr3, _ = _loop({}, ref, nrm, rd, T0, *args, iters=12)
    assert n == n2 == n3 == 12
    assert np.array_equal(tr, tr2) and np.array_equal(tr, tr3)


def test_level_records_follow_the_reference():
    """Every grid level's records hold the reference's points and normals
    (pmx_grid_level_records).  The levels finer than the cold one build on a
    side stream from the packed normals, which the context stream packs after
    their upload: the side stream waits for that (the side_start event,
    pmx_chain.hip build_levels_cold).  A new reference on the same context
    each time, so a level built from stale normals would hold the previous
    cloud's."""
    ctx = P.Context(0, np.float32)
    for seed in (1, 2, 3):
        ref, nrm = reference_cloud(300_000, seed=seed)
        ctx.set_reference(ref, nrm)
        n_levels = 0
        while True:
            try:
                ids, pts, nn = ctx.level_records(n_levels)
            except P.InvalidParameter:  # (past the last level)
                break
            assert np.array_equal(np.sort(ids), np.arange(len(ref)))
            assert np.array_equal(pts[:, :3], ref[ids, :3]), f"level {n_levels}: points"
            assert np.array_equal(nn[:, :3], nrm[ids]), f"level {n_levels}: normals"
            n_levels += 1
        assert n_levels >= 2
    ctx.close()
