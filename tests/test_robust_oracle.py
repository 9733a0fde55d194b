"""RobustOutlierFilter in the CPU oracle (oracle/pmo_impl.inc pmo_robust_weights)
pinned two ways, without a GPU:

* against an independent numpy restatement of robustFiltering
  (OutlierFiltersImpl.cpp:494-598) and of the Matches scale estimators
  (Matches.cpp:88-129), every robust function x scale estimator, with +inf
  distances, the approximation cut and the nbIterationForScale schedule;
* against the reference's own regression fixture: the oracle ICP with the
  defaultRobustOutlierFilter.yaml chain (KDTreeMatcher knn 10, cauchy / mad /
  tuning 1, point-to-point, Counter 40 + Differential) on icp_data
  cloud.00001 -> cloud.00000 lands within the 3 % rule of utest.cpp:81-160 of
  the stored defaultRobustOutlierFilter.ref_trans.

Tolerances: float weights to 2 ulp-ish (rtol 1e-6; exp / pow are libm on one
side, numpy on the other), double 1e-13.
"""
import numpy as np
import pytest

from helpers import hom, rel_displacement

FCTS = ["cauchy", "welsch", "sc", "gm", "tukey", "huber", "L1", "student"]
BERG = {"cauchy": 4.3040, "tukey": 7.0589, "huber": 2.0138}


class NpRobust:
    """numpy restatement of the reference object (constructor + robustFiltering)."""

    def __init__(self, dtype, fct="cauchy", tuning=1.0, scale="mad", nb=0, approx=np.inf):
        T = np.dtype(dtype).type
        self.T, self.fct, self.scale_est, self.nb = T, fct, scale, nb
        self.k = T(tuning)
        self.target = T(0)
        if scale == "berg":
            self.target = T(tuning)
            if fct in BERG:
                self.k = T(BERG[fct])
        self.sqa = T(np.inf) if np.isinf(approx) else T(T(approx) ** 2)
        self.it, self.scale = 1, T(0)

    def weights(self, d):
        T = self.T
        rec = self.it <= self.nb or self.nb == 0
        fin = d[np.isfinite(d)]
        if self.scale_est == "mad" and rec:
            med = np.sort(fin)[len(fin) // 2]
            dev = np.abs(fin - med).astype(T)
            self.scale = T(np.sqrt(np.sort(dev)[len(dev) // 2]))
        elif self.scale_est == "std" and rec:
            s = np.sum(d.astype(np.float64))
            mean = T(s / d.size)
            c = (d - mean).astype(T)
            var = T(T(np.sum((c * c).astype(np.float64))) / T(d.size - 1))
            self.scale = T(np.sqrt(T(np.sqrt(var))))
        elif self.scale_est == "berg" and rec:
            if self.it == 1:
                q = np.partition(fin, int(T(len(fin)) * T(0.5)))[int(T(len(fin)) * T(0.5))]
                self.scale = T(1.9 * float(T(np.sqrt(q))))
            else:
                self.scale = T(T(0.85) * (self.scale - self.target) + self.target)
        elif self.scale_est == "none":
            self.scale = T(1)
        self.it += 1
        with np.errstate(all="ignore"):
            e2 = (d / (self.scale * self.scale)).astype(T)
            k, k2 = self.k, T(self.k * self.k)
            one = T(1)
            f = self.fct
            if f == "cauchy":
                w = one / (one + e2 / k2)
            elif f == "welsch":
                w = np.exp(-e2 / k2)
            elif f == "sc":
                s = (k + e2).astype(T)
                w = np.where(e2 >= k, T(4.0 * float(k2)) * (one / (s * s)), one)
            elif f == "gm":
                s = (k + e2).astype(T)
                w = k2 * (one / (s * s))
            elif f == "tukey":
                a = (one - e2 / k2).astype(T)
                w = np.where(e2 >= k2, T(0), a * a)
            elif f == "huber":
                w = np.where(e2 >= k2, k * (one / np.sqrt(e2)), one)
            elif f == "L1":
                w = one / np.sqrt(e2)
            else:
                dd = T(3)
                w = np.power(one + e2 / k, -(k + dd) / T(2)) * (k + dd) * (one / (k + e2))
            w = w.astype(T)
            w = np.where(w <= T(1e-50), T(1e-50), w).astype(T)
            if not np.isinf(self.sqa):
                w = np.where(e2 >= self.sqa, T(0), w).astype(T)
        return w


def _dists(dtype, n=2000, k=3, seed=0, inf_frac=0.05):
    rng = np.random.default_rng(seed)
    d = (rng.gamma(2.0, 0.02, (n, k)) ** 2).astype(dtype)
    d[rng.random((n, k)) < inf_frac] = np.inf
    return np.sort(d, axis=1)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("fct", FCTS)
@pytest.mark.parametrize("scale", ["mad", "std", "berg", "none"])
def test_robust_weights_match_numpy(oracle, dtype, fct, scale):
    tol = 1e-6 if dtype == np.float32 else 1e-13
    for approx, nb in ((np.inf, 0), (0.5, 2)):
        inf_frac = 0.0 if scale == "std" else 0.05  # (std over +inf is NaN in the reference too)
        p = {"robustFct": fct, "scaleEstimator": scale, "tuning": 0.7, "nbIterationForScale": nb,
             "approximation": approx}
        r = oracle.make_robust(p)
        ref = NpRobust(dtype, fct, 0.7, scale, nb, approx)
        for it in range(4):  # the schedule: recompute, keep, berg's convergence
            d = _dists(dtype, seed=it, inf_frac=inf_frac)
            rc, w = oracle.robust_weights(r, d, np.zeros(d.shape, np.int32))
            assert rc == 0
            wn = ref.weights(d)
            np.testing.assert_allclose(r.scale, float(ref.scale), rtol=tol)
            np.testing.assert_allclose(w, wn, rtol=tol, atol=tol)  # (tukey near e2 = k2 cancels)
            assert r.iteration == it + 2


def test_robust_mad_empty_raises(oracle):
    r = oracle.make_robust({"scaleEstimator": "mad"})
    d = np.full((10, 2), np.inf, np.float32)
    rc, _ = oracle.robust_weights(r, d, np.zeros(d.shape, np.int32))
    assert rc == oracle.E_EMPTY_QUANTILE  # Matches.cpp:106-107 "no outlier to filter"


def test_oracle_icp_robust_config_matches_ref_trans(golden, oracle):
    """defaultRobustOutlierFilter.yaml through the oracle ICP vs the reference's
    stored result (utest.cpp:81-160)."""
    g, kat = golden
    c = oracle.make_cfg(knn=10, filters=(("RobustOutlierFilter", {"robustFct": "cauchy", "scaleEstimator": "mad",
                                                                    "tuning": 1}),),
                        minimizer="PointToPointErrorMinimizer", counter_max=40,
                        differential=dict(minDiffRotErr=0.001, minDiffTransErr=0.01, smoothLength=4), threads=8)
    rc, T, st, _ = oracle.icp(c, hom(g["vtk1"], np.float32), hom(g["vtk0"], np.float32))
    assert rc == 0
    refT = np.array(kat["icp_data_ref_trans"]["defaultRobustOutlierFilter"])
    err = rel_displacement(T, refT, g["vtk1"])
    print(f"oracle robust icp: rel err {err:.5f}, iterations {st.iterations}")
    assert err < kat["icp_data_rel_tol"]


@pytest.mark.parametrize("scale,nb", [("berg", 0), ("mad", 3)])
def test_oracle_icp_keeps_robust_state_across_calls(golden, oracle, scale, nb):
    """pmo_icp_keep: the filter object outlives a compute() (the reference's ICP
    owns its chain, OutlierFiltersImpl.cpp:500-540).  Its first call equals
    pmo_icp's; the iteration counter advances by the iterations run (one
    robustFiltering per iteration) on both calls, and the second call differs
    from a fresh filter's compute."""
    g, _ = golden
    p = {"robustFct": "huber" if scale == "berg" else "cauchy", "scaleEstimator": scale, "tuning": 0.05 if
         scale == "berg" else 1, "nbIterationForScale": nb}
    filt = (("RobustOutlierFilter", p),)
    rd, ref = hom(g["vtk1"], np.float32), hom(g["vtk0"], np.float32)
    mk = lambda: oracle.make_cfg(knn=3, filters=filt, minimizer="PointToPointErrorMinimizer", counter_max=6,
                                 threads=8)
    c = mk()
    rc, T1, s1, _ = oracle.icp(c, rd, ref, keep_robust=True)
    rc0, T0, s0, _ = oracle.icp(mk(), rd, ref)
    assert rc == rc0 == 0 and np.array_equal(T1, T0) and s1.iterations == s0.iterations
    assert c.robust.iteration == 1 + s1.iterations
    it1 = c.robust.iteration
    rc, T2, s2, _ = oracle.icp(c, rd, ref, keep_robust=True)
    assert rc == 0 and c.robust.iteration == it1 + s2.iterations
    # the schedule carried over: past nbIterationForScale (mad) the scale is
    # kept, and berg never re-runs its first-call estimate — so the second
    # call is not a fresh filter's compute
    rcf, Tf, _, _ = oracle.icp(mk(), rd, ref)
    assert rcf == 0
    assert not np.array_equal(T2, Tf)
