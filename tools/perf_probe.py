"""Device-time probe of the per-iteration kernels (development tool).

python tools/perf_probe.py N M k iters [f64] [brute]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from libpointmatcher_amd import _capi as P  # noqa: E402
from libpointmatcher_amd.synth import reading_cloud, reference_cloud, t_gt  # noqa: E402


def main():
    a = sys.argv[1:]
    N = int(a[0]) if len(a) > 0 else 1_000_000
    M = int(a[1]) if len(a) > 1 else 1_000_000
    k = int(a[2]) if len(a) > 2 else 1
    iters = int(a[3]) if len(a) > 3 else 5
    dt = np.float64 if "f64" in a else np.float32
    search = 0 if "brute" in a else 1
    ref, nrm = reference_cloud(M, dt)
    rd = reading_cloud(N, dt)
    ctx = P.Context(0, dt)
    ctx.set_search(search)
    t0 = time.perf_counter()
    ctx.set_reference(ref, nrm)
    ctx.set_reading(rd)
    t_setup = time.perf_counter() - t0
    T = (t_gt() if "aligned" in a else np.eye(4)).astype(dt)
    ctx.match(T, knn=k)
    ctx.outlier("TrimmedDistOutlierFilter", 0, ratio=0.85)
    ctx.p2plane_system()
    ctx.timing(True)
    t0 = time.perf_counter()
    for _ in range(iters):
        ctx.match(T, knn=k)
        ctx.outlier("TrimmedDistOutlierFilter", 0, ratio=0.85)
        A, b, st = ctx.p2plane_system()
    t1 = time.perf_counter()
    ms, n = ctx.timing_read()
    per = ms / n
    print(f"N={N} M={M} k={k} {dt.__name__} search={search} options={os.environ.get('PMX_OPTS', '')!r}: setup {t_setup:.2f}s, "
          f"iter {1e3 * (t1 - t0) / iters:.3f} ms wall, match {per:.3f} ms, visited/query {st.visited / N:.1f}, "
          f"{st.visited / (per * 1e-3) / 1e9:.1f} Gpair/s, kept={st.kept}, fallback={st.fallback_queries}")


if __name__ == "__main__":
    main()
