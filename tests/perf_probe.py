"""Quick device-time probe of the per-iteration kernels (development tool).

python tests/perf_probe.py N M k iters dtype
"""
import sys
import time

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from libpointmatcher_amd import _capi as P  # noqa: E402
from libpointmatcher_amd.synth import reading_cloud, reference_cloud  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    M = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    iters = int(sys.argv[4]) if len(sys.argv) > 4 else 5
    dt = np.float64 if (len(sys.argv) > 5 and sys.argv[5] == "f64") else np.float32
    ref, nrm = reference_cloud(M, dt)
    rd = reading_cloud(N, dt)
    ctx = P.Context(0, dt)
    ctx.set_reference(ref, nrm)
    ctx.set_reading(rd)
    T = np.eye(4, dtype=dt)
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
    pairs = N * M
    per = ms / n
    print(f"N={N} M={M} k={k} {dt.__name__}: iter {1e3 * (t1 - t0) / iters:.3f} ms wall, "
          f"match kernel {per:.3f} ms avg over {n}; {pairs / (per * 1e-3) / 1e12:.3f} Tpair/s; "
          f"{8 * pairs / (per * 1e-3) / 1e12:.1f} TFLOP/s(8/pair); kept={st.kept}")


if __name__ == "__main__":
    main()
