"""Setup timeline of ICP::compute's prepare (development tool): prepares the
bench configuration's clouds three times on one context with
PMX_OPTS=setup_trace=1 (the library prints each phase), and prints the host-side
prepare wall time and the stats' reference / reading parts.
usage: PMX_OPTS=setup_trace=1 python tools/setup_trace.py [c3|c5]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from libpointmatcher_amd.icp import ICP  # noqa: E402
from libpointmatcher_amd.synth import reading_cloud, reference_cloud  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
N, M, dtype, knn, filters, minimizer = bench.CONFIGS[cfg]
ref, nrm = reference_cloud(M, dtype)
rd = reading_cloud(N, dtype)
icp = ICP(dtype)
icp.load_yaml(bench.chain_yaml(knn, filters, minimizer, 1, 10))
nrm_in = nrm if minimizer.startswith("PointToPlane") else None
# (the GPU at its working clocks first: a few whole ICPs, as bench.py's warm-up)
t_end = time.perf_counter() + 0.3
while time.perf_counter() < t_end:
    icp.prepare(rd, ref, nrm_in)
    icp.iterate(10)
for rep in range(4):
    print(f"--- prepare {rep}", file=sys.stderr, flush=True)
    t = time.perf_counter()
    icp.prepare(rd, ref, nrm_in)
    dt = time.perf_counter() - t
    st = icp.stats()
    print(f"prepare {rep}: {dt * 1e3:.3f} ms  reference {st.reference_preprocessing_duration * 1e3:.3f}"
          f"  reading {st.reading_preprocessing_duration * 1e3:.3f}", file=sys.stderr, flush=True)
icp.close()
