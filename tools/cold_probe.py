"""Cold (first-iteration) match time, twice in one process (development tool):
separates one-time launch costs from the misaligned search itself."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from libpointmatcher_amd.icp import ICP  # noqa: E402
from libpointmatcher_amd.synth import reading_cloud, reference_cloud  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
N, M, dtype, knn, filters, minimizer = bench.CONFIGS[cfg]
ref, nrm = reference_cloud(M, dtype)
rd = reading_cloud(N, dtype)
icp = ICP(dtype)
icp.load_yaml(bench.chain_yaml(knn, filters, minimizer, 1, 100))
for rep in range(3):
    icp.prepare(rd, ref, nrm if minimizer.startswith("PointToPlane") else None)
    icp.timing(True)
    icp.iterate(1)
    ms, n = icp.timing_read()
    icp.timing(True)
    icp.iterate(1)
    ms2, n2 = icp.timing_read()
    print(f"{cfg} rep {rep}: first match {ms / max(n, 1):.3f} ms, second {ms2 / max(n2, 1):.3f} ms", flush=True)
