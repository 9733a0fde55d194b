"""Per-wave profile of the cold tile match (development tool): one ICP of
the bench configuration with PMX_OPTS=tile_prof=1 (the library prints the cold
form's per-wave durations, rounds and copied points to stderr).
usage: PMX_OPTS=tile_prof=1 python tools/tile_prof.py [c3|c5|...] [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from libpointmatcher_amd.icp import ICP  # noqa: E402
from libpointmatcher_amd.synth import reading_cloud, reference_cloud  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
N, M, dtype, knn, filters, minimizer = bench.CONFIGS[cfg]
ref, nrm = reference_cloud(M, dtype)
rd = reading_cloud(N, dtype)
icp = ICP(dtype)
icp.load_yaml(bench.chain_yaml(knn, filters, minimizer, 1, 3))
nrm_in = nrm if minimizer.startswith("PointToPlane") else None
for _ in range(reps):
    icp.prepare(rd, ref, nrm_in)
    icp.iterate(3)
icp.close()
