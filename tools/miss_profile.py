"""Full searches per iteration of a C3 ICP (development tool).

Runs the device-loop ICP once for its pose trace, then replays the same poses
through the per-module context API (match, TrimmedDist, point-to-plane
system) and prints per iteration: the match time (HIP events), the pair
evaluations and the queries that took the full search (the temporal-reuse
certificate failed).  The reference is centred by its mean as ICP::compute
does; the poses are the loop's T_iter before each iteration.
usage: python tools/miss_profile.py [config] [iterations]
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from libpointmatcher_amd import _capi as P  # noqa: E402
from libpointmatcher_amd.icp import ICP  # noqa: E402
from libpointmatcher_amd.synth import reading_cloud, reference_cloud  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 40
N, M, dtype, knn, filters, minimizer = bench.CONFIGS[cfg]
ref, nrm = reference_cloud(M, dtype)
rd = reading_cloud(N, dtype)
icp = ICP(dtype)
icp.load_yaml(bench.chain_yaml(knn, filters, minimizer, 1, iters))
icp.keep_trace(True)
icp.compute(rd, ref, nrm)
tr = icp.trace()
icp.close()

mean = ref[:, :3].astype(np.float64).mean(0).astype(dtype)
refc = ref.copy()
refc[:, :3] -= mean
rdc = rd.copy()
rdc[:, :3] -= mean
ctx = P.Context(0, dtype)
ctx.set_search(1)
ctx.set_reference(refc, nrm)
ctx.set_reading(rdc)
poses = [np.eye(4, dtype=dtype)] + [t for t in tr[:-1]]
for i, Ti in enumerate(poses):
    ctx.timing(True)
    ctx.match(Ti.astype(dtype), knn=knn)
    ms, n = ctx.timing_read()
    ctx.timing(False)
    for name, p in filters:
        ctx.outlier(name, 0, **p)
    _, _, st = ctx.p2plane_system()
    print(json.dumps({"it": i, "match_us": round(1e3 * ms / max(n, 1), 2), "visited": int(st.visited),
                      "full_searches": int(st.fallback_queries), "kept": int(st.kept)}), flush=True)
ctx.close()
