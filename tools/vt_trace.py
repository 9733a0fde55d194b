"""Timeline of the VarTrimmed partial-sum walk at C3 (development tool).

Runs the C3 ICP for a few iterations (for a realistic pose), then one match +
VarTrimmedDist at that pose through the context API with PMX_OPTS=vt_trace=1: the
library prints every step of vt_cumsum_kernel's walk (100 MHz real-time
stamps) to stderr.
usage: PMX_OPTS=vt_trace=1 python tools/vt_trace.py [iterations]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from libpointmatcher_amd import _capi as P  # noqa: E402
from libpointmatcher_amd.icp import ICP  # noqa: E402
from libpointmatcher_amd.synth import reading_cloud, reference_cloud  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
N, M, dtype, knn, filters, minimizer = bench.CONFIGS["c3v"]
ref, nrm = reference_cloud(M, dtype)
rd = reading_cloud(N, dtype)
icp = ICP(dtype)
icp.load_yaml(bench.chain_yaml(knn, filters, minimizer, 1, iters))
icp.keep_trace(True)
icp.compute(rd, ref, nrm)
T = icp.trace()[-1]
icp.close()
mean = ref[:, :3].astype(np.float64).mean(0).astype(dtype)
refc, rdc = ref.copy(), rd.copy()
refc[:, :3] -= mean
rdc[:, :3] -= mean
ctx = P.Context(0, dtype)
ctx.set_reference(refc, nrm)
ctx.set_reading(rdc)
for rep in range(2):
    ctx.match(T.astype(dtype), knn=knn)
    name, p = filters[0]
    ctx.outlier(name, 0, **p)
    cum = ctx.vartrim_partial_sums()
    print(f"rep {rep}: {cum.shape[0]} partial sums", flush=True)
ctx.close()
