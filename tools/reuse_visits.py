"""Development probe: per-match pair counts of test_temporal_reuse_stays_exact's
pose sequence (grid matcher, one context), for the current env knobs."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from libpointmatcher_amd import _capi as P  # noqa: E402
from libpointmatcher_amd.synth import reading_cloud, reference_cloud, t_gt  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 1
ref, nrm = reference_cloud(100_000)
rd = reading_cloud(20_000)
ctx = P.Context(0, np.float32)
ctx.set_search(1)
ctx.set_reference(ref, nrm)
ctx.set_reading(rd)
Tg = t_gt().astype(np.float32)
out = []
mirror = os.environ.get("PROBE_MIRROR") == "1"
for T in (np.eye(4, dtype=np.float32), Tg, Tg, Tg, Tg):
    ctx.match(T, knn=k, max_dist=np.inf)
    if mirror:
        ctx.get_matches()
    ctx.outlier("NullOutlierFilter", 0)
    _, _, st = ctx.p2plane_system()
    out.append(int(st.visited))
ctx.close()
print("k", k, "env", {e: os.environ.get(e) for e in ("PMX_COOP_MAX", "PMX_REUSE_CAND")}, "visits", out)
