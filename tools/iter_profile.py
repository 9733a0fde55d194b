"""Per-iteration match statistics of one C3 ICP through the device loop
(development tool): match kernel time (HIP events), pair evaluations and the
queries that took the full search (temporal-reuse certificate failed), and
the quantile window's hit / miss count.  One JSON line per iteration."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from libpointmatcher_amd import _capi  # noqa: E402
from libpointmatcher_amd.synth import reading_cloud, reference_cloud  # noqa: E402

N = int(os.environ.get("PROF_N", "1000000"))
iters = int(os.environ.get("PROF_ITERS", "40"))
ref, nrm = reference_cloud(N, np.float32)
rd = reading_cloud(N, np.float32)
ctx = _capi.Context(0, np.float32)
ctx.set_reference(ref, nrm)
ctx.set_reading(rd)
ctx.loop_begin(filters=[("TrimmedDistOutlierFilter", 0.85)], checkers=[("CounterTransformationChecker", iters)])
prev_hits = (0, 0)
for i in range(iters):
    ctx.timing(True)
    st = ctx.loop_run(1)
    ms, n = ctx.timing_read()
    hits = ctx.loop_select_stats()
    print(json.dumps({"iter": i, "match_ms": ms / max(n, 1), "pairs_per_query": st.last.visited / N,
                      "full_search_frac": st.last.fallback_queries / N, "kept": st.last.kept,
                      "window_hit": hits[0] - prev_hits[0], "limit": st.last.limit}), flush=True)
    prev_hits = hits
    if st.done:
        break
ctx.close()
