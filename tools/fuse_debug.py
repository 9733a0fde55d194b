"""Fused vs module-sequence device loop, iteration by iteration (development
tool): the first iteration whose T_iter differs, with the window verdicts."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from libpointmatcher_amd import _capi  # noqa: E402
from libpointmatcher_amd.synth import reading_cloud, reference_cloud  # noqa: E402

dt = np.float64 if "f64" in sys.argv else np.float32
N = int(os.environ.get("DBG_N", "50000"))
ref, nrm = reference_cloud(60000, dt)
rd = reading_cloud(N, dt)
runs = {}
for fused in ("1", "0"):
    os.environ["PMX_FUSED"] = fused
    ctx = _capi.Context(0, dt)
    ctx.set_reference(ref, nrm)
    ctx.set_reading(rd)
    ctx.loop_begin(filters=[("TrimmedDistOutlierFilter", 0.85)], checkers=[("CounterTransformationChecker", 20)],
                   keep_trace=True)
    rows = []
    for i in range(20):
        st = ctx.loop_run(1)
        rows.append({"T": np.array(st.T_iter[:16]).reshape(4, 4), "kept": st.last.kept, "limit": st.last.limit,
                     "rejP": st.last.rejected_points, "rejM": st.last.rejected_matches, "nz": st.last.nonzero_weights,
                     "sel": ctx.loop_select_stats()})
    runs[fused] = rows
    ctx.close()
for i, (a, b) in enumerate(zip(runs["1"], runs["0"])):
    print(json.dumps({"iter": i, "dT": float(np.abs(a["T"] - b["T"]).max()), "kept": [a["kept"], b["kept"]],
                      "limit": [a["limit"], b["limit"]], "rejP": [a["rejP"], b["rejP"]], "rejM": [a["rejM"], b["rejM"]],
                      "nz": [a["nz"], b["nz"]], "sel_fused": a["sel"]}), flush=True)
