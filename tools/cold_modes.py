"""Cold (initial-pose) grid match at C3 under the search variants (development
tool): per-lane shell search at each first level, the LDS tile kernel and the
octant-first search.  Each variant runs in its own process (the knobs are read
at context creation).  Prints one JSON line per variant."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, sys, time
import numpy as np
sys.path.insert(0, %r)
from libpointmatcher_amd import _capi
from libpointmatcher_amd.synth import reading_cloud, reference_cloud
N = int(os.environ.get("COLD_N", "1000000"))
ref, nrm = reference_cloud(N, np.float32)
rd = reading_cloud(N, np.float32)
out = []
for rep in range(3):
    ctx = _capi.Context(0, np.float32)
    ctx.set_reference(ref, nrm)
    ctx.set_reading(rd)
    ctx.timing(True)
    ctx.match(np.eye(4, dtype=np.float32), knn=1)
    ctx.outlier("TrimmedDistOutlierFilter", 0, ratio=0.85)
    A, b, st = ctx.p2plane_system()
    ms, n = ctx.timing_read()
    out.append((ms / max(n, 1), st.visited / N, st.fallback_queries))
    ctx.close()
print(json.dumps({"env": {k: v for k, v in os.environ.items() if k.startswith("PMX_")},
                  "cold_ms": [o[0] for o in out], "pairs_per_query": out[-1][1]}), flush=True)
""" % ROOT

VARIANTS = [{"PMX_GRID_FIRST_PPC": str(p)} for p in (2, 4, 8, 16, 32, 64)]
VARIANTS += [{"PMX_GRID_MODE": "tile"}, {"PMX_GRID_MODE": "octant"},
             {"PMX_GRID_MODE": "tile", "PMX_GRID_FIRST_PPC": "4"}]
if len(sys.argv) > 1:
    VARIANTS = [dict(kv.split("=", 1) for kv in a.split(",")) for a in sys.argv[1:]]

for v in VARIANTS:
    env = dict(os.environ)
    env.update(v)
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
    line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else json.dumps({"env": v, "error": r.stderr[-400:]})
    print(line, flush=True)
