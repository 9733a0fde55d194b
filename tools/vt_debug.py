"""VarTrimmed partial sums on the spread/jump parity data, with the walk's
trace (development tool): prints the first differing sums and the walk's
steps.  usage: PMX_OPTS=vt_trace=1 python tools/vt_debug.py [jump|decades] [f32|f64]"""
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "tests"))
from libpointmatcher_amd import _capi as P  # noqa: E402
from test_gpu_kernels import _spread_clouds  # noqa: E402

data = sys.argv[1] if len(sys.argv) > 1 else "jump"
dtype = np.float64 if len(sys.argv) > 2 and sys.argv[2] == "f64" else np.float32
rng = np.random.default_rng(11)
ref, rd = _spread_clouds(64, dtype, rng, data == "jump")
ctx = P.Context(0, dtype)
ctx.set_reference(ref)
ctx.set_reading(rd)
ctx.match(np.eye(4, dtype=dtype), knn=1)
ctx.outlier("VarTrimmedDistOutlierFilter", 0, minRatio=0.05, maxRatio=0.99, **{"lambda": 2.35})
d, _ = ctx.get_matches()
cum = ctx.vartrim_partial_sums()
ctx.close()
keys = np.sort(d[np.isfinite(d) & (d > 0)].astype(dtype))
rc = np.cumsum(keys, dtype=dtype)
U = np.uint32 if dtype == np.float32 else np.uint64
bad = np.flatnonzero(cum.view(U) != rc.view(U))
print("n", len(keys), "bad", bad.size, "range", bad[:1], bad[-1:])
first_big = int(np.argmax(keys > 1e-3))
print("first big key", first_big)
for i in list(range(max(0, bad[0] - 3), bad[0] + 12)) if bad.size else []:
    print(i, repr(keys[i]), repr(cum[i]), repr(rc[i]), int(cum.view(U)[i]) - int(rc.view(U)[i]))
