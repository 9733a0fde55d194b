"""Where a fresh process's first prepare goes (development tool): the
library load, the context creation (HIP runtime + the grid module's
preload), the first reference (setup kernels' modules loaded on first
launch), the first reading, and the same two calls again.
Usage: python tools/first_use.py [c3]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))


def main(cfg="c3"):
    t0 = time.perf_counter()
    from bench import CONFIGS
    from libpointmatcher_amd.synth import reading_cloud, reference_cloud
    N, M, dtype, *_ = CONFIGS[cfg]
    ref, nrm = reference_cloud(M, dtype)
    rd = reading_cloud(N, dtype)
    t1 = time.perf_counter()
    from libpointmatcher_amd import _capi as P
    t2 = time.perf_counter()
    ctx = P.Context(0, dtype)
    t3 = time.perf_counter()
    ctx.set_reference(ref, nrm)
    ctx.sync() if hasattr(ctx, "sync") else None
    t4 = time.perf_counter()
    ctx.set_reading(rd)
    ctx.sync() if hasattr(ctx, "sync") else None
    t5 = time.perf_counter()
    ctx.set_reference(ref, nrm)
    ctx.set_reading(rd)
    ctx.sync() if hasattr(ctx, "sync") else None
    t6 = time.perf_counter()
    ms = lambda a, b: round((b - a) * 1e3, 1)
    print({"clouds_ms": ms(t0, t1), "library_load_ms": ms(t1, t2), "context_create_ms": ms(t2, t3),
           "first_reference_ms": ms(t3, t4), "first_reading_ms": ms(t4, t5), "again_both_ms": ms(t5, t6)})
    ctx.close()


if __name__ == "__main__":
    main(*sys.argv[1:])
