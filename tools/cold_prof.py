"""Per-wave profile of the cold tile form at a BASELINE config (development
tool): runs the config's first match a few times with tile_prof=2 and keeps
the last run's raw words (start / end stamps in 100 MHz ticks, rounds |
fallback lanes << 32, points copied) in tile_prof_<cfg>.npy.
Usage: python tools/cold_prof.py [c3] [out_dir]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from bench import CONFIGS  # noqa: E402
from libpointmatcher_amd import _capi as P  # noqa: E402
from libpointmatcher_amd.synth import reading_cloud, reference_cloud  # noqa: E402


def main(cfg="c3", out="."):
    N, M, dtype, knn, filters, minimizer = CONFIGS[cfg]
    ref, nrm = reference_cloud(M, dtype)
    rd = reading_cloud(N, dtype)
    ctx = P.Context(0, dtype)
    ctx.set_option("tile_prof", 2)
    ctx.set_reference(ref, nrm)
    for _ in range(4):
        ctx.set_reading(rd)
        ctx.loop_begin(knn=knn, filters=[(f, *p.values()) for f, p in filters], minimizer=minimizer,
                       checkers=[("CounterTransformationChecker", 1)], T0=np.eye(4, dtype=dtype))
        ctx.loop_run(1)
    ctx.close()
    w = np.fromfile("tile_prof.bin", dtype=np.uint64).reshape(-1, 4)
    os.remove("tile_prof.bin")
    np.save(os.path.join(out, f"tile_prof_{cfg}.npy"), w)
    d = (w[:, 1] - w[:, 0]) * 0.01
    fin = w[:, 0] + (w[:, 3] >> 32)  # (the wave's end after its fallback walks)
    fb = (w[:, 2] >> 32) > 0
    print(cfg, "waves", len(w), "span us", (w[:, 1].max() - w[:, 0].min()) * 0.01,
          "span with fallback us", (fin.max() - w[:, 0].min()) * 0.01, "sum us", d.sum(),
          "p50/p90/p99/max", np.percentile(d, [50, 90, 99, 100]), "fallback waves", int(fb.sum()),
          "lanes", int((w[:, 2] >> 32).sum()), "their walk us max", ((fin - w[:, 1]) * 0.01)[fb].max() if fb.any() else 0)


if __name__ == "__main__":
    main(*sys.argv[1:])
