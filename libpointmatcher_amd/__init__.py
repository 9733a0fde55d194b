"""libpointmatcher_amd — an MI355X-native ICP inner loop behind libpointmatcher's
Matcher / OutlierFilter / ErrorMinimizer interfaces.

Layout:
  csrc/*.hip        HIP kernels for gfx950 + the C ABI of include/pmx.h
  csrc/host/*.cpp   host C++ ICP chain (PointMatcher<T>::ICP restated, YAML
                    config, registry) calling the C ABI — lib/libpmx_icp.so
  _capi.py          ctypes binding of the C ABI (tests / bench plumbing)
  icp.py            ctypes binding of the host ICP chain
  synth.py          deterministic synthetic clouds of the benchmark configs
"""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

__all__ = ["build", "HERE", "ROOT"]


def build(jobs: int = 8) -> None:
    """Compile libpmx.so (HIP, gfx950) and libpmx_icp.so in-tree."""
    subprocess.check_call(["make", "-s", "-C", HERE, f"-j{jobs}", "all"])
