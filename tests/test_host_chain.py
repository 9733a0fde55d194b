"""Host-side logic that runs without a GPU: the C-ABI libraries load and export
every declared symbol, the YAML chain loader and registry behave like the
reference's (ICP.cpp:116-167, Registrar.h:98-135, Parametrizable.cpp:170-192),
and the product path fails loudly (no CPU fallback) when no GPU is present.
"""
import ctypes
import os
import re

import numpy as np
import pytest

from helpers import chain_yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(pmx_[a-z0-9_]+)\s*\(", txt)))


@pytest.mark.parametrize("header,lib", [("pmx.h", "libpmx.so"), ("pmx_icp.h", "libpmx_icp.so")])
def test_c_abi_exports_every_declared_symbol(header, lib):
    from libpointmatcher_amd import _capi
    _capi.lib()
    l = ctypes.CDLL(os.path.join(ROOT, "libpointmatcher_amd", "lib", lib))
    names = declared(header)
    assert len(names) >= 10
    missing = [n for n in names if not hasattr(l, n)]
    assert not missing, missing


def test_capi_python_binding_covers_header():
    from libpointmatcher_amd import _capi
    assert set(declared("pmx.h")) == set(_capi.EXPORTS)


def test_no_gpu_fails_loudly():
    from libpointmatcher_amd import _capi
    if _capi.device_count() > 0:
        pytest.skip("GPU present")
    with pytest.raises(_capi.PmxError):
        _capi.Context(0, np.float32)
    from libpointmatcher_amd.icp import ICP
    icp = ICP(np.float32)
    icp.load_yaml(chain_yaml())
    pts = np.ones((10, 4), np.float32)
    with pytest.raises(RuntimeError, match="pmx_ctx_create failed"):
        icp.compute(pts, pts, np.ones((10, 3), np.float32))


REF_DATA = "/root/reference/examples/data"


def test_yaml_loads_reference_chain_files():
    from libpointmatcher_amd.icp import ICP
    icp = ICP(np.float32)
    icp.load_yaml(chain_yaml(knn=4, maxdist=0.5, filters=[("MaxDistOutlierFilter", {"maxDist": 0.05}),
                                                         ("NullOutlierFilter", {})],
                             differential=dict(minDiffRotErr=0.001, minDiffTransErr=0.01, smoothLength=4)))
    icp.set_default()
    yaml_default_identity = """
readingDataPointsFilters:
  - IdentityDataPointsFilter:

referenceDataPointsFilters:
  - SamplingSurfaceNormalDataPointsFilter:
      knn: 10
      ratio: 1.0
      samplingMethod: 0
      averageExistingDescriptors: 0

matcher:
  KDTreeMatcher:
    knn: 1
    epsilon: 0

outlierFilters:
  - TrimmedDistOutlierFilter:
      ratio: 1.0

errorMinimizer:
  PointToPlaneErrorMinimizer

transformationCheckers:
  - CounterTransformationChecker:
      maxIterationCount: 40
  - DifferentialTransformationChecker:
      minDiffRotErr: 0.001
      minDiffTransErr: 0.01
      smoothLength: 4

inspector:
  NullInspector
#  VTKFileInspector

logger:
  NullLogger
"""
    icp.load_yaml(yaml_default_identity)  # examples/data/default-identity.yaml


BAD_MODULE_TYPE = """
FAKE_MODULE_NAME:
  - RandomSamplingDataPointsFilter:
      prob: 0.5
matcher:
  KDTreeMatcher:
    knn: 1
errorMinimizer:
  PointToPlaneErrorMinimizer
inspector:
  NullInspector
"""

BAD_PARAMETER = """
readingDataPointsFilters:
  - RandomSamplingDataPointsFilter:
      FAKE_PARAM: 0.5
      prob: 0.5
matcher:
  KDTreeMatcher:
    knn: 1
"""


def test_yaml_errors_like_reference():
    # examples/data/unit_tests/badIcpConfig_*.yaml (utest/ui/IO.cpp:23-28)
    from libpointmatcher_amd import icp as I
    icp = I.ICP(np.float32)
    with pytest.raises(I.InvalidModuleType, match="FAKE_MODULE_NAME"):
        icp.load_yaml(BAD_MODULE_TYPE)
    with pytest.raises(I.InvalidParameter, match="FAKE_PARAM"):
        icp.load_yaml(BAD_PARAMETER)
    # bounds (Parametrizable.cpp:170-192): ratio in [1e-7, 1]
    with pytest.raises(I.InvalidParameter, match="larger than maximum"):
        icp.load_yaml(chain_yaml(filters=[("TrimmedDistOutlierFilter", {"ratio": 1.5})]))
    with pytest.raises(I.InvalidParameter, match="smaller than minimum"):
        icp.load_yaml(chain_yaml(knn=0))
    with pytest.raises(I.InvalidElement, match="NoSuchMatcher"):
        icp.load_yaml("matcher:\n  NoSuchMatcher\n")
    with pytest.raises(I.InvalidParameter, match="minRatio"):
        icp.load_yaml(chain_yaml(filters=[("VarTrimmedDistOutlierFilter", {"minRatio": 0.9, "maxRatio": 0.5})]))
    # a module without parameters rejects any parameter
    with pytest.raises(I.InvalidParameter, match="dos not use any parameter"):
        icp.load_yaml("errorMinimizer:\n  PointToPointErrorMinimizer:\n    foo: 1\n")
    # missing inspector -> reset -> runtime error at compute (ICP.cpp:271-276)
    icp.load_yaml("matcher:\n  KDTreeMatcher\nerrorMinimizer:\n  PointToPointErrorMinimizer\n")
    pts = np.ones((4, 4), np.float32)
    with pytest.raises(RuntimeError, match="inspector"):
        icp.compute(pts, pts)


def test_robust_outlier_filter_parameter_errors():
    # RobustOutlierFilter's constructor checks (OutlierFiltersImpl.cpp:409-417, 447-450)
    from libpointmatcher_amd import icp as I
    icp = I.ICP(np.float32)
    for bad, msg in ((dict(robustFct="foo"), "Invalid robust function name."),
                     (dict(scaleEstimator="foo"), "Invalid scale estimator name."),
                     (dict(distanceType="foo"), "Invalid distance type name."),
                     (dict(tuning=0), "smaller than minimum"),
                     (dict(nbIterationForScale=101), "larger than maximum")):
        with pytest.raises(I.InvalidParameter, match=msg):
            icp.load_yaml(chain_yaml(filters=[("RobustOutlierFilter", bad)]))
    icp.load_yaml(chain_yaml(filters=[("RobustOutlierFilter", dict(robustFct="student", scaleEstimator="berg",
                                                                   approximation="inf"))]))


def test_yaml_inf_and_numbers():
    from libpointmatcher_amd import icp as I
    icp = I.ICP(np.float64)
    icp.load_yaml(chain_yaml(maxdist="inf", filters=[("MaxDistOutlierFilter", {"maxDist": "inf"})]))
    with pytest.raises(I.InvalidParameter):
        icp.load_yaml(chain_yaml(maxdist="-1"))


def test_add_descriptor_rejects_bad_arguments():
    """pmx_icp_add_descriptor is guarded (no exception crosses the C ABI) and
    the Python binding accepts only the two cloud names."""
    from libpointmatcher_amd.icp import ICP, lib
    from libpointmatcher_amd._capi import InvalidParameter
    icp = ICP(np.float32)
    with pytest.raises(ValueError, match="reading"):
        icp.add_descriptor("readings", "maxSearchDist", np.ones(4, np.float32))
    l = lib()
    v = np.ones(4, np.float32)
    assert l.pmx_icp_add_descriptor(icp.h, 0, b"d", 1, v.ctypes.data_as(ctypes.c_void_p), -1) == -3
    assert l.pmx_icp_add_descriptor(icp.h, 0, b"d", 1, v.ctypes.data_as(ctypes.c_void_p), 1 << 62) == -3
    assert l.pmx_icp_add_descriptor(icp.h, 2, b"d", 1, v.ctypes.data_as(ctypes.c_void_p), 4) == -3
    assert "bad arguments" in l.pmx_icp_last_error(icp.h).decode()
    icp.add_descriptor("reading", "maxSearchDist", v)  # a well-formed one is staged
    _ = InvalidParameter


def test_sequence_without_map_is_identity():
    """ICPSequence::compute with no map returns the identity and an empty
    setMap is ignored (ICP.cpp:477-481, 599-604); neither touches the GPU."""
    from libpointmatcher_amd.icp import ICPSequence
    from libpointmatcher_amd.synth import reading_cloud

    for dt in (np.float32, np.float64):
        s = ICPSequence(dt)
        s.set_default()
        np.testing.assert_array_equal(s.compute(reading_cloud(50, dt)), np.eye(4, dtype=dt))
        assert not s.set_map(np.zeros((0, 4), dt))
        assert not s.has_map()
        assert not s.prepare(reading_cloud(50, dt))
        s.close()
