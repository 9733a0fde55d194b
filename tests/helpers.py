"""Shared test helpers (test infrastructure)."""
import numpy as np


def hom(a, dtype=None):
    a = np.asarray(a)
    dtype = dtype or a.dtype
    return np.hstack([a, np.ones((a.shape[0], 1))]).astype(dtype)


def pca_normals(pts, k=10):
    """Unit normals by PCA over the k nearest neighbours (scipy cKDTree) —
    stands in for the reference's SurfaceNormal filter when a test needs
    reference normals on a cloud that has none."""
    from scipy.spatial import cKDTree

    tree = cKDTree(pts)
    _, idx = tree.query(pts, k=k)
    nb = pts[idx]
    c = nb - nb.mean(axis=1, keepdims=True)
    cov = np.einsum("nki,nkj->nij", c, c)
    w, v = np.linalg.eigh(cov)
    return v[:, :, 0]


def quat(R):
    """Eigen Quaternion(Matrix3) -> (x, y, z, w)."""
    t = R[0, 0] + R[1, 1] + R[2, 2]
    q = np.zeros(4)
    if t > 0:
        t = np.sqrt(t + 1.0)
        q[3] = 0.5 * t
        t = 0.5 / t
        q[0] = (R[2, 1] - R[1, 2]) * t
        q[1] = (R[0, 2] - R[2, 0]) * t
        q[2] = (R[1, 0] - R[0, 1]) * t
    else:
        i = 0
        if R[1, 1] > R[0, 0]:
            i = 1
        if R[2, 2] > R[i, i]:
            i = 2
        j, k = (i + 1) % 3, (i + 2) % 3
        t = np.sqrt(R[i, i] - R[j, j] - R[k, k] + 1.0)
        q[i] = 0.5 * t
        t = 0.5 / t
        q[3] = (R[k, j] - R[j, k]) * t
        q[j] = (R[j, i] + R[i, j]) * t
        q[k] = (R[k, i] + R[i, k]) * t
    return q


def angular_distance(Ra, Rb):
    a, b = quat(Ra), quat(Rb)
    a = a / np.linalg.norm(a)
    b = b / np.linalg.norm(b)
    d = abs(np.dot(a, b))
    return 2 * np.arccos(min(1.0, d))


def validate3d(T, V, tol):
    """utest/utest.h:64-85: translation-norm difference and rotation angle."""
    dt = abs(np.linalg.norm(V[:3, 3]) - np.linalg.norm(T[:3, 3]))
    da = angular_distance(np.asarray(T[:3, :3], np.float64), np.asarray(V[:3, :3], np.float64))
    return dt < tol and da < tol, dt, da


def validate2d(T, V, tol):
    """utest/utest.h:49-62: translation norm and acos(T00)."""
    dt = abs(np.linalg.norm(V[:2, 2]) - np.linalg.norm(T[:2, 2]))
    da = abs(np.arccos(np.clip(V[0, 0], -1, 1)) - np.arccos(np.clip(T[0, 0], -1, 1)))
    return dt < tol and da < tol, dt, da


def rel_displacement(curT, refT, pts):
    """utest/utest.cpp:139-153: median |curT p - refT p| / median |curT p|."""
    P = hom(pts, np.float64).T
    a = np.abs(np.asarray(curT, np.float64) @ P - np.asarray(refT, np.float64) @ P)
    b = np.abs(np.asarray(curT, np.float64) @ P)
    return np.median(a) / np.median(b)


def planar_grid():
    """utest/utest.cpp:167-183 (icpSingular): 10x10 grid, d=0.1, z=0 / z=1."""
    nX = nY = 10
    d = np.float32(0.1)
    oX = -(nX * d / 2)
    oY = -(nY * d / 2)
    pts = np.zeros((nX * nY, 4), np.float32)
    for x in range(nX):
        for y in range(nY):
            pts[x * nY + y] = [d * x + oX, d * y + oY, 0, 1]
    pts1 = pts.copy()
    pts1[:, 2] = 1
    return pts, pts1


CHAIN_P2PLANE = """
readingDataPointsFilters:
  - IdentityDataPointsFilter:
matcher:
  KDTreeMatcher:
    knn: {knn}
    epsilon: 0
    maxDist: {maxdist}
outlierFilters:
{filters}
errorMinimizer:
  {minimizer}
transformationCheckers:
  - CounterTransformationChecker:
      maxIterationCount: {maxit}
{diff}
inspector:
  NullInspector
logger:
  NullLogger
"""


def chain_yaml(knn=1, maxdist="inf", filters=(("TrimmedDistOutlierFilter", {"ratio": 0.85}),),
               minimizer="PointToPlaneErrorMinimizer", maxit=40, differential=None, bound=None):
    if filters:
        fl = []
        for name, p in filters:
            if p:
                fl.append(f"  - {name}:\n" + "".join(f"      {k}: {v}\n" for k, v in p.items()))
            else:
                fl.append(f"  - {name}\n")
        ftxt = "".join(fl)
    else:
        ftxt = ""
    diff = ""
    if differential:
        diff = ("  - DifferentialTransformationChecker:\n" +
                "".join(f"      {k}: {v}\n" for k, v in differential.items()))
    if bound:
        diff += ("  - BoundTransformationChecker:\n" +
                 "".join(f"      {k}: {v}\n" for k, v in bound.items()))
    return CHAIN_P2PLANE.format(knn=knn, maxdist=maxdist, filters=ftxt, minimizer=minimizer, maxit=maxit,
                                diff=diff)
