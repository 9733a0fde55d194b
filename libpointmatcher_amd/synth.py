"""Deterministic synthetic clouds for the benchmark configurations.

Surface: area-weighted samples on the inner faces of the box
[-10,10] x [-6,6] x [-3,3] plus a sphere of radius 3 centred at (2, 1, 0.5),
with analytic unit normals (constrains all 6 DOF).  Reference: M samples,
seed 1, no noise.  Reading: N samples, seed 2, isotropic Gaussian noise
sigma = 0.01, then mapped by T_gt^-1 (3 degrees about normalize(1,2,3),
translation (0.05, -0.03, 0.02)), so ICP(reading -> reference) recovers T_gt.
numpy's PCG64 makes the clouds identical on every machine with numpy 2.x.
"""
from __future__ import annotations

import numpy as np

BOX = (10.0, 6.0, 3.0)
SPHERE_C = np.array([2.0, 1.0, 0.5])
SPHERE_R = 3.0


def t_gt():
    ax = np.array([1.0, 2.0, 3.0])
    ax /= np.linalg.norm(ax)
    a = np.deg2rad(3.0)
    K = np.array([[0, -ax[2], ax[1]], [ax[2], 0, -ax[0]], [-ax[1], ax[0], 0]])
    R = np.eye(3) + np.sin(a) * K + (1 - np.cos(a)) * K @ K
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = [0.05, -0.03, 0.02]
    return T


def surface(n, seed):
    """n points (float64) and unit normals on the box+sphere surface."""
    rng = np.random.default_rng(seed)
    X, Y, Z = BOX
    areas = np.array([4 * Y * Z, 4 * Y * Z, 4 * X * Z, 4 * X * Z, 4 * X * Y, 4 * X * Y,
                      4 * np.pi * SPHERE_R ** 2])
    counts = rng.multinomial(n, areas / areas.sum())
    P, Nn = [], []
    specs = [(0, +X), (0, -X), (1, +Y), (1, -Y), (2, +Z), (2, -Z)]
    half = np.array(BOX)
    for (axis, val), c in zip(specs, counts[:6]):
        p = rng.uniform(-1.0, 1.0, size=(c, 3)) * half
        p[:, axis] = val
        nn = np.zeros((c, 3))
        nn[:, axis] = -np.sign(val)  # inner faces: normal points inside
        P.append(p)
        Nn.append(nn)
    c = counts[6]
    v = rng.normal(size=(c, 3))
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    P.append(SPHERE_C + SPHERE_R * v)
    Nn.append(v)
    P = np.concatenate(P)
    Nn = np.concatenate(Nn)
    perm = rng.permutation(n)
    return P[perm], Nn[perm]


def reference_cloud(M, dtype=np.float32, seed=1):
    """(M, 4) homogeneous reference and (M, 3) normals."""
    P, Nn = surface(M, seed)
    feat = np.hstack([P, np.ones((M, 1))])
    return feat.astype(dtype), Nn.astype(dtype)


def reading_cloud(N, dtype=np.float32, seed=2, noise=0.01):
    """(N, 4) homogeneous reading = T_gt^-1 (surface + noise)."""
    P, _ = surface(N, seed)
    rng = np.random.default_rng(seed + 1000)
    P = P + rng.normal(scale=noise, size=P.shape)
    Ti = np.linalg.inv(t_gt())
    P = P @ Ti[:3, :3].T + Ti[:3, 3]
    return np.hstack([P, np.ones((N, 1))]).astype(dtype)


def random_cloud(n, rows=4, seed=0, dtype=np.float32, scale=1.0):
    rng = np.random.default_rng(seed)
    p = rng.uniform(-scale, scale, size=(n, rows - 1))
    return np.hstack([p, np.ones((n, 1))]).astype(dtype)
