"""Generate the committed golden fixtures from the reference's own test data.

Run once in the build container (where /root/reference exists):
    python tests/golden/make_fixtures.py
Outputs (data only, no reference source) go to tests/golden/:
  - clouds.npz: the point clouds the reference's tests load
      (examples/data/car_cloud400.csv [with nx,ny,nz], car_cloud401.csv,
       2D_oneBox.csv, 2D_twoBoxes.csv, cloud.00000.vtk, cloud.00001.vtk),
      stored as float32 (n, D) arrays;
  - kat.json: known answers transcribed from the reference tests
      (utest/utest.cpp:346-356 validT2d/validT3d; utest/utest.h:49-85
       tolerances; utest/ui/Outliers.cpp:126-152 VarTrimmed KAT), the
      examples/data/icp_data/*.ref_trans regression transforms and the
      icp_data/*.yaml chain configurations they are the answers for (test
      inputs of utest.cpp:81-160, loaded unchanged by the GPU chain).
"""
import json
import os
import re

import numpy as np

REF = "/root/reference/examples/data"
OUT = os.path.dirname(os.path.abspath(__file__))


def load_csv(path):
    with open(path) as f:
        lines = [l.strip() for l in f if l.strip()]
    header = None
    if re.match(r"^[A-Za-z]", lines[0]):
        header = [h.strip() for h in lines[0].split(",")]
        lines = lines[1:]
    rows = [[float(x) for x in re.split(r"[,\s]+", l) if x] for l in lines]
    return header, np.array(rows, dtype=np.float64)


def load_vtk_points(path):
    with open(path) as f:
        toks = f.read().split()
    i = toks.index("POINTS")
    n = int(toks[i + 1])
    vals = np.array([float(x) for x in toks[i + 3: i + 3 + 3 * n]], dtype=np.float64)
    return vals.reshape(n, 3)


def main():
    clouds = {}
    h, a = load_csv(os.path.join(REF, "car_cloud400.csv"))
    assert h[:3] == ["x", "y", "z"] and h[3:6] == ["nx", "ny", "nz"], h
    clouds["car400"] = a[:, :3].astype(np.float32)
    clouds["car400_normals"] = a[:, 3:6].astype(np.float32)
    _, a = load_csv(os.path.join(REF, "car_cloud401.csv"))
    clouds["car401"] = a[:, :3].astype(np.float32)
    _, a = load_csv(os.path.join(REF, "2D_oneBox.csv"))
    clouds["box1"] = a[:, :2].astype(np.float32)
    _, a = load_csv(os.path.join(REF, "2D_twoBoxes.csv"))
    clouds["box2"] = a[:, :2].astype(np.float32)
    clouds["vtk0"] = load_vtk_points(os.path.join(REF, "cloud.00000.vtk")).astype(np.float32)
    clouds["vtk1"] = load_vtk_points(os.path.join(REF, "cloud.00001.vtk")).astype(np.float32)
    np.savez_compressed(os.path.join(OUT, "clouds.npz"), **clouds)

    ref_trans = {}
    d = os.path.join(REF, "icp_data")
    for fn in sorted(os.listdir(d)):
        if fn.endswith(".ref_trans"):
            with open(os.path.join(d, fn)) as f:
                vals = [float(x) for x in f.read().split()]
            ref_trans[fn[:-len(".ref_trans")]] = np.array(vals).reshape(4, 4).tolist()
    configs = {}
    for fn in sorted(os.listdir(d)):
        if fn.endswith(".yaml"):
            with open(os.path.join(d, fn)) as f:
                configs[fn[:-len(".yaml")]] = f.read()

    kat = {
        # utest/utest.cpp:346-356 (reading = 2D_twoBoxes / car_cloud401,
        # reference = 2D_oneBox / car_cloud400; utest.cpp:335-338)
        "validT2d": [[0.987498, 0.157629, 0.0859918],
                     [-0.157629, 0.987498, 0.203247],
                     [0, 0, 1]],
        "validT3d": [[0.982304, 0.166685, -0.0854066, 0.0446816],
                     [-0.150189, 0.973488, 0.172524, 0.191998],
                     [0.111899, -0.156644, 0.981296, -0.0356313],
                     [0, 0, 0, 1]],
        # utest/utest.h:60-61 and :81-82
        "tol2d": 0.05,
        "tol3d": 0.1,
        # utest/ui/Outliers.cpp:126-152
        "vartrim": {"dists": [4, 5, 5, 5, 5], "minRatio": 1e-7, "maxRatio": 1.0,
                    "lambda0_w": [1, 0, None, None, None], "lambda1_w": [1, 1, None, None, None]},
        # utest/utest.cpp:81-160: median relative displacement < 3 %
        "icp_data_rel_tol": 0.03,
        "icp_data_ref_trans": ref_trans,
        "icp_data_configs": configs,
    }
    with open(os.path.join(OUT, "kat.json"), "w") as f:
        json.dump(kat, f, indent=1)
    print("wrote", sorted(clouds), len(ref_trans), "ref_trans")


if __name__ == "__main__":
    main()
