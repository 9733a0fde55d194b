"""DataPoints::load for .csv / .vtk (libpointmatcher_amd/csrc/host/pm_io.cpp,
reference IO.cpp:374-389, loadCSV :535-800, loadVTK :948-1252).  Host code:
these tests run without a GPU.

Pinned by the reference's own data files where they are present (the
examples/data clouds the golden fixtures were extracted from: same values
as tests/golden/clouds.npz) and by files written here in every layout the
loaders take: header / no header, the reference's delimiters, supported and
unknown columns (the label table's order, spans grown by repeated names, a
missing pad added), VTK ASCII and big-endian BINARY, POLYDATA cell blocks
skipped, UNSTRUCTURED_GRID, SCALARS (LOOKUP_TABLE) / NORMALS / VECTORS /
COLOR_SCALARS / FIELD arrays, and the reference's error messages.
"""
import os

import numpy as np
import pytest

from libpointmatcher_amd.icp import load_cloud

REF = "/root/reference/examples/data"


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference data not present")
def test_reference_files_match_golden(golden):
    g, _ = golden
    c = load_cloud(os.path.join(REF, "car_cloud400.csv"))
    assert c.feature_labels == [("x", 1), ("y", 1), ("z", 1), ("pad", 1)]
    assert c.descriptor_labels == [("normals", 3)]
    np.testing.assert_array_equal(c.features[:, :3], g["car400"].astype(np.float32))
    np.testing.assert_array_equal(c.descriptor("normals"), g["car400_normals"].astype(np.float32))
    c = load_cloud(os.path.join(REF, "2D_oneBox.csv"))
    assert c.features.shape[1] == 3 and np.all(c.features[:, 2] == 1)
    np.testing.assert_array_equal(c.features[:, :2], g["box1"].astype(np.float32))
    c = load_cloud(os.path.join(REF, "cloud.00000.vtk"))
    np.testing.assert_array_equal(c.features[:, :3], g["vtk0"])


def test_csv_header_labels_and_values(tmp_path):
    rng = np.random.default_rng(0)
    v = rng.normal(size=(50, 8)).round(6)
    p = tmp_path / "a.csv"
    names = ["foo", "x", "nz", "y", "ny", "intensity", "nx", "z"]
    with open(p, "w") as f:
        f.write(",".join(names) + "\n")
        for row in v:
            f.write(" , ".join(f"{x:.6f}" for x in row) + "\n")
    for dt in (np.float32, np.float64):
        c = load_cloud(p, dt)
        assert c.feature_labels == [("x", 1), ("y", 1), ("z", 1), ("pad", 1)]
        # table order (normals, intensity), then the unknown column
        assert c.descriptor_labels == [("normals", 3), ("intensity", 1), ("foo", 1)]
        ref = np.array([[float(f"{x:.6f}") for x in row] for row in v])
        np.testing.assert_array_equal(c.features[:, :3], ref[:, [1, 3, 7]].astype(dt))
        np.testing.assert_array_equal(c.descriptor("normals"), ref[:, [6, 4, 2]].astype(dt))
        np.testing.assert_array_equal(c.descriptor("foo")[:, 0], ref[:, 0].astype(dt))
        assert np.all(c.features[:, 3] == 1)


def test_csv_no_header_and_delimiters(tmp_path):
    p = tmp_path / "b.csv"
    p.write_text("1.5 2.5,3.5\n-1e-3\t, 4E2 ;+7\n\nignored after an empty line\n")
    c = load_cloud(p)
    assert c.features.shape == (2, 4)
    np.testing.assert_array_equal(c.features, np.array([[1.5, 2.5, 3.5, 1], [-1e-3, 400, 7, 1]], np.float32))
    # a first line with a tab / ';' / letter is a header (IO.cpp:571-580: only " ,+-.1234567890Ee" is data)
    ph = tmp_path / "h.csv"
    ph.write_text("1\t2\n3 4\n")
    c = load_cloud(ph)
    assert c.descriptor_labels == [("1", 1), ("2", 1)] and c.feature_labels == [("pad", 1)]
    p2 = tmp_path / "c.csv"
    p2.write_text("1 2 3 4\n")
    with pytest.raises(RuntimeError, match="columns"):
        load_cloud(p2)
    p3 = tmp_path / "d.csv"
    p3.write_text("x,y\n1,2\n1,2,3\n")
    with pytest.raises(RuntimeError, match="too many elements"):
        load_cloud(p3)
    p4 = tmp_path / "e.csv"
    p4.write_text("x,y,z\n1,2\n")
    with pytest.raises(RuntimeError, match="not enough elements"):
        load_cloud(p4)


def _vtk(path, pts, binary, dataset="POLYDATA", extra=b""):
    n = len(pts)
    with open(path, "wb") as f:
        f.write(b"# vtk DataFile Version 3.0\ntest\n" + (b"BINARY" if binary else b"ASCII") + b"\n")
        f.write(b"DATASET " + dataset.encode() + b"\n")
        f.write(f"POINTS {n} float\n".encode())
        if binary:
            f.write(pts.astype(">f4").tobytes() + b"\n")
        else:
            f.write(b"".join(f"{a:.7g} {b:.7g} {c:.7g}\n".encode() for a, b, c in pts))
        f.write(extra)


def test_vtk_ascii_and_binary(tmp_path):
    rng = np.random.default_rng(1)
    pts = rng.normal(size=(40, 3)).astype(np.float32)
    nrm = rng.normal(size=(40, 3)).astype(np.float32)
    sc = rng.normal(size=40).astype(np.float32)
    n = len(pts)
    for binary in (False, True):
        if binary:
            extra = (f"VERTICES {n} {2 * n}\n".encode() + np.array([[1, i] for i in range(n)], ">i4").tobytes() +
                     f"\nPOINT_DATA {n}\nNORMALS normals float\n".encode() + nrm.astype(">f4").tobytes() +
                     b"\nSCALARS densities float 1\nLOOKUP_TABLE default\n" + sc.astype(">f4").tobytes() + b"\n")
        else:
            extra = (f"VERTICES {n} {2 * n}\n".encode() + b"".join(f"1 {i}\n".encode() for i in range(n)) +
                     f"POINT_DATA {n}\nNORMALS normals float\n".encode() +
                     b"".join(f"{a:.7g} {b:.7g} {c:.7g}\n".encode() for a, b, c in nrm) +
                     b"SCALARS densities float 1\nLOOKUP_TABLE default\n" +
                     b"".join(f"{a:.7g}\n".encode() for a in sc))
        p = tmp_path / f"a{int(binary)}.vtk"
        _vtk(p, pts, binary, extra=extra)
        c = load_cloud(p)
        assert c.feature_labels == [("x", 1), ("y", 1), ("z", 1), ("pad", 1)]
        assert c.descriptor_labels == [("normals", 3), ("densities", 1)]
        exp_p = pts if binary else np.array([[np.float32(f"{x:.7g}") for x in r] for r in pts])
        np.testing.assert_array_equal(c.features[:, :3], exp_p)
        exp_n = nrm if binary else np.array([[np.float32(f"{x:.7g}") for x in r] for r in nrm])
        np.testing.assert_array_equal(c.descriptor("normals"), exp_n)


def test_vtk_unstructured_field_and_errors(tmp_path):
    pts = np.arange(12, dtype=np.float32).reshape(4, 3)
    extra = (b"CELLS 4 8\n1 0\n1 1\n1 2\n1 3\nCELL_TYPES 4\n1\n1\n1\n1\nPOINT_DATA 4\n"
             b"FIELD FieldData 1\nvel 2 4 float\n1 2\n3 4\n5 6\n7 8\n"
             b"COLOR_SCALARS color 3\n0.1 0.2 0.3\n0.4 0.5 0.6\n0.7 0.8 0.9\n1 1 1\n")
    p = tmp_path / "u.vtk"
    _vtk(p, pts, False, "UNSTRUCTURED_GRID", extra)
    c = load_cloud(p, np.float64)
    assert c.descriptor_labels == [("vel", 2), ("color", 3)]
    np.testing.assert_array_equal(c.descriptor("vel"), np.arange(1, 9).reshape(4, 2))
    bad = tmp_path / "bad.vtk"
    bad.write_bytes(b"# vtk DataFile Version 3.0\nx\nASCII\nDATASET STRUCTURED_POINTS\n")
    with pytest.raises(RuntimeError, match="Wrong data type"):
        load_cloud(bad)
    bad.write_bytes(b"not vtk\n")
    with pytest.raises(RuntimeError, match="magic header"):
        load_cloud(bad)
    mis = tmp_path / "m.vtk"
    _vtk(mis, pts, False, extra=b"POINT_DATA 3\n")
    with pytest.raises(RuntimeError, match="different than POINT_DATA"):
        load_cloud(mis)
    with pytest.raises(RuntimeError, match="extension"):
        load_cloud(tmp_path / "x.ply")


def test_vtk_malformed_blocks_rejected(tmp_path):
    """Point data before POINTS, a repeated POINTS block or a negative count
    raise instead of leaving short descriptor rows (over-read)."""
    head = b"# vtk DataFile Version 3.0\nx\nASCII\nDATASET POLYDATA\n"
    pts = b"POINTS 2 float\n0 0 0\n1 1 1\n"
    p = tmp_path / "f.vtk"
    p.write_bytes(head + b"FIELD FieldData 1\nTIME 1 1 double\n0.5\n" + pts)
    with pytest.raises(RuntimeError, match="before POINTS"):
        load_cloud(p)
    p.write_bytes(head + b"SCALARS d float 1\nLOOKUP_TABLE default\n1\n2\n" + pts)
    with pytest.raises(RuntimeError, match="before POINTS"):
        load_cloud(p)
    p.write_bytes(head + pts + b"POINTS 3 float\n0 0 0\n1 1 1\n2 2 2\n")
    with pytest.raises(RuntimeError, match="second POINTS"):
        load_cloud(p)
    p.write_bytes(head + b"POINTS -4 float\n")
    with pytest.raises(RuntimeError, match="bad POINTS count"):
        load_cloud(p)
    # well-formed point data after POINTS still loads
    p.write_bytes(head + pts + b"POINT_DATA 2\nSCALARS d float 1\nLOOKUP_TABLE default\n1\n2\n")
    c = load_cloud(p)
    assert c.descriptor_labels == [("d", 1)]
    np.testing.assert_array_equal(c.descriptor("d")[:, 0], [1, 2])
