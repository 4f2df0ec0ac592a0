"""output_results (boussinesq_model.tpp:1566-1680) as dcp_write_vtu: the VTU
of DataOut::build_patches(2) with the Postprocessor's fields (host-only)."""
import xml.etree.ElementTree as ET

import numpy as np

import dcp


def _arrays(path):
    root = ET.parse(path).getroot()
    piece = root.find("UnstructuredGrid/Piece")
    out = {"npts": int(piece.get("NumberOfPoints")), "ncells": int(piece.get("NumberOfCells"))}
    for da in root.iter("DataArray"):
        name = da.get("Name") or "points"
        out[name] = np.array(da.text.split(), dtype=np.float64)
    return out


def test_vtu_patches_and_fields(tmp_path):
    m = dcp.HostMesh(refine=1)
    rng = np.random.default_rng(3)
    # velocity = the node coordinates (a Q2 field), p = 2 + x-coordinate-free constant, T = T0
    u = np.zeros(m.n_u + m.n_p)
    u[:m.n_u] = m.node_xyz.reshape(-1)
    u[m.n_u:] = 2.0 + rng.uniform(-1, 1, m.n_p)
    path = tmp_path / "boussinesq-00000.0000.vtu"
    m.write_vtu(path, u, m.T0, partition=0)
    a = _arrays(path)
    assert a["npts"] == 27 * m.n_cells and a["ncells"] == 8 * m.n_cells
    assert a["connectivity"].size == 8 * a["ncells"]
    assert np.all(a["types"] == 12)                        # VTK_HEXAHEDRON
    assert np.array_equal(a["offsets"], 8 * np.arange(1, a["ncells"] + 1))
    vel = a["velocity"].reshape(-1, 3)
    pts = a["points"].reshape(-1, 3)
    # every patch point carries a nodal velocity value (the lattice = the Q2 nodes)
    assert np.allclose(np.sort(np.unique(np.round(vel, 12), axis=0), axis=0),
                       np.sort(np.unique(np.round(m.node_xyz, 12), axis=0), axis=0))
    # the patch corners are the cell vertices under any mapping: there the
    # velocity field (= the node coordinates) equals the point; the other
    # lattice points are placed by DataOut's MappingQ1, off the curved nodes
    d = np.linalg.norm(vel - pts, axis=1).reshape(m.n_cells, 27)
    corners = [i + 3 * j + 9 * k for k in (0, 2) for j in (0, 2) for i in (0, 2)]
    assert d[:, corners].max() < 1e-12
    assert d.max() < 0.5
    # Q1 fields interpolated inside their vertex range; partition constant
    assert a["T"].min() >= m.T0.min() - 1e-12 and a["T"].max() <= m.T0.max() + 1e-12
    assert a["p"].min() >= u[m.n_u:].min() - 1e-12 and a["p"].max() <= u[m.n_u:].max() + 1e-12
    assert np.all(a["partition"] == 0)


def test_pvtu_record(tmp_path):
    import ctypes as C
    names = [b"boussinesq-00000.0000.vtu", b"boussinesq-00000.0001.vtu"]
    arr = (C.c_char_p * 2)(*names)
    path = tmp_path / "boussinesq-00000.pvtu"
    assert dcp.lib().dcp_write_pvtu_record(str(path).encode(), 2, arr) == 0
    root = ET.parse(path).getroot()
    assert [p.get("Source") for p in root.iter("Piece")] == [n.decode() for n in names]
    assert [d.get("Name") for d in root.iter("PDataArray") if d.get("Name")] == \
        ["velocity", "p", "T", "partition"]
