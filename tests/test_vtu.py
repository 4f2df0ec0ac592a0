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


def _one_cell_feec(J, x0, sign_w, sign_u):
    """A hand-built one-cell FEEC mesh: the affine cell x = x0 + J xi."""
    import ctypes as C
    v = dcp.FeecMeshView()
    X = np.array([x0 + J @ np.array([i & 1, (i >> 1) & 1, i >> 2], float) for i in range(8)])
    keep = {"X": np.ascontiguousarray(X.reshape(-1)), "cw": np.arange(12, dtype=np.int32),
            "cu": np.arange(6, dtype=np.int32), "sw": np.asarray(sign_w, np.int8),
            "su": np.asarray(sign_u, np.int8), "d": np.ones(1), "ct": np.arange(8, dtype=np.int32),
            "wf": np.zeros(12, np.uint8), "uf": np.zeros(6, np.uint8)}
    v.n_cells, v.n_w, v.n_u, v.n_p, v.n_T = 1, 12, 6, 1, 8
    for name, key, ct in (("cell_w", "cw", C.c_int32), ("sign_w", "sw", C.c_int8),
                          ("cell_u", "cu", C.c_int32), ("sign_u", "su", C.c_int8),
                          ("cell_vertices", "X", C.c_double), ("cell_diameter", "d", C.c_double),
                          ("cell_T_dofs", "ct", C.c_int32), ("w_fixed", "wf", C.c_uint8),
                          ("u_fixed", "uf", C.c_uint8)):
        setattr(v, name, keep[key].ctypes.data_as(C.POINTER(ct)))
    return v, X, keep


def test_feec_vtu_reproduces_constant_fields(tmp_path):
    """FEEC output_results (boussineq_model_FEEC.tpp:1917-2030) on one affine
    cell: the lowest-order Nedelec interpolant of a constant vorticity W
    (edge dofs = the tangential integrals, here (J^T W)_axis) and the RT
    interpolant of a constant velocity U (face dofs = the reference fluxes,
    (det J J^-1 U)_axis) are exact, so every vertex must carry W and U through
    the covariant / contravariant Piola maps, with the orientation signs
    undone; p is the cell value, T the vertex values."""
    rng = np.random.default_rng(12)
    J = np.eye(3) + 0.3 * rng.uniform(-1, 1, (3, 3))
    x0 = rng.uniform(-1, 1, 3)
    W, U = rng.uniform(-1, 1, 3), rng.uniform(-1, 1, 3)
    sw, su = rng.choice([-1, 1], 12), rng.choice([-1, 1], 6)
    v, X, keep = _one_cell_feec(J, x0, sw, su)
    line_axis = [1, 1, 0, 0, 1, 1, 0, 0, 2, 2, 2, 2]
    w_ref = J.T @ W
    u_ref = np.linalg.det(J) * np.linalg.solve(J, U)
    x = np.zeros(12 + 6 + 1)
    x[:12] = [sw[l] * w_ref[line_axis[l]] for l in range(12)]
    x[12:18] = [su[f] * u_ref[f // 2] for f in range(6)]
    x[18] = 3.25
    T = rng.uniform(0, 1, 8)
    path = tmp_path / "feec-00000.0000.vtu"
    rc = dcp.lib().dcp_write_feec_vtu(v, dcp._ptr(x), dcp._ptr(T), 0, str(path).encode())
    assert rc == dcp.DCP_OK
    a = _arrays(path)
    assert a["npts"] == 8 and a["ncells"] == 1 and np.all(a["types"] == 12)
    assert np.allclose(a["points"].reshape(-1, 3), X, rtol=0, atol=1e-15)
    assert np.allclose(a["vorticity"].reshape(-1, 3), W[None, :], rtol=0, atol=1e-13)
    assert np.allclose(a["velocity"].reshape(-1, 3), U[None, :], rtol=0, atol=1e-13)
    assert np.all(a["p"] == 3.25) and np.allclose(a["T"], T, rtol=0, atol=0)
    # VTK_HEXAHEDRON from the lexicographic vertices: bottom face counter-clockwise
    assert list(a["connectivity"].astype(int)) == [0, 1, 3, 2, 4, 5, 7, 6]


def test_feec_vtu_on_the_shell(tmp_path):
    """The shell's FEEC topology: one hexahedron per cell, p constant per cell,
    T at the vertices, and the pvtu record naming the vorticity array too."""
    m = dcp.HostMesh(refine=1, feec=True)
    f = m.feec
    rng = np.random.default_rng(4)
    x = rng.uniform(-1, 1, f.n)
    path = tmp_path / "feec-00001.0000.vtu"
    f.write_vtu(path, x, m.T0)
    a = _arrays(path)
    assert a["npts"] == 8 * f.n_cells and a["ncells"] == f.n_cells
    assert np.allclose(a["points"].reshape(-1, 8, 3), f.cell_vertices, rtol=0, atol=0)
    assert np.array_equal(a["p"].reshape(-1, 8), np.repeat(x[f.n_w + f.n_u:, None], 8, axis=1))
    assert np.array_equal(a["T"].reshape(-1, 8), m.T0[f.cell_T_dofs])
    assert np.all(np.isfinite(a["vorticity"])) and np.all(np.isfinite(a["velocity"]))
    import ctypes as C
    pv = tmp_path / "feec-00001.pvtu"
    pieces = (C.c_char_p * 1)(b"feec-00001.0000.vtu")
    assert dcp.lib().dcp_write_feec_pvtu_record(str(pv).encode(), 1, pieces) == dcp.DCP_OK
    txt = pv.read_text()
    assert 'Name="vorticity"' in txt and 'Name="velocity"' in txt and "feec-00001.0000.vtu" in txt


def test_periodic_feec_one_cell_across_is_rejected():
    """FEEC on the cuboid identifies the x = 1 / y = 1 edges and faces with
    their x = 0 / y = 0 partners (feec_mesh.cpp); with one cell across
    (refinement 0) a cell would hold the same dof twice, which the concurrent
    scatter cannot take: refused up front."""
    import pytest
    with pytest.raises(dcp.DcpError) as e:
        dcp.HostMesh(cuboid=True, refine=0, feec=True)
    assert e.value.code == dcp.DCP_ERR_UNSUPPORTED
    m = dcp.HostMesh(cuboid=True, refine=1, feec=True)
    assert m.feec.n_p == 8
