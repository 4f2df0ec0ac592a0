"""Host setup (mesh / DoFs / constraints) — the data setup_dofs() produces
(boussinesq_model.tpp:184-412) restated without deal.II."""
import numpy as np
import pytest

import dcp

# SURVEY §6 size table: cells 6*8^r, n_u = 3*(6(2N)^2+2)(2N+1), n_p = (6N^2+2)(N+1)
@pytest.mark.parametrize("r", [0, 1, 2, 3])
def test_shell_sizes(r):
    m = dcp.HostMesh(refine=r)
    N = 2 ** r
    assert m.n_cells == 6 * 8 ** r
    assert m.n_u == 3 * (6 * (2 * N) ** 2 + 2) * (2 * N + 1)
    assert m.n_p == (6 * N ** 2 + 2) * (N + 1)
    assert m.n_T == m.n_p


def test_dof_layout_component_wise():
    m = dcp.HostMesh(refine=2)
    d = m.cell_nse_dofs
    # FESystem order: vertex v -> 4v..4v+3 (u_x,u_y,u_z,p); velocity blocks first
    for v in range(8):
        assert np.all(d[:, 4 * v + 1] == d[:, 4 * v] + 1)
        assert np.all(d[:, 4 * v + 2] == d[:, 4 * v] + 2)
        assert np.all(d[:, 4 * v + 3] >= m.n_u)
    assert np.all(d[:, 32:] < m.n_u)
    # distribute_dofs numbers on first encounter: first cell gets the lowest indices
    assert sorted(d[0, [0, 4, 8, 12, 16, 20, 24, 28]] // 3) == list(range(8))
    assert np.all(np.unique(d[:, :32:4]) % 3 == 0)
    # every dof appears
    assert len(np.unique(d)) == m.n_u + m.n_p


def test_shell_geometry_and_boundaries():
    m = dcp.HostMesh(refine=2, R0=1.0, R1=3.0, normals="radial")
    r = np.linalg.norm(m.node_xyz, axis=1)
    # vertices lie on the spheres; the other boundary support points are the
    # cubic map's image (MappingQ(3)), within its interpolation error
    rv = np.linalg.norm(m.cell_geometry[:, [0, 3, 12, 15, 48, 51, 60, 63]], axis=2)
    assert np.allclose(rv.min(), 1.0, rtol=0, atol=1e-14) and np.allclose(rv.max(), 3.0, rtol=0, atol=1e-14)
    assert np.isclose(r.min(), 1.0, atol=1e-4) and np.isclose(r.max(), 3.0, atol=1e-4)
    # inner sphere: no-slip on all 3 components; outer: one no-normal-flux line per node
    nc = m.nse_constraints
    n_in = np.sum(np.abs(r - 1.0) < 1e-3)
    n_out = np.sum(np.abs(r - 3.0) < 1e-3)
    assert n_in == n_out == 6 * (2 * 4) ** 2 + 2
    assert len(nc.line_dof) == 3 * n_in + n_out
    lens = np.diff(nc.entry_ptr)
    assert np.all(nc.inhomogeneity == 0)
    # no-normal-flux: u_k = -sum n_d/n_k u_d; check n . u = 0 for u = tangential
    for li in np.nonzero(lens > 0)[0][:50]:
        dof = nc.line_dof[li]
        node, k = divmod(dof, 3)
        n = m.node_xyz[node] / np.linalg.norm(m.node_xyz[node])
        # dominant component (deal.II tie-breaking prefers the later one on ties)
        assert abs(n[k]) >= np.abs(n).max() - 1e-9
        w = np.zeros(3)
        for e in range(nc.entry_ptr[li], nc.entry_ptr[li + 1]):
            assert nc.entry_dof[e] // 3 == node
            w[nc.entry_dof[e] % 3] = nc.entry_w[e]
        for d in range(3):
            if d != k:
                assert np.isclose(w[d], -n[d] / n[k])
    # temperature: Dirichlet with the initial temperature on the inner sphere
    tc = m.T_constraints
    assert np.all(np.diff(tc.entry_ptr) == 0)
    assert np.allclose(tc.inhomogeneity, m.T0[tc.line_dof])


def test_initial_temperature_function():
    m = dcp.HostMesh(refine=1)
    # two Gaussians at (1.7,0,0) and (0,2.3,0), covariance 20 I (R0=1, R1=3)
    cov = 20.0
    norm = np.sqrt(cov ** 3) / np.sqrt((2 * np.pi) ** 3)
    x = m.node_xyz[m.cell_nse_dofs[:, 0] // 3]
    T_expect = [norm * (np.exp(-0.5 * cov * np.sum((p - [1.7, 0, 0]) ** 2)) +
                        np.exp(-0.5 * cov * np.sum((p - [0, 2.3, 0]) ** 2))) for p in x]
    vertex_T = m.T0[m.cell_T_dofs[:, 0]]
    assert np.allclose(vertex_T, T_expect, rtol=1e-12, atol=1e-300)


def test_cube_sizes_and_constraints():
    m = dcp.HostMesh(cuboid=True, refine=2)
    N = 4
    assert m.n_cells == N ** 3
    assert m.n_u == 3 * (2 * N + 1) ** 3
    nc = m.nse_constraints
    # periodic x/y faces are identity constraints to the opposite face
    lens = np.diff(nc.entry_ptr)
    ones = nc.entry_w[nc.entry_ptr[:-1][lens == 1]]
    assert np.all(np.isin(ones, [1.0])) or len(ones) > 0


def test_cell_diameter():
    m = dcp.HostMesh(cuboid=True, refine=1)
    assert np.allclose(m.cell_diameter, np.sqrt(3) * 0.5)
