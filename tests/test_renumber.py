"""DoFRenumbering::Cuthill_McKee + component_wise of the NSE dofs
(boussinesq_model.tpp:198-204), applied by setup_dofs when the
Schur-complement solver is selected: dcp_host_mesh_renumber_cuthill_mckee
against the oracle's numpy restatement of deal.II's reorder_Cuthill_McKee, and
the renumbered system is the same system up to the permutation.

Parity with deal.II's own numbers is as pinned as the first-encounter
numbering it starts from (the reference's DoFHandler order is not available
here): the restatement is checked, the start order is this mesh's."""
import os

import numpy as np
import pytest

import dcp
import oracle_py

CUBE_PRM = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs",
                        "aqua_planet_cube_test_3d.prm")
CASES = [dict(refine=1), dict(refine=2), dict(cuboid=True, refine=2), dict(cuboid=True, refine=3)]


def levels(m):
    """Depth of the ILU(0) dependency chain of the velocity block (forward)."""
    import scipy.sparse as sp
    d = m.cell_nse_dofs[:, [4 * v + c for v in range(8) for c in range(3)] + list(range(32, 89))]
    r = np.repeat(d, d.shape[1], axis=1).ravel()
    c = np.tile(d, (1, d.shape[1])).ravel()
    A = sp.csr_matrix((np.ones(r.size), (r, c)), shape=(m.n_u, m.n_u))
    lev = np.zeros(m.n_u, np.int64)
    for i in range(m.n_u):
        cs = A.indices[A.indptr[i]:A.indptr[i + 1]]
        cs = cs[cs < i]
        if cs.size:
            lev[i] = lev[cs].max() + 1
    return int(lev.max()) + 1


@pytest.mark.parametrize("kw", CASES, ids=lambda k: "%s-r%d" % ("cube" if k.get("cuboid") else
                                                               "shell", k["refine"]))
def test_renumbering_matches_the_restatement(kw):
    a = dcp.HostMesh(**kw)
    b = dcp.HostMesh(cuthill_mckee=True, **kw)
    new, dmap = oracle_py.cuthill_mckee_nse(a.cell_nse_dofs, a.n_vnodes, a.n_u, a.n_p)
    # a permutation, node-major in the velocity block, blocks kept
    assert np.array_equal(np.sort(new), np.arange(a.n_vnodes))
    assert np.array_equal(np.sort(dmap), np.arange(a.n_u + a.n_p))
    assert np.all(dmap[a.n_u:] >= a.n_u)
    assert np.array_equal(b.cell_nse_dofs, dmap[a.cell_nse_dofs])
    xyz = np.empty_like(a.node_xyz)
    xyz[new] = a.node_xyz
    assert np.array_equal(b.node_xyz, xyz)
    # the constraints: the same lines and entries over the new numbers
    ca, cb = a.nse_constraints, b.nse_constraints
    la = {int(dmap[d]): (sorted((int(dmap[ca.entry_dof[k]]), float(ca.entry_w[k]))
                                for k in range(ca.entry_ptr[i], ca.entry_ptr[i + 1])),
                         float(ca.inhomogeneity[i])) for i, d in enumerate(ca.line_dof)}
    lb = {int(d): ([(int(cb.entry_dof[k]), float(cb.entry_w[k]))
                    for k in range(cb.entry_ptr[i], cb.entry_ptr[i + 1])], float(cb.inhomogeneity[i]))
          for i, d in enumerate(cb.line_dof)}
    assert la == lb
    assert np.all(np.diff(cb.line_dof) > 0)
    # the T numbering is untouched
    assert np.array_equal(a.cell_T_dofs, b.cell_T_dofs) and np.array_equal(a.T0, b.T0)


def test_renumbering_shortens_the_ilu_chain():
    a = dcp.HostMesh(cuboid=True, refine=2)
    b = dcp.HostMesh(cuboid=True, refine=2, cuthill_mckee=True)
    assert levels(b) < 0.6 * levels(a)


def test_renumbered_system_is_the_permuted_system():
    rp = dcp.load_prm(CUBE_PRM)
    ph = dcp.physics_from_params(rp)
    a = dcp.HostMesh(cuboid=True, refine=1, length=rp.length)
    b = dcp.HostMesh(cuboid=True, refine=1, length=rp.length, cuthill_mckee=True)
    _, dmap = oracle_py.cuthill_mckee_nse(a.cell_nse_dofs, a.n_vnodes, a.n_u, a.n_p)
    rng = np.random.default_rng(3)
    ua = 0.1 * rng.uniform(-1, 1, a.n_u + a.n_p)
    ub = np.empty_like(ua)
    ub[dmap] = ua
    oa, ob = oracle_py.Model(ph, a), oracle_py.Model(ph, b)
    oa.assemble_nse_system(ua, a.T0)
    ob.assemble_nse_system(ub, b.T0)
    ra, rb = oa.nse_rhs(), ob.nse_rhs()
    assert np.array_equal(rb[dmap], ra)


# ---------------------------------------------------------------------------
# deal.II's own distribute_dofs order on the 6-cell hyper_shell
# (dcp_host_mesh_renumber_dealii; the coarse cells of GridGenerator::
# hyper_shell are restated from deal.II 9.2, which is not in this image:
# unpinned against deal.II itself, checked here for its defining properties).

def _first_encounter(cells, dofs_of, lo, hi):
    """True when walking the cells in order meets the dofs in [lo, hi) in
    increasing, gap-free order (what distribute_dofs produces)."""
    seen = lo - 1
    for c in cells:
        d = dofs_of[c]
        d = d[(d >= lo) & (d < hi)]
        new = np.unique(d[d > seen])
        if new.size:
            if new[0] != seen + 1 or new[-1] != seen + new.size:
                return False
            seen = new[-1]
    return seen == hi - 1


@pytest.mark.parametrize("refine,tdeg", [(0, 1), (1, 1), (2, 1), (2, 2), (3, 1)])
def test_dealii_order_is_first_encounter_over_dealii_cells(refine, tdeg):
    m = dcp.HostMesh(refine=refine, temperature_degree=tdeg, dealii_order=True)
    cells = m.dealii_cells
    assert np.array_equal(np.sort(cells), np.arange(m.n_cells))
    # each coarse cell's children stay together (refine_global's level order)
    n3 = 8 ** refine
    assert all(len(set((cells[q * n3:(q + 1) * n3] // n3).tolist())) == 1 for q in range(6))
    assert _first_encounter(cells, m.cell_nse_dofs, 0, m.n_u)
    assert _first_encounter(cells, m.cell_nse_dofs, m.n_u, m.n_u + m.n_p)
    assert _first_encounter(cells, m.cell_T_dofs, 0, m.n_T)
    # velocity stays node-major (component_wise {0,0,0,1} keeps the order)
    v = m.cell_nse_dofs[:, :32].reshape(-1, 8, 4)
    assert np.all(v[:, :, 1] == v[:, :, 0] + 1) and np.all(v[:, :, 2] == v[:, :, 0] + 2)


def test_dealii_order_first_cell_geometry():
    """The first active cell is the bottom coarse cell's child 0...0: its local
    z runs from the outer sphere inwards, so dofs 0..3 (vertices 0-3) sit on the
    outer sphere, vertex 0 at the corner direction (-1,-1,-1)."""
    R0, R1, r = 1.0, 3.0, 2
    m = dcp.HostMesh(refine=r, R0=R0, R1=R1, dealii_order=True)
    x = m.node_xyz
    rad = np.linalg.norm(x[:8], axis=1)
    assert np.allclose(rad[:4], R1, rtol=1e-13)
    assert np.allclose(rad[4:8], R1 - (R1 - R0) / 2 ** r, rtol=1e-13)
    assert np.allclose(x[0], -R1 / np.sqrt(3) * np.ones(3), rtol=1e-13)
    # local x of the bottom cell is world +x (vertex 1 on the arc from corner
    # (-1,-1,-1) towards (+1,-1,-1): y = z), local y is world +y (x = z)
    assert x[1][0] > x[0][0] and x[1][1] == pytest.approx(x[1][2], rel=1e-13)
    assert x[2][1] > x[0][1] and x[2][0] == pytest.approx(x[2][2], rel=1e-13)
    # pressure dof 0 / temperature dof 0 at that vertex
    c0 = m.dealii_cells[0]
    v0 = [v for v in range(8) if m.cell_nse_dofs[c0][4 * v] == 0]
    assert len(v0) == 1       # the mesh cell's own frame differs; find deal.II's vertex 0
    assert m.cell_nse_dofs[c0][4 * v0[0] + 3] == m.n_u and m.cell_T_dofs[c0][v0[0]] == 0
    assert m.T0[0] == pytest.approx(0.0, abs=1e-30)   # outer sphere: the Gaussian's tail


def test_dealii_order_is_the_same_problem_permuted():
    a = dcp.HostMesh(refine=2)
    b = dcp.HostMesh(refine=2, dealii_order=True)
    # old -> new dof maps from the cell dof tables (same cells, same local order)
    dmap = np.full(a.n_u + a.n_p, -1)
    dmap[a.cell_nse_dofs.ravel()] = b.cell_nse_dofs.ravel()
    assert np.array_equal(np.sort(dmap), np.arange(a.n_u + a.n_p))
    tmap = np.full(a.n_T, -1)
    tmap[a.cell_T_dofs.ravel()] = b.cell_T_dofs.ravel()
    assert np.array_equal(np.sort(tmap), np.arange(a.n_T))
    assert np.array_equal(b.T0[tmap], a.T0)
    xyz = np.empty_like(a.node_xyz)
    xyz[dmap[:a.n_u:3] // 3] = a.node_xyz
    assert np.array_equal(b.node_xyz, xyz)
    for ca, cb, mp in ((a.nse_constraints, b.nse_constraints, dmap),
                       (a.T_constraints, b.T_constraints, tmap)):
        la = {int(mp[d]): (sorted((int(mp[ca.entry_dof[k]]), float(ca.entry_w[k]))
                                  for k in range(ca.entry_ptr[i], ca.entry_ptr[i + 1])),
                           float(ca.inhomogeneity[i])) for i, d in enumerate(ca.line_dof)}
        lb = {int(d): (sorted((int(cb.entry_dof[k]), float(cb.entry_w[k]))
                              for k in range(cb.entry_ptr[i], cb.entry_ptr[i + 1])),
                       float(cb.inhomogeneity[i])) for i, d in enumerate(cb.line_dof)}
        assert la == lb
    # the oracle's assembled right-hand side is the permuted one
    ph = dcp.classic_physics()
    rng = np.random.default_rng(5)
    ua = 0.1 * rng.uniform(-1, 1, a.n_u + a.n_p)
    ub = np.empty_like(ua)
    ub[dmap] = ua
    oa, ob = oracle_py.Model(ph, a), oracle_py.Model(ph, b)
    oa.assemble_nse_system(ua, a.T0)
    ob.assemble_nse_system(ub, b.T0)
    assert np.allclose(ob.nse_rhs()[dmap], oa.nse_rhs(), rtol=0, atol=1e-13 * np.abs(oa.nse_rhs()).max())


def test_dealii_order_then_cuthill_mckee():
    """The Schur configs: Cuthill-McKee from deal.II's order (as setup_dofs)."""
    b = dcp.HostMesh(refine=1, dealii_order=True, cuthill_mckee=True)
    c = dcp.HostMesh(refine=1, dealii_order=True)
    _, dmap = oracle_py.cuthill_mckee_nse(c.cell_nse_dofs, c.n_vnodes, c.n_u, c.n_p)
    assert np.array_equal(b.cell_nse_dofs, dmap[c.cell_nse_dofs])
    assert np.array_equal(b.cell_T_dofs, c.cell_T_dofs)
    with pytest.raises(dcp.DcpError):
        dcp.HostMesh(cuboid=True, refine=1, dealii_order=True)


@pytest.mark.gpu
def test_dealii_order_time_step_on_the_gpu():
    """One classic time step (r=2) in deal.II's dof order and in the mesh's:
    the same FGMRES count, the NSE / temperature solutions equal up to the
    permutation (Krylov sums run in another order: rounding-level)."""
    a = dcp.HostMesh(refine=2)
    b = dcp.HostMesh(refine=2, dealii_order=True)
    dmap = np.full(a.n_u + a.n_p, -1)
    dmap[a.cell_nse_dofs.ravel()] = b.cell_nse_dofs.ravel()
    tmap = np.full(a.n_T, -1)
    tmap[a.cell_T_dofs.ravel()] = b.cell_T_dofs.ravel()
    res = []
    for m in (a, b):
        ctx = dcp.Context()
        ctx.set_physics(dcp.classic_physics())
        ctx.upload_mesh(m)
        u = np.zeros(m.n_u + m.n_p)
        for f, v in ((dcp.NSE_SOLUTION, u), (dcp.OLD_NSE_SOLUTION, u), (dcp.T_SOLUTION, m.T0),
                     (dcp.OLD_T_SOLUTION, m.T0)):
            ctx.set_state(f, v)
        ctx.assemble_nse_system()
        ctx.build_nse_preconditioner()
        ctx.assemble_temperature_matrix()
        rc, outer, _ = ctx.solve_nse()
        ctx.assemble_temperature_rhs()
        rcT, _, _ = ctx.solve_temperature()
        assert rc == 0 and rcT == 0
        res.append((outer, ctx.get_state(dcp.NSE_SOLUTION), ctx.get_state(dcp.T_SOLUTION)))
        ctx.close()
    (oa, ua, Ta), (ob, ub, Tb) = res
    assert oa == ob
    assert np.linalg.norm(ub[dmap] - ua) <= 1e-9 * np.linalg.norm(ua)
    assert np.linalg.norm(Tb[tmap] - Ta) <= 1e-9 * np.linalg.norm(Ta)
