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
