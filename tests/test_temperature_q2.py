"""FE_Q(2) temperature in the 3D classic model (temperature_fe(2),
boussinesq_model.tpp:30; data/aqua_planet.prm and aqua_planet_test_3d.prm set
temperature degree = 2): 27 temperature dofs per cell, QGauss(4) for the
temperature matrices and rhs (:834, :990), and the Q2 temperature inside the
NSE right-hand side's density term (:594-597).

CPU: the host mesh, the upload's validation and the rank partition take the
27-dof layout. GPU: device vs oracle at 1e-12 (assembly) / 1e-10 (CG iterate)."""
import numpy as np
import pytest

import dcp
import oracle_py

SEED = 20261018


def rel_max(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300)


def rel2(a, b):
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


def test_host_mesh_and_partition_take_q2_temperature():
    m = dcp.HostMesh(refine=2, temperature_degree=2)
    assert m.cell_T_dofs.shape == (m.n_cells, 27)
    assert m.n_T == m.n_u // 3            # one dof per Q2 support point
    assert m.check() > 0
    # the Dirichlet values of the inner sphere sit on all 9 points of each inner face
    assert len(m.T_constraints.line_dof) == 6 * 4 ** 2 * 4 + 2
    owned = 0
    for r in range(3):
        info = dcp.partition_info(m, r, 3)
        owned += info["nTo"]
    assert owned == m.n_T


def q2_physics():
    ph = dcp.classic_physics()
    ph.temperature_degree = 2
    return ph


@pytest.fixture(scope="module")
def setup():
    m = dcp.HostMesh(refine=2, temperature_degree=2)
    ph = q2_physics()
    ctx = dcp.Context()
    ctx.set_physics(ph)
    ctx.upload_mesh(m)
    return m, ph, ctx, oracle_py.Model(ph, m)


@pytest.mark.gpu
def test_q2_temperature_matrix_rhs_and_solve(setup):
    m, ph, ctx, orc = setup
    rng = np.random.default_rng(SEED)
    u = 0.1 * rng.uniform(-1, 1, m.n_u + m.n_p)
    T = m.T0 + 0.05 * rng.uniform(-1, 1, m.n_T)
    ctx.set_state(dcp.NSE_SOLUTION, u)
    ctx.set_state(dcp.OLD_T_SOLUTION, T)
    ctx.set_state(dcp.T_SOLUTION, T)
    ctx.assemble_temperature_matrix()
    ctx.assemble_temperature_rhs()
    orc.assemble_temperature_matrix()
    orc.assemble_temperature_rhs(T, u)
    import scipy.sparse as sp
    n = m.n_T
    rg, cg, vg = ctx.T_matrix_csr()
    Ag = sp.csr_matrix((vg, cg, rg), shape=(n, n))
    ro, co, vo = orc.T_matrix_csr()
    Ao = sp.csr_matrix((vo, co, ro), shape=(n, n))
    assert abs(Ag - Ao).max() / abs(Ao).max() < 1e-12
    assert rel_max(ctx.get_state(dcp.T_RHS), orc.T_rhs()) < 1e-12
    rc, its, _ = ctx.solve_temperature()
    rco, To, itso = orc.solve_temperature(T)
    assert rc == rco == 0 and its == itso
    assert rel2(ctx.get_state(dcp.T_SOLUTION), To) < 1e-10


@pytest.mark.gpu
def test_q2_temperature_in_nse_rhs(setup):
    """The density term of the NSE rhs reads the FE_Q(2) temperature."""
    m, ph, ctx, orc = setup
    rng = np.random.default_rng(SEED + 1)
    u = rng.uniform(-1, 1, m.n_u + m.n_p)
    T = m.T0 + 0.1 * rng.uniform(-1, 1, m.n_T)
    ctx.set_state(dcp.OLD_NSE_SOLUTION, u)
    ctx.set_state(dcp.OLD_T_SOLUTION, T)
    K, f = ctx.cell_nse_system(0, m.n_cells)
    worst = 0.0
    for c in range(0, m.n_cells, 7):
        Ko, fo = oracle_py.cell_nse_system(ph, m.cell_geometry[c], u[m.cell_nse_dofs[c]],
                                           T[m.cell_T_dofs[c]])
        worst = max(worst, rel_max(f[c], fo), rel_max(K[c], Ko))
    assert worst < 1e-12, worst
    ctx.assemble_nse_system()
    orc.assemble_nse_system(u, T)
    assert rel_max(ctx.get_state(dcp.NSE_RHS), orc.nse_rhs()) < 1e-12


@pytest.mark.gpu
def test_q2_temperature_schur_steps_match_oracle():
    """Two steps of data/aqua_planet.prm's setting (Q2 temperature, Cuthill-McKee,
    Schur-complement solver) at refinement 2 on the device and in the oracle."""
    m = dcp.HostMesh(refine=2, temperature_degree=2, cuthill_mckee=True)
    ph = q2_physics()
    ctx = dcp.Context()
    ctx.set_physics(ph)
    ctx.upload_mesh(m)
    orc = oracle_py.Model(ph, m)
    u = np.zeros(m.n_u + m.n_p)
    T = m.T0.copy()
    for f, v in ((dcp.OLD_NSE_SOLUTION, u), (dcp.NSE_SOLUTION, u), (dcp.OLD_T_SOLUTION, T),
                 (dcp.T_SOLUTION, T)):
        ctx.set_state(f, v)
    ctx.assemble_temperature_matrix()
    orc.assemble_temperature_matrix()
    for step in range(2):
        ctx.assemble_nse_system()
        rc, its, _ = ctx.solve_nse_schur()
        ctx.assemble_temperature_rhs()
        rcT, _, _ = ctx.solve_temperature()
        ctx.advance_state()
        orc.assemble_nse_system(u, T)
        rco, u_new, itso, _ = orc.solve_nse_schur(u)
        orc.assemble_temperature_rhs(T, u_new)
        _, T_new, _ = orc.solve_temperature(T)
        u, T = u_new, T_new
        assert rc == rco == 0 and rcT == 0 and its == itso
        # the reference's inner rule (1e-6 CGs): rounding reaches ~1e-8 (see
        # test_parity_gpu_2d.py); the iteration counts must agree exactly
        assert rel2(ctx.get_state(dcp.NSE_SOLUTION), u) < 1e-7
        assert rel2(ctx.get_state(dcp.T_SOLUTION), T) < 1e-7
