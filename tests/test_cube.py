"""BASELINE C2: data/aqua_planet_cube_test_3d.prm on the device, classic
Q2/Q1 (overrides: use FEEC solver = false, nse velocity degree = 2) at
refine 3 -- the periodic unit cube of planet_geometry.tpp:29-58 with
x/y periodicity (DoFTools::make_periodicity_constraints,
boussinesq_model.tpp:265-285), no-slip at z = 0 and no normal flux at z = 1.
On the cuboid the Coriolis term (boussinesq_model.tpp:615-621) and the
vertical gravity (core_model_data.tpp:86-95) are on.

The device folds every periodic identity into the cell maps; the original
maps route each image's constrained diagonal (|K_ii| or the average) to the
image itself. Compared with the oracle (whose AffineConstraints is general):
element matrices, the assembled nse_matrix / rhs, the preconditioner
diagonals and the temperature system at 1e-12; the matrix-free operator
against the assembled one at 1e-13."""
import os

import numpy as np
import pytest
import scipy.sparse as sp

import dcp
import oracle_py

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEED = 20261016


def rel_max(a, b):
    return np.max(np.abs(np.asarray(a) - np.asarray(b))) / max(np.max(np.abs(b)), 1e-300)


def csr(rp, cols, vals, n):
    return sp.csr_matrix((vals, cols, rp), shape=(n, n))


@pytest.fixture(scope="module")
def cube():
    rp = dcp.load_prm(os.path.join(ROOT, "configs", "aqua_planet_cube_test_3d.prm"))
    ph = dcp.physics_from_params(rp)
    assert ph.cuboid == 1 and ph.omega != 0.0
    m = dcp.HostMesh(cuboid=True, refine=3, length=rp.length)
    ctx = dcp.Context()
    ctx.set_physics(ph)
    ctx.upload_mesh(m)
    rng = np.random.default_rng(SEED)
    u = rng.uniform(-1, 1, m.n_u + m.n_p)
    T = m.T0 + 0.1 * rng.uniform(-1, 1, m.n_T)
    ctx.set_state(dcp.OLD_NSE_SOLUTION, u)
    ctx.set_state(dcp.OLD_T_SOLUTION, T)
    ctx.set_state(dcp.NSE_SOLUTION, u)
    orc = oracle_py.Model(ph, m)
    yield m, ph, ctx, orc, u, T
    ctx.close()


def test_cube_element_matrices(cube):
    m, ph, ctx, _, u, T = cube
    K, f = ctx.cell_nse_system(0, m.n_cells)
    for c in range(0, m.n_cells, 7):
        Ko, fo = oracle_py.cell_nse_system(ph, m.cell_geometry[c], u[m.cell_nse_dofs[c]],
                                           T[m.cell_T_dofs[c]])
        assert rel_max(K[c], Ko) < 1e-12
        assert rel_max(f[c], fo) < 1e-12


@pytest.mark.parametrize("full", [False, True], ids=["operator-form", "velocity-block"])
def test_cube_assembled_system(cube, full):
    m, ph, ctx, orc, u, T = cube
    n = m.n_u + m.n_p
    ctx.set_assemble_velocity_block(full)
    ctx.assemble_nse_system()
    ctx.set_assemble_velocity_block(False)
    orc.assemble_nse_system(u, T)
    Ag = csr(*ctx.nse_matrix_csr(), n)
    Ao = csr(*orc.nse_matrix_csr(), n)
    assert abs(Ag - Ao).max() / abs(Ao).max() < 1e-12
    # same pattern rows for the periodic images: the diagonal only
    assert rel_max(ctx.get_state(dcp.NSE_RHS), orc.nse_rhs()) < 1e-12
    # the Coriolis term is on: the rhs differs from the omega = 0 one
    ph0 = dcp.physics_from_params(dcp.load_prm(os.path.join(ROOT, "configs",
                                                            "aqua_planet_cube_test_3d.prm")))
    ph0.omega = 0.0
    orc0 = oracle_py.Model(ph0, m)
    orc0.assemble_nse_system(u, T)
    assert rel_max(orc0.nse_rhs(), orc.nse_rhs()) > 1e-3


def test_cube_preconditioner_and_temperature(cube):
    m, ph, ctx, orc, u, T = cube
    ctx.assemble_nse_system()
    ctx.build_nse_preconditioner()
    orc.assemble_nse_system(u, T)
    orc.build_nse_preconditioner()
    a_g, p_g = ctx.precond_diagonals()
    a_o, p_o = orc.precond_diagonals()
    assert rel_max(a_g, a_o) < 1e-12
    assert rel_max(p_g, p_o) < 1e-12
    ctx.assemble_temperature_matrix()
    ctx.assemble_temperature_rhs()
    orc.assemble_temperature_matrix()
    orc.assemble_temperature_rhs(T, u)
    Tg = csr(*ctx.T_matrix_csr(), m.n_T)
    To = csr(*orc.T_matrix_csr(), m.n_T)
    assert abs(Tg - To).max() / abs(To).max() < 1e-12
    assert rel_max(ctx.get_state(dcp.T_RHS), orc.T_rhs()) < 1e-12


def test_cube_matrix_free_operator(cube):
    m, ph, ctx, orc, u, T = cube
    ctx.assemble_nse_system()
    n = m.n_u + m.n_p
    A = csr(*ctx.nse_matrix_csr(), n)
    x = np.random.default_rng(SEED + 1).uniform(-1, 1, n)
    for mode in (1, 2):
        ctx.set_matrix_free(mode)
        assert rel_max(ctx.nse_vmult(x), A @ x) < 1e-13, mode
        assert rel_max(ctx.velocity_vmult(x[:m.n_u]), A[:m.n_u, :m.n_u] @ x[:m.n_u]) < 1e-13
    ctx.set_matrix_free(1)
    # and the oracle's product with its own matrix
    orc.assemble_nse_system(u, T)
    assert rel_max(ctx.nse_vmult(x), orc.nse_vmult(x)) < 1e-12


def test_cube_repeated_operator_form_assembly(cube):
    """On the periodic cube the velocity pattern holds the periodic images'
    diagonal-only rows, which no cell's scatter position reaches (A is
    zero-filled and added, not stored at first touch). Three operator-form
    assemblies with different states on the module's context, each against the
    oracle: B^T / B as the solve reads them, the rhs and S = B D_A^-1 B^T at
    1e-12; then the full export (velocity block materialised) at 1e-12."""
    m, ph, ctx, orc, u0, T0 = cube
    info = ctx.scatter_info()
    print("scatter info (touched, nnzb, first touch):", info)
    assert info["A"][0] < info["A"][1] and not info["A"][2]
    assert info["Bt"][0] == info["Bt"][1]
    rng = np.random.default_rng(SEED + 9)
    n = m.n_u + m.n_p
    for i in range(3):
        u = rng.uniform(-1, 1, n)
        T = m.T0 + 0.1 * rng.uniform(-1, 1, m.n_T)
        ctx.set_state(dcp.OLD_NSE_SOLUTION, u)
        ctx.set_state(dcp.OLD_T_SOLUTION, T)
        ctx.assemble_nse_system()
        ctx.build_nse_preconditioner()
        orc.assemble_nse_system(u, T)
        orc.build_nse_preconditioner()
        Ao = csr(*orc.nse_matrix_csr(), n)
        rp, cols, vals = ctx.coupling_csr("Bt")
        Bt_g = sp.csr_matrix((vals, cols, rp), shape=(m.n_u, m.n_p))
        rp, cols, vals = ctx.coupling_csr("B")
        B_g = sp.csr_matrix((vals, cols, rp), shape=(m.n_p, m.n_u))
        Bt_o, B_o = Ao[:m.n_u, m.n_u:], Ao[m.n_u:, :m.n_u]
        assert abs(Bt_g - Bt_o).max() / abs(Bt_o).max() < 1e-12, i
        assert abs(B_g - B_o).max() / abs(B_o).max() < 1e-12, i
        assert rel_max(ctx.get_state(dcp.NSE_RHS), orc.nse_rhs()) < 1e-12, i
        p = rng.uniform(-1, 1, m.n_p)
        assert rel_max(ctx.schur_vmult(p), orc.schur_vmult(p)) < 1e-12, i
    Ag = csr(*ctx.nse_matrix_csr(), n)
    assert abs(Ag - Ao).max() / abs(Ao).max() < 1e-12
    # leave the module state as the fixture made it
    ctx.set_state(dcp.OLD_NSE_SOLUTION, u0)
    ctx.set_state(dcp.OLD_T_SOLUTION, T0)
