"""DCP_OPT_ELEMENT_MFMA: the velocity-velocity node-pair sums of the NSE
element matrix (local_assemble_nse_system, boussinesq_model.tpp:597-640) as
v_mfma_f64_16x16x4_f64 Gram tiles instead of FP64 VALU tiles.

Against the oracle at the assembly bar (1e-12 relative to the largest entry)
and against the VALU path at 1e-13 (only the summation order differs); what
does not involve the velocity block (B^T, B, rhs, constrained diagonals) must
be bitwise the VALU path's. Shell r=2 (radially separable geometry) and the
periodic cube r=2 of BASELINE C2 (MappingQ(3) from the support points,
Coriolis and vertical gravity on)."""
import os

import numpy as np
import pytest
import scipy.sparse as sp

import dcp
import oracle_py

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEED = 20261017


def rel_max(a, b):
    return np.max(np.abs(np.asarray(a) - np.asarray(b))) / max(np.max(np.abs(b)), 1e-300)


def csr(rp, cols, vals, n):
    return sp.csr_matrix((vals, cols, rp), shape=(n, n))


def meshes():
    ph = dcp.classic_physics()
    yield "shell", dcp.HostMesh(refine=2), ph
    rp = dcp.load_prm(os.path.join(ROOT, "configs", "aqua_planet_cube_test_3d.prm"))
    yield "cube", dcp.HostMesh(cuboid=True, refine=2, length=rp.length), \
        dcp.physics_from_params(rp)


@pytest.fixture(scope="module", params=["shell", "cube"])
def case(request):
    name, m, ph = [c for c in meshes() if c[0] == request.param][0]
    rng = np.random.default_rng(SEED)
    u = rng.uniform(-1, 1, m.n_u + m.n_p)
    T = m.T0 + 0.1 * rng.uniform(-1, 1, m.n_T)
    return m, ph, u, T


def run(m, ph, u, T, mfma):
    ctx = dcp.Context()
    ctx.set_physics(ph)
    ctx.upload_mesh(m)
    ctx.set_element_mfma(mfma)
    ctx.set_state(dcp.OLD_NSE_SOLUTION, u)
    ctx.set_state(dcp.OLD_T_SOLUTION, T)
    K, f = ctx.cell_nse_system(0, m.n_cells)
    ctx.set_assemble_velocity_block(True)
    ctx.assemble_nse_system()
    n = m.n_u + m.n_p
    A = csr(*ctx.nse_matrix_csr(), n)
    rhs = ctx.get_state(dcp.NSE_RHS)
    ctx.close()
    return K, f, A, rhs


def test_element_matrices_mfma(case):
    m, ph, u, T = case
    K, f, _, _ = run(m, ph, u, T, True)
    Kv, fv, _, _ = run(m, ph, u, T, False)
    assert rel_max(K, Kv) < 1e-13
    assert np.array_equal(f, fv)
    worst = 0.0
    for c in range(0, m.n_cells, 3):
        Ko, _ = oracle_py.cell_nse_system(ph, m.cell_geometry[c], u[m.cell_nse_dofs[c]],
                                          T[m.cell_T_dofs[c]])
        worst = max(worst, rel_max(K[c], Ko))
    assert worst < 1e-12, worst
    # the velocity block stays node-pair symmetric
    Kvv = K[:, :, :]
    assert rel_max(Kvv, np.transpose(Kvv, (0, 2, 1))) < 1e-13


def test_assembled_velocity_block_mfma(case):
    m, ph, u, T = case
    n = m.n_u + m.n_p
    _, _, A, rhs = run(m, ph, u, T, True)
    _, _, Av, rhsv = run(m, ph, u, T, False)
    assert np.array_equal(rhs, rhsv)
    # B^T / B blocks bitwise, velocity block at rounding level
    nu = m.n_u
    assert abs(A[:nu, nu:] - Av[:nu, nu:]).max() == 0.0
    assert abs(A[nu:, :nu] - Av[nu:, :nu]).max() == 0.0
    assert abs(A - Av).max() / abs(Av).max() < 1e-13
    orc = oracle_py.Model(ph, m)
    orc.assemble_nse_system(u, T)
    Ao = csr(*orc.nse_matrix_csr(), n)
    assert abs(A - Ao).max() / abs(Ao).max() < 1e-12
    assert rel_max(rhs, orc.nse_rhs()) < 1e-12
