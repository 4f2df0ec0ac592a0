"""The temperature system in Kronecker form (kernels/temperature_sep.hip,
csrc/tsep.cpp) against the oracle's assemble_temperature_matrix / _rhs
(oracle.cpp, restating boussinesq_model.tpp:748-1020) and against the colour
kernels it replaces on the layered shell (DCP_T_SEPARABLE=0).

Bars: assembled entries and rhs at 1e-12 relative to the largest entry (only
the summation order differs: lateral x radial integrals instead of 27-point
cell sums), the two device paths at 1e-13, repeated assemblies bitwise."""
import numpy as np
import pytest
import scipy.sparse as sp

import dcp
import oracle_py

pytestmark = pytest.mark.gpu

SEED = 20261018


def rel_max(a, b):
    return float(np.max(np.abs(np.asarray(a) - np.asarray(b))) / max(np.max(np.abs(b)), 1e-300))


def csr(ctx, n):
    rp, cols, vals = ctx.T_matrix_csr()
    return sp.csr_matrix((vals, cols, rp), shape=(n, n))


def make_ctx(m, ph, separable, monkeypatch):
    if separable:
        monkeypatch.delenv("DCP_T_SEPARABLE", raising=False)
    else:
        monkeypatch.setenv("DCP_T_SEPARABLE", "0")
    ctx = dcp.Context()
    ctx.set_physics(ph)
    ctx.upload_mesh(m)
    monkeypatch.delenv("DCP_T_SEPARABLE", raising=False)
    return ctx


def state(m, seed):
    rng = np.random.default_rng(seed)
    u = rng.uniform(-1, 1, m.n_u + m.n_p)
    T = m.T0 + 0.1 * rng.uniform(-1, 1, m.n_T)
    return u, T


def assemble(ctx, u, T):
    ctx.set_state(dcp.OLD_T_SOLUTION, T)
    ctx.set_state(dcp.NSE_SOLUTION, u)
    ctx.assemble_temperature_matrix()
    ctx.assemble_temperature_rhs()
    return ctx.T_matrix_csr()[2].copy(), ctx.get_state(dcp.T_RHS)


@pytest.mark.parametrize("refine", [1, 2, 3])
def test_separable_temperature_matches_oracle_and_colour_kernels(monkeypatch, refine):
    m = dcp.HostMesh(refine=refine)
    ph = dcp.classic_physics()
    new = make_ctx(m, ph, True, monkeypatch)
    old = make_ctx(m, ph, False, monkeypatch)
    lay = new.temperature_layout()
    assert lay["separable"] and lay["kinds"] == (1 if refine <= 1 else 2), lay
    assert lay["layers"] == 2 ** refine and not old.temperature_layout()["separable"]
    u, T = state(m, SEED + refine)
    orc = oracle_py.Model(ph, m)
    orc.assemble_temperature_matrix()
    orc.assemble_temperature_rhs(T, u)
    rp, cols, vals = orc.T_matrix_csr()
    To = sp.csr_matrix((vals, cols, rp), shape=(m.n_T, m.n_T))
    vn, rn = assemble(new, u, T)
    vo, ro = assemble(old, u, T)
    Tn, Tc = csr(new, m.n_T), csr(old, m.n_T)
    assert abs(Tn - To).max() / abs(To).max() < 1e-12
    assert abs(Tn - Tc).max() / abs(Tc).max() < 1e-13
    assert rel_max(rn, orc.T_rhs()) < 1e-12
    assert rel_max(rn, ro) < 1e-13
    # the lift is exercised: inhomogeneous Dirichlet values on the shell
    fixed = m.T_constraints.line_dof
    assert np.any(m.T_constraints.inhomogeneity != 0.0) and len(fixed) > 0
    # deterministic: a second assembly is bitwise the first
    v2, r2 = assemble(new, u, T)
    assert np.array_equal(v2, vn) and np.array_equal(r2, rn)
    new.close()
    old.close()


def test_separable_temperature_dt_change_between_matrix_and_rhs(monkeypatch):
    """T_matrix = M + dt K belongs to assemble_temperature_rhs (:975-978): a
    time step set between the two calls must reach it (the matrix pass formed
    it with the old dt)."""
    m = dcp.HostMesh(refine=2)
    ph = dcp.classic_physics()
    new = make_ctx(m, ph, True, monkeypatch)
    old = make_ctx(m, ph, False, monkeypatch)
    u, T = state(m, SEED + 7)
    for ctx in (new, old):
        ctx.set_state(dcp.OLD_T_SOLUTION, T)
        ctx.set_state(dcp.NSE_SOLUTION, u)
        ctx.assemble_temperature_matrix()
        ctx.set_time_step(0.37 * ph.time_step)
        ctx.assemble_temperature_rhs()
    assert abs(csr(new, m.n_T) - csr(old, m.n_T)).max() / abs(csr(old, m.n_T)).max() < 1e-13
    assert rel_max(new.get_state(dcp.T_RHS), old.get_state(dcp.T_RHS)) < 1e-13
    # and the CG on it takes the same number of steps to the same solution
    rn = new.solve_temperature()
    ro = old.solve_temperature()
    assert rn[1] == ro[1]
    assert rel_max(new.get_state(dcp.T_SOLUTION), old.get_state(dcp.T_SOLUTION)) < 1e-12
    new.close()
    old.close()


def test_non_separable_meshes_keep_colour_kernels(monkeypatch):
    """A warped shell is no longer a separable map (and a partition or the
    periodic cube is no column x layer product): the colour kernels run, and
    still match the oracle."""
    ph = dcp.classic_physics()
    warped = dcp.HostMesh(refine=2)
    X = warped.cell_geometry.reshape(-1, 3)
    X += 0.02 * np.sin(3.0 * X[:, [1, 2, 0]]) * np.cos(2.0 * X[:, [2, 0, 1]])
    for m in (warped,):
        ctx = make_ctx(m, ph, True, monkeypatch)
        assert not ctx.temperature_layout()["separable"]
        u, T = state(m, SEED + 11)
        _, r = assemble(ctx, u, T)
        orc = oracle_py.Model(ph, m)
        orc.assemble_temperature_matrix()
        orc.assemble_temperature_rhs(T, u)
        assert rel_max(r, orc.T_rhs()) < 1e-12
        ctx.close()
