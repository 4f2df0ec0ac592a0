"""B^T of nse_matrix in Kronecker form (kernels/bt_kron.hip, csrc/btkron.cpp)
against the oracle's assemble_nse_system (oracle.cpp, restating
boussinesq_model.tpp:626-637 scattered at :677-687) and against the B^T row
tasks it replaces on one GPU (DCP_BT_KRON=0).

Bars: B^T and B at 1e-12 relative to the largest entry against the oracle
(only the summation order differs: lateral columns x layers instead of
cells), 1e-13 against the row tasks, B = (B^T)^T bitwise, repeated assemblies
bitwise, and the constrained (no-normal-flux) rows condensed as the tasks do."""
import numpy as np
import pytest
import scipy.sparse as sp

import dcp
import oracle_py

pytestmark = pytest.mark.gpu

SEED = 20261019


def block_csr(ctx, key, shape):
    rp, cols, vals = ctx.coupling_csr(key)
    return sp.csr_matrix((vals, cols, rp), shape=shape)


def make_ctx(m, ph, kron, monkeypatch):
    monkeypatch.setenv("DCP_BT_KRON", "1" if kron else "0")
    ctx = dcp.Context()
    ctx.set_physics(ph)
    ctx.upload_mesh(m)
    monkeypatch.delenv("DCP_BT_KRON", raising=False)
    return ctx


@pytest.mark.parametrize("refine", [1, 2, 3])
def test_kronecker_bt_matches_oracle_and_row_tasks(monkeypatch, refine):
    m = dcp.HostMesh(refine=refine)
    ph = dcp.classic_physics()
    rng = np.random.default_rng(SEED + refine)
    u = rng.uniform(-1, 1, m.n_u + m.n_p)
    T = m.T0 + 0.1 * rng.uniform(-1, 1, m.n_T)
    new = make_ctx(m, ph, True, monkeypatch)
    old = make_ctx(m, ph, False, monkeypatch)
    lay = new.assembly_layout()
    assert lay["bt_kronecker"] and lay["bt_lateral_pairs"] > 0 and lay["bt_constrained_entries"] > 0
    assert not old.assembly_layout()["bt_kronecker"]
    for ctx in (new, old):
        ctx.set_state(dcp.OLD_NSE_SOLUTION, u)
        ctx.set_state(dcp.OLD_T_SOLUTION, T)
        ctx.assemble_nse_system()
    orc = oracle_py.Model(ph, m)
    orc.assemble_nse_system(u, T)
    for key, shape in (("Bt", (m.n_u, m.n_p)), ("B", (m.n_p, m.n_u))):
        G, C = block_csr(new, key, shape), block_csr(old, key, shape)
        rp, cols, vals = orc.nse_block_csr(key)
        O = sp.csr_matrix((vals, cols, rp), shape=shape)
        assert abs(G - O).max() / abs(O).max() < 1e-12, key
        assert abs(G - C).max() / abs(C).max() < 1e-13, key
        assert G.nnz == C.nnz
    Bt, B = block_csr(new, "Bt", (m.n_u, m.n_p)), block_csr(new, "B", (m.n_p, m.n_u))
    assert abs(B - Bt.T).max() == 0.0
    # the whole operator and the rhs the solve reads
    x = rng.uniform(-1, 1, m.n_u + m.n_p)
    yn, yo = new.nse_vmult(x), old.nse_vmult(x)
    assert np.max(np.abs(yn - yo)) <= 1e-13 * np.max(np.abs(yo))
    assert np.array_equal(new.get_state(dcp.NSE_RHS), old.get_state(dcp.NSE_RHS))
    # deterministic
    v1 = new.coupling_csr("Bt")[2].copy()
    new.assemble_nse_system()
    assert np.array_equal(new.coupling_csr("Bt")[2], v1)
    new.close()
    old.close()


@pytest.mark.parametrize("refine", [2, 3])
def test_kronecker_constrained_diagonals(monkeypatch, refine):
    """The constrained-row diagonals (no-normal-flux nodes: the |K_ii| of the
    cells holding the node, what AffineConstraints puts on a constrained row)
    in Kronecker form (k_cdk_diag, assembly.hip) against the cell pass +
    con_gather (DCP_CDIAG_KRON=0): the velocity apply and the Stokes apply at
    1e-13, the velocity apply against the oracle's assembled nse_matrix at
    1e-12, bitwise repeatable, and a time
    step change (dt / Re in K_ii) followed by the next assembly."""
    m = dcp.HostMesh(refine=refine)
    ph = dcp.classic_physics()
    rng = np.random.default_rng(SEED + 40 + refine)
    u = rng.uniform(-1, 1, m.n_u + m.n_p)
    T = m.T0 + 0.1 * rng.uniform(-1, 1, m.n_T)
    x = rng.uniform(-1, 1, m.n_u + m.n_p)
    out = {}
    for kron in ("1", "0"):
        monkeypatch.setenv("DCP_CDIAG_KRON", kron)
        ctx = make_ctx(m, ph, True, monkeypatch)
        monkeypatch.delenv("DCP_CDIAG_KRON", raising=False)
        ctx.set_state(dcp.OLD_NSE_SOLUTION, u)
        ctx.set_state(dcp.OLD_T_SOLUTION, T)
        ctx.assemble_nse_system()
        r = [ctx.velocity_vmult(x[:m.n_u]), ctx.nse_vmult(x), None]
        ctx.assemble_nse_system()
        r.append(ctx.velocity_vmult(x[:m.n_u]))
        ctx.set_time_step(0.5 * ph.time_step)
        ctx.assemble_nse_system()
        r.append(ctx.velocity_vmult(x[:m.n_u]))
        out[kron] = r
        ctx.close()
    k, c = out["1"], out["0"]
    for a, b in zip(k[:2], c[:2]):
        assert np.max(np.abs(a - b)) <= 1e-13 * np.max(np.abs(b))
    assert np.array_equal(k[0], k[3])
    assert np.max(np.abs(k[4] - c[4])) <= 1e-13 * np.max(np.abs(c[4]))
    assert not np.allclose(k[4], k[0], rtol=1e-6)  # dt entered K_ii
    # the velocity apply, constrained rows included, against the oracle's
    # assembled nse_matrix (velocity block) times x
    orc = oracle_py.Model(ph, m)
    orc.assemble_nse_system(u, T)
    xv = x.copy()
    xv[m.n_u:] = 0.0
    yo = orc.nse_vmult(xv)[:m.n_u]
    assert np.max(np.abs(k[0] - yo)) <= 1e-12 * np.max(np.abs(yo))


def test_kronecker_bt_solve_matches_row_tasks(monkeypatch):
    """The block-preconditioned solve on either B^T: equal FGMRES / inner
    counts, iterates at 1e-10 (the inner GMRES held at a fixed step count, so
    no tolerance decision sits on a rounding difference)."""
    m = dcp.HostMesh(refine=2)
    ph = dcp.classic_physics()
    out = []
    for kron in (True, False):
        ctx = make_ctx(m, ph, kron, monkeypatch)
        ctx.set_state(dcp.OLD_NSE_SOLUTION, np.zeros(m.n_u + m.n_p))
        ctx.set_state(dcp.OLD_T_SOLUTION, m.T0)
        ctx.copy_state(dcp.NSE_SOLUTION, dcp.OLD_NSE_SOLUTION)
        ctx.assemble_nse_system()
        ctx.build_nse_preconditioner()
        rc, outer, inner = ctx.solve_nse()
        out.append((rc, outer, inner, ctx.get_state(dcp.NSE_SOLUTION)))
        ctx.close()
    (r0, o0, i0, x0), (r1, o1, i1, x1) = out
    assert r0 == r1 and o0 == o1
    assert abs(i0 - i1) <= max(2, i1 // 50)
    assert np.linalg.norm(x0 - x1) <= 1e-8 * np.linalg.norm(x1)


def test_partitioned_and_periodic_meshes_keep_row_tasks(monkeypatch):
    """Not the one-GPU layered shell (a warped shell is no separable map):
    the Kronecker form is refused and B^T still matches the oracle."""
    m = dcp.HostMesh(refine=2)
    X = m.cell_geometry.reshape(-1, 3)
    X += 0.02 * np.sin(3.0 * X[:, [1, 2, 0]]) * np.cos(2.0 * X[:, [2, 0, 1]])
    ph = dcp.classic_physics()
    ctx = make_ctx(m, ph, True, monkeypatch)
    assert not ctx.assembly_layout()["bt_kronecker"]
    u = np.random.default_rng(SEED).uniform(-1, 1, m.n_u + m.n_p)
    ctx.set_state(dcp.OLD_NSE_SOLUTION, u)
    ctx.set_state(dcp.OLD_T_SOLUTION, m.T0)
    ctx.assemble_nse_system()
    orc = oracle_py.Model(ph, m)
    orc.assemble_nse_system(u, m.T0)
    G = block_csr(ctx, "Bt", (m.n_u, m.n_p))
    rp, cols, vals = orc.nse_block_csr("Bt")
    O = sp.csr_matrix((vals, cols, rp), shape=(m.n_u, m.n_p))
    assert abs(G - O).max() / abs(O).max() < 1e-12
    ctx.close()
