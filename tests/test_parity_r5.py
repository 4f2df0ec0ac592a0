"""Oracle parity at the size the bench measures (refine 5: 196,608 cells,
4,995,528 NSE dofs), with the kernels the bench's default step runs.

The oracle (oracle/oracle.cpp, test infrastructure) runs live on the host:
the full assemble_nse_system with AffineConstraints distribute into CSR
(boussinesq_model.tpp:550-687, 691-740), build_nse_preconditioner (:479-542),
the temperature matrix and rhs (:748-1020), SchurComplement::vmult
(schur_complement.hpp:143-150) as B (D_A^-1 (B^T p)) and
BlockSchurPreconditioner::vmult (block_schur_preconditioner.hpp:42-70). Its
cell loops run on up to 16 host threads with bitwise the serial results
(tests/test_oracle_kat.py::test_threaded_assembly_is_the_serial_assembly).

The GPU side is configured as bench.py's default step: operator-form
assembly (B^T by row tasks, the rhs through the pencil kernel and the node
gather, the constrained diagonals over the constrained cells), the explicit
Schur complement in the structured-column SELL layout (k_sell_spmv<.., 2>),
the s-step inner Schur GMRES, the matrix-free [A B^T; B 0] apply.

Bars: assembled entries and operator applies 1e-12 relative to the largest
entry (only the summation order differs); the block preconditioner with its
inner Schur GMRES held at 56 steps (two restart cycles of 28, no tolerance
decision for rounding to flip) 1e-10 relative in the 2-norm.

DCP_PARITY_REFINE overrides the refinement (e.g. 4 where host memory is
short); the module prints which size ran, its wall times and the peak host
memory."""
import os
import resource
import time

import numpy as np
import pytest
import scipy.sparse as sp

import dcp
import oracle_py

pytestmark = pytest.mark.gpu

REFINE = int(os.environ.get("DCP_PARITY_REFINE", "5"))
SEED = 20261015


def rel_max(a, b):
    return np.max(np.abs(np.asarray(a) - np.asarray(b))) / max(np.max(np.abs(b)), 1e-300)


def rel2(a, b):
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


def peak_rss_gb():
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6


class Big:
    """The module's shared state, built stage by stage by the tests below (in
    file order, each well under two minutes, so no single test sits silent
    for long): the mesh and the GPU context, then the oracle's pattern, its
    assembly, its preconditioner and temperature system."""
    m = ph = ctx = orc = u = T = None


@pytest.fixture(scope="module")
def big():
    b = Big()
    yield b
    if b.ctx is not None:
        b.ctx.close()
    oracle_py.set_threads(1)


def _need(b, *names):
    for n in names:
        if getattr(b, n) is None:
            pytest.skip(f"earlier stage did not run ({n})")


def test_r5_gpu_setup_runs_the_bench_layout(big):
    """The GPU step of the bench's default configuration. The parity below is
    about the bench's kernels: the structured-column S (8 bytes per entry,
    columns formed from the row's level) must be the layout in use."""
    t0 = time.time()
    big.m = m = dcp.HostMesh(refine=REFINE)
    big.ph = ph = dcp.classic_physics()
    rng = np.random.default_rng(SEED)
    n = m.n_u + m.n_p
    # a moving state (every rhs term: advection, buoyancy of a perturbed T)
    big.u = u = rng.uniform(-1, 1, n)
    big.T = T = m.T0 + 0.1 * rng.uniform(-1, 1, m.n_T)
    t_mesh = time.time() - t0
    t0 = time.time()
    ctx = dcp.Context()
    ctx.set_physics(ph)
    ctx.set_schur_explicit(True)
    ctx.set_gram_schmidt("sstep")
    ctx.upload_mesh(m)
    ctx.set_state(dcp.OLD_NSE_SOLUTION, u)
    ctx.set_state(dcp.OLD_T_SOLUTION, T)
    ctx.set_state(dcp.NSE_SOLUTION, u)
    ctx.assemble_nse_system()
    ctx.build_nse_preconditioner()
    ctx.assemble_temperature_matrix()
    ctx.assemble_temperature_rhs()
    big.ctx = ctx
    lay = ctx.schur_layout()
    print(f"\nparity at refine {REFINE}: {m.n_cells} cells, {n} NSE dofs, {m.n_T} T dofs; "
          f"mesh {t_mesh:.1f} s, GPU setup {time.time() - t0:.1f} s; schur layout {lay}")
    assert lay["col_bytes"] == 0, lay


def test_r5_oracle_pattern(big):
    """setup_nse_matrices / setup_temperature_matrices (boussinesq_model.tpp:79-180)
    in the oracle: the constrained sparsity patterns."""
    _need(big, "m")
    threads = oracle_py.usable_threads()
    oracle_py.set_threads(threads)
    t0 = time.time()
    big.orc = oracle_py.Model(big.ph, big.m)
    print(f"\noracle patterns on {threads} threads: {time.time() - t0:.1f} s; "
          f"peak host memory {peak_rss_gb():.1f} GB")


def test_r5_rhs_and_coupling_blocks(big):
    """Operator-form rhs and B^T / B (coupling_csr: what the solve reads)
    against the oracle's assemble_nse_system (element matrices and
    distribute_local_to_global, :550-687)."""
    _need(big, "ctx", "orc")
    m, ctx, orc = big.m, big.ctx, big.orc
    t0 = time.time()
    orc.assemble_nse_system(big.u, big.T)
    print(f"\noracle assemble_nse_system: {time.time() - t0:.1f} s; "
          f"peak host memory {peak_rss_gb():.1f} GB")
    t0 = time.time()
    assert rel_max(ctx.get_state(dcp.NSE_RHS), orc.nse_rhs()) < 1e-12
    for key, shape in (("Bt", (m.n_u, m.n_p)), ("B", (m.n_p, m.n_u))):
        rp, cols, vals = ctx.coupling_csr(key)
        G = sp.csr_matrix((vals, cols, rp), shape=shape)
        rp, cols, vals = orc.nse_block_csr(key)
        O = sp.csr_matrix((vals, cols, rp), shape=shape)
        err = abs(G - O).max() / abs(O).max()
        print(f"{key}: nnz GPU {G.nnz} oracle {O.nnz}, max rel {err:.2e}")
        assert err < 1e-12, key
    print(f"rhs + coupling compared in {time.time() - t0:.1f} s")


def test_r5_preconditioner_and_temperature(big):
    """build_nse_preconditioner's Jacobi diagonals (:479-542) and the
    temperature matrix / rhs (:748-1020)."""
    _need(big, "ctx", "orc")
    m, ctx, orc = big.m, big.ctx, big.orc
    t0 = time.time()
    orc.build_nse_preconditioner()
    orc.assemble_temperature_matrix()
    orc.assemble_temperature_rhs(big.T, big.u)
    print(f"\noracle preconditioner + temperature system: {time.time() - t0:.1f} s")
    a_g, p_g = ctx.precond_diagonals()
    a_o, p_o = orc.precond_diagonals()
    assert rel_max(a_g, a_o) < 1e-12
    assert rel_max(p_g, p_o) < 1e-12
    rp, cols, vals = ctx.T_matrix_csr()
    Tg = sp.csr_matrix((vals, cols, rp), shape=(m.n_T, m.n_T))
    rp, cols, vals = orc.T_matrix_csr()
    To = sp.csr_matrix((vals, cols, rp), shape=(m.n_T, m.n_T))
    assert abs(Tg - To).max() / abs(To).max() < 1e-12
    assert rel_max(ctx.get_state(dcp.T_RHS), orc.T_rhs()) < 1e-12


def test_r5_operator_applies(big):
    """The structured-column S apply against the oracle's composite
    B (D_A^-1 (B^T p)); the matrix-free [A B^T; B 0] x and A x against the
    assembled nse_matrix products."""
    _need(big, "ctx", "orc")
    m, ctx, orc = big.m, big.ctx, big.orc
    rng = np.random.default_rng(SEED + 1)
    p = rng.uniform(-1, 1, m.n_p)
    e = rel_max(ctx.schur_vmult(p), orc.schur_vmult(p))
    print(f"S p: max rel {e:.2e}")
    assert e < 1e-12
    x = rng.uniform(-1, 1, m.n_u + m.n_p)
    yo = orc.nse_vmult(x)
    e = rel_max(ctx.nse_vmult(x), yo)
    print(f"[A B^T; B 0] x: max rel {e:.2e}")
    assert e < 1e-12
    xv = x.copy()
    xv[m.n_u:] = 0.0
    yv = orc.nse_vmult(xv)[:m.n_u]
    assert rel_max(ctx.velocity_vmult(x[:m.n_u]), yv) < 1e-12


def test_r5_block_preconditioner_fixed_inner_sstep(big):
    """BlockSchurPreconditioner::vmult with the inner Schur GMRES held at 56
    steps (DCP_OPT_BLOCK_FIXED_INNER, the same hook in the oracle): the s-step
    Newton-basis Arnoldi with block CGS2 + Cholesky QR on the GPU against
    deal.II's modified Gram-Schmidt in the oracle."""
    _need(big, "ctx", "orc")
    m, ctx, orc = big.m, big.ctx, big.orc
    x = np.random.default_rng(SEED + 2).uniform(-1, 1, m.n_u + m.n_p)
    x[m.n_u:] -= x[m.n_u:].mean()
    ctx.set_block_fixed_inner(56)
    orc.set_block_fixed_inner(56)
    try:
        t0 = time.time()
        dg, itg = ctx.block_preconditioner_vmult(x)
        t_g = time.time() - t0
        t0 = time.time()
        do, ito = orc.block_preconditioner_vmult(x)
        t_o = time.time() - t0
    finally:
        ctx.set_block_fixed_inner(0)
        orc.set_block_fixed_inner(0)
    e_p = rel2(dg[m.n_u:], do[m.n_u:])
    e = rel2(dg, do)
    print(f"block preconditioner, 56 inner steps: GPU {t_g:.2f} s, oracle {t_o:.1f} s, "
          f"rel2 {e:.2e} (pressure {e_p:.2e}); peak host memory {peak_rss_gb():.1f} GB")
    assert itg == ito == 56
    assert e < 1e-10 and e_p < 1e-10
