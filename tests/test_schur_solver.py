"""solve_NSE_Schur_complement (boussinesq_model.tpp:1248-1414), the
use_schur_complement_solver path of the classic model that the cube prm
(BASELINE C2) selects: GMRES on S = B A^-1 B^T (A^-1: InverseMatrix = CG
preconditioned by LA::PreconditionILU, i.e. Trilinos ILU(0) of A), left
preconditioned by ApproximateInverseMatrix = CG on B ILU^-1 B^T, then
u = A^-1 (f - B^T p).

CPU: the oracle's restatement converges on the shell and the periodic cube.
GPU: dcp_solve_nse_schur against the oracle at 1e-9 (nested inexact solves)
with equal Schur GMRES and A^-1 counts, on the shell (classic prm) and the cube (cube prm physics:
Coriolis, vertical gravity, periodic images), and dcp_run on the cube prm.

The reference renumbers the NSE dofs with Cuthill_McKee before this solver
(:198-204); ILU(0) depends on the order, so both sides factor the numbering
the mesh arrives with: the first-encounter one and the Cuthill-McKee one
(cube-r2-cm, dcp_host_mesh_renumber_cuthill_mckee) that the reference's
setup_dofs gives this solver (parity with Trilinos' Ifpack unpinned)."""
import os

import numpy as np
import pytest

import dcp
import oracle_py

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CUBE_PRM = os.path.join(ROOT, "configs", "aqua_planet_cube_test_3d.prm")


def case(name):
    if name.startswith("cube-r2"):
        rp = dcp.load_prm(CUBE_PRM)
        ph = dcp.physics_from_params(rp)
        return dcp.HostMesh(cuboid=True, refine=2, length=rp.length,
                            cuthill_mckee=name.endswith("-cm")), ph
    refine = int(name[-1])
    return dcp.HostMesh(refine=refine), dcp.classic_physics()


def oracle_solve(m, ph, u, T, fixed_inner=0):
    orc = oracle_py.Model(ph, m)
    orc.set_schur_fixed_inner(fixed_inner)
    orc.assemble_nse_system(u, T)
    return orc.solve_nse_schur(u)


@pytest.mark.parametrize("name", ["shell-r1", "cube-r2", "cube-r2-cm"])
def test_oracle_schur_solver_converges(name):
    m, ph = case(name)
    u, T = np.zeros(m.n_u + m.n_p), m.T0.copy()
    rc, x, its, na = oracle_solve(m, ph, u, T)
    # A^-1 solves: the rhs, one per S apply (GMRES: the initial residual and one
    # per step), the velocity
    assert rc == 0 and 0 < its < 30 and na == its + 3
    assert np.all(np.isfinite(x)) and np.linalg.norm(x) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["shell-r1", "cube-r2", "cube-r2-cm"])
def test_gpu_schur_solver_matches_oracle(name):
    m, ph = case(name)
    rng = np.random.default_rng(7)
    u = 0.1 * rng.uniform(-1, 1, m.n_u + m.n_p)
    T = m.T0 + 0.05 * rng.uniform(-1, 1, m.n_T)
    ctx = dcp.Context()
    ctx.set_physics(ph)
    ctx.upload_mesh(m)
    for f, v in ((dcp.OLD_NSE_SOLUTION, u), (dcp.NSE_SOLUTION, u), (dcp.OLD_T_SOLUTION, T),
                 (dcp.T_SOLUTION, T)):
        ctx.set_state(f, v)
    ctx.assemble_nse_system()
    rc, its, na = ctx.solve_nse_schur()
    x = ctx.get_state(dcp.NSE_SOLUTION)
    rco, xo, itso, nao = oracle_solve(m, ph, ctx.get_state(dcp.OLD_NSE_SOLUTION), T)
    ctx.close()
    assert rc == rco == 0
    assert (its, na) == (itso, nao)
    # the solve nests inexact solves (CG at 1e-6 inside GMRES at 1e-6, the
    # preconditioner another CG at 1e-6): operator rounding at 1e-16 (FMA
    # contraction, the block SpMV's sum order) reaches ~1e-10 of the result
    # (1.5e-10 measured on the r=1 shell), hence 1e-9
    assert np.linalg.norm(x - xo) <= 1e-9 * np.linalg.norm(xo)


@pytest.mark.gpu
@pytest.mark.parametrize("name,k", [("shell-r1", 40), ("cube-r2-cm", 8)])
def test_gpu_schur_solver_fixed_inner_1e10(name, k):
    """With DCP_OPT_SCHUR_FIXED_INNER both inner CGs run a fixed number of
    steps in the oracle and on the device (no early-stop decision for rounding
    to flip), and the Schur solve agrees to 1e-10 — the north-star bar."""
    m, ph = case(name)
    rng = np.random.default_rng(11)
    u = 0.1 * rng.uniform(-1, 1, m.n_u + m.n_p)
    T = m.T0 + 0.05 * rng.uniform(-1, 1, m.n_T)
    ctx = dcp.Context()
    ctx.set_physics(ph)
    ctx.upload_mesh(m)
    # k below the CG's exact convergence on the mesh: steps past it divide by
    # round-off-level residuals, where no two implementations agree
    ctx.set_schur_fixed_inner(k)
    for f, v in ((dcp.OLD_NSE_SOLUTION, u), (dcp.NSE_SOLUTION, u), (dcp.OLD_T_SOLUTION, T),
                 (dcp.T_SOLUTION, T)):
        ctx.set_state(f, v)
    ctx.assemble_nse_system()
    rc, its, na = ctx.solve_nse_schur()
    x = ctx.get_state(dcp.NSE_SOLUTION)
    rco, xo, itso, nao = oracle_solve(m, ph, ctx.get_state(dcp.OLD_NSE_SOLUTION), T, k)
    ctx.close()
    assert rc == rco and (its, na) == (itso, nao)
    assert np.linalg.norm(x - xo) <= 1e-10 * np.linalg.norm(xo)


@pytest.mark.gpu
def test_run_cube_prm_uses_the_schur_solver():
    """dcp_run with the cube prm (use schur complement solver = true): the
    first step runs the Schur-complement solve, as run() does (:1896-1898),
    on the Cuthill-McKee numbering setup_dofs gives it."""
    rp = dcp.load_prm(CUBE_PRM)
    assert rp.use_schur_complement_solver == 1
    rp.use_FEEC_solver = 0  # the classic model (BASELINE C2 overrides)
    rp.nse_velocity_degree = 2
    ph = dcp.physics_from_params(rp)
    m = dcp.HostMesh(cuboid=True, refine=2, length=rp.length, cuthill_mckee=True)
    ctx = dcp.Context()
    ctx.set_physics(ph)
    ctx.upload_mesh(m)
    for f, v in ((dcp.OLD_NSE_SOLUTION, np.zeros(m.n_u + m.n_p)),
                 (dcp.NSE_SOLUTION, np.zeros(m.n_u + m.n_p)), (dcp.OLD_T_SOLUTION, m.T0),
                 (dcp.T_SOLUTION, m.T0)):
        ctx.set_state(f, v)
    rc, rep, _ = ctx.run(rp, max_steps=1)
    ctx.close()
    assert rc == 0 and rep.steps == 1
    assert rep.fgmres_outer == 0 and rep.schur_inner > 0


@pytest.mark.gpu
def test_schur_solver_after_reupload_with_another_numbering():
    """The ILU(0) structure (pattern, levels, A_val positions) is built once per
    mesh: uploading the Cuthill-McKee copy of the same mesh (same n_u, other
    numbering) into the same context must rebuild it, so the second solve
    matches the oracle on the new numbering exactly like a fresh context."""
    rng = np.random.default_rng(11)
    ctx = dcp.Context()
    try:
        for name in ("cube-r2", "cube-r2-cm"):
            m, ph = case(name)
            u = 0.1 * rng.uniform(-1, 1, m.n_u + m.n_p)
            T = m.T0.copy()
            ctx.set_physics(ph)
            ctx.upload_mesh(m)
            for f, v in ((dcp.OLD_NSE_SOLUTION, u), (dcp.NSE_SOLUTION, u),
                         (dcp.OLD_T_SOLUTION, T), (dcp.T_SOLUTION, T)):
                ctx.set_state(f, v)
            ctx.assemble_nse_system()
            rc, its, na = ctx.solve_nse_schur()
            x = ctx.get_state(dcp.NSE_SOLUTION)
            rco, xo, itso, nao = oracle_solve(m, ph, ctx.get_state(dcp.OLD_NSE_SOLUTION), T)
            assert rc == rco == 0 and (its, na) == (itso, nao), name
            assert np.linalg.norm(x - xo) <= 1e-9 * np.linalg.norm(xo), name
    finally:
        ctx.close()
