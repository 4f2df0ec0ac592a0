"""dcp_run (csrc/driver.cpp): the reference's time loop (boussinesq_model.tpp:
1841-1926) over the C ABI, against the same calls made one by one from Python,
and the dcp_aquaplanet executable (source/main.cxx -p <prm>)."""
import math
import os
import subprocess

import numpy as np
import pytest

import dcp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PRM = os.path.join(ROOT, "configs", "aqua_planet_shell_test_3d-classic.prm")


def fresh(rp, m):
    ctx = dcp.Context()
    ctx.set_physics(dcp.physics_from_params(rp))
    ctx.upload_mesh(m)
    u = np.zeros(m.n_u + m.n_p)
    for f, v in ((dcp.NSE_SOLUTION, u), (dcp.OLD_NSE_SOLUTION, u), (dcp.T_SOLUTION, m.T0),
                 (dcp.OLD_T_SOLUTION, m.T0)):
        ctx.set_state(f, v)
    return ctx


@pytest.mark.gpu
@pytest.mark.parametrize("interval", [1, 2])
def test_run_matches_step_by_step_calls(interval):
    """interval = NSE solver interval: the NSE system is reassembled AND solved
    only on step 0 and every interval-th step (run(), :1865-1881, and
    solve_NSE_block_preconditioned's own guard, :1135-1137)."""
    rp = dcp.load_prm(PRM)
    rp.initial_global_refinement = 1
    rp.adapt_time_step = 1           # recompute_time_step from step 1 on
    rp.final_time = 100.0
    rp.physics.nse_solver_interval = interval
    m = dcp.HostMesh(refine=1, R0=rp.R0, R1=rp.R1, length=rp.length)
    nsteps = 3
    ctx = fresh(rp, m)
    rc, rep, steps = ctx.run(rp, max_steps=nsteps)
    assert rc == dcp.DCP_OK and rep.steps == nsteps and len(steps) == nsteps
    u_run, T_run = ctx.get_state(dcp.NSE_SOLUTION), ctx.get_state(dcp.T_SOLUTION)
    ctx.close()

    ctx = fresh(rp, m)
    dt = rp.physics.time_step
    t = 0.0
    for n in range(nsteps):
        cfl = ctx.cfl_number()
        nse_step = n % interval == 0
        if n > 0 and nse_step and rp.adapt_time_step:
            deg = max(rp.physics.temperature_degree, rp.nse_velocity_degree)
            dt = (0.25 / (2.1 * 3 * math.sqrt(3))) / (deg * cfl)
            ctx.set_time_step(dt)
        ctx.max_velocity()
        assert steps[n].time_step == dt and steps[n].time_index == t
        if nse_step:
            ctx.assemble_nse_system()
            ctx.build_nse_preconditioner()
        ctx.assemble_temperature_matrix()
        ctx.assemble_temperature_rhs()
        if nse_step:
            rcn, outer, inner = ctx.solve_nse()
            assert outer > 0
        else:
            rcn, outer, inner = 0, 0, 0
        assert (rcn, outer, inner) == (0, steps[n].fgmres_outer, steps[n].schur_inner)
        ctx.solve_temperature()
        ctx.advance_state()
        t += dt / rp.physics.nse_solver_interval
    assert steps[interval].time_step != steps[0].time_step  # the adaptive step took effect
    assert np.array_equal(ctx.get_state(dcp.NSE_SOLUTION), u_run)
    assert np.array_equal(ctx.get_state(dcp.T_SOLUTION), T_run)
    ctx.close()


@pytest.mark.gpu
def test_executable_runs_the_classic_prm():
    exe = os.path.join(ROOT, "3d-dycoreplanet_amd", "dcp_aquaplanet")
    out = subprocess.run([exe, "-p", PRM, "--refine", "2"], capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stderr
    # the classic prm runs exactly one step (time_index += dt > final_time, Q24)
    assert out.stdout.count("Time step ") == 1
    assert "1 steps to t=" in out.stdout


def test_executable_requires_a_parameter_file():
    exe = os.path.join(ROOT, "3d-dycoreplanet_amd", "dcp_aquaplanet")
    out = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert out.returncode == 1 and "-p" in out.stderr


@pytest.mark.gpu
def test_executable_writes_vtu_output(tmp_path):
    """--output: output_results before the loop and after each step
    (boussinesq_model.tpp:1840/1907), NAME-XXXXX.0000.vtu + NAME-XXXXX.pvtu."""
    exe = os.path.join(ROOT, "3d-dycoreplanet_amd", "dcp_aquaplanet")
    out = subprocess.run([exe, "-p", PRM, "--refine", "1", "--output", str(tmp_path),
                          "--output-stem", "aqua"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    names = sorted(p.name for p in tmp_path.iterdir())
    assert names == ["aqua-00000.0000.vtu", "aqua-00000.pvtu",
                     "aqua-00001.0000.vtu", "aqua-00001.pvtu"]
    text = (tmp_path / "aqua-00001.0000.vtu").read_text()
    n_cells = dcp.HostMesh(refine=1).n_cells
    assert 'NumberOfCells="%d"' % (8 * n_cells) in text  # 8 hexahedra per cell
    assert 'Source="aqua-00001.0000.vtu"' in (tmp_path / "aqua-00001.pvtu").read_text()


def _calls(ctx, name):
    """Calls of a TimerOutput section; 0 for a section never entered (the
    library knows only sections that ran)."""
    try:
        return ctx.timer_section(name)[0]
    except dcp.DcpError:
        return 0


@pytest.mark.gpu
def test_solver_history_and_timer_sections():
    """§5 auxiliaries: SolverControl(..., log_history = true, log_result = true)
    of the FGMRES solve (boussinesq_model.tpp:1166-1169) and the TimerOutput
    sections under the reference's names (:483-1572)."""
    rp = dcp.load_prm(PRM)
    m = dcp.HostMesh(refine=2)
    ctx = fresh(rp, m)
    ctx.set_log_history(True)
    ctx.assemble_nse_system()
    ctx.build_nse_preconditioner()
    ctx.assemble_temperature_matrix()
    ctx.assemble_temperature_rhs()
    rc, outer, inner = ctx.solve_nse()
    ctx.solve_temperature()
    assert rc == 0
    steps, vals, res = ctx.solver_history(0)
    # one check per FGMRES restart head (step 0) and per iteration from j = 1
    assert res == 1 and steps[0] == 0 and steps[-1] == outer and len(steps) == outer + 1
    tol = 1e-8 * np.linalg.norm(ctx.get_state(dcp.NSE_RHS))
    assert vals[-1] <= tol < vals[-2]
    assert np.all(np.diff(vals) <= 1e-12 * vals[0])  # least-squares residuals never grow
    assert ctx.solver_history(1)[2] == 0                 # the fallback did not run
    lines = ctx.deallog(2)
    assert lines[0].startswith("DEAL:FGMRES::Check 0\t") and lines[-1].startswith(
        f"DEAL:FGMRES::Convergence step {outer} value ")
    for name in ("   Assemble NSE system", "   Build NSE preconditioner",
                 "   Assembly NSE preconditioner", "   Assemble temperature matrices",
                 "   Assemble temperature RHS", "   Solve Stokes system",
                 "   Solve temperature system"):
        calls, sec = ctx.timer_section(name)
        assert calls == 1 and sec > 0, name
    assert ctx.timer_section("   Assembly NSE preconditioner")[1] <= \
        ctx.timer_section("   Build NSE preconditioner")[1]
    summary = ctx.timer_summary()
    assert "Total wallclock time elapsed since start" in summary and "Solve Stokes system" in summary
    with pytest.raises(dcp.DcpError):
        ctx.timer_section("no such section")
    ctx.close()


FEEC_PRM = os.path.join(ROOT, "configs", "aqua_planet_shell_test_3d-feec.prm")


def fresh_feec(rp, m):
    ctx = dcp.Context()
    ctx.set_physics(dcp.physics_from_params(rp))
    ctx.upload_feec_mesh(m)
    x0 = np.zeros(m.feec.n)
    for f, v in ((dcp.NSE_SOLUTION, x0), (dcp.OLD_NSE_SOLUTION, x0), (dcp.T_SOLUTION, m.T0),
                 (dcp.OLD_T_SOLUTION, m.T0)):
        ctx.set_state(f, v)
    return ctx


@pytest.mark.gpu
def test_run_feec_with_schur_complement_solver_is_the_reference_no_op():
    """FEEC with use_schur_complement_solver (FEEC.tpp:2264-2298): run() skips
    build_nse_preconditioner and calls solve_NSE_Schur_complement, whose body is
    commented out (:1480-1500): nse_solution keeps its value, no FGMRES
    iterations, no preconditioner section, the temperature still solves. The
    same run with the block preconditioner builds it and solves."""
    rp = dcp.load_prm(FEEC_PRM)
    rp.initial_global_refinement = 1
    m = dcp.HostMesh(refine=1, feec=True, R0=rp.R0, R1=rp.R1, length=rp.length)
    rng = np.random.default_rng(2)
    out = {}
    for schur in (1, 0):
        rp.use_schur_complement_solver = schur
        ctx = fresh_feec(rp, m)
        x0 = np.zeros(m.feec.n)
        x0[:m.feec.n_w + m.feec.n_u] = 0.01 * rng.uniform(-1, 1, m.feec.n_w + m.feec.n_u)
        x0[m.feec.fixed.astype(bool)] = 0
        ctx.set_state(dcp.NSE_SOLUTION, x0)
        ctx.set_state(dcp.OLD_NSE_SOLUTION, x0)
        rc, rep, steps = ctx.run(rp, max_steps=1)
        out[schur] = (rc, rep, ctx.get_state(dcp.NSE_SOLUTION), x0,
                      _calls(ctx, "   Build NSE FEEC preconditioner"),
                      _calls(ctx, "   Solve NSE system"))
        ctx.close()
    rc, rep, x, x0, n_prec, n_solve = out[1]
    assert rc == dcp.DCP_OK and rep.steps == 1 and rep.fgmres_outer == 0
    assert np.array_equal(x, x0) and n_prec == 0 and n_solve == 0 and rep.T_cg > 0
    rc, rep, x, x0, n_prec, n_solve = out[0]
    assert rc == dcp.DCP_OK and rep.fgmres_outer > 0 and n_prec == 1 and n_solve == 1
    assert not np.array_equal(x, x0)


@pytest.mark.gpu
def test_run_feec_without_block_preconditioner():
    """use block preconditioner feec = false (FEEC.tpp:1420-1431): run() skips
    build_nse_preconditioner (:2264-2276) and the solve is the identity-
    preconditioned GMRES(100); one step against the step-by-step calls with the
    option set directly (bitwise)."""
    rp = dcp.load_prm(FEEC_PRM)
    rp.initial_global_refinement = 1
    rp.use_block_preconditioner_feec = 0
    rp.use_schur_complement_solver = 0
    m = dcp.HostMesh(refine=1, feec=True, R0=rp.R0, R1=rp.R1, length=rp.length)
    ctx = fresh_feec(rp, m)
    rc, rep, steps = ctx.run(rp, max_steps=1)
    x_run = ctx.get_state(dcp.NSE_SOLUTION)
    n_prec = _calls(ctx, "   Build NSE FEEC preconditioner")
    ctx.close()
    assert rc == dcp.DCP_OK and rep.fgmres_outer > 0 and n_prec == 0
    ctx = fresh_feec(rp, m)
    ctx.set_feec_block_preconditioner(False)
    ctx.set_feec_zero_mean(bool(rp.correct_pressure_to_zero_mean))
    ctx.set_time_step(rp.physics.time_step)
    ctx.cfl_number()
    ctx.feec_assemble_nse_system()
    rc2, it = ctx.feec_solve_nse()
    assert rc2 == dcp.DCP_OK and it == rep.fgmres_outer
    assert np.array_equal(ctx.get_state(dcp.NSE_SOLUTION), x_run)
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["feec-degree-2", "classic-degree-1", "direct-solver"])
def test_run_rejects_what_the_device_path_does_not_implement(case):
    """dcp_run refuses up front (DCP_ERR_UNSUPPORTED, nothing stepped) instead
    of silently running another discretisation: FEEC with nse velocity degree
    != 1 (FE_Nedelec/RT/DGQ(degree - 1), FEEC.tpp:21-30), the classic model
    with degree != 2, and the MUMPS branch the reference itself throws on
    (:1886-1893)."""
    feec = case.startswith("feec")
    rp = dcp.load_prm(FEEC_PRM if feec else PRM)
    rp.initial_global_refinement = 1
    if case == "feec-degree-2":
        rp.nse_velocity_degree = 2
    elif case == "classic-degree-1":
        rp.nse_velocity_degree = 1
    else:
        rp.use_direct_solver = 1
    m = dcp.HostMesh(refine=1, feec=feec, R0=rp.R0, R1=rp.R1, length=rp.length)
    ctx = fresh_feec(rp, m) if feec else fresh(rp, m)
    with pytest.raises(dcp.DcpError) as e:
        ctx.run(rp, max_steps=1)
    assert e.value.code == dcp.DCP_ERR_UNSUPPORTED
    assert _calls(ctx, "   Assemble NSE system") == 0
    ctx.close()


CUBE_PRM = os.path.join(ROOT, "configs", "aqua_planet_cube_test_3d.prm")


@pytest.mark.gpu
def test_run_feec_cube_prm_against_the_oracle():
    """data/aqua_planet_cube_test_3d.prm: FEEC on the periodic cuboid with the
    Schur-complement switch, i.e. run() reassembles the NSE system every step
    and leaves nse_solution as it is (FEEC.tpp:1480-1500), and the temperature
    (periodic in x, y: identity lines folded at upload, FEEC.tpp:435-463)
    diffuses and advects with the given RT velocity. Three dcp_run steps
    against the oracle's assemble / CG step by step: CG counts within one
    (the second step's CG ends at its 1e-12 threshold: a 1e-15 perturbation of
    the oracle's own old temperature moves it between 25 and 26 steps,
    test_feec.py::test_cube_temperature_cg_count_is_rounding_sensitive),
    temperature at 1e-10, periodic images equal to their partners."""
    import oracle_py
    rp = dcp.load_prm(CUBE_PRM)
    rp.initial_global_refinement = 2
    m = dcp.HostMesh(cuboid=True, refine=2, feec=True, length=rp.length)
    f = m.feec
    rng = np.random.default_rng(11)
    x0 = np.zeros(f.n)
    x0[:f.n_w + f.n_u] = 0.05 * rng.uniform(-1, 1, f.n_w + f.n_u)
    x0[f.fixed.astype(bool)] = 0
    ctx = fresh_feec(rp, m)
    ctx.set_state(dcp.NSE_SOLUTION, x0)
    ctx.set_state(dcp.OLD_NSE_SOLUTION, x0)
    nsteps = 3
    rc, rep, steps = ctx.run(rp, max_steps=nsteps)
    assert rc == dcp.DCP_OK and rep.steps == nsteps
    T_run = ctx.get_state(dcp.T_SOLUTION)
    assert np.array_equal(ctx.get_state(dcp.NSE_SOLUTION), x0)
    assert _calls(ctx, "   Assemble NSE system") == nsteps
    ctx.close()
    orc = oracle_py.FeecModel(dcp.physics_from_params(rp), m)
    T = m.T0.copy()
    for n in range(nsteps):
        orc.assemble_nse_system(x0, T)
        orc.assemble_temperature(T, x0)
        rcT, T, itT = orc.solve_temperature(T)
        assert rcT == 0 and abs(itT - steps[n].T_cg) <= 1
    assert np.linalg.norm(T_run - T) <= 1e-10 * np.linalg.norm(T)
    cs = m.T_constraints
    for l, d in enumerate(cs.line_dof):
        b, e = cs.entry_ptr[l], cs.entry_ptr[l + 1]
        if e - b == 1 and cs.entry_w[b] == 1.0:
            assert T_run[d] == T_run[cs.entry_dof[b]]


@pytest.mark.gpu
def test_executable_runs_the_cube_prm():
    exe = os.path.join(ROOT, "3d-dycoreplanet_amd", "dcp_aquaplanet")
    out = subprocess.run([exe, "-p", CUBE_PRM, "--refine", "2", "--max-steps", "3"],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.count("Time step ") == 3
