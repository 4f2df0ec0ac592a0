#!/usr/bin/env python3
"""Generates the regression fixtures in tests/golden/ from the CPU oracle.

These vectors are oracle outputs (parity with deal.II is unpinned: the
reference cannot be built in this image and ships no golden data, see
DESIGN.md section 3). They freeze the restatement so that any change to the
oracle or to the host mesh/DoF setup shows up as a diff, and give the GPU
tests a fixed target that does not need the oracle at run time.

Cases (classic shell physics, data/aqua_planet_shell_test_3d-classic.prm):
  shell_r1.npz       refine 1 (48 cells): cell 0..3 element matrices/rhs for the
                     physical state (u=0, T0) and a seeded random state, the
                     assembled nse rhs, preconditioner diagonals, one full time
                     step's NSE solution / iteration counts, temperature solution.
  shell_r3_step.npz  refine 3 (3,072 cells, 81,912 NSE dofs): one full time step
                     from the physical state (about 15 min of oracle time: ~29,000
                     inner Schur GMRES iterations): iteration counts, the NSE and
                     temperature solutions, the assembled rhs.
  shell_r4_step.npz  BASELINE config 3 (classic prm, refine 4: 24,576 cells, 634,600
                     NSE dofs): one full time step. On the reference geometry the
                     reference's inner Schur GMRES stagnates at its 5000-iteration
                     cap in both FGMRES attempts (NoConvergence): the
                     fixture holds the assembled rhs, the iteration counts of that
                     failure and the temperature step.
  feec_r4_step.npz   BASELINE config 4: data/aqua_planet_shell_test_3d-feec.prm at
                     refine 4 (24,576 cells; Nedelec/RT/DGQ0 + Q1 temperature),
                     one full FEEC time step from u = 0 and the initial temperature:
                     assembled rhs, GMRES(100) iterations and solution, temperature
                     solution (FeecModel, boussineq_model_FEEC.tpp:2238-2300).
usage: python tests/golden/make_golden.py [r1|r3|r4|feec4]
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (os.path.join(ROOT, "3d-dycoreplanet_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import dcp  # noqa: E402  (host mesh/prm helpers only: no device calls)
import oracle_py  # noqa: E402

SEED = 20261015


def states(m):
    rng = np.random.default_rng(SEED)
    u_r = rng.uniform(-1, 1, m.n_u + m.n_p)
    T_r = m.T0 + 0.1 * rng.uniform(-1, 1, m.n_T)
    return {"physical": (np.zeros(m.n_u + m.n_p), m.T0.copy()), "random": (u_r, T_r)}


def make(refine=1):
    m = dcp.HostMesh(refine=refine)
    ph = dcp.classic_physics()
    out = {"n": np.array([m.n_cells, m.n_u, m.n_p, m.n_T], np.int64),
           "cell_nse_dofs": m.cell_nse_dofs.astype(np.int32),
           "cell_T_dofs": m.cell_T_dofs.astype(np.int32),
           "cell_geometry": m.cell_geometry.copy()}
    for name, (u, T) in states(m).items():
        K = np.zeros((4, 89, 89))
        f = np.zeros((4, 89))
        for c in range(4):
            K[c], f[c] = oracle_py.cell_nse_system(ph, m.cell_geometry[c], u[m.cell_nse_dofs[c]],
                                                   T[m.cell_T_dofs[c]])
        out[f"{name}_K"], out[f"{name}_f"] = K, f
        orc = oracle_py.Model(ph, m)
        orc.assemble_nse_system(u, T)
        out[f"{name}_rhs"] = orc.nse_rhs()
        out[f"{name}_u"], out[f"{name}_T"] = u, T
    # one full time step from the physical state (run(), boussinesq_model.tpp:1867-1905)
    u, T = states(m)["physical"]
    orc = oracle_py.Model(ph, m)
    orc.assemble_nse_system(u, T)
    orc.build_nse_preconditioner()
    orc.assemble_temperature_matrix()
    orc.assemble_temperature_rhs(T, u)
    a_diag, p_diag = orc.precond_diagonals()
    rc, x, outer, inner = orc.solve_nse(u)
    rcT, Tn, itT = orc.solve_temperature(T)
    out.update(A_diag=a_diag, Mp_diag=p_diag, T_rhs=orc.T_rhs(), nse_solution=x,
               T_solution=Tn, iters=np.array([rc, outer, inner, rcT, itT], np.int64))
    return out


def make_step(refine):
    m = dcp.HostMesh(refine=refine)
    ph = dcp.classic_physics()
    u, T = states(m)["physical"]
    orc = oracle_py.Model(ph, m)
    orc.assemble_nse_system(u, T)
    rhs = orc.nse_rhs()
    orc.build_nse_preconditioner()
    orc.assemble_temperature_matrix()
    orc.assemble_temperature_rhs(T, u)
    rc, x, outer, inner = orc.solve_nse(u)
    rcT, Tn, itT = orc.solve_temperature(T)
    return {"n": np.array([m.n_cells, m.n_u, m.n_p, m.n_T], np.int64), "nse_rhs": rhs,
            "T_rhs": orc.T_rhs(), "nse_solution": x, "T_solution": Tn,
            "iters": np.array([rc, outer, inner, rcT, itT], np.int64)}


def make_feec_step(refine=4):
    rp = dcp.load_prm(os.path.join(ROOT, "configs", "aqua_planet_shell_test_3d-feec.prm"))
    ph = dcp.physics_from_params(rp)
    m = dcp.HostMesh(cuboid=False, refine=refine, R0=rp.R0, R1=rp.R1, length=rp.length,
                     temperature_degree=ph.temperature_degree, feec=True)
    f = m.feec
    x0, T0 = np.zeros(f.n), m.T0.copy()
    orc = oracle_py.FeecModel(ph, m, zero_mean=bool(rp.correct_pressure_to_zero_mean))
    orc.assemble_nse_system(x0, T0)
    rhs = orc.rhs()
    orc.assemble_preconditioner()
    orc.assemble_temperature(T0, x0)
    T_rhs = orc.T_rhs()
    rc, x, it = orc.solve_nse(x0)
    rcT, Tn, itT = orc.solve_temperature(T0)
    vs = orc.velocity_stats(x)
    return {"n": np.array([f.n_cells, f.n_w, f.n_u, f.n_p, m.n_T], np.int64), "nse_rhs": rhs,
            "T_rhs": T_rhs, "nse_solution": x, "T_solution": Tn,
            "velocity_stats": np.asarray(vs, np.float64),
            "iters": np.array([rc, it, rcT, itT], np.int64)}


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "r1"
    if which == "r1":
        np.savez_compressed(os.path.join(HERE, "shell_r1.npz"), **make(1))
        print("wrote", os.path.join(HERE, "shell_r1.npz"))
    elif which == "feec4":
        np.savez_compressed(os.path.join(HERE, "feec_r4_step.npz"), **make_feec_step(4))
        print("wrote", os.path.join(HERE, "feec_r4_step.npz"))
    elif which == "r4":
        np.savez_compressed(os.path.join(HERE, "shell_r4_step.npz"), **make_step(4))
        print("wrote", os.path.join(HERE, "shell_r4_step.npz"))
    elif which == "r3":
        np.savez_compressed(os.path.join(HERE, "shell_r3_step.npz"), **make_step(3))
        print("wrote", os.path.join(HERE, "shell_r3_step.npz"))
