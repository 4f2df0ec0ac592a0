"""The two-dimensional model, Standard::BoussinesqModel<2>
(boussinesq_model.inst.cc:8; data/aqua_planet_test_2d.prm, BASELINE config C1):
host mesh / DoFs / constraints (dcp_host_mesh2d_create), the upload's host
validation (dcp_mesh2d_check) and the oracle's 2D element and model level
(oracle/oracle.cpp, orc2d_*), on the CPU.

Parity of the 2D restatement with deal.II itself is unpinned (deal.II is not in
this image and the reference holds no 2D output); the element-level checks
below are known answers of the weak forms (areas, divergence of constants, the
sign of the 2D Coriolis term Q3) that do not depend on the oracle's code."""
import math

import numpy as np
import pytest
import scipy.sparse as sp

import dcp
import oracle_py

R0, R1, L = 1.0, 3.0, 0.1   # data/aqua_planet_test_2d.prm: R0 = 1, atm height 2, length 0.1


def physics_2d(**kw):
    rp = dcp.load_prm("configs/aqua_planet_test_2d.prm")
    ph = dcp.physics_from_params(rp)
    for k, v in kw.items():
        setattr(ph, k, v)
    return ph


@pytest.mark.parametrize("refine", [0, 1, 2, 3])
def test_mesh_counts(refine):
    m = dcp.HostMesh2D(refine=refine, R0=R0, R1=R1, length=L, temperature_degree=2)
    nc = 12 * 4 ** refine
    ring = 12 * 2 ** refine            # cells around, vertices per circle
    layers = 2 ** refine               # cells across the shell
    n_vert = ring * (layers + 1)
    n_nodes = (2 * ring) * (2 * layers + 1)   # Q2 support points
    assert m.n_cells == nc
    assert m.n_p == n_vert
    assert m.n_vnodes == n_nodes and m.n_u == 2 * n_nodes
    assert m.n_T == n_nodes
    # no-slip: both components of the 2 ring inner-circle points; no-normal-flux: one
    assert len(m.nse_constraints.line_dof) == 2 * (2 * ring) + 2 * ring
    assert len(m.T_constraints.line_dof) == 2 * ring
    assert m.check() <= 8
    q1 = dcp.HostMesh2D(refine=refine, R0=R0, R1=R1, length=L, temperature_degree=1)
    assert q1.n_T == n_vert and q1.cell_T_dofs.shape == (nc, 4)
    assert len(q1.T_constraints.line_dof) == ring


def test_geometry_and_boundaries():
    m = dcp.HostMesh2D(refine=2, R0=R0, R1=R1, length=L)
    r = np.linalg.norm(m.node_xy, axis=1)
    # support points are MappingQ(3) images: on the cubic arc, not the circle
    assert r.min() == pytest.approx(R0 / L, rel=1e-5)
    assert r.max() == pytest.approx(R1 / L, rel=1e-5)
    # the inner-circle dofs are exactly the no-slip lines (both components, no entries)
    nc = m.nse_constraints
    lines = dict(zip(nc.line_dof.tolist(), range(len(nc.line_dof))))
    inner = np.where(np.abs(r - R0 / L) < 1e-3)[0]
    outer = np.where(np.abs(r - R1 / L) < 1e-3)[0]
    assert len(inner) == len(outer) == 2 * 12 * 4
    for n in inner:
        for c in range(2):
            l = lines[2 * n + c]
            assert nc.entry_ptr[l + 1] == nc.entry_ptr[l]
    # no-normal-flux: u_k = w u_other with w = -n_other / n_k (mapping normal ~ radial)
    for n in outer:
        k = [c for c in range(2) if 2 * n + c in lines]
        assert len(k) == 1
        l = lines[2 * n + k[0]]
        assert nc.entry_ptr[l + 1] - nc.entry_ptr[l] <= 1
        if nc.entry_ptr[l + 1] > nc.entry_ptr[l]:
            e = nc.entry_ptr[l]
            assert nc.entry_dof[e] == 2 * n + 1 - k[0]
            x = m.node_xy[n] / np.linalg.norm(m.node_xy[n])
            assert nc.entry_w[e] == pytest.approx(-x[1 - k[0]] / x[k[0]], abs=1e-3)
    # the cubic support points of boundary cells lie on the circles
    g = m.cell_geometry
    rr = np.linalg.norm(g, axis=2)
    on_inner = np.abs(rr[:, 12:16] - R0 / L).max(axis=1)
    on_outer = np.abs(rr[:, 0:4] - R1 / L).max(axis=1)
    assert np.sum(on_inner < 1e-12) == 12 * 4 and np.sum(on_outer < 1e-12) == 12 * 4


def test_initial_temperature_and_dirichlet_values():
    m = dcp.HostMesh2D(refine=3, R0=R0, R1=R1, length=L, temperature_degree=2)
    tc = m.T_constraints
    # the Dirichlet values are the initial temperature at those dofs
    assert np.allclose(m.T0[tc.line_dof], tc.inhomogeneity, rtol=0, atol=1e-15)
    # TemperatureInitialValues<2>: two Gaussians of height sqrt(det C)/(2 pi),
    # C = 20/((R1-R0)/2) (scaled radii), centres rotated by 2 alpha = 2 pi/3
    cov = 20.0 / ((R1 - R0) / L / 2.0)
    peak = cov / (2 * math.pi)
    assert m.T0.max() <= peak * (1 + 1e-12)
    assert m.T0.max() > 0.5 * peak
    a = 2 * math.pi / 3
    c1 = (R0 + (R1 - R0) * 0.35) / L * np.array([math.cos(a), math.sin(a)])
    hottest = m.node_xy[np.argmax(m.T0)]
    c2 = (R0 + (R1 - R0) * 0.65) / L * np.array([-math.sin(a), math.cos(a)])
    assert min(np.linalg.norm(hottest - c1), np.linalg.norm(hottest - c2)) < 1.0


def test_cuthill_mckee_2d_is_a_consistent_renumbering():
    a = dcp.HostMesh2D(refine=2, R0=R0, R1=R1, length=L)
    b = dcp.HostMesh2D(refine=2, R0=R0, R1=R1, length=L, cuthill_mckee=True)
    assert np.array_equal(np.sort(np.unique(b.cell_nse_dofs)), np.arange(b.n_u + b.n_p))
    # the permutation maps a's cell dofs onto b's, component-preserving and node-major
    perm = np.full(a.n_u + a.n_p, -1)
    perm[a.cell_nse_dofs.ravel()] = b.cell_nse_dofs.ravel()
    assert np.array_equal(np.sort(perm), np.arange(a.n_u + a.n_p))
    vel = np.arange(a.n_u)
    assert np.array_equal(perm[vel] % 2, vel % 2)
    assert np.array_equal(perm[vel[0::2]] + 1, perm[vel[1::2]])
    assert np.all(perm[a.n_u:] >= a.n_u)
    # the support points follow the renumbering
    assert np.allclose(b.node_xy[perm[vel[0::2]] // 2], a.node_xy)
    # constraints follow too
    assert set(perm[a.nse_constraints.line_dof].tolist()) == set(b.nse_constraints.line_dof.tolist())
    # and the bandwidth of the velocity-node graph shrinks
    def bandwidth(m):
        nodes = m.cell_nse_dofs[:, [0, 3, 6, 9, 12, 14, 16, 18, 20]] // 2
        return max(int(r.max() - r.min()) for r in nodes)
    assert bandwidth(b) < bandwidth(a)


def test_check_rejects_non_local_constraints():
    m = dcp.HostMesh2D(refine=1, R0=R0, R1=R1, length=L)
    nc = m.nse_constraints
    # a line whose entry points at a far-away dof is not node-local
    k = int(np.argmax(np.diff(nc.entry_ptr) == 1))
    bad = dcp.ConstraintSet(nc.line_dof, nc.entry_ptr, nc.entry_dof.copy(), nc.entry_w,
                            nc.inhomogeneity)
    bad.entry_dof[nc.entry_ptr[k]] = (int(nc.entry_dof[nc.entry_ptr[k]]) + m.n_u // 2) % m.n_u
    with pytest.raises(dcp.DcpError) as e:
        m.check(nse_constraints=bad)
    assert e.value.code in (dcp.DCP_ERR_UNSUPPORTED, dcp.DCP_ERR_INVALID)
    # inhomogeneous NSE constraints are not supported
    inh = dcp.ConstraintSet(nc.line_dof, nc.entry_ptr, nc.entry_dof, nc.entry_w,
                            nc.inhomogeneity + 1.0)
    with pytest.raises(dcp.DcpError):
        m.check(nse_constraints=inh)


# ---------------------------------------------------------------------------
# oracle, element level: known answers of the weak forms


def cell_area(g16):
    """Integral of 1 over the MappingQ(3) cell: Gauss 6x6 on the cubic map."""
    x, w = np.polynomial.legendre.leggauss(6)
    x, w = (x + 1) / 2, w / 2
    gl = np.array([0.0, 0.27639320225002103036, 0.72360679774997896964, 1.0])

    def lag(i, t):
        v = 1.0
        for j in range(4):
            if j != i:
                v *= (t - gl[j]) / (gl[i] - gl[j])
        return v

    def dlag(i, t, h=1e-6):
        return (lag(i, t + h) - lag(i, t - h)) / (2 * h)

    area = 0.0
    for a, wa in zip(x, w):
        for b, wb in zip(x, w):
            J = np.zeros((2, 2))
            for t in range(16):
                i, j = t % 4, t // 4
                J[:, 0] += g16[t] * dlag(i, a) * lag(j, b)
                J[:, 1] += g16[t] * lag(i, a) * dlag(j, b)
            area += wa * wb * np.linalg.det(J)
    return area


def test_element_known_answers():
    m = dcp.HostMesh2D(refine=1, R0=R0, R1=R1, length=L, temperature_degree=2)
    ph = physics_2d(time_step=1.0, gravity_constant=0.0)
    vel = [i for i in range(22) if (i < 12 and i % 3 != 2) or i >= 12]
    comp = np.array([i % 3 if i < 12 else (i - 12) % 2 for i in range(22)])
    pres = [2, 5, 8, 11]
    for c in (0, 5, 17, 40):
        g = m.cell_geometry[c]
        area = cell_area(g)
        # u = (1, 0) everywhere: advection 0, f_i = int phi_i . (u + 2 cross_2d(u)),
        # cross_2d(u) = (u_y, -u_x) = (0, -1)  ->  sum f_x = area, sum f_y = -2 area
        u = np.zeros(22)
        u[[i for i in vel if comp[i] == 0]] = 1.0
        T = np.full(9, ph.temperature_ref)
        K, f = oracle_py.cell_nse_system_2d(ph, g, u, T)
        fx = sum(f[i] for i in vel if comp[i] == 0)
        fy = sum(f[i] for i in vel if comp[i] == 1)
        assert fx == pytest.approx(area, rel=1e-9)
        assert fy == pytest.approx(-2 * area, rel=1e-9)
        # velocity mass of one component sums to the area; divergence of a constant is 0
        Kv = K[np.ix_(vel, vel)]
        assert np.allclose(Kv, Kv.T, rtol=0, atol=1e-12 * np.abs(Kv).max())
        Bt = K[np.ix_(pres, vel)]
        assert np.allclose(Bt @ np.array([1.0 if comp[i] == 0 else 0.0 for i in vel]), 0, atol=1e-12)
        assert np.allclose(K[np.ix_(vel, pres)], Bt.T, rtol=0, atol=0)
        assert np.all(K[np.ix_(pres, pres)] == 0)
        # temperature: mass sums to the area, stiffness annihilates constants
        M, S = oracle_py.cell_temperature_matrix_2d(ph, g)
        assert M.sum() == pytest.approx(area, rel=1e-9)
        assert np.allclose(S @ np.ones(9), 0, atol=1e-12 * np.abs(S).max())


def test_oracle_2d_schur_solve_converges():
    m = dcp.HostMesh2D(refine=2, R0=R0, R1=R1, length=L, temperature_degree=2, cuthill_mckee=True)
    ph = physics_2d()
    o = oracle_py.Model(ph, m)
    u0 = np.zeros(m.n_u + m.n_p)
    o.assemble_nse_system(u0, m.T0)
    rc, x, its, n_inv = o.solve_nse_schur(u0)
    assert rc == 0 and its > 0 and n_inv == its + 3  # rhs, A x0, one per step, u
    n = m.n_u + m.n_p
    A = sp.csr_matrix((o.nse_matrix_csr()[2], o.nse_matrix_csr()[1], o.nse_matrix_csr()[0]),
                      shape=(n, n))
    b = o.nse_rhs()
    # the pressure is solved as dt p and rescaled: [A B^T; B 0] [u; dt p] = rhs
    y = x.copy()
    y[m.n_u:] *= ph.time_step
    r = A @ y - b
    r[m.nse_constraints.line_dof] = 0.0   # constrained rows hold the diagonal only
    # the inner solves stop at 1e-6 relative (InverseMatrix, the Schur GMRES)
    assert np.linalg.norm(r) / np.linalg.norm(b) < 1e-4
    # constraints hold: no-slip rows are zero, no-normal-flux rows follow their entry
    nc = m.nse_constraints
    for l, d in enumerate(nc.line_dof):
        v = sum(nc.entry_w[k] * x[nc.entry_dof[k]] for k in range(nc.entry_ptr[l], nc.entry_ptr[l + 1]))
        assert x[d] == pytest.approx(v, abs=1e-14)
    # the block-preconditioned path (solve_NSE_block_preconditioned) on this
    # configuration: its inner GMRES on S = B D_A^-1 B^T (identity
    # preconditioner, 1e-6 |src_p|) stalls on the near-null constant-pressure
    # mode (cf. tests/test_schur_pin.py for 3D r >= 4); with a small cap both
    # FGMRES attempts end in NoConvergence, as the reference's would
    assert o.solve_nse(u0)[0] == -4   # the preconditioner has not been built
    o.build_nse_preconditioner()
    o.set_inner_max_steps(200)
    rc2, _, outer, inner = o.solve_nse(u0)
    assert rc2 == 1 and outer == 0 and inner >= 2 * 200


def test_oracle_2d_temperature_step():
    m = dcp.HostMesh2D(refine=2, R0=R0, R1=R1, length=L, temperature_degree=2)
    ph = physics_2d()
    o = oracle_py.Model(ph, m)
    u0 = np.zeros(m.n_u + m.n_p)
    o.assemble_temperature_matrix()
    o.assemble_temperature_rhs(m.T0, u0)
    rc, T, its = o.solve_temperature(m.T0)
    assert rc == 0 and its > 0
    # at rest, one implicit diffusion step: Dirichlet values kept, maximum principle-ish
    tc = m.T_constraints
    assert np.allclose(T[tc.line_dof], tc.inhomogeneity, atol=1e-14)
    assert T.max() <= m.T0.max() * (1 + 1e-6)
    assert abs(T - m.T0).max() > 0
