"""Known-answer tests pinning the CPU oracle's finite-element arithmetic.

The reference ships no golden vectors (test/test_dummy.cc only prints), so the
oracle (oracle/oracle.cpp, a restatement of boussinesq_model.tpp) is pinned by
closed-form element matrices on an affine cell, by structural identities and
by solver-tolerance properties. All element integrals below are exact under
QGauss(3) (degree <= 5 polynomials on an affine cell)."""
import numpy as np
import pytest

import dcp
import oracle_py

h = 0.5
M1 = h / 30 * np.array([[4, 2, -1], [2, 16, 2], [-1, 2, 4]])      # 1D Q2 mass
K1 = 1 / (3 * h) * np.array([[7, -8, 1], [-8, 16, -8], [1, -8, 7]])  # 1D Q2 stiffness
I1 = h / 6 * np.array([1, 4, 1])                                  # 1D Q2 integrals
# 1D mixed: int L1_v(x) dL2_a/dx dx on [0,h] (Q1 value x Q2 derivative)
X1 = np.array([[-5 / 6, 2 / 3, 1 / 6], [-1 / 6, -2 / 3, 5 / 6]])
# 1D Q1-Q2 value products (pressure shape x velocity shape), on [0,h]
V1 = h * np.array([[1 / 6, 1 / 3, 0], [0, 1 / 3, 1 / 6]])
HIER2LEX = [0, 2, 6, 8, 18, 20, 24, 26, 3, 5, 1, 7, 21, 23, 19, 25, 9, 11, 15, 17, 12, 14, 10, 16,
            4, 22, 13]


def kron3(a, b, c):
    # lexicographic (x fastest): index = i + 3j + 9k -> kron(z, y, x)
    return np.kron(c, np.kron(b, a))


GL = np.array([0.0, 0.5 - 0.5 / np.sqrt(5.0), 0.5 + 0.5 / np.sqrt(5.0), 1.0])


def cube_geom(h):
    """MappingQ(3) support points of the affine cube [0,h]^3 (64, lexicographic
    over the Gauss-Lobatto points)."""
    g = np.zeros((64, 3))
    for n in range(64):
        g[n] = [h * GL[n % 4], h * GL[(n // 4) % 4], h * GL[n // 16]]
    return g


def cube_nodes(h):
    """The 27 Q2 support points of the same cube (lexicographic)."""
    g = np.zeros((27, 3))
    for n in range(27):
        g[n] = [h * (n % 3) / 2, h * ((n // 3) % 3) / 2, h * (n // 9) / 2]
    return g


def sysdof(i):
    if i < 32:
        return (i % 4, i // 4 if i % 4 == 3 else HIER2LEX[i // 4])
    return ((i - 32) % 3, HIER2LEX[8 + (i - 32) // 3])


def velocity_block(K):
    """Reorder the 81x81 velocity block of an FESystem matrix into [comp][lex]."""
    idx = np.zeros((3, 27), int)
    for i in range(89):
        c, l = sysdof(i)
        if c < 3:
            idx[c, l] = i
    return K[np.ix_(idx.ravel(), idx.ravel())], idx


def test_mass_block_closed_form(classic):
    ph = dcp.classic_physics(time_step=0.0)
    K, f = oracle_py.cell_nse_system(ph, cube_geom(h), np.zeros(89), np.full(8, 2.0))
    A, _ = velocity_block(K)
    M3 = kron3(M1, M1, M1)
    for c in range(3):
        assert np.allclose(A[27 * c:27 * c + 27, 27 * c:27 * c + 27], M3, rtol=1e-13, atol=1e-16)
    assert np.allclose(A[0:27, 27:54], 0)


def test_viscous_block_closed_form():
    dt = 0.1
    ph = dcp.classic_physics(time_step=dt)
    K, _ = oracle_py.cell_nse_system(ph, cube_geom(h), np.zeros(89), np.full(8, 2.0))
    A, _ = velocity_block(K)
    nu = dt / 100.0
    M3 = kron3(M1, M1, M1)
    L3 = kron3(K1, M1, M1) + kron3(M1, K1, M1) + kron3(M1, M1, K1)
    # 2/Re eps:eps = 1/Re (grad.grad delta_cc' + d_c' s_a d_c s_b)
    # coupling block (c, c'): sum_q w d_c' s_a d_c s_b, from 1D factors with
    # Cx[a][b] = int L_a L_b' (scale free)
    Cx = np.array([[-1 / 2, 2 / 3, -1 / 6], [-2 / 3, 0, 2 / 3], [1 / 6, -2 / 3, 1 / 2]])
    ops = {}
    for c in range(3):
        for cp in range(3):
            f = [M1, M1, M1]
            if c == cp:
                f[c] = K1
            else:
                f[cp] = Cx.T        # d/dx_c' on a (row), value on b
                f[c] = Cx           # value on a, d/dx_c on b
            ops[(c, cp)] = kron3(*f)
    for c in range(3):
        for cp in range(3):
            expect = nu * ops[(c, cp)] + (M3 + nu * L3 if c == cp else 0)
            got = A[27 * c:27 * c + 27, 27 * cp:27 * cp + 27]
            assert np.allclose(got, expect, rtol=1e-12, atol=1e-15), (c, cp)


def test_divergence_block_closed_form():
    ph = dcp.classic_physics()
    K, _ = oracle_py.cell_nse_system(ph, cube_geom(h), np.zeros(89), np.full(8, 2.0))
    _, idx = velocity_block(K)
    pidx = [4 * v + 3 for v in range(8)]
    for c in range(3):
        Bt = K[np.ix_(idx[c], pidx)]           # -div phi_u * phi_p, rows velocity
        fac = [V1.T, V1.T, V1.T]
        fac[c] = X1.T                          # derivative on the velocity factor
        expect = -np.kron(fac[2], np.kron(fac[1], fac[0]))
        assert np.allclose(Bt, expect, rtol=1e-12, atol=1e-15)
        assert np.allclose(K[np.ix_(pidx, idx[c])], Bt.T, rtol=0, atol=0)
    assert np.all(K[np.ix_(pidx, pidx)] == 0)


def test_rhs_gravity_cuboid():
    ph = dcp.classic_physics(time_step=0.3)
    ph.cuboid = 1
    ph.gravity_constant = 2.0
    K, f = oracle_py.cell_nse_system(ph, cube_geom(h), np.zeros(89), np.full(8, ph.temperature_ref))
    _, idx = velocity_block(K)
    # u0 = 0, rho = 1: f_(a,z) = -dt * g * int s_a ; x,y components 0
    assert np.allclose(f[idx[2]], -0.3 * 2.0 * kron3(I1, I1, I1), rtol=1e-13)
    assert np.allclose(f[idx[0]], 0) and np.allclose(f[idx[1]], 0)


def test_rhs_advection_and_coriolis_linear_field():
    # u0 = (y, 0, 0) on the cuboid: (u.grad)u = 0; Coriolis 2 Omega x u = (0, 2 w y, 0)
    ph = dcp.classic_physics(time_step=0.2)
    ph.cuboid = 1
    ph.omega = 1.5
    g = cube_nodes(h)
    u = np.zeros(89)
    for i in range(89):
        c, l = sysdof(i)
        if c == 0:
            u[i] = g[l, 1]
    K, f = oracle_py.cell_nse_system(ph, cube_geom(h), u, np.full(8, ph.temperature_ref))
    _, idx = velocity_block(K)
    M3 = kron3(M1, M1, M1)
    yv = g[:, 1]
    assert np.allclose(f[idx[0]], M3 @ yv, rtol=1e-12)                       # mass * u0
    assert np.allclose(f[idx[1]], -0.2 * 2 * 1.5 * (M3 @ yv), rtol=1e-12)    # -dt 2 (Omega x u)
    # z: gravity only
    assert np.allclose(f[idx[2]], -0.2 * 1.0 * kron3(I1, I1, I1), rtol=1e-12)


def test_shell_totals():
    m = dcp.HostMesh(refine=2)
    ph = dcp.classic_physics()
    o = oracle_py.Model(ph, m)
    o.build_nse_preconditioner()
    _, Mp = o.precond_diagonals()
    # pressure mass diagonal sums to the integral of the squared Q1 shapes;
    # sum over all 89x89 local pressure mass entries = volume. Check via T mass:
    o.assemble_temperature_matrix()
    vol = 4 / 3 * np.pi * (27 - 1)
    rp, cols, vals = o.T_matrix_csr()
    assert Mp.sum() > 0 and np.isfinite(vals).all()


def test_solver_tolerances_honoured():
    m = dcp.HostMesh(refine=1)
    ph = dcp.classic_physics()
    o = oracle_py.Model(ph, m)
    u = np.zeros(m.n_u + m.n_p)
    T = m.T0.copy()
    o.assemble_nse_system(u, T)
    o.build_nse_preconditioner()
    rc, x, outer, inner = o.solve_nse(u)
    assert rc == 0 and outer > 0 and inner > 0
    rhs = o.nse_rhs()
    xs = x.copy()
    xs[m.n_u:] *= ph.time_step    # system is in the dt-scaled pressure
    res = o.nse_vmult(xs) - rhs
    # constrained rows carry only the diagonal; compare on free rows
    free = np.ones(m.n_u + m.n_p, bool)
    free[m.nse_constraints.line_dof] = False
    assert np.linalg.norm(res[free]) <= 1.01e-8 * np.linalg.norm(rhs)
    o.assemble_temperature_matrix()
    o.assemble_temperature_rhs(T, x)
    rc, Tn, it = o.solve_temperature(T)
    assert rc == 0 and it > 0
    # Dirichlet values restored by distribute()
    tc = m.T_constraints
    assert np.allclose(Tn[tc.line_dof], tc.inhomogeneity)


def _schur_parts(r, normals, all_cells=True):
    import scipy.sparse as sp
    m = dcp.HostMesh(refine=r, normals=normals, mapping_q_on_all_cells=all_cells)
    ph = dcp.classic_physics()
    o = oracle_py.Model(ph, m)
    o.assemble_nse_system(np.zeros(m.n_u + m.n_p), m.T0)
    o.build_nse_preconditioner()
    n = m.n_u + m.n_p
    rp, c, v = o.nse_matrix_csr()
    A = sp.csr_matrix((v, c, rp), shape=(n, n))
    Ad, _ = o.precond_diagonals()
    return m, o, A[m.n_u:, :m.n_u], A[:m.n_u, m.n_u:], Ad


def test_constant_pressure_mode_is_near_null():
    """DESIGN.md 'no-normal-flux normals': under MappingQ(3) and QGauss(3) the
    divergence block no longer integrates grad(phi_i) exactly (the cofactor of
    a cubic map times grad phi exceeds degree 5 per direction), so B^T 1 does
    not vanish on interior rows and the constant pressure is a near-null, not a
    null, vector of S whatever the boundary normals: O(1e-6) at r = 2 with the
    cubic map on every cell, O(1e-2) on the interface layer with deal.II 9.2's
    MappingQ (cubic boundary cells against trilinear interior cells)."""
    m, o, B, Bt, Ad = _schur_parts(2, "consistent")
    v = np.abs(Bt @ np.ones(m.n_p))
    assert 1e-8 < v.max() < 1e-5
    m, o, B, Bt, Ad = _schur_parts(2, "consistent", all_cells=False)
    assert np.abs(Bt @ np.ones(m.n_p)).max() > 1e-3
    m, o, B, Bt, Ad = _schur_parts(2, "radial")
    S = (B @ (Bt.multiply(1 / Ad[:, None]))).toarray()
    w = np.linalg.eigvalsh(0.5 * (S + S.T))
    assert w[0] < 1e-3 * w[1]
    one = np.ones(m.n_p) / np.sqrt(m.n_p)
    assert np.isclose(one @ S @ one, w[0], rtol=0.1)


def test_shell_solve_converges_r2():
    """r = 2 with the reference's geometry (MappingQ(3), deal.II 9.2) and
    no-normal-flux normals: 27 FGMRES iterations, ~1900 inner."""
    m = dcp.HostMesh(refine=2)
    o = oracle_py.Model(dcp.classic_physics(), m)
    u = np.zeros(m.n_u + m.n_p)
    o.assemble_nse_system(u, m.T0)
    o.build_nse_preconditioner()
    rc, x, outer, inner = o.solve_nse(u)
    assert rc == 0 and outer < 40 and inner < 2000


@pytest.mark.parametrize("cuboid", [False, True])
def test_structural_zero_loops_are_the_literal_loops(cuboid):
    """orc_cell_nse_system / orc_cell_nse_preconditioner skip the FESystem's
    structural zeros and sum every other term in the order of the literal
    89 x 89 loops of boussinesq_model.tpp:626-637 / :421-464: every entry must
    be bitwise the literal one (numpy equality, so +0 == -0), on every cell of
    a mesh, with a random state."""
    m = dcp.HostMesh(cuboid=cuboid, refine=1 if cuboid else 2)
    ph = dcp.classic_physics()
    ph.cuboid = int(cuboid)
    rng = np.random.default_rng(7)
    u = rng.uniform(-1, 1, m.n_u + m.n_p)
    T = rng.uniform(-1, 1, m.n_T)
    for c in range(m.n_cells):
        g, ul, Tl = m.cell_geometry[c], u[m.cell_nse_dofs[c]], T[m.cell_T_dofs[c]]
        K, f = oracle_py.cell_nse_system(ph, g, ul, Tl)
        Kl, fl = oracle_py.cell_nse_system_literal(ph, g, ul, Tl)
        assert np.array_equal(K, Kl) and np.array_equal(f, fl), c
        assert np.array_equal(oracle_py.cell_nse_preconditioner(ph, g),
                              oracle_py.cell_nse_preconditioner_literal(ph, g)), c


def test_threaded_assembly_is_the_serial_assembly():
    """The oracle's cell loops on several threads (element work in parallel, the
    copier by row ranges in cell order) give bitwise the serial cell-order
    copier's matrix, rhs, preconditioner diagonals and temperature system."""
    m = dcp.HostMesh(refine=2)
    ph = dcp.classic_physics()
    rng = np.random.default_rng(11)
    u = rng.uniform(-1, 1, m.n_u + m.n_p)
    T = m.T0 + 0.1 * rng.uniform(-1, 1, m.n_T)
    out = []
    try:
        for th in (1, 4):
            oracle_py.set_threads(th)
            orc = oracle_py.Model(ph, m)
            orc.assemble_nse_system(u, T)
            orc.build_nse_preconditioner()
            orc.assemble_temperature_matrix()
            orc.assemble_temperature_rhs(T, u)
            out.append([*orc.nse_matrix_csr(), orc.nse_rhs(), *orc.precond_diagonals(),
                        *orc.T_matrix_csr(), orc.T_rhs(), orc.nse_vmult(u),
                        orc.schur_vmult(u[m.n_u:])])
    finally:
        oracle_py.set_threads(1)
    for a, b in zip(*out):
        assert np.array_equal(a, b)
    # the block accessor is the slice of the full CSR
    import scipy.sparse as sp
    n = m.n_u + m.n_p
    A = sp.csr_matrix((out[0][2], out[0][1], out[0][0]), shape=(n, n))
    orc = oracle_py.Model(ph, m)
    orc.assemble_nse_system(u, T)
    for key, blk in (("Bt", A[:m.n_u, m.n_u:]), ("B", A[m.n_u:, :m.n_u]), ("A", A[:m.n_u, :m.n_u])):
        rp, cols, vals = orc.nse_block_csr(key)
        S = sp.csr_matrix((vals, cols, rp), shape=blk.shape)
        assert (S != blk).nnz == 0, key
