"""ORACLE — TEST INFRASTRUCTURE ONLY. ctypes binding of oracle/build/liboracle.so,
the CPU restatement of the reference hot path (see oracle.h). Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
Parity status vs deal.II: unpinned (see oracle.h)."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")


class OrcPhysics(C.Structure):
    _fields_ = [
        ("time_step", C.c_double), ("one_over_reynolds", C.c_double),
        ("one_over_peclet", C.c_double), ("expansion_coefficient", C.c_double),
        ("temperature_ref", C.c_double), ("gravity_scale", C.c_double),
        ("gravity_constant", C.c_double), ("coriolis_scale", C.c_double),
        ("omega", C.c_double), ("cuboid", C.c_int), ("nse_solver_interval", C.c_int),
        ("temperature_degree", C.c_int),
    ]


class OrcConstraints(C.Structure):
    _fields_ = [
        ("n_lines", C.c_int), ("line_dof", C.c_void_p), ("entry_ptr", C.c_void_p),
        ("entry_dof", C.c_void_p), ("entry_w", C.c_void_p), ("inhomogeneity", C.c_void_p),
    ]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} missing: run `make -C oracle`")
        L = C.CDLL(LIB_PATH)
        P, I, D = C.c_void_p, C.c_int, C.c_double
        L.orc_cell_nse_system.argtypes = [P, P, P, P, P, P]
        L.orc_cell_nse_preconditioner.argtypes = [P, P, P]
        L.orc_cell_temperature_matrix.argtypes = [P, P, P, P]
        L.orc_cell_temperature_rhs.argtypes = [P, P, P, P, P, P, P]
        L.orc_create.argtypes = [P, I, P, P, P, I, I, I, P, P]
        L.orc_create.restype = P
        L.orc_destroy.argtypes = [P]
        L.orc_set_time_step.argtypes = [P, D]
        L.orc_assemble_nse_system.argtypes = [P, P, P]
        L.orc_build_nse_preconditioner.argtypes = [P]
        L.orc_assemble_temperature_matrix.argtypes = [P]
        L.orc_assemble_temperature_rhs.argtypes = [P, P, P]
        L.orc_nse_matrix_nnz.argtypes = [P]
        L.orc_nse_matrix_nnz.restype = C.c_long
        L.orc_nse_matrix_csr.argtypes = [P, P, P, P]
        L.orc_nse_rhs.argtypes = [P, P]
        L.orc_nse_block_csr.argtypes = [P, I, P, P, P]
        L.orc_nse_block_csr.restype = C.c_long
        L.orc_cell_nse_system_literal.argtypes = [P, P, P, P, P, P]
        L.orc_cell_nse_preconditioner_literal.argtypes = [P, P, P]
        L.orc_precond_diagonals.argtypes = [P, P, P]
        L.orc_T_matrix_nnz.argtypes = [P]
        L.orc_T_matrix_nnz.restype = C.c_long
        L.orc_T_matrix_csr.argtypes = [P, P, P, P]
        L.orc_T_rhs.argtypes = [P, P]
        L.orc_nse_vmult.argtypes = [P, P, P]
        L.orc_schur_vmult.argtypes = [P, P, P]
        L.orc_block_preconditioner_vmult.argtypes = [P, P, P, I, P]
        L.orc_solve_nse.argtypes = [P, P, P, P, I]
        L.orc_solve_temperature.argtypes = [P, P, P]
        L.orc_solve_nse_schur.argtypes = [P, P, P, P]
        L.orc_assemble_nse_system_threads.argtypes = [P, P, P, I]
        L.orc_set_inner_max_steps.argtypes = [P, I]
        L.orc_set_schur_fixed_inner.argtypes = [P, I]
        L.orc_set_ilu_blocks.argtypes = [P, P]
        L.orc_set_block_fixed_inner.argtypes = [P, I]
        L.orc_set_threads.argtypes = [I]
        L.orc_fgmres_outer.argtypes = [P, P, I, P]
        L.orc_schur_gmres_sample.argtypes = [I, I, P, P, P, P, P, P, P, P, P, I]
        L.orc_schur_gmres_sample.restype = D
        L.orc_a_solve_iterations.argtypes = [P]
        L.orc_a_solve_iterations.restype = C.c_long
        L.orc_max_velocity.argtypes = [P, P]
        L.orc_max_velocity.restype = D
        L.orc_cfl.argtypes = [P, P, P]
        L.orc_cfl.restype = D
        L.orc_feec_cell_system.argtypes = [P, P, P, P, P, P, P]
        L.orc_feec_cell_preconditioner.argtypes = [P, P, P, P]
        L.orc_feec_create.argtypes = [P, I, P, P, P, P, I, I, I, P, I, P, P]
        L.orc_feec_create.restype = P
        L.orc_feec_destroy.argtypes = [P]
        L.orc_feec_set_zero_mean.argtypes = [P, I]
        L.orc_feec_set_fixed_inner.argtypes = [P, I]
        L.orc_feec_set_block_preconditioner.argtypes = [P, I]
        L.orc_feec_assemble_nse_system.argtypes = [P, P, P]
        L.orc_feec_assemble_preconditioner.argtypes = [P]
        L.orc_feec_matrix_nnz.argtypes = [P, I]
        L.orc_feec_matrix_nnz.restype = C.c_long
        L.orc_feec_matrix_csr.argtypes = [P, I, P, P, P]
        L.orc_feec_rhs.argtypes = [P, P]
        L.orc_feec_assemble_temperature.argtypes = [P, P, P]
        L.orc_feec_T_rhs.argtypes = [P, P]
        L.orc_feec_solve_nse.argtypes = [P, P, P]
        L.orc_feec_solve_temperature.argtypes = [P, P, P]
        L.orc_feec_velocity_stats.argtypes = [P, P, P]
        L.orc2d_cell_nse_system.argtypes = [P, P, P, P, P, P]
        L.orc2d_cell_nse_preconditioner.argtypes = [P, P, P]
        L.orc2d_cell_temperature_matrix.argtypes = [P, P, P, P]
        L.orc2d_cell_temperature_rhs.argtypes = [P, P, P, P, P, P, P]
        L.orc2d_create.argtypes = [P, I, P, P, P, I, I, I, P, P]
        L.orc2d_create.restype = P
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def physics(ph) -> OrcPhysics:
    """Convert a dcp.Physics (same field layout) to OrcPhysics."""
    o = OrcPhysics()
    for name, _ in OrcPhysics._fields_:
        setattr(o, name, getattr(ph, name))
    return o


def cell_nse_system(ph, geom64, u_local, T_local):
    K = np.zeros((89, 89))
    f = np.zeros(89)
    o = physics(ph)
    lib().orc_cell_nse_system(C.byref(o), _p(np.ascontiguousarray(geom64, np.float64)),
                              _p(np.ascontiguousarray(u_local, np.float64)),
                              _p(np.ascontiguousarray(T_local, np.float64)), _p(K), _p(f))
    return K, f


def cell_nse_system_literal(ph, geom64, u_local, T_local):
    """The literal 89 x 89 loop of local_assemble_nse_system (checker of the
    structural-zero loop cell_nse_system uses)."""
    K = np.zeros((89, 89))
    f = np.zeros(89)
    o = physics(ph)
    lib().orc_cell_nse_system_literal(C.byref(o), _p(np.ascontiguousarray(geom64, np.float64)),
                                      _p(np.ascontiguousarray(u_local, np.float64)),
                                      _p(np.ascontiguousarray(T_local, np.float64)), _p(K), _p(f))
    return K, f


def cell_nse_preconditioner_literal(ph, geom64):
    P = np.zeros((89, 89))
    o = physics(ph)
    lib().orc_cell_nse_preconditioner_literal(C.byref(o),
                                              _p(np.ascontiguousarray(geom64, np.float64)), _p(P))
    return P


def set_threads(n):
    """Threads of the oracle's cell loops and operator applies (bitwise the
    serial results)."""
    lib().orc_set_threads(int(n))


def usable_threads(cap=16):
    """Cores this process may use, capped (the GPU box's CPU share is 16)."""
    import os
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    return max(1, min(cap, n))


def cell_nse_preconditioner(ph, geom64):
    P = np.zeros((89, 89))
    o = physics(ph)
    lib().orc_cell_nse_preconditioner(C.byref(o), _p(np.ascontiguousarray(geom64, np.float64)), _p(P))
    return P


def cell_nse_system_2d(ph, geom16, u_local, T_local):
    """local_assemble_nse_system at dim = 2: K [22][22], f [22]."""
    K = np.zeros((22, 22))
    f = np.zeros(22)
    o = physics(ph)
    lib().orc2d_cell_nse_system(C.byref(o), _p(np.ascontiguousarray(geom16, np.float64)),
                                _p(np.ascontiguousarray(u_local, np.float64)),
                                _p(np.ascontiguousarray(T_local, np.float64)), _p(K), _p(f))
    return K, f


def cell_temperature_matrix_2d(ph, geom16):
    n = (ph.temperature_degree + 1) ** 2
    M, K = np.zeros((n, n)), np.zeros((n, n))
    o = physics(ph)
    lib().orc2d_cell_temperature_matrix(C.byref(o), _p(np.ascontiguousarray(geom16, np.float64)),
                                        _p(M), _p(K))
    return M, K


class Model:
    """Global oracle model over a dcp.HostMesh (or a dcp.HostMesh2D: the 2D
    model, orc2d_create)."""

    def __init__(self, ph, mesh):
        self.ph = physics(ph)
        self.dim = getattr(mesh, "dim", 3)
        if self.dim == 2:
            self.ph.temperature_degree = mesh.temperature_degree
        self.mesh = mesh
        self._keep = []

        def cons(cs):
            s = OrcConstraints(len(cs.line_dof), _p(cs.line_dof).value, _p(cs.entry_ptr).value,
                               _p(cs.entry_dof).value, _p(cs.entry_w).value,
                               _p(cs.inhomogeneity).value)
            self._keep.append(cs)
            return s

        self._nc, self._tc = cons(mesh.nse_constraints), cons(mesh.T_constraints)
        self._cd = np.ascontiguousarray(mesh.cell_nse_dofs, np.int32)
        self._td = np.ascontiguousarray(mesh.cell_T_dofs, np.int32)
        self._g = np.ascontiguousarray(mesh.cell_geometry, np.float64)
        create = lib().orc2d_create if self.dim == 2 else lib().orc_create
        self.h = create(C.byref(self.ph), mesh.n_cells, _p(self._cd), _p(self._td), _p(self._g),
                        mesh.n_u, mesh.n_p, mesh.n_T, C.byref(self._nc), C.byref(self._tc))

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_destroy(self.h)
            self.h = None

    def set_time_step(self, dt):
        self.ph.time_step = dt
        lib().orc_set_time_step(self.h, dt)

    def assemble_nse_system(self, old_nse, old_T):
        lib().orc_assemble_nse_system(self.h, _p(np.ascontiguousarray(old_nse, np.float64)),
                                      _p(np.ascontiguousarray(old_T, np.float64)))

    def assemble_nse_system_threads(self, old_nse, old_T, threads):
        """WorkStream-style assembly on `threads` threads (bitwise the serial one)."""
        lib().orc_assemble_nse_system_threads(
            self.h, _p(np.ascontiguousarray(old_nse, np.float64)),
            _p(np.ascontiguousarray(old_T, np.float64)), int(threads))

    def set_inner_max_steps(self, n):
        """Timing hook: cap of the inner Schur GMRES (the reference's 5000)."""
        lib().orc_set_inner_max_steps(self.h, int(n))

    def set_block_fixed_inner(self, k):
        """Parity hook: the block preconditioner's inner Schur GMRES runs
        exactly k steps with no tolerance test (0 = the reference's rule)."""
        lib().orc_set_block_fixed_inner(self.h, int(k))

    def set_schur_fixed_inner(self, k):
        """Parity hook: the Schur solver's inner CGs run exactly k steps (0 = off)."""
        lib().orc_set_schur_fixed_inner(self.h, int(k))

    def set_ilu_blocks(self, owner):
        """The Schur solver's ILU as on P ranks (Trilinos ILU, overlap 0): owner
        = the rank of every velocity dof; None restores the one-rank factor."""
        if owner is None:
            self._ilu_owner = None
            lib().orc_set_ilu_blocks(self.h, None)
            return
        self._ilu_owner = np.ascontiguousarray(owner, np.int32)
        lib().orc_set_ilu_blocks(self.h, _p(self._ilu_owner))

    def build_nse_preconditioner(self):
        lib().orc_build_nse_preconditioner(self.h)

    def assemble_temperature_matrix(self):
        lib().orc_assemble_temperature_matrix(self.h)

    def assemble_temperature_rhs(self, old_T, nse_solution):
        lib().orc_assemble_temperature_rhs(self.h, _p(np.ascontiguousarray(old_T, np.float64)),
                                           _p(np.ascontiguousarray(nse_solution, np.float64)))

    def nse_matrix_csr(self):
        nnz = lib().orc_nse_matrix_nnz(self.h)
        n = self.mesh.n_u + self.mesh.n_p
        rp, cols, vals = np.zeros(n + 1, np.int32), np.zeros(nnz, np.int32), np.zeros(nnz)
        lib().orc_nse_matrix_csr(self.h, _p(rp), _p(cols), _p(vals))
        return rp, cols, vals

    def nse_block_csr(self, which):
        """One block of nse_matrix as (rowptr, cols, vals): "A" (0,0), "Bt" (0,1),
        "B" (1,0), with block-local columns."""
        w = {"A": 0, "Bt": 1, "B": 2}[which]
        nnz = lib().orc_nse_block_csr(self.h, w, None, None, None)
        nr = self.mesh.n_p if which == "B" else self.mesh.n_u
        rp, cols, vals = np.zeros(nr + 1, np.int32), np.zeros(nnz, np.int32), np.zeros(nnz)
        lib().orc_nse_block_csr(self.h, w, _p(rp), _p(cols), _p(vals))
        return rp, cols, vals

    def nse_rhs(self):
        out = np.zeros(self.mesh.n_u + self.mesh.n_p)
        lib().orc_nse_rhs(self.h, _p(out))
        return out

    def precond_diagonals(self):
        a, p = np.zeros(self.mesh.n_u), np.zeros(self.mesh.n_p)
        lib().orc_precond_diagonals(self.h, _p(a), _p(p))
        return a, p

    def T_matrix_csr(self):
        nnz = lib().orc_T_matrix_nnz(self.h)
        rp, cols, vals = np.zeros(self.mesh.n_T + 1, np.int32), np.zeros(nnz, np.int32), np.zeros(nnz)
        lib().orc_T_matrix_csr(self.h, _p(rp), _p(cols), _p(vals))
        return rp, cols, vals

    def T_rhs(self):
        out = np.zeros(self.mesh.n_T)
        lib().orc_T_rhs(self.h, _p(out))
        return out

    def nse_vmult(self, src):
        dst = np.zeros(self.mesh.n_u + self.mesh.n_p)
        lib().orc_nse_vmult(self.h, _p(np.ascontiguousarray(src, np.float64)), _p(dst))
        return dst

    def schur_vmult(self, src):
        dst = np.zeros(self.mesh.n_p)
        lib().orc_schur_vmult(self.h, _p(np.ascontiguousarray(src, np.float64)), _p(dst))
        return dst

    def block_preconditioner_vmult(self, src, do_solve_A=False):
        dst = np.zeros(self.mesh.n_u + self.mesh.n_p)
        it = C.c_int(0)
        lib().orc_block_preconditioner_vmult(self.h, _p(np.ascontiguousarray(src, np.float64)),
                                             _p(dst), int(do_solve_A), C.byref(it))
        return dst, it.value

    def solve_nse(self, nse_solution, max_outer=40):
        x = np.array(nse_solution, dtype=np.float64, copy=True)
        o, i = C.c_int(0), C.c_int(0)
        rc = lib().orc_solve_nse(self.h, _p(x), C.byref(o), C.byref(i), int(max_outer))
        return rc, x, o.value, i.value

    def fgmres_outer(self, nse_solution, k):
        """Timing hook: the first FGMRES(30) cut at k outer iterations, no
        fallback -> (outer iterations done, inner Schur GMRES iterations)."""
        i = C.c_int(0)
        o = lib().orc_fgmres_outer(self.h, _p(np.ascontiguousarray(nse_solution, np.float64)),
                                   int(k), C.byref(i))
        return o, i.value

    def a_solve_iterations(self):
        """AztecOO A-GMRES iterations of the last solve_nse (do_solve_A fallback)."""
        return int(lib().orc_a_solve_iterations(self.h))

    def solve_temperature(self, T):
        x = np.array(T, dtype=np.float64, copy=True)
        it = C.c_int(0)
        rc = lib().orc_solve_temperature(self.h, _p(x), C.byref(it))
        return rc, x, it.value

    def solve_nse_schur(self, sol):
        """solve_NSE_Schur_complement: (rc, solution, Schur GMRES steps, A^-1 solves)."""
        x = np.array(sol, dtype=np.float64, copy=True)
        it, na = C.c_int(0), C.c_int(0)
        rc = lib().orc_solve_nse_schur(self.h, _p(x), C.byref(it), C.byref(na))
        return rc, x, it.value, na.value

    def max_velocity(self, sol):
        return lib().orc_max_velocity(self.h, _p(np.ascontiguousarray(sol, np.float64)))

    def cfl(self, sol):
        return lib().orc_cfl(self.h, _p(np.ascontiguousarray(sol, np.float64)),
                             _p(np.ascontiguousarray(self.mesh.cell_diameter, np.float64)))


# ---- FEEC variant (ExteriorCalculus::BoussinesqModel<3>) -------------------

def feec_cell_system(ph, X8, sign19, dofv19, T_local):
    K, f = np.zeros((19, 19)), np.zeros(19)
    o = physics(ph)
    lib().orc_feec_cell_system(C.byref(o), _p(np.ascontiguousarray(X8, np.float64)),
                               _p(np.ascontiguousarray(sign19, np.int8)),
                               _p(np.ascontiguousarray(dofv19, np.float64)),
                               _p(np.ascontiguousarray(T_local, np.float64)), _p(K), _p(f))
    return K, f


def feec_cell_preconditioner(ph, X8, sign19):
    P = np.zeros((19, 19))
    o = physics(ph)
    lib().orc_feec_cell_preconditioner(C.byref(o), _p(np.ascontiguousarray(X8, np.float64)),
                                       _p(np.ascontiguousarray(sign19, np.int8)), _p(P))
    return P


class FeecModel:
    """Global FEEC oracle over dcp.HostMesh(feec=True)."""

    def __init__(self, ph, mesh, zero_mean=True):
        f = mesh.feec
        self.f = f
        self.ph = physics(ph)
        self._a = [np.ascontiguousarray(f.cell_dofs, np.int32), np.ascontiguousarray(f.signs, np.int8),
                   np.ascontiguousarray(f.cell_vertices, np.float64),
                   np.ascontiguousarray(f.fixed, np.uint8), np.ascontiguousarray(f.cell_T_dofs, np.int32),
                   np.ascontiguousarray(f.cell_diameter, np.float64)]
        cs = mesh.T_constraints
        self._tc = OrcConstraints(len(cs.line_dof), _p(cs.line_dof).value, _p(cs.entry_ptr).value,
                                  _p(cs.entry_dof).value, _p(cs.entry_w).value,
                                  _p(cs.inhomogeneity).value)
        self._keep = cs
        a = self._a
        self.h = lib().orc_feec_create(C.byref(self.ph), f.n_cells, _p(a[0]), _p(a[1]), _p(a[2]),
                                       _p(a[3]), f.n_w, f.n_u, f.n_p, _p(a[4]), f.n_T,
                                       C.byref(self._tc), _p(a[5]))
        lib().orc_feec_set_zero_mean(self.h, int(zero_mean))

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_feec_destroy(self.h)
            self.h = None

    def assemble_nse_system(self, old_nse, old_T):
        lib().orc_feec_assemble_nse_system(self.h, _p(np.ascontiguousarray(old_nse, np.float64)),
                                           _p(np.ascontiguousarray(old_T, np.float64)))

    def assemble_preconditioner(self):
        lib().orc_feec_assemble_preconditioner(self.h)

    def matrix_csr(self, which=0):
        nnz = lib().orc_feec_matrix_nnz(self.h, which)
        n = self.f.n
        rp, cols, vals = np.zeros(n + 1, np.int32), np.zeros(nnz, np.int32), np.zeros(nnz)
        lib().orc_feec_matrix_csr(self.h, which, _p(rp), _p(cols), _p(vals))
        return rp, cols, vals

    def rhs(self):
        out = np.zeros(self.f.n)
        lib().orc_feec_rhs(self.h, _p(out))
        return out

    def assemble_temperature(self, old_T, nse_solution):
        lib().orc_feec_assemble_temperature(self.h, _p(np.ascontiguousarray(old_T, np.float64)),
                                            _p(np.ascontiguousarray(nse_solution, np.float64)))

    def T_rhs(self):
        out = np.zeros(self.f.n_T)
        lib().orc_feec_T_rhs(self.h, _p(out))
        return out

    def set_fixed_inner(self, k):
        """Test hook (DCP_OPT_FEEC_FIXED_INNER): both inner GMRES run exactly k steps."""
        lib().orc_feec_set_fixed_inner(self.h, int(k))

    def set_block_preconditioner(self, on):
        """use_block_preconditioner_feec; off: identity-preconditioned GMRES(100)."""
        lib().orc_feec_set_block_preconditioner(self.h, int(bool(on)))

    def solve_nse(self, sol):
        x = np.array(sol, dtype=np.float64, copy=True)
        it = C.c_int(0)
        rc = lib().orc_feec_solve_nse(self.h, _p(x), C.byref(it))
        return rc, x, it.value

    def solve_temperature(self, T):
        x = np.array(T, dtype=np.float64, copy=True)
        it = C.c_int(0)
        rc = lib().orc_feec_solve_temperature(self.h, _p(x), C.byref(it))
        return rc, x, it.value

    def velocity_stats(self, sol):
        out = np.zeros(2)
        lib().orc_feec_velocity_stats(self.h, _p(np.ascontiguousarray(sol, np.float64)), _p(out))
        return out


def schur_gmres_sample(Bt, B, A_inv, src_p, k):
    """CPU baseline sample: k steps of deal.II's SolverGMRES on
    S = B (D_A^-1 (B^T p)) from the CSR triples Bt (n_u x n_p) and B (n_p x n_u).
    Returns (seconds, iterate)."""
    (btp, btc, btv), (bp, bc, bv) = Bt, B
    n_u, n_p = len(btp) - 1, len(bp) - 1
    arr = [np.ascontiguousarray(a, t) for a, t in ((btp, np.int32), (btc, np.int32), (btv, np.float64),
                                                      (bp, np.int32), (bc, np.int32), (bv, np.float64),
                                                      (A_inv, np.float64), (src_p, np.float64))]
    dst = np.zeros(n_p)
    sec = lib().orc_schur_gmres_sample(n_u, n_p, *[_p(a) for a in arr], _p(dst), int(k))
    return sec, dst


def cuthill_mckee_nse(cell_nse_dofs, n_vnodes, n_u, n_p):
    """Checker for dcp_host_mesh_renumber_cuthill_mckee: deal.II's
    SparsityTools::reorder_Cuthill_McKee (sparsity_tools.cc, called by
    DoFRenumbering::Cuthill_McKee at boussinesq_model.tpp:200) restated in
    numpy on support points, then component_wise (:204). Returns (node_new,
    dof_map old -> new)."""
    import scipy.sparse as sp
    nc = cell_nse_dofs.shape[0]
    vel = cell_nse_dofs[:, [4 * v for v in range(8)] + list(range(32, 89, 3))] // 3
    vnode_p = np.full(n_p, -1, np.int64)
    for v in range(8):
        vnode_p[cell_nse_dofs[:, 4 * v + 3] - n_u] = cell_nse_dofs[:, 4 * v] // 3
    ndof = np.full(n_vnodes, 3, np.int64)
    ndof[vnode_p] = 4
    rows = np.repeat(vel, 27, axis=1).ravel()
    cols = np.tile(vel, (1, 27)).ravel()
    A = sp.csr_matrix((np.ones(rows.size, np.int8), (rows, cols)), shape=(n_vnodes, n_vnodes))
    A.sum_duplicates()
    A.data[:] = 1
    coord = np.asarray(A @ ndof).ravel()  # row length of every dof at the node
    ptr, idx = A.indptr, A.indices
    new = np.full(n_vnodes, -1, np.int64)

    def start():  # find_unnumbered_starting_index: first of least coordination
        free = np.flatnonzero(new < 0)
        return int(free[np.argmin(coord[free])])

    last = np.array([start()])
    new[last] = 0
    nxt = 1
    while nxt < n_vnodes:
        cand = np.unique(np.concatenate([idx[ptr[n]:ptr[n + 1]] for n in last]))
        cand = cand[new[cand] < 0]
        if cand.size == 0:
            cand = np.array([start()])
        order = cand[np.argsort(coord[cand], kind="stable")]
        new[order] = np.arange(nxt, nxt + order.size)
        nxt += order.size
        last = order
    newp = np.empty(n_p, np.int64)
    newp[np.argsort(new[vnode_p], kind="stable")] = np.arange(n_p)
    dmap = np.empty(n_u + n_p, np.int64)
    dmap[:n_u] = 3 * new[np.arange(n_u) // 3] + np.arange(n_u) % 3
    dmap[n_u:] = n_u + newp
    return new, dmap
