#!/usr/bin/env python3
"""Pins the r >= 4 failure mode of the inner Schur GMRES outside the builder's
own GMRES restatement.

At refine R (default 4, BASELINE config 3) the oracle assembles the classic
prm's NSE system, builds S = B diag(A_inv) B^T exactly as
SchurComplement::vmult applies it (schur_complement.hpp:143-150, the
A-Jacobi of Q9), and forms src_p of the first non-trivial preconditioner
call of the first FGMRES (the pressure block of v_1; v_0 = b/|b| has a zero
pressure block). Then:
  * scipy.sparse.linalg.gmres (restart 28 = SolverGMRES's max_n_tmp_vectors - 2,
    identity preconditioner, rtol 1e-6 relative to |src_p|, x0 = 0, 5,000
    iterations = the reference's SolverControl(5000, 1e-6 |src_p|)) and its
    per-iteration residual estimate;
  * the oracle's own inner GMRES on the same src_p (deal.II's SolverGMRES
    restated) for its count;
  * the three smallest eigenpairs of S (shift-invert Lanczos) and the overlap
    of the smallest eigenvector with the constant pressure vector.
Writes tests/golden/schur_scipy_r<R>.npz. Test infrastructure only: runs on
the CPU, reads nothing from /root/reference."""
import os
import sys
import time

import numpy as np
import scipy
import scipy.sparse as sp
import scipy.sparse.linalg as spla

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-dycoreplanet_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import dcp  # noqa: E402
import oracle_py  # noqa: E402


def schur_problem(refine, threads=8):
    """(S, src_p, oracle model, mesh) of the first non-trivial preconditioner
    call of the refine-`refine` classic step."""
    m = dcp.HostMesh(refine=refine)
    orc = oracle_py.Model(dcp.classic_physics(), m)
    u = np.zeros(m.n_u + m.n_p)
    orc.assemble_nse_system_threads(u, m.T0, threads)
    orc.build_nse_preconditioner()
    n = m.n_u + m.n_p
    rp, cols, vals = orc.nse_matrix_csr()
    M = sp.csr_matrix((vals, cols, rp), shape=(n, n))
    Bt = M[:m.n_u, m.n_u:]
    B = M[m.n_u:, :m.n_u]
    a_diag, _ = orc.precond_diagonals()
    S = (B @ sp.diags(1.0 / a_diag) @ Bt).tocsr()
    # FGMRES (deal.II SolverFGMRES, x0 = 0 at the reference's first step):
    # v_0 = b/|b|, z_0 = P v_0, aux = A z_0 - (aux.v_0) v_0, v_1 = aux/|aux|
    b = orc.nse_rhs()
    v0 = b / np.linalg.norm(b)
    z0, it0 = orc.block_preconditioner_vmult(v0)
    aux = orc.nse_vmult(z0)
    aux -= (aux @ v0) * v0
    v1 = aux / np.linalg.norm(aux)
    return S, v1[m.n_u:].copy(), v1, orc, m, it0


def scipy_gmres(S, src, maxit=5000, restart=28):
    hist = []
    x, info = spla.gmres(S, src, x0=np.zeros_like(src), rtol=1e-6, atol=0.0, restart=restart,
                         maxiter=int(np.ceil(maxit / restart)), callback=hist.append,
                         callback_type="pr_norm")
    hist = np.asarray(hist[:maxit]) * np.linalg.norm(src)  # pr_norm is relative to |b|
    true_res = np.linalg.norm(src - S @ x)
    return x, info, hist, true_res


def main():
    refine = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    t0 = time.time()
    S, src, v1, orc, m, it0 = schur_problem(refine)
    print(f"refine {refine}: n_p {m.n_p}, nnz(S) {S.nnz}, setup {time.time() - t0:.1f} s", flush=True)
    assert S.shape == (m.n_p, m.n_p)
    # S as the oracle applies it (same operator, summation order aside)
    q = np.random.default_rng(3).uniform(-1, 1, m.n_p)
    assert np.linalg.norm(S @ q - orc.schur_vmult(q)) <= 1e-12 * np.linalg.norm(S @ q)
    t0 = time.time()
    x, info, hist, true_res = scipy_gmres(S, src)
    print(f"scipy gmres: info {info}, {len(hist)} iterations, final estimate "
          f"{hist[-1] / np.linalg.norm(src):.3e}, true {true_res / np.linalg.norm(src):.3e} "
          f"({time.time() - t0:.1f} s)", flush=True)
    # the oracle's SolverGMRES on the same right-hand side (full block vector
    # with the velocity part zero: only src_p enters the inner solve)
    srcv = np.zeros(m.n_u + m.n_p)
    srcv[m.n_u:] = src
    _, it_orc = orc.block_preconditioner_vmult(srcv)
    print(f"oracle SolverGMRES: {it_orc} iterations (-1: NoConvergence at its cap)", flush=True)
    # smallest eigenpairs of the symmetric positive semi-definite S
    t0 = time.time()
    lmax = spla.eigsh(S, k=1, which="LA", return_eigenvectors=False, tol=1e-6)[0]
    w, V = spla.eigsh(S, k=3, sigma=-1e-9 * lmax, which="LM", tol=1e-10)
    order = np.argsort(w)
    w, V = w[order], V[:, order]
    ones = np.ones(m.n_p) / np.sqrt(m.n_p)
    overlap = np.abs(V.T @ ones)
    print(f"eigenvalues of S: smallest {w}, largest {lmax:.4e}; |<v_min, 1/sqrt(n)>| = "
          f"{overlap} ({time.time() - t0:.1f} s)", flush=True)
    out = os.path.join(ROOT, "tests", "golden", f"schur_scipy_r{refine}.npz")
    np.savez_compressed(out, refine=refine, n_p=m.n_p, nnz_S=S.nnz, src_norm=np.linalg.norm(src),
                        src_mean=src.mean(), hist=hist.astype(np.float32), info=info,
                        true_res=true_res, oracle_its=it_orc, eig_small=w, eig_max=lmax,
                        overlap_const=overlap, const_rayleigh=ones @ (S @ ones),
                        scipy_version=scipy.__version__)
    print("wrote", out)


if __name__ == "__main__":
    main()
