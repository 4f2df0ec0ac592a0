"""BASELINE config C5's mesh (classic prm, global refinement 6: 1,572,864
cells, 38.0 M velocity + 1.6 M pressure dofs) on ONE GPU, through the code
paths only this size takes: the s-step inner Schur GMRES block as five
launches (the basis no longer fits the resident grid of the one-launch
kernel; the same path several GPUs run), S formation and the matrix-free
operator at 39.6 M dofs. No oracle runs at this size (the CPU
restatement's CSR alone would be ~100 GB); the checks are size-independent:
s-step against classical Gram-Schmidt twice (the same Krylov space), the
inner residual, symmetry / linearity of the operators, determinism, and the
device memory per stage (tools/r6_probe.py records the same stages)."""
import ctypes as C

import numpy as np
import pytest

import dcp

pytestmark = pytest.mark.gpu


def _mem_used_gb():
    free, total = C.c_size_t(0), C.c_size_t(0)
    dcp.hip().hipMemGetInfo(C.byref(free), C.byref(total))
    return (total.value - free.value) / 1e9


def test_refine6_one_gpu_sstep_five_launch_block():
    m = dcp.HostMesh(refine=6)
    assert (m.n_cells, m.n_p) == (1_572_864, 1_597_570)
    mem = {"context": _mem_used_gb()}
    ctx = dcp.Context()
    ctx.set_physics(dcp.classic_physics())
    ctx.upload_mesh(m)
    mem["upload"] = _mem_used_gb()
    n = m.n_u + m.n_p
    u = np.zeros(n)
    for f, v in ((dcp.OLD_NSE_SOLUTION, u), (dcp.NSE_SOLUTION, u), (dcp.OLD_T_SOLUTION, m.T0),
                 (dcp.T_SOLUTION, m.T0)):
        ctx.set_state(f, v)
    ctx.assemble_nse_system()
    r1 = ctx.get_state(dcp.NSE_RHS)
    ctx.assemble_nse_system()
    assert np.array_equal(r1, ctx.get_state(dcp.NSE_RHS)) and np.all(np.isfinite(r1))
    ctx.build_nse_preconditioner()
    mem["preconditioner"] = _mem_used_gb()
    rng = np.random.default_rng(6)
    x, y = rng.uniform(-1, 1, n), rng.uniform(-1, 1, n)
    Mx, My, Mxy = ctx.nse_vmult(x), ctx.nse_vmult(y), ctx.nse_vmult(x + 2 * y)
    scale = np.linalg.norm(Mx) + 2 * np.linalg.norm(My)
    assert np.linalg.norm(Mxy - Mx - 2 * My) / scale < 1e-12
    assert abs(y @ Mx - x @ My) / (np.linalg.norm(x) * np.linalg.norm(My)) < 1e-12
    p = rng.uniform(-1, 1, m.n_p)
    q = rng.uniform(-1, 1, m.n_p)
    Sp, Sq = ctx.schur_vmult(p), ctx.schur_vmult(q)
    assert abs(q @ Sp - p @ Sq) / (np.linalg.norm(p) * np.linalg.norm(Sq)) < 1e-12
    assert p @ Sp > 0 and q @ Sq > 0
    # 56 inner steps (two restart cycles of 28) of BlockSchurPreconditioner::vmult
    src = np.zeros(n)
    src[m.n_u:] = p - p.mean()
    ctx.set_block_fixed_inner(56)
    res = {}
    for gs in ("sstep", "classical2"):
        ctx.set_gram_schmidt(gs)
        dst, its = ctx.block_preconditioner_vmult(src)
        assert its == 56
        # dst_p = -y (block_schur_preconditioner.hpp:48-51)
        r = ctx.schur_vmult(-dst[m.n_u:]) - src[m.n_u:]
        res[gs] = (dst, np.linalg.norm(r) / np.linalg.norm(src[m.n_u:]))
        mem["inner_" + gs] = _mem_used_gb()
    ctx.set_block_fixed_inner(0)
    ctx.close()
    print("device memory (GB) per stage:", {k: round(v, 2) for k, v in mem.items()})
    print("inner residual reduction after 56 steps:", {k: v[1] for k, v in res.items()})
    (ds, rs), (dc, rc) = res["sstep"], res["classical2"]
    # the same 56-dimensional Krylov minimiser, two orthogonalisations
    assert rs < 0.5 and rc < 0.5
    assert abs(rs - rc) <= 1e-6 * rc
    assert np.linalg.norm(ds - dc) <= 1e-6 * np.linalg.norm(dc)
    assert max(mem.values()) < 200.0
