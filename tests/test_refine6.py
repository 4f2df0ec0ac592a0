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


def _c5_step(ctx, m, u, T, src):
    """The rank's part of config C5's step at fixed inner steps: assembly,
    preconditioner, temperature system, BlockSchurPreconditioner::vmult of
    `src` (through the state buffers: the operator seam takes the rank's local
    vectors, which set_state lays out from the global vector), the
    temperature CG."""
    import ctypes as C
    for f, v in ((dcp.OLD_NSE_SOLUTION, u), (dcp.OLD_T_SOLUTION, T), (dcp.T_SOLUTION, T)):
        ctx.set_state(f, v)
    out = {}
    ctx.assemble_nse_system()
    out["rhs"] = ctx.get_state(dcp.NSE_RHS)
    ctx.build_nse_preconditioner()
    ctx.assemble_temperature_matrix()
    ctx.assemble_temperature_rhs()
    out["T_rhs"] = ctx.get_state(dcp.T_RHS)
    ctx.set_state(dcp.NSE_SOLUTION, src)
    it = C.c_int(0)
    ctx._check(dcp.lib().dcp_block_preconditioner_vmult(
        ctx._h, C.c_void_p(ctx.device_ptr(dcp.NSE_SOLUTION)),
        C.c_void_p(ctx.device_ptr(dcp.OLD_NSE_SOLUTION)), 0, C.byref(it)), True)
    out["inner"] = it.value
    out["dst"] = ctx.get_state(dcp.OLD_NSE_SOLUTION)
    out["T"] = ctx.solve_temperature()
    out["Tx"] = ctx.get_state(dcp.T_SOLUTION)
    out["mp"] = ctx.matrix_powers_info()
    out["mem"] = dcp.Context.device_memory()
    return out


def test_refine6_c5_eight_rank_decomposition():
    """BASELINE config C5 (classic prm, refine 6: 1,572,864 cells, 39.6 M NSE
    dofs) decomposed over 8 ranks -- the p4est-style split, two ghost layers,
    halos, the depth-4 matrix-powers ghost rows of S -- in an in-process group
    on one GPU, against the same step on one GPU: the rhs and temperature rhs
    at 1e-12, BlockSchurPreconditioner::vmult (block_schur_preconditioner.hpp:
    42-70) with its s-step inner Schur GMRES held at 56 steps at 1e-10, the
    temperature CG (:1417-1476) count within one and its solution at 1e-10;
    device memory per rank and in total printed (dcp_device_memory per rank
    thread, hipMemGetInfo for the device)."""
    import threading
    import time
    world = 8
    t0 = time.time()
    m = dcp.HostMesh(refine=6)
    ph = dcp.classic_physics()
    rng = np.random.default_rng(66)
    n = m.n_u + m.n_p
    u = np.zeros(n)
    u[:m.n_u] = 0.05 * rng.uniform(-1, 1, m.n_u)
    T = m.T0.copy()
    src = rng.uniform(-1, 1, n)
    src[m.n_u:] -= src[m.n_u:].mean()
    t_mesh = time.time() - t0
    base = _mem_used_gb()
    t0 = time.time()
    ctx = dcp.Context()
    ctx.set_physics(ph)
    ctx.set_gram_schmidt("sstep")
    ctx.set_block_fixed_inner(56)
    ctx.upload_mesh(m)
    ref = _c5_step(ctx, m, u, T, src)
    ref["device_gb"] = _mem_used_gb() - base
    ctx.close()
    t_one = time.time() - t0
    t0 = time.time()
    g = dcp.Group(world)
    results, errors = [None] * world, []
    peak = [0.0]
    ready = threading.Barrier(world)

    def run(rank):
        try:
            c = dcp.Context(rank=rank, world_size=world, group=g)
            c.set_physics(ph)
            c.set_gram_schmidt("sstep")
            c.set_block_fixed_inner(56)
            c.upload_mesh(m)
            results[rank] = _c5_step(c, m, u, T, src)
            ready.wait(timeout=600)
            if rank == 0:
                peak[0] = _mem_used_gb() - base
            ready.wait(timeout=600)
            c.close()
        except Exception as e:  # noqa: BLE001
            errors.append((rank, repr(e)))
            ready.abort()

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=900)
    g.close()
    t_group = time.time() - t0
    assert not errors, errors
    per_rank = [r["mem"]["peak"] / 1e9 for r in results]
    print(f"\nC5 refine 6: {m.n_cells} cells, {n} NSE dofs; mesh {t_mesh:.0f} s, one GPU "
          f"{t_one:.0f} s, 8 ranks {t_group:.0f} s")
    print(f"device memory: one GPU {ref['device_gb']:.1f} GB (library peak "
          f"{ref['mem']['peak'] / 1e9:.1f} GB); 8 ranks: per-rank library peak "
          f"{[round(x, 1) for x in per_rank]} GB, sum {sum(per_rank):.1f} GB, device "
          f"{peak[0]:.1f} GB")
    print("matrix powers per rank (ghost rows depth<=1,2,3; depth-4 halo entries per block):",
          [(r["mp"]["rows"], r["mp"]["halo_recv"]) for r in results])

    def merged(key):
        v = np.zeros_like(ref[key])
        for r in results:
            nz = r[key] != 0
            v[nz] = r[key][nz]
        return v

    rel = lambda a, b: np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300)  # noqa: E731
    e_rhs, e_T = rel(merged("rhs"), ref["rhs"]), rel(merged("T_rhs"), ref["T_rhs"])
    dst = merged("dst")
    e_dst = np.linalg.norm(dst - ref["dst"]) / np.linalg.norm(ref["dst"])
    e_Tx = rel(merged("Tx"), ref["Tx"])
    print(f"rhs {e_rhs:.1e}, T rhs {e_T:.1e}, block preconditioner {e_dst:.1e} "
          f"(bitwise: {np.array_equal(dst, ref['dst'])}), T CG {ref['T'][1]} vs "
          f"{[r['T'][1] for r in results]}, T solution {e_Tx:.1e}")
    assert e_rhs < 1e-12 and e_T < 1e-12
    assert ref["inner"] == 56 and all(r["inner"] == 56 for r in results)
    assert all(r["mp"]["built"] for r in results)
    assert e_dst < 1e-10
    assert all(abs(r["T"][1] - ref["T"][1]) <= 1 for r in results)
    assert e_Tx < 1e-10
    assert peak[0] < 250.0
