"""The 2D model (Standard::BoussinesqModel<2>, data/aqua_planet_test_2d.prm)
on several ranks: dcp_mesh2d_upload on a P-rank context keeps the rank's
cells and two ghost layers (localize_2d: cells sharing a vertex), the
velocity as scalar owned / ghost dofs, halos for u, p and T.

CPU: every rank's local mesh passes the 2D upload's validation, halo lists
pair up, ownership covers every dof once (in-process and over gloo).
GPU (in-process groups on one GPU): the block-preconditioned step against one
GPU (assembly 1e-12, iterate 1e-10 with the inner GMRES held at k steps, equal
FGMRES counts, T 1e-10), and the Schur-complement solver (the prm's solver)
against the oracle's block-Jacobi ILU of the same partition at 1e-10."""
import os
import threading

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import dcp
import oracle_py

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
R0, R1, L = 1.0, 3.0, 0.1


def make_mesh(refine=2, cm=True):
    return dcp.HostMesh2D(refine=refine, R0=R0, R1=R1, length=L, temperature_degree=2,
                          cuthill_mckee=cm)


def physics():
    rp = dcp.load_prm(os.path.join(ROOT, "configs", "aqua_planet_test_2d.prm"))
    ph = dcp.physics_from_params(rp)
    ph.temperature_degree = 2
    return ph


def velocity_owner(m, world):
    """Rank of every (scalar) velocity dof: the rank of the lowest cell holding
    it (partition.cpp localize_2d; rank r owns cells [r N / P, (r + 1) N / P))."""
    start = [r * m.n_cells // world for r in range(world + 1)]
    owner = np.full(m.n_u, -1, np.int64)
    r = 0
    for c in range(m.n_cells):
        while c >= start[r + 1]:
            r += 1
        d = m.cell_nse_dofs[c]
        d = d[d < m.n_u]
        owner[d[owner[d] < 0]] = r
    return owner.astype(np.int32)


@pytest.mark.parametrize("refine,world", [(2, 2), (2, 3), (3, 8)])
def test_partition_2d_covers_and_pairs(refine, world):
    m = make_mesh(refine)
    infos = {f: [dcp.mesh2d_partition_info(m, r, world, f) for r in range(world)] for f in "upT"}
    i0 = infos["u"]
    assert sum(i["n_owned_cells"] for i in i0) == m.n_cells
    assert sum(i["nuo"] for i in i0) == m.n_u
    assert sum(i["npo"] for i in i0) == m.n_p
    assert sum(i["nTo"] for i in i0) == m.n_T
    owner = velocity_owner(m, world)
    for r in range(world):
        assert i0[r]["nuo"] == int(np.sum(owner == r))
    for f in "upT":
        for r, i in enumerate(infos[f]):
            for s, ids in i["send"].items():
                assert np.array_equal(ids, infos[f][s]["recv"][r])


def _gloo_2d_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = make_mesh(2)
        mine = {}
        for f in "upT":
            info = dcp.mesh2d_partition_info(m, rank, world, f)
            mine[f] = {"send": {k: v.tolist() for k, v in info["send"].items()},
                       "recv": {k: v.tolist() for k, v in info["recv"].items()}}
        allinfo = [None] * world
        dist.all_gather_object(allinfo, mine)
        ok = True
        for f in "upT":
            for s, ids in mine[f]["send"].items():
                ok &= allinfo[s][f]["recv"].get(rank, []) == ids
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


def test_partition_2d_halo_consistency_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gloo_2d_worker, args=(r, world, 29641, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}


def _group(world, body):
    g = dcp.Group(world)
    results, errors = [None] * world, []

    def run(rank):
        try:
            ctx = dcp.Context(rank=rank, world_size=world, group=g)
            results[rank] = body(ctx)
            ctx.close()
        except Exception as e:  # noqa: BLE001
            errors.append((rank, repr(e)))

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    g.close()
    assert not errors, errors
    return results


def merged(results, key, like):
    v = np.zeros_like(like)
    for r in results:
        nz = r[key] != 0
        v[nz] = r[key][nz]
    return v


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3, 8])
def test_group_2d_block_preconditioned_step_matches_single_gpu(world):
    m = make_mesh(2, cm=False)
    ph = physics()
    rng = np.random.default_rng(5)
    u = np.zeros(m.n_u + m.n_p)
    u[:m.n_u] = 0.05 * rng.uniform(-1, 1, m.n_u)
    T = m.T0.copy()

    def step(ctx):
        ctx.set_physics(ph)
        ctx.upload_mesh2d(m)
        ctx.set_block_fixed_inner(40)
        for f, v in ((dcp.OLD_NSE_SOLUTION, u), (dcp.NSE_SOLUTION, u),
                     (dcp.OLD_T_SOLUTION, T), (dcp.T_SOLUTION, T)):
            ctx.set_state(f, v)
        out = {}
        ctx.assemble_nse_system()
        out["rhs"] = ctx.get_state(dcp.NSE_RHS)
        ctx.build_nse_preconditioner()
        ctx.assemble_temperature_matrix()
        ctx.assemble_temperature_rhs()
        out["T_rhs"] = ctx.get_state(dcp.T_RHS)
        out["nse"] = ctx.solve_nse()
        out["x"] = ctx.get_state(dcp.NSE_SOLUTION)
        out["T"] = ctx.solve_temperature()
        out["Tx"] = ctx.get_state(dcp.T_SOLUTION)
        out["vmax"] = ctx.max_velocity()
        return out

    ref_ctx = dcp.Context()
    ref = step(ref_ctx)
    ref_ctx.close()
    results = _group(world, step)
    rel = lambda a, b: np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300)  # noqa: E731
    assert rel(merged(results, "rhs", ref["rhs"]), ref["rhs"]) < 1e-12
    assert rel(merged(results, "T_rhs", ref["T_rhs"]), ref["T_rhs"]) < 1e-12
    x = merged(results, "x", ref["x"])
    print("2D group", world, "FGMRES", ref["nse"][1], "inner", ref["nse"][2], "x rel2",
          np.linalg.norm(x - ref["x"]) / np.linalg.norm(ref["x"]))
    assert np.linalg.norm(x - ref["x"]) <= 1e-10 * np.linalg.norm(ref["x"])
    assert rel(merged(results, "Tx", ref["Tx"]), ref["Tx"]) < 1e-10
    for r in results:
        assert r["nse"][:3] == ref["nse"][:3]
        assert abs(r["T"][1] - ref["T"][1]) <= 1
        assert np.isclose(r["vmax"], ref["vmax"], rtol=1e-10)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3, 8])
def test_group_2d_schur_solver_block_jacobi_ilu_matches_oracle(world):
    m = make_mesh(2, cm=True)
    ph = physics()
    k = 40
    u0 = np.zeros(m.n_u + m.n_p)

    def solve(ctx):
        ctx.set_physics(ph)
        ctx.upload_mesh2d(m)
        ctx.set_schur_fixed_inner(k)
        for f, v in ((dcp.OLD_NSE_SOLUTION, u0), (dcp.NSE_SOLUTION, u0),
                     (dcp.OLD_T_SOLUTION, m.T0)):
            ctx.set_state(f, v)
        ctx.assemble_nse_system()
        rc, its, n_inv = ctx.solve_nse_schur()
        return {"rc": rc, "its": its, "n_inv": n_inv, "x": ctx.get_state(dcp.NSE_SOLUTION)}

    results = _group(world, solve)
    orc = oracle_py.Model(ph, m)
    orc.set_schur_fixed_inner(k)
    orc.set_ilu_blocks(velocity_owner(m, world))
    orc.assemble_nse_system(u0, m.T0)
    rco, xo, itso, n_invo = orc.solve_nse_schur(u0)
    x = merged(results, "x", xo)
    print("2D Schur group", world, itso, n_invo, np.linalg.norm(x - xo) / np.linalg.norm(xo))
    for r in results:
        assert r["rc"] == rco and (r["its"], r["n_inv"]) == (itso, n_invo)
    assert np.linalg.norm(x - xo) <= 1e-10 * np.linalg.norm(xo)
