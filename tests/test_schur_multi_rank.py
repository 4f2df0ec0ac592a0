"""The Schur-complement solver (solve_NSE_Schur_complement,
boussinesq_model.tpp:1248-1414) on several ranks, as the cube prm (BASELINE
C2) runs it under MPI: Trilinos' PreconditionILU has zero overlap, so each
rank factors ILU(0) of its owned diagonal block of A (block Jacobi over the
ranks) and the preconditioner -- hence the iterates -- depend on the
partition. The oracle restates exactly that (orc_set_ilu_blocks: the couplings
between ranks dropped before the factorisation) for the library's partition
(the owner of a dof is the rank of the lowest cell that has it, cells split in
equal contiguous ranges).

CPU: that ownership rule reproduces the partition's owned counts.
GPU: in-process groups of 2 and 3 ranks on the periodic cube and the shell
against the oracle with the same blocks, inner CGs held at k steps
(DCP_OPT_SCHUR_FIXED_INNER): equal Schur GMRES / A^-1 counts, solution at 1e-10."""
import os
import threading

import numpy as np
import pytest

import dcp
import oracle_py

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CUBE_PRM = os.path.join(ROOT, "configs", "aqua_planet_cube_test_3d.prm")


def velocity_owner(m, world):
    """The rank owning every velocity dof (partition.cpp: the rank of the lowest
    cell holding the support point; rank r owns cells [r N / P, (r + 1) N / P))."""
    start = [r * m.n_cells // world for r in range(world + 1)]
    node_owner = np.full(m.n_u // 3, -1, np.int64)
    r = 0
    for c in range(m.n_cells):
        while c >= start[r + 1]:
            r += 1
        d = m.cell_nse_dofs[c]
        nodes = d[d < m.n_u] // 3
        new = nodes[node_owner[nodes] < 0]
        node_owner[new] = r
    return np.repeat(node_owner, 3).astype(np.int32)


def case(name):
    if name.startswith("cube"):
        rp = dcp.load_prm(CUBE_PRM)
        return dcp.HostMesh(cuboid=True, refine=2, length=rp.length), dcp.physics_from_params(rp)
    return dcp.HostMesh(refine=2), dcp.classic_physics()


@pytest.mark.parametrize("name,world", [("cube", 2), ("cube", 3), ("shell", 3)])
def test_velocity_owner_rule_matches_the_partition(name, world):
    m, _ = case(name)
    owner = velocity_owner(m, world)
    for r in range(world):
        assert int(np.sum(owner == r)) // 3 == dcp.partition_info(m, r, world)["nvo"]


@pytest.mark.gpu
@pytest.mark.parametrize("name,world,k", [("cube", 2, 8), ("cube", 3, 8), ("shell", 2, 40),
                                          ("shell", 8, 40)])
def test_group_schur_solver_block_jacobi_ilu_matches_oracle(name, world, k):
    m, ph = case(name)
    rng = np.random.default_rng(23)
    u = 0.1 * rng.uniform(-1, 1, m.n_u + m.n_p)
    T = m.T0 + 0.05 * rng.uniform(-1, 1, m.n_T)
    g = dcp.Group(world)
    results, errors = [None] * world, []

    def run(rank):
        try:
            ctx = dcp.Context(rank=rank, world_size=world, group=g)
            ctx.set_physics(ph)
            ctx.upload_mesh(m)
            ctx.set_schur_fixed_inner(k)
            for f, v in ((dcp.OLD_NSE_SOLUTION, u), (dcp.NSE_SOLUTION, u),
                         (dcp.OLD_T_SOLUTION, T), (dcp.T_SOLUTION, T)):
                ctx.set_state(f, v)
            ctx.assemble_nse_system()
            rc, its, na = ctx.solve_nse_schur()
            results[rank] = (rc, its, na, ctx.get_state(dcp.NSE_SOLUTION),
                             ctx.get_state(dcp.OLD_NSE_SOLUTION))
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
    x = np.zeros(m.n_u + m.n_p)
    u_old = np.zeros(m.n_u + m.n_p)
    for r in results:
        nz = r[3] != 0
        x[nz] = r[3][nz]
        nz = r[4] != 0
        u_old[nz] = r[4][nz]
    orc = oracle_py.Model(ph, m)
    orc.set_schur_fixed_inner(k)
    orc.set_ilu_blocks(velocity_owner(m, world))
    orc.assemble_nse_system(u_old, T)
    rco, xo, itso, nao = orc.solve_nse_schur(u_old)
    print(name, world, "Schur GMRES", itso, "A^-1 solves", nao,
          "rel2", np.linalg.norm(x - xo) / np.linalg.norm(xo))
    for rc, its, na, _, _ in results:
        assert rc == rco and (its, na) == (itso, nao)
    assert np.linalg.norm(x - xo) <= 1e-10 * np.linalg.norm(xo)
