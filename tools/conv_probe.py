"""Convergence of solve_NSE_block_preconditioned (dcp_solve_nse) on the GPU
for the shell geometry variants: MappingQ(3) on boundary cells only (deal.II
9.2) or on all cells, and the no-normal-flux normals (consistent / radial /
deal.II mapped-face). One line per case: rc, FGMRES outer, Schur inner,
seconds. usage: R=2,3,4 python tools/conv_probe.py"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "3d-dycoreplanet_amd"))
import numpy as np  # noqa: E402
import dcp  # noqa: E402

Rs = [int(r) for r in os.environ.get("R", "2,3,4").split(",")]
modes = os.environ.get("MODES", "0:mapping,0:consistent,1:mapping,1:consistent,0:radial").split(",")
for R in Rs:
    for md in modes:
        allc, normals = md.split(":")
        m = dcp.HostMesh(refine=R, normals=normals, mapping_q_on_all_cells=allc == "1")
        ctx = dcp.Context(device=0)
        ctx.set_physics(dcp.classic_physics())
        ctx.upload_mesh(m)
        u = np.zeros(m.n_u + m.n_p)
        for f, v in ((dcp.OLD_NSE_SOLUTION, u), (dcp.NSE_SOLUTION, u), (dcp.OLD_T_SOLUTION, m.T0),
                     (dcp.T_SOLUTION, m.T0)):
            ctx.set_state(f, v)
        ctx.assemble_nse_system()
        ctx.build_nse_preconditioner()
        t0 = time.perf_counter()
        rc, outer, inner = ctx.solve_nse()
        print("r=%d all_cells=%s normals=%-10s rc=%d outer=%d inner=%d %.2fs"
              % (R, allc, normals, rc, outer, inner, time.perf_counter() - t0), flush=True)
        ctx.close()
