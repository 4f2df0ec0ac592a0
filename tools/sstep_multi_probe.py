"""The s-step block in its three-launch form (DCP_OPT_FUSED_CHAIN = 0) at
refine R: 50 inner iterations of one block_preconditioner_vmult, timed, with
the residual reduction. Usage: R=5 python3 tools/sstep_multi_probe.py"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "3d-dycoreplanet_amd"))
import numpy as np  # noqa: E402
import dcp  # noqa: E402

R = int(os.environ.get("R", "5"))
m = dcp.HostMesh(refine=R)
ctx = dcp.Context()
ctx.set_physics(dcp.classic_physics())
ctx.set_gram_schmidt(os.environ.get("GS", "sstep"))
ctx.upload_mesh(m)
ctx.set_fused_chain(os.environ.get("FUSED", "0") == "1")
n = m.n_u + m.n_p
ctx.set_state(dcp.OLD_NSE_SOLUTION, np.zeros(n))
ctx.set_state(dcp.OLD_T_SOLUTION, m.T0)
ctx.assemble_nse_system()
ctx.build_nse_preconditioner()
ctx.set_inner_max_steps(int(os.environ.get("STEPS", "50")))
p = np.random.default_rng(6).uniform(-1, 1, m.n_p)
src = np.zeros(n)
src[m.n_u:] = p - p.mean()
print("R", R, "n_p", m.n_p, "start", flush=True)
t0 = time.perf_counter()
dst, its = ctx.block_preconditioner_vmult(src)
dt = time.perf_counter() - t0
r = ctx.schur_vmult(dst[m.n_u:]) - src[m.n_u:]
print("R", R, "its", its, "s", round(dt, 4), "residual reduction",
      float(np.linalg.norm(r) / np.linalg.norm(src[m.n_u:])), flush=True)
ctx.close()
