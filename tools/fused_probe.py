"""Fused vs per-step Gram-Schmidt chain on one block-preconditioner apply,
optionally with the re-orthogonalisation forced (DCP_TEST_FORCE_REORTH_AT)."""
import hashlib
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "3d-dycoreplanet_amd"))
import numpy as np  # noqa: E402
import dcp  # noqa: E402

R = int(os.environ.get("R", "2"))
m = dcp.HostMesh(refine=R)
x = np.random.default_rng(20261015 + R).uniform(-1, 1, m.n_u + m.n_p)
ctx = dcp.Context()
ctx.set_physics(dcp.classic_physics())
ctx.upload_mesh(m)
ctx.set_state(dcp.OLD_NSE_SOLUTION, np.zeros(m.n_u + m.n_p))
ctx.set_state(dcp.OLD_T_SOLUTION, m.T0)
ctx.assemble_nse_system()
ctx.build_nse_preconditioner()
for fused in (True, False, True, False):
    ctx.set_fused_chain(fused)
    y, it = ctx.block_preconditioner_vmult(x)
    print(os.environ.get("DCP_TEST_FORCE_REORTH_AT"), "fused" if fused else "per-step", it,
          hashlib.sha1(y.tobytes()).hexdigest()[:10], float(y[-1]), flush=True)
