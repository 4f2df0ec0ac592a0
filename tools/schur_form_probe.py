"""Times build_nse_preconditioner (the explicit S = B D_A^-1 B^T formation,
k_schur_form) at refine R for every build/var/libdcp_*.so, and checks the
formed S bitwise across variants through S x for a fixed x."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "3d-dycoreplanet_amd"))
import glob  # noqa: E402
import numpy as np  # noqa: E402
import dcp  # noqa: E402

R = int(os.environ.get("R", "5"))
m = dcp.HostMesh(refine=R)
ref = None
x = np.random.default_rng(3).uniform(-1, 1, m.n_p)
for path in sorted(glob.glob(os.path.join(os.path.dirname(dcp.__file__), "build/var/libdcp_*.so"))) \
        or [dcp.LIB_PATH]:
    dcp._lib = dcp.load_library(path)
    ctx = dcp.Context(device=0)
    ctx.set_physics(dcp.classic_physics())
    ctx.upload_mesh(m)
    ctx.set_state(dcp.OLD_NSE_SOLUTION, np.zeros(m.n_u + m.n_p))
    ctx.set_state(dcp.OLD_T_SOLUTION, m.T0)
    ctx.assemble_nse_system()
    ms = []
    for _ in range(5):
        ctx.build_nse_preconditioner()
        ms.append(ctx.timings()["build_precond_ms"])
    y = ctx.schur_vmult(x)
    if ref is None:
        ref = y
    ctx.close()
    print(json.dumps({"variant": os.path.basename(path), "build_precond_ms": ms,
                      "bitwise_first_variant": bool(np.array_equal(y, ref))}), flush=True)
