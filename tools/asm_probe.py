"""assemble_nse_system at refine R (default 5) with the default options, six
times (a PMC / kernel-statistics target: one configuration only)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "3d-dycoreplanet_amd"))
import numpy as np  # noqa: E402
import dcp  # noqa: E402

R = int(os.environ.get("R", "5"))
m = dcp.HostMesh(refine=R)
rng = np.random.default_rng(1)
u = np.zeros(m.n_u + m.n_p)
u[:m.n_u] = 0.05 * rng.uniform(-1, 1, m.n_u)
ctx = dcp.Context()
ctx.set_physics(dcp.classic_physics())
ctx.upload_mesh(m)
ctx.set_state(dcp.OLD_NSE_SOLUTION, u)
ctx.set_state(dcp.OLD_T_SOLUTION, m.T0)
ms = []
for _ in range(6):
    ctx.assemble_nse_system()
    ms.append(round(ctx.timings()["assemble_nse_ms"], 4))
ctx.close()
print(json.dumps({"refine": R, "assemble_nse_ms": ms}), flush=True)
