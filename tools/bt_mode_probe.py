#!/usr/bin/env python3
"""assemble_nse_system at refine R under the k_bt_tasks store / placement
modes (DCP_BT_MODE, assembly.hip): median assembly time per mode over
alternating rounds, and a digest of B^T (every mode must be bitwise equal)."""
import hashlib
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "3d-dycoreplanet_amd"))
import numpy as np  # noqa: E402
import dcp  # noqa: E402

R = int(os.environ.get("R", "5"))
MODES = [int(x) for x in os.environ.get("MODES", "0,1,2,3").split(",")]
m = dcp.HostMesh(refine=R)
rng = np.random.default_rng(1)
u = np.zeros(m.n_u + m.n_p)
u[:m.n_u] = 0.05 * rng.uniform(-1, 1, m.n_u)
ctx = dcp.Context()
ctx.set_physics(dcp.classic_physics())
ctx.upload_mesh(m)
ctx.set_state(dcp.OLD_NSE_SOLUTION, u)
ctx.set_state(dcp.OLD_T_SOLUTION, m.T0)
times = {md: [] for md in MODES}
digest = {}
for rnd in range(4):
    for md in MODES:
        os.environ["DCP_BT_MODE"] = str(md)
        for _ in range(8):
            ctx.assemble_nse_system()
            times[md].append(ctx.timings()["assemble_nse_ms"])
        if rnd == 0:
            digest[md] = hashlib.sha256(ctx.coupling_csr("Bt")[2].tobytes()).hexdigest()[:16]
for md in MODES:
    t = times[md]
    print(f"mode {md}: median {np.median(t) * 1e3:.1f} us  min {np.min(t) * 1e3:.1f} us  "
          f"B^T digest {digest[md]}", flush=True)
ctx.close()
