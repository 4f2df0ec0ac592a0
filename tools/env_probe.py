"""assemble_nse_system at refine R under each value of an environment switch
read at assembly or upload time (`python3 tools/env_probe.py VAR v1 v2 ...`,
a fresh context per value): one JSON line per value, median of REPS, B^T and
the rhs bitwise against the first value."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "3d-dycoreplanet_amd"))
import numpy as np  # noqa: E402
import dcp  # noqa: E402

R = int(os.environ.get("R", "5"))
REPS = int(os.environ.get("REPS", "12"))
var, values = sys.argv[1], sys.argv[2:]
m = dcp.HostMesh(refine=R)
ref = None
for val in values:
    os.environ[var] = val
    ctx = dcp.Context(device=0)
    ctx.set_physics(dcp.classic_physics())
    ctx.upload_mesh(m)
    ctx.set_state(dcp.OLD_NSE_SOLUTION, np.zeros(m.n_u + m.n_p))
    ctx.set_state(dcp.OLD_T_SOLUTION, m.T0)
    ms = []
    for _ in range(REPS):
        ctx.assemble_nse_system()
        ms.append(ctx.timings()["assemble_nse_ms"])
    bt = ctx.coupling_csr("Bt")[2]
    rhs = ctx.get_state(dcp.NSE_RHS)
    if ref is None:
        ref = (bt, rhs)
    same = bool(np.array_equal(bt, ref[0]) and np.array_equal(rhs, ref[1]))
    ctx.close()
    print(json.dumps({var: val, "ms_median": float(np.median(ms[2:])), "ms": ms,
                      "bitwise_first": same}), flush=True)
