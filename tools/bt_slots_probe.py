"""assemble_nse_system at refine R with the B^T tasks of 16 (default), 32
(128 entries, two per lane) and 8 slots (DCP_BT_SLOTS, read at upload): one
JSON line per setting, median of reps, B^T and the rhs bitwise against 16."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "3d-dycoreplanet_amd"))
import numpy as np  # noqa: E402
import dcp  # noqa: E402

R = int(os.environ.get("R", "5"))
m = dcp.HostMesh(refine=R)
ref = None
for sl in ("16", "32", "8", "16"):
    os.environ["DCP_BT_SLOTS"] = sl
    ctx = dcp.Context(device=0)
    ctx.set_physics(dcp.classic_physics())
    ctx.upload_mesh(m)
    ctx.set_state(dcp.OLD_NSE_SOLUTION, np.zeros(m.n_u + m.n_p))
    ctx.set_state(dcp.OLD_T_SOLUTION, m.T0)
    ms = []
    for _ in range(8):
        ctx.assemble_nse_system()
        ms.append(ctx.timings()["assemble_nse_ms"])
    bt = ctx.coupling_csr("Bt")[2]
    rhs = ctx.get_state(dcp.NSE_RHS)
    if ref is None:
        ref = (bt, rhs)
    same = bool(np.array_equal(bt, ref[0]) and np.array_equal(rhs, ref[1]))
    ctx.close()
    print(json.dumps({"slots": sl, "ms_median": float(np.median(ms[2:])), "ms": ms,
                      "bitwise_16": same}), flush=True)
