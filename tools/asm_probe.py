"""Times assemble_nse_system at refine R (default 5) and prints a checksum of
the assembled matrix at refine 3 (to compare kernel variants bit for bit)."""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "3d-dycoreplanet_amd"))
import numpy as np  # noqa: E402
import dcp  # noqa: E402


def run(refine, reps, export=False):
    m = dcp.HostMesh(refine=refine)
    ctx = dcp.Context(device=0)
    ctx.set_physics(dcp.classic_physics())
    ctx.upload_mesh(m)
    ctx.set_state(dcp.OLD_NSE_SOLUTION, np.zeros(m.n_u + m.n_p))
    ctx.set_state(dcp.OLD_T_SOLUTION, m.T0)
    ms = []
    for _ in range(reps):
        ctx.assemble_nse_system()
        ms.append(ctx.timings()["assemble_nse_ms"])
    h = None
    if export:
        rp, ci, v = ctx.nse_matrix_csr()
        h = hashlib.sha1(np.ascontiguousarray(v).tobytes()).hexdigest()[:16]
        h += "/" + hashlib.sha1(ctx.get_state(dcp.NSE_RHS).tobytes()).hexdigest()[:8]
    ctx.close()
    return ms, h


ms3, h3 = run(3, 2, export=True)
ms, _ = run(int(os.environ.get("R", "5")), 4)
print(json.dumps({"variant": os.environ.get("DCP_ASM_WRITE", "0"), "ms": ms, "hash_r3": h3}),
      flush=True)
