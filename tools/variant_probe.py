"""Times assemble_nse_system at refine R for every build/var/libdcp_k.so
(tools/variant_probe.sh): one JSON line per variant, median of reps."""
import glob
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
for path in sorted(glob.glob(os.path.join(os.path.dirname(dcp.__file__),
                                         "build/var/libdcp_%s.so" % os.environ.get("VAR", "*")))):
    dcp._lib = dcp.load_library(path)
    ctx = dcp.Context(device=0)
    ctx.set_physics(dcp.classic_physics())
    ctx.upload_mesh(m)
    if os.environ.get("VB") == "1":  # time the full scatter with the velocity block
        ctx.set_assemble_velocity_block(True)
    ctx.set_state(dcp.OLD_NSE_SOLUTION, np.zeros(m.n_u + m.n_p))
    ctx.set_state(dcp.OLD_T_SOLUTION, m.T0)
    ms = []
    for _ in range(int(os.environ.get("REPS", "6"))):
        ctx.assemble_nse_system()
        ms.append(ctx.timings()["assemble_nse_ms"])
    # B^T and the rhs bitwise against the first variant
    bt = ctx.coupling_csr("Bt")[2]
    rhs = ctx.get_state(dcp.NSE_RHS)
    if ref is None:
        ref = (bt, rhs)
    same = bool(np.array_equal(bt, ref[0]) and np.array_equal(rhs, ref[1]))
    ctx.close()
    print(json.dumps({"variant": os.path.basename(path), "ms_median": float(np.median(ms[1:])),
                      "ms": ms, "bitwise_first_variant": same}), flush=True)
