"""Assembles the refine-5 shell a few times with the library named by VAR
(build/var/libdcp_<VAR>.so, tools/variant_probe.sh) for counter passes."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "3d-dycoreplanet_amd"))
import numpy as np  # noqa: E402
import dcp  # noqa: E402

var = os.environ.get("VAR")
if var:
    dcp._lib = dcp.load_library(os.path.join(os.path.dirname(dcp.__file__),
                                             f"build/var/libdcp_{var}.so"))
m = dcp.HostMesh(refine=int(os.environ.get("R", "5")))
ctx = dcp.Context(device=0)
ctx.set_physics(dcp.classic_physics())
ctx.upload_mesh(m)
ctx.set_state(dcp.OLD_NSE_SOLUTION, np.zeros(m.n_u + m.n_p))
ctx.set_state(dcp.OLD_T_SOLUTION, m.T0)
for _ in range(2):
    ctx.assemble_nse_system()
print(ctx.timings()["assemble_nse_ms"])
ctx.close()
