"""Back-to-back operator applies at refine R (default 5) on device buffers,
one HIP event pair per batch (dcp_time_operator): ms per apply of the
matrix-free Stokes operator, its velocity block and the Schur complement,
batches of REPS applies, BATCHES times. One JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "3d-dycoreplanet_amd"))
import numpy as np  # noqa: E402
import dcp  # noqa: E402

R = int(os.environ.get("R", "5"))
REPS = int(os.environ.get("REPS", "20"))
BATCHES = int(os.environ.get("BATCHES", "5"))
m = dcp.HostMesh(refine=R)
ctx = dcp.Context()
ctx.set_physics(dcp.classic_physics())
ctx.upload_mesh(m)
rng = np.random.default_rng(3)
u = np.zeros(m.n_u + m.n_p)
u[:m.n_u] = 0.05 * rng.uniform(-1, 1, m.n_u)
ctx.set_state(dcp.OLD_NSE_SOLUTION, u)
ctx.set_state(dcp.OLD_T_SOLUTION, m.T0)
ctx.assemble_nse_system()
ctx.build_nse_preconditioner()
n = m.n_u + m.n_p
out = {"refine": R, "reps": REPS}
NVEC = int(os.environ.get("NVEC", "8"))  # 8 x 40 MB sources: more than the 256 MB cache
lens = {"nse": n, "velocity": m.n_u, "schur": m.n_p}
with dcp.DeviceBuffer(n * NVEC) as s, dcp.DeviceBuffer(n * NVEC) as d:
    s.upload(rng.uniform(-1, 1, n * NVEC))
    for which in ("nse", "velocity", "schur"):
        for nv in (1, NVEC):
            ms = [ctx.time_operator(which, REPS, s.ptr, d.ptr, nv) for _ in range(BATCHES)]
            out["%s_ms_nvec%d" % (which, nv)] = [round(x, 5) for x in ms]
out["nvec"] = NVEC
ctx.close()
print(json.dumps(out), flush=True)
