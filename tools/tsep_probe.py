#!/usr/bin/env python3
"""Timing variants of the separable temperature assembly (DCP_TSEP_PROBE bits,
kernels/temperature_sep.hip) on the refine-R shell: per variant the median of
REPS assemble_temperature_matrix / _rhs phase times (HIP events around each
call). Probe values are diagnostic only (their results are wrong)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-dycoreplanet_amd"))
import numpy as np  # noqa: E402
import dcp  # noqa: E402

R = int(os.environ.get("R", "5"))
REPS = int(os.environ.get("REPS", "20"))
PROBES = [int(x) for x in os.environ.get("PROBES", "0,1,2,3,4,6,8,32,40").split(",")]
PTS = [x for x in os.environ.get("PTS", "4").split(",")]
m = dcp.HostMesh(refine=R)
ctx = dcp.Context()
ctx.set_physics(dcp.classic_physics())
ctx.upload_mesh(m)
ctx.set_state(dcp.OLD_T_SOLUTION, m.T0)
ctx.set_state(dcp.NSE_SOLUTION, np.random.default_rng(1).uniform(-1, 1, m.n_u + m.n_p))
print("layout", ctx.temperature_layout(), flush=True)
for pt, p in [(pt, p) for pt in PTS for p in PROBES]:
    os.environ["DCP_TSEP_PROBE"] = str(p)
    os.environ["DCP_TSEP_PT"] = pt
    tm, tr = [], []
    for _ in range(REPS):
        ctx.assemble_temperature_matrix()
        ctx.assemble_temperature_rhs()
        t = ctx.timings()
        tm.append(t["assemble_T_matrix_ms"])
        tr.append(t["assemble_T_rhs_ms"])
    print(f"pt {pt} probe {p:3d}: matrix {np.median(tm[2:]) * 1e3:8.1f} us  rhs {np.median(tr[2:]) * 1e3:8.1f} us",
          flush=True)
os.environ["DCP_TSEP_PROBE"] = "0"
ctx.close()
