"""B^T by rows (k_bt_coltab + k_bt_tasks) with the rhs in cell order (pencil +
gather), the same with the per-colour rhs kernel (DCP_ASM_RHS_CELL_ORDER=0)
and the cell scatter (DCP_BT_ROWS=0) at refine R (default 5):
assemble_nse_system time per variant, max relative differences."""
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
out = {"refine": R}
res = {}
for variant, env in (("1", {"DCP_BT_ROWS": "1", "DCP_ASM_RHS_CELL_ORDER": "1", "DCP_BT_SLOTS": "8"}),
                     ("16", {"DCP_BT_ROWS": "1", "DCP_ASM_RHS_CELL_ORDER": "1", "DCP_BT_SLOTS": "16"}),
                     ("h", {"DCP_BT_ROWS": "1", "DCP_ASM_RHS_CELL_ORDER": "0", "DCP_BT_SLOTS": "8"}),
                     ("0", {"DCP_BT_ROWS": "0", "DCP_ASM_RHS_CELL_ORDER": "1", "DCP_BT_SLOTS": "8"})):
    os.environ.update(env)
    ctx = dcp.Context()
    ctx.set_physics(dcp.classic_physics())
    ctx.upload_mesh(m)
    ctx.set_state(dcp.OLD_NSE_SOLUTION, u)
    ctx.set_state(dcp.OLD_T_SOLUTION, m.T0)
    ms = []
    for _ in range(6):
        ctx.assemble_nse_system()
        ms.append(ctx.timings()["assemble_nse_ms"])
    rp, ci, v = ctx.coupling_csr("Bt")
    res[variant] = (v, ctx.get_state(dcp.NSE_RHS))
    out[{"1": "ms_bt_rows", "16": "ms_bt_rows_16_slots", "h": "ms_bt_rows_halfwave_rhs",
         "0": "ms_cell_scatter"}[variant]] = \
        [round(x, 4) for x in ms]
    ctx.close()
(v1, r1), (v0, r0) = res["1"], res["0"]
out["bt_rel_max"] = float(np.max(np.abs(v1 - v0)) / np.max(np.abs(v0)))
out["rhs_bitwise"] = bool(np.array_equal(r1, r0))
out["rhs_rel_max"] = float(np.max(np.abs(r1 - r0)) / np.max(np.abs(r0)))
out["rhs_halfwave_bitwise_cell_scatter"] = bool(np.array_equal(res["h"][1], r0))
out["bt_16_bitwise_8_slots"] = bool(np.array_equal(res["1"][0], res["16"][0]))
print(json.dumps(out), flush=True)
