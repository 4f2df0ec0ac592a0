"""Phase timing of the DCGS2 step kernel (k_dcgs2_step) from the per-workgroup
realtime stamps of a -DDCP_DCGS_TIMING=k probe build (build/var/libdcp_ts<k>.so,
tools/variant_probe.sh SRC=krylov): entry spread (dispatch ramp), loads +
local products, hand-over publish, result wait, update, bookkeeping, in us."""
import ctypes as C
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
for path in sorted(glob.glob(os.path.join(os.path.dirname(dcp.__file__), "build/var/libdcp_ts*.so"))):
    dcp._lib = dcp.load_library(path)
    ctx = dcp.Context(device=0)
    ctx.set_physics(dcp.classic_physics())
    ctx.set_gram_schmidt("dcgs2")
    ctx.upload_mesh(m)
    ctx.set_state(dcp.OLD_NSE_SOLUTION, np.zeros(m.n_u + m.n_p))
    ctx.set_state(dcp.OLD_T_SOLUTION, m.T0)
    ctx.assemble_nse_system()
    ctx.build_nse_preconditioner()
    ctx.set_inner_max_steps(28)
    x = np.random.default_rng(1).uniform(-1, 1, m.n_u + m.n_p)
    x[m.n_u:] -= x[m.n_u:].mean()
    res = []
    for rep in range(6):
        ctx.block_preconditioner_vmult(x)
        ts = np.zeros(256 * 8, dtype=np.uint64)
        dcp.lib().dcp_probe_dcgs_timestamps(ts.ctypes.data_as(C.c_void_p))
        ts = ts.reshape(256, 8).astype(np.float64) / 100.0  # 100 MHz -> us
        nb = int(np.count_nonzero(ts[:, 0]))
        t = ts[:nb] - ts[:nb, 0].min()
        res.append({"workgroups": nb, "entry_spread": float(t[:, 0].max()),
                    "loads_products_med": float(np.median(t[:, 1] - t[:, 0])),
                    "loads_products_max": float((t[:, 1] - t[:, 0]).max()),
                    "last_publish": float(t[:, 2].max()),
                    "reducers_done": float(t[:64, 3].max()),
                    "results_first": float(t[:, 4].min()), "results_last": float(t[:, 4].max()),
                    "update_med": float(np.median(t[:, 5] - t[:, 4])),
                    "end_last": float(t[:, 5].max()), "bookkeeping": float(t[0, 6] - t[0, 5])})
    print(json.dumps({"variant": os.path.basename(path), "runs": res[2:]}), flush=True)
    ctx.close()
