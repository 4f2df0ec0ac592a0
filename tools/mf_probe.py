"""Times the matrix-free Stokes apply (dcp_nse_vmult, DCP_OPT_MATRIX_FREE) at
refine R for every build/var/libdcp_*.so (tools/variant_probe.sh), device
buffers only: one JSON line per variant (median over batches of 20 applies)."""
import ctypes as C
import glob
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "3d-dycoreplanet_amd"))
import numpy as np  # noqa: E402
import dcp  # noqa: E402

R = int(os.environ.get("R", "5"))
m = dcp.HostMesh(refine=R)
hip = C.CDLL("libamdhip64.so")
libs = sorted(glob.glob(os.path.join(os.path.dirname(dcp.__file__),
                                   "build/var/libdcp_%s.so" % os.environ.get("VAR", "*"))))
for path in libs or [dcp.LIB_PATH]:
    dcp._lib = dcp.load_library(path)
    ctx = dcp.Context(device=0)
    ctx.set_physics(dcp.classic_physics())
    ctx.upload_mesh(m)
    ctx.set_state(dcp.OLD_NSE_SOLUTION, np.zeros(m.n_u + m.n_p))
    ctx.set_state(dcp.OLD_T_SOLUTION, m.T0)
    ctx.assemble_nse_system()
    n = m.n_u + m.n_p
    x = np.random.default_rng(1).uniform(-1, 1, n)
    res = {}
    for mf in (1, 2, 0):
        ctx.set_matrix_free(mf)
        with dcp.DeviceBuffer(n) as ds, dcp.DeviceBuffer(n) as dd:
            ds.upload(x)
            f = dcp.lib().dcp_nse_vmult
            for _ in range(3):
                f(ctx._h, C.c_void_p(ds.ptr), C.c_void_p(dd.ptr))
            hip.hipDeviceSynchronize()
            ts = []
            for _ in range(5):
                t0 = time.perf_counter()
                for _ in range(20):
                    f(ctx._h, C.c_void_p(ds.ptr), C.c_void_p(dd.ptr))
                hip.hipDeviceSynchronize()
                ts.append((time.perf_counter() - t0) / 20 * 1e3)
            y = dd.download()
        res[{1: "mf", 2: "mf_colour", 0: "assembled"}[mf]] = (float(np.median(ts)), y)
    ya = res["assembled"][1]
    d = {k: float(np.max(np.abs(v[1] - ya)) / np.max(np.abs(ya))) for k, v in res.items()}
    print(json.dumps({"variant": os.path.basename(path), "R": R,
                      **{k + "_ms": v[0] for k, v in res.items()},
                      "rel_diff": d}), flush=True)
    ctx.close()
