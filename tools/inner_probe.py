"""Times the inner Schur GMRES (dcp_block_preconditioner_vmult on device
buffers) at refine R for every build/var/libdcp_*.so: one JSON line per
variant with microseconds per inner iteration (median of 4 calls)."""
import ctypes as C
import glob
import hashlib
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
    if os.environ.get("GS"):
        ctx.set_gram_schmidt(os.environ["GS"])
    ctx.upload_mesh(m)
    ctx.set_state(dcp.OLD_NSE_SOLUTION, np.zeros(m.n_u + m.n_p))
    ctx.set_state(dcp.OLD_T_SOLUTION, m.T0)
    ctx.assemble_nse_system()
    ctx.build_nse_preconditioner()
    n = m.n_u + m.n_p
    x = np.random.default_rng(1).uniform(-1, 1, n)
    x[m.n_u:] -= x[m.n_u:].mean()
    per = []
    with dcp.DeviceBuffer(n) as ds, dcp.DeviceBuffer(n) as dd:
        ds.upload(x)
        for rep in range(int(os.environ.get("REPS", "5"))):
            it = C.c_int(0)
            hip.hipDeviceSynchronize()
            t0 = time.perf_counter()
            dcp.lib().dcp_block_preconditioner_vmult(ctx._h, C.c_void_p(ds.ptr),
                                                     C.c_void_p(dd.ptr), 0, C.byref(it))
            hip.hipDeviceSynchronize()
            dt = time.perf_counter() - t0
            if rep:
                per.append(dt / max(it.value, 1) * 1e6)
        digest = hashlib.sha1(dd.download().tobytes()).hexdigest()[:12]
    print(json.dumps({"variant": os.path.basename(path), "inner_its": it.value,
                      "us_per_inner_it": float(np.median(per)), "result_sha1": digest}),
          flush=True)
    ctx.close()
