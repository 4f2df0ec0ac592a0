"""Repeats one NSE solve per configuration and prints (rc, outer, inner, hash)
of every run: a configuration whose lines differ is nondeterministic."""
import hashlib
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "3d-dycoreplanet_amd"))
import numpy as np  # noqa: E402
import dcp  # noqa: E402

R = int(os.environ.get("R", "1"))
REPS = int(os.environ.get("REPS", "4"))
m = dcp.HostMesh(refine=R)
u = np.zeros(m.n_u + m.n_p)
for name, env, fused in (("all on", {}, True), ("per-step chain", {}, False),
                         ("events", {"DCP_SCHUR_READY_FLAG": "0"}, True),
                         ("no ahead", {"DCP_SCHUR_AHEAD": "0"}, True),
                         ("no ahead, per-step", {"DCP_SCHUR_AHEAD": "0"}, False)):
    for k in ("DCP_SCHUR_READY_FLAG", "DCP_SCHUR_AHEAD"):
        os.environ.pop(k, None)
    os.environ.update(env)
    ctx = dcp.Context()
    ctx.set_physics(dcp.classic_physics())
    ctx.upload_mesh(m)
    ctx.set_fused_chain(fused)
    ctx.set_state(dcp.OLD_NSE_SOLUTION, u)
    ctx.set_state(dcp.OLD_T_SOLUTION, m.T0)
    ctx.assemble_nse_system()
    ctx.build_nse_preconditioner()
    out = []
    xin = np.random.default_rng(7).uniform(-1, 1, m.n_u + m.n_p)
    for r in range(REPS):
        if os.environ.get("MODE") == "prec":
            x, inner = ctx.block_preconditioner_vmult(xin, do_solve_A=False)
            out.append((inner, hashlib.sha1(x.tobytes()).hexdigest()[:10],
                        float(np.abs(x[m.n_u:]).max())))
            continue
        ctx.set_state(dcp.NSE_SOLUTION, u)
        rc, outer, inner = ctx.solve_nse()
        x = ctx.get_state(dcp.NSE_SOLUTION)
        out.append((rc, outer, inner, hashlib.sha1(x.tobytes()).hexdigest()[:10]))
    print(name, out, flush=True)
    ctx.close()
