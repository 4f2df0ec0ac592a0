"""Diagnostics of the in-process multi-rank time step vs one GPU (r=2)."""
import os
import sys
import threading

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "3d-dycoreplanet_amd"))
import dcp  # noqa: E402
from test_multi_rank import _time_step  # noqa: E402

world = int(os.environ.get("W", "2"))
explicit = os.environ.get("EXPLICIT", "1") == "1"
m = dcp.HostMesh(refine=int(os.environ.get("R", "2")))
ph = dcp.classic_physics()
rng = np.random.default_rng(7)
u = np.zeros(m.n_u + m.n_p)
u[:m.n_u] = 0.05 * rng.uniform(-1, 1, m.n_u)
T = m.T0.copy()
ctx = dcp.Context()
ctx.set_physics(ph)
ctx.set_schur_explicit(explicit)
ctx.upload_mesh(m)
ref = _time_step(ctx, m, u, T)
ctx.close()
g = dcp.Group(world)
res = [None] * world


def run(r):
    c = dcp.Context(rank=r, world_size=world, group=g)
    c.set_physics(ph)
    c.set_schur_explicit(explicit)
    c.upload_mesh(m)
    res[r] = _time_step(c, m, u, T)
    c.close()


th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
[t.start() for t in th]
[t.join() for t in th]
for k in ("x", "Tx", "rhs"):
    v = np.zeros_like(ref[k])
    for r in res:
        nz = r[k] != 0
        v[nz] = r[k][nz]
    d = v - ref[k]
    if k == "x":
        nu = m.n_u
        print("vel rel", np.linalg.norm(d[:nu]) / np.linalg.norm(ref[k][:nu]),
              "p rel", np.linalg.norm(d[nu:]) / np.linalg.norm(ref[k][nu:]),
              "p mean diff", d[nu:].mean(), "p rel (mean-free)",
              np.linalg.norm(d[nu:] - d[nu:].mean()) / np.linalg.norm(ref[k][nu:]))
        print("zeros merged", np.sum(v == 0), np.sum(ref[k] == 0))
    print(k, np.linalg.norm(d) / np.linalg.norm(ref[k]))
print("ref iters", ref["nse"], ref["T"], [r["nse"] for r in res], [r["T"] for r in res])
