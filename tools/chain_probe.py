"""Bitwise reproducibility of the inner Schur GMRES at refine R (default 5):
block_preconditioner_vmult (do_solve_A = false) three ways — fused chain twice,
per-step chain once — and, when they differ, where (first differing entry,
inner counts). usage: R=5 python tools/chain_probe.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "3d-dycoreplanet_amd"))
import numpy as np  # noqa: E402
import dcp  # noqa: E402

R = int(os.environ.get("R", "5"))
m = dcp.HostMesh(refine=R)
ctx = dcp.Context()
ctx.set_physics(dcp.classic_physics())
ctx.upload_mesh(m)
u = np.zeros(m.n_u + m.n_p)
ctx.set_state(dcp.OLD_NSE_SOLUTION, u)
ctx.set_state(dcp.OLD_T_SOLUTION, m.T0)
ctx.assemble_nse_system()
ctx.build_nse_preconditioner()
x = np.random.default_rng(20261015 + R).uniform(-1, 1, m.n_u + m.n_p)
res = []
ahead = os.environ.get("DCP_SCHUR_AHEAD", "1")
for fused in (True, True, False, False):
    ctx.set_fused_chain(fused)
    y, it = ctx.block_preconditioner_vmult(x, do_solve_A=False)
    res.append((fused, it, y))
    print("ahead=%s fused=%d inner=%d |y|=%.17g" % (ahead, fused, it, np.linalg.norm(y)), flush=True)
for k in range(1, len(res)):
    a, b = res[0][2], res[k][2]
    d = np.nonzero(a != b)[0]
    print("run0 vs run%d: %d entries differ%s" % (k, len(d), "" if not len(d) else
          ", first %d (%r vs %r), max rel %.3e" % (d[0], a[d[0]], b[d[0]],
                                                   np.max(np.abs(a - b)) / np.max(np.abs(a)))))
