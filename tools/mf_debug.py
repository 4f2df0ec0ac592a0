"""Locates matrix-free vs assembled mismatches on a small shell: prints the
worst dofs (velocity node / component or pressure dof) and, per pressure dof,
its incidence count."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "3d-dycoreplanet_amd"))
import numpy as np  # noqa: E402
import dcp  # noqa: E402

import glob  # noqa: E402
R = int(os.environ.get("R", "1"))
m = dcp.HostMesh(refine=R)
libs = sorted(glob.glob(os.path.join(os.path.dirname(dcp.__file__), "build/var/libdcp_*.so")))
for path in libs or [dcp.LIB_PATH]:
  dcp._lib = dcp.load_library(path)
  print(os.path.basename(path))
  ctx = dcp.Context()
  ctx.set_physics(dcp.classic_physics())
  ctx.upload_mesh(m)
  ctx.set_state(dcp.OLD_NSE_SOLUTION, np.zeros(m.n_u + m.n_p))
  ctx.set_state(dcp.OLD_T_SOLUTION, m.T0)
  ctx.assemble_nse_system()
  rng = np.random.default_rng(5)
  for name, x in (("random", rng.uniform(-1, 1, m.n_u + m.n_p)),
                  ("u only", np.r_[rng.uniform(-1, 1, m.n_u), np.zeros(m.n_p)]),
                  ("p only", np.r_[np.zeros(m.n_u), rng.uniform(-1, 1, m.n_p)])):
      ctx.set_matrix_free(0)
      ya = ctx.nse_vmult(x)
      ctx.set_matrix_free(1)
      ym = ctx.nse_vmult(x)
      d = np.abs(ym - ya)
      sc = np.max(np.abs(ya))
      bad = np.nonzero(d > 1e-12 * sc)[0]
      print(name, "n_u", m.n_u, "n_p", m.n_p, "bad", len(bad), "bad_u", int(np.sum(bad < m.n_u)),
            "bad_p", int(np.sum(bad >= m.n_u)), "max rel", float(d.max() / sc))
      print("  first bad", bad[:20].tolist())
  ctx.close()
