#!/usr/bin/env python3
"""assemble_nse_system at refine R with the Kronecker-form B^T (default) and
with the B^T row tasks (DCP_BT_KRON=0): medians over alternating rounds, and
the largest relative B^T difference between the two. PROBES sets
DCP_BTK_PROBE per timing row; the probe variants of round 6 (no A reads, no
stores, direct stores, staging forms) were measured and then removed from the
kernel, so today every value times the real kernels (the logs under
profiles/r06/ keep those measurements)."""
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
ctxs = {}
for kron in ("1", "0"):
    os.environ["DCP_BT_KRON"] = kron
    c = dcp.Context()
    c.set_physics(dcp.classic_physics())
    c.upload_mesh(m)
    c.set_state(dcp.OLD_NSE_SOLUTION, u)
    c.set_state(dcp.OLD_T_SOLUTION, m.T0)
    ctxs[kron] = c
    print("layout", kron, c.assembly_layout(), flush=True)
PROBES = os.environ.get("PROBES", "0").split(",")
keys = [("1", p) for p in PROBES] + [("0", "0")]
times = {k: [] for k in keys}
for rnd in range(4):
    for k in keys:
        os.environ["DCP_BTK_PROBE"] = k[1]
        c = ctxs[k[0]]
        for _ in range(8):
            c.assemble_nse_system()
            times[k].append(c.timings()["assemble_nse_ms"])
os.environ["DCP_BTK_PROBE"] = "0"
for c in ctxs.values():
    c.assemble_nse_system()
a, b = ctxs["1"].coupling_csr("Bt")[2], ctxs["0"].coupling_csr("Bt")[2]
print("B^T max rel diff", float(np.max(np.abs(a - b)) / np.max(np.abs(b))), flush=True)
for k in keys:
    print(f"DCP_BT_KRON={k[0]} probe {k[1]}: median {np.median(times[k]) * 1e3:.1f} us  "
          f"min {np.min(times[k]) * 1e3:.1f} us", flush=True)
for c in ctxs.values():
    c.close()
