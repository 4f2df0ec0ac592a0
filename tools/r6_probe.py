#!/usr/bin/env python3
"""BASELINE config C5's mesh (classic prm, global refinement 6: 1,572,864
cells, 38.0 M velocity + 1.6 M pressure + 1.6 M temperature dofs) on ONE GPU:
operator-form assemble_nse_system, build_nse_preconditioner (the explicit
Schur complement S), temperature assembly, matrix-free nse_matrix products,
S products and 50 inner Schur GMRES steps (DCP_OPT_INNER_MAX_STEPS), with
size-independent property checks and the device memory after each stage
(hipMemGetInfo). One JSON line. Usage: R=6 python3 tools/r6_probe.py"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-dycoreplanet_amd"))
import numpy as np  # noqa: E402
import dcp  # noqa: E402

R = int(os.environ.get("R", "6"))
GS = os.environ.get("GS", "dcgs2")
out = {"refine": R, "gram_schmidt": GS}
hip = dcp.hip()


def mem_used_gb():
    free, total = C.c_size_t(0), C.c_size_t(0)
    hip.hipMemGetInfo(C.byref(free), C.byref(total))
    return (total.value - free.value) / 1e9


def stage(name, t0):
    out.setdefault("stages", {})[name] = {"s": round(time.perf_counter() - t0, 3),
                                          "device_mem_gb": round(mem_used_gb(), 3)}
    print(name, out["stages"][name], flush=True)


t0 = time.perf_counter()
m = dcp.HostMesh(refine=R)
out["sizes"] = {"cells": m.n_cells, "n_u": m.n_u, "n_p": m.n_p, "n_T": m.n_T}
stage("host_mesh", t0)
t0 = time.perf_counter()
ctx = dcp.Context()
base = mem_used_gb()
out["device_mem_gb_context"] = round(base, 3)
ctx.set_physics(dcp.classic_physics())
ctx.set_gram_schmidt(GS)
ctx.upload_mesh(m)
stage("upload", t0)
n = m.n_u + m.n_p
u = np.zeros(n)
ctx.set_state(dcp.OLD_NSE_SOLUTION, u)
ctx.set_state(dcp.NSE_SOLUTION, u)
ctx.set_state(dcp.OLD_T_SOLUTION, m.T0)
ctx.set_state(dcp.T_SOLUTION, m.T0)
t0 = time.perf_counter()
ctx.assemble_nse_system()
r1 = ctx.get_state(dcp.NSE_RHS)
ctx.assemble_nse_system()
r2 = ctx.get_state(dcp.NSE_RHS)
tm = ctx.timings()
stage("assemble_nse_system", t0)
checks = {"rhs_deterministic": bool(np.array_equal(r1, r2)),
          "rhs_finite": bool(np.all(np.isfinite(r1)))}
t0 = time.perf_counter()
ctx.build_nse_preconditioner()
ctx.assemble_temperature_matrix()
ctx.assemble_temperature_rhs()
tm2 = ctx.timings()
stage("preconditioner_and_T", t0)
out["phase_ms"] = {"assemble_nse": tm["assemble_nse_ms"], "build_precond": tm2["build_precond_ms"],
                   "assemble_T_matrix": tm2["assemble_T_matrix_ms"],
                   "assemble_T_rhs": tm2["assemble_T_rhs_ms"]}
out["assembled_dofs_per_s"] = n / (tm["assemble_nse_ms"] * 1e-3)
rng = np.random.default_rng(6)
x, y = rng.uniform(-1, 1, n), rng.uniform(-1, 1, n)
t0 = time.perf_counter()
Mx, My, Mxy = ctx.nse_vmult(x), ctx.nse_vmult(y), ctx.nse_vmult(x + 2 * y)
stage("stokes_applies", t0)
scale = np.linalg.norm(Mx) + 2 * np.linalg.norm(My)
checks["stokes_linear_rel"] = float(np.linalg.norm(Mxy - Mx - 2 * My) / scale)
checks["stokes_symmetric_rel"] = float(abs(y @ Mx - x @ My) / (np.linalg.norm(x) * np.linalg.norm(My)))
p, q = rng.uniform(-1, 1, m.n_p), rng.uniform(-1, 1, m.n_p)
Sp, Sq = ctx.schur_vmult(p), ctx.schur_vmult(q)
checks["schur_symmetric_rel"] = float(abs(q @ Sp - p @ Sq) / (np.linalg.norm(p) * np.linalg.norm(Sq)))
checks["schur_psd"] = bool(p @ Sp > 0 and q @ Sq > 0)
# 50 inner Schur GMRES steps of BlockSchurPreconditioner::vmult
ctx.set_inner_max_steps(50)
src = np.zeros(n)
src[m.n_u:] = p - p.mean()
t0 = time.perf_counter()
dst, its = ctx.block_preconditioner_vmult(src)
stage("inner_gmres_50", t0)
# at the cap the inner GMRES throws NoConvergence before dst_p = -y
# (block_schur_preconditioner.hpp:48-51), so dst_p holds the iterate y
r = ctx.schur_vmult(dst[m.n_u:]) - src[m.n_u:]
checks["inner_steps"] = its
checks["inner_residual_reduction"] = float(np.linalg.norm(r) / np.linalg.norm(src[m.n_u:]))
out["checks"] = checks
out["ok"] = bool(checks["rhs_deterministic"] and checks["rhs_finite"] and
                 checks["stokes_linear_rel"] < 1e-12 and checks["stokes_symmetric_rel"] < 1e-12 and
                 checks["schur_symmetric_rel"] < 1e-12 and checks["schur_psd"] and its == 50 and
                 checks["inner_residual_reduction"] < 1.0)
out["device_mem_gb_peak_stage"] = max(v["device_mem_gb"] for v in out["stages"].values())
ctx.close()
print(json.dumps(out), flush=True)
sys.exit(0 if out["ok"] else 1)
