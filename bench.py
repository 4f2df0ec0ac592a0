#!/usr/bin/env python3
"""Benchmark of the Boussinesq per-time-step hot path on MI355X.

Workload (BASELINE.json metric): 3D hypershell, classic Q2/Q1 Taylor-Hood,
global refinement 5 (196,608 cells, 4,995,528 NSE dofs + 202,818 T dofs),
data/aqua_planet_shell_test_3d-classic.prm physics, the reference initial state
(u = 0, two-Gaussian temperature), synthetic mesh (hyper_shell refined with
SphericalManifold's rules, MappingQ(3) cell maps as deal.II 9.2's MappingQ).

One "step" = one full reference time step (Standard::BoussinesqModel::run body,
boussinesq_model.tpp:1843-1926): assemble_nse_system, build_nse_preconditioner,
assemble_temperature_matrix/_rhs, solve_NSE_block_preconditioned (FGMRES with
the block-Schur preconditioner and its inner GMRES), solve_temperature,
get_cfl_number/get_maximal_velocity. Every step restarts from the initial
state (the classic configuration runs exactly this one step, Q24).

Output: one JSON line (rank 0). value = assembled NSE DoFs/s of the
assemble_nse_system phase; GMRES iteration rates, per-phase times, the
Schur-complement apply roofline and the CPU oracle baseline ride along.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
# idle OpenMP workers of the CPU-baseline legs sleep instead of spinning
# (read when libgomp loads, i.e. before libdcp.so / liboracle.so)
os.environ.setdefault("OMP_WAIT_POLICY", "passive")
sys.path.insert(0, os.path.join(ROOT, "3d-dycoreplanet_amd"))

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# measured on this GPU model (tools/stream_probe.hip, 1 GiB arrays, best of 10):
# the read / copy / triad ceilings every frac is also reported against
CEILING_FILE = "profiles/r04c_stream_probe.json"


def measured_ceilings():
    path = os.path.join(ROOT, CEILING_FILE)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    return {"read_GBps": 1e3 * d["read_TBps"], "copy_GBps": 1e3 * d["copy_TBps"],
            "triad_GBps": 1e3 * d["triad_TBps"], "source": CEILING_FILE}
# rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE summaries (tools/pmc_summary.py) of the
# roofline kernel, per (refine, schur mode): HBM bytes per launch
PMC_SUMMARIES = {(5, "explicit"): ("profiles/r04j_pmc_inner_r5.json", "k_sell_spmv<true, 2>")}
# rocprofv3 --kernel-trace --stats of the same workload (durations of the
# orthogonalisation launches, for their roofline): the CGS2 chain (bench) and
# the s-step block (inner probe)
# PMC (2 FETCH + WRITE) of the same launches (tools/pmc_inner.sh)
CHAIN_PMC = {(5, "sstep"): "profiles/r05/r05ab_pmc_inner_sstep_r5.json"}
CHAIN_STATS = {(5, "classical2"): "profiles/r03a_bench_r5_kernel_stats.csv",
               (5, "sstep"): "profiles/r05/r05zd_bench_r5_kernel_stats.csv"}
# the operator-form assembly's kernels (tools/bt_rows_probe.py) and their
# launches per assembly (the rhs kernel once per colour class)
PMC_ASM = {5: ("profiles/r06/r06_pmc_asm_r5.json",
               {"k_btk_lateral": 1, "k_btk_entries": 1, "k_mf_pencil": 1, "k_mf_gather": 1,
                "k_cdk_diag": 1})}
# (k_bt_coltab / k_bt_laytab run once at upload)
# the same for the matrix-free Stokes apply (pencil kernel + dof gather); the
# kernel names must be found in the summary (no stale profile of other kernels)
PMC_MF = {5: ("profiles/r06/r06_pmc_mf_r5.json", ("k_mf_pencil<true, true, false>",
                                                  "k_mf_gather<true>"))}
# rocprofv3 --kernel-trace of the default refine-5 step alone (bench.py
# --no-converging-leg --no-other-gs --no-cpu-baseline), per-kernel durations
# with the early-exit launches of stopped Krylov cycles split off
# (tools/trace_summary.py): the source of roofline_chain and of the trace
# cross-checks of the in-step HIP-event rooflines
TRACE = {(5, "sstep"): "profiles/r06/r06_trace_r5.json"}


def trace_summary(refine, gs):
    path = TRACE.get((refine, gs))
    if path is None or not os.path.exists(os.path.join(ROOT, path)):
        return None
    with open(os.path.join(ROOT, path)) as f:
        d = json.load(f)
    d["path"] = path
    return d


def trace_kernel(tr, key):
    """The one kernel of the trace summary whose name contains key, or None."""
    if tr is None:
        return None
    hits = [(k, v) for k, v in tr["kernels"].items() if key in k]
    return hits[0] if len(hits) == 1 else None


def pmc_asm_traffic(refine):
    """HBM bytes of one operator-form assembly from the committed PMC summary:
    FETCH + WRITE as counted, and with the gfx950 2x FETCH correction (which
    holds for wide coalesced streams; the rhs kernel's node gathers are short
    reads counted in full, so the truth lies between the two)."""
    ent = PMC_ASM.get(refine)
    if ent is None or not os.path.exists(os.path.join(ROOT, ent[0])):
        return None
    with open(os.path.join(ROOT, ent[0])) as f:
        ctr = json.load(f)["counters"]
    fetch = write = 0.0
    for key, launches in ent[1].items():
        fk = [v["mean_kB"] for k, v in ctr["FETCH_SIZE"].items() if key in k]
        wk = [v["mean_kB"] for k, v in ctr["WRITE_SIZE"].items() if key in k]
        if len(fk) != 1 or len(wk) != 1:  # missing or ambiguous: no stale numbers
            return None
        fetch += launches * fk[0] * 1e3
        write += launches * wk[0] * 1e3
    return {"fetch_plus_write": fetch + write, "two_fetch_plus_write": 2 * fetch + write,
            "write": write, "source": ent[0]}


def pmc_mf_traffic(refine):
    """HBM bytes of one matrix-free Stokes apply (both launches) from the
    committed PMC summary: (bytes, None), or (None, why)."""
    ent = PMC_MF.get(refine)
    if ent is None or not os.path.exists(os.path.join(ROOT, ent[0])):
        return None, "no PMC summary for this refinement"
    with open(os.path.join(ROOT, ent[0])) as f:
        tb = json.load(f)["traffic_bytes"]
    parts = []
    for key in ent[1]:
        hits = [v for k, v in tb.items() if key in k]
        if len(hits) != 1:
            return None, f"{ent[0]}: kernel {key!r} found {len(hits)} times (stale profile?)"
        parts.append(hits[0])
    return sum(parts), None


def pmc_traffic(refine, mode, n_p):
    """HBM bytes per launch of the roofline kernel from the committed PMC
    summary of the same workload, or None when none was collected. The
    summary's traffic_bytes is 2 FETCH + WRITE (gfx950 FETCH_SIZE counts half
    of wide coalesced streaming reads); the gathered x (8 n_p bytes, short
    scattered reads counted in full) is taken back out of the doubling."""
    ent = PMC_SUMMARIES.get((refine, mode))
    if ent is None or not os.path.exists(os.path.join(ROOT, ent[0])):
        return None
    with open(os.path.join(ROOT, ent[0])) as f:
        tb = json.load(f)["traffic_bytes"]
    hits = [v for k, v in tb.items() if ent[1] in k]
    return hits[0] - 8.0 * n_p if hits else None


def back_to_back_applies(ctx, ls, nvec=8, reps=48, batches=8, warm=3):
    """Median ms per apply of the matrix-free Stokes operator and of its
    velocity block over `batches` batches of `reps` back-to-back applies
    (dcp_time_operator: one HIP event pair per batch on the context's stream),
    the first `warm` batches dropped, sources rotating over nvec vectors."""
    import dcp
    n = ls["n_u"] + ls["n_p"]
    try:
        with dcp.DeviceBuffer(n * nvec) as src, dcp.DeviceBuffer(n * nvec) as dst:
            src.upload(np.random.default_rng(5).uniform(-1, 1, n * nvec))
            res = {}
            for which in ("nse", "velocity"):
                ms = [ctx.time_operator(which, reps, src.ptr, dst.ptr, nvec)
                      for _ in range(batches)]
                res[which + "_ms"] = float(np.median(ms[warm:]))
                res[which + "_batches_ms"] = [round(x, 5) for x in ms]
    except dcp.DcpError as e:  # e.g. no room for the 2 x nvec vectors: the in-step figure stays
        print("back-to-back applies skipped: %s" % e, file=sys.stderr)
        return None
    res["what"] = ("median of %d batches (after %d warm-up batches) of %d back-to-back applies, "
                   "one HIP event pair per batch, sources rotating over %d vectors of %d MB"
                   % (batches - warm, warm, reps, nvec, 8 * n // 1000000))
    return res


def chain_roofline_trace(refine, n_p, gs):
    """roofline_chain from the committed kernel trace of the default step
    alone (TRACE): per k_sstep_block<KL> template the average over its working
    launches (early exits of stopped cycles split off), bytes (KL + 5) 8 n_p."""
    tr = trace_summary(refine, gs)
    if tr is None or gs != "sstep":
        return None
    key = "k_sstep_block<"
    rows = []
    for name, v in tr["kernels"].items():
        if key not in name:
            continue
        kl = int(name.split(key)[1].split(",")[0].split(">")[0])
        rows.append((kl, v["full_calls"], v["avg_ns_full"], v["early_exit_calls"]))
    if not rows:
        return None
    per = {kl: {"bytes": (kl + 5.0) * 8 * n_p, "avg_us": ns * 1e-3, "launches": c,
                "early_exits_dropped": ee,
                "achieved": (kl + 5.0) * 8 * n_p / (ns * 1e-9) / 1e9} for kl, c, ns, ee in rows}
    tot_b = sum(c * (kl + 5.0) * 8 * n_p for kl, c, _, _ in rows)
    tot_t = sum(c * ns * 1e-9 for _, c, ns, _ in rows)
    ach = tot_b / tot_t / 1e9
    out = {"kernel": "s-step block k_sstep_block<KL> (one launch per 4 inner Arnoldi columns: "
                     "BCGS2 + Cholesky QR + Hessenberg/Givens)",
           "bound": "hbm", "source": tr["path"], "rule": tr.get("early_exit_rule"),
           "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
           "per_template": per, "traffic": None}
    pmc = CHAIN_PMC.get((refine, gs))
    if pmc and os.path.exists(os.path.join(ROOT, pmc)):
        with open(os.path.join(ROOT, pmc)) as f:
            tb = json.load(f)["traffic_bytes"]
        for name, v in tb.items():
            if key in name:
                kl = int(name.split(key)[1].split(",")[0].split(">")[0])
                if kl in per:
                    per[kl]["traffic"] = v
        if all("traffic" in per[kl] for kl in per):
            calls = {kl: c for kl, c, _, _ in rows}
            out["traffic"] = sum(calls[kl] * per[kl]["traffic"] for kl in per) / sum(calls.values())
            out["traffic_source"] = pmc
    return out


def chain_roofline(refine, n_p, gs):
    """The orthogonalisation launches of the inner Schur GMRES from the
    committed kernel statistics (rocprofv3 --kernel-trace --stats).
    classical2: k_cgs2_chain<KL>, one launch per Arnoldi column k: the k+1
    basis vectors read once (registers for both passes) + w read + q written
    = (k + 3) 8 n_p bytes; template KL serves k = KL-4..KL-1, on average
    (KL + 0.5) 8 n_p. sstep: k_sstep_block<KL>, one launch per block of 4
    columns starting at k = KL-4: the k+1 basis vectors + the 4 Newton vectors
    read, the 4 new basis vectors written = (KL + 5) 8 n_p. Bound: HBM,
    although at refine 5 the basis sits in the 256 MB MALL and the launches
    are hand-off latency bound."""
    path = CHAIN_STATS.get((refine, gs))
    if path is None or not os.path.exists(os.path.join(ROOT, path)):
        return None
    import csv
    key, extra = ("k_cgs2_chain<", 0.5) if gs == "classical2" else ("k_sstep_block<", 5.0)
    rows = []
    with open(os.path.join(ROOT, path)) as f:
        for r in csv.DictReader(f):
            name = r["Name"]
            if key not in name:
                continue
            kl = int(name.split(key)[1].split(",")[0].split(">")[0])
            rows.append((kl, int(r["Calls"]), float(r["AverageNs"])))
    if not rows:
        return None
    per = {kl: {"bytes": (kl + extra) * 8 * n_p, "avg_us": ns * 1e-3,
                "achieved": (kl + extra) * 8 * n_p / (ns * 1e-9) / 1e9} for kl, _, ns in rows}
    tot_b = sum(calls * (kl + extra) * 8 * n_p for kl, calls, _ in rows)
    tot_t = sum(calls * ns * 1e-9 for _, calls, ns in rows)
    ach = tot_b / tot_t / 1e9
    what = ("fused CGS2 orthogonalisation chain k_cgs2_chain<KL> (one launch per inner "
            "Arnoldi column)" if gs == "classical2" else
            "s-step block k_sstep_block<KL> (one launch per 4 inner Arnoldi columns: BCGS2 + "
            "Cholesky QR + Hessenberg/Givens)")
    out = {"kernel": what, "bound": "hbm", "source": path,
           "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
           "per_template": per, "traffic": None}
    pmc = CHAIN_PMC.get((refine, gs))
    if pmc and os.path.exists(os.path.join(ROOT, pmc)):
        with open(os.path.join(ROOT, pmc)) as f:
            tb = json.load(f)["traffic_bytes"]
        for name, v in tb.items():
            if key in name:
                kl = int(name.split(key)[1].split(",")[0].split(">")[0])
                if kl in per:
                    per[kl]["traffic"] = v
        calls = {kl: c for kl, c, _ in rows}
        if all("traffic" in per[kl] for kl in per):
            # per launch, averaged over the launches of the profile
            out["traffic"] = sum(calls[kl] * per[kl]["traffic"] for kl in per) / sum(calls.values())
            out["traffic_source"] = pmc
    return out


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--refine", type=int, default=5)
    ap.add_argument("--prm", default=os.path.join(ROOT, "configs",
                                                  "aqua_planet_shell_test_3d-classic.prm"))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-back-to-back", action="store_true",
                    help="skip the back-to-back matrix-free apply timing after the steps")
    ap.add_argument("--no-converging-leg", action="store_true",
                    help="skip the converging refine-3 step (GMRES outer iter/s)")
    ap.add_argument("--no-other-gs", action="store_true",
                    help="skip the one-step legs of the other Gram-Schmidt variants (a kernel "
                         "trace of the default step alone)")
    ap.add_argument("--schur", choices=["explicit", "composite"], default="explicit",
                    help="explicit: formed S = B D^-1 B^T (default); composite: B^T, Jacobi, B")
    ap.add_argument("--gram-schmidt", choices=["modified", "classical2", "dcgs2", "sstep"],
                    default="sstep",
                    help="inner Schur GMRES orthogonalisation (DCP_OPT_GRAM_SCHMIDT): modified "
                         "(deal.II's), classical2 / dcgs2 (classical twice, one launch per "
                         "step), sstep (blocks of 4 Newton-basis steps, one orthogonalisation "
                         "launch per block; DESIGN 9a); all device-resident cycles but modified")
    ap.add_argument("--variant", choices=["classic", "feec"], default="classic",
                    help="feec: ExteriorCalculus model of config 4 (feec prm, refine 4, 1 GPU)")
    ap.add_argument("--shared-device", action="store_true",
                    help="rehearsal: every rank on device 0 (one-GPU box), gloo bootstrap")
    ap.add_argument("--probe-schur", type=int, default=0,
                    help="PMC probe: only N Schur-complement applies after one assembly")
    ap.add_argument("--dry-launch", action="store_true",
                    help="launch rehearsal: every rank sets up torch.distributed (gloo) and the "
                         "communicator id broadcast, reports its env and stops before any GPU call")
    args = ap.parse_args()
    argv = sys.argv[1:]
    args.refine_set = any(a.startswith("--refine") for a in argv)
    args.prm_set = any(a.startswith("--prm") for a in argv)
    return args


def schur_bytes(m, nnzb_bt, nnzb_b):
    """Algorithmic HBM bytes of one Schur-complement apply B D_A^-1 B^T
    (schur_complement.hpp:143-150) on the block-CSR layout:
    B^T: 3x1 blocks (24 B values + 4 B column) + row pointers, gathered p (8 n_p),
    tmp1 write (8 n_u); Jacobi: tmp1 + inv-diag read, tmp2 write (24 n_u);
    B: 1x3 blocks (24 + 4 B) + row pointers, gathered tmp2 (8 n_u), dst (8 n_p)."""
    n_v = m.n_u // 3
    bt = 28 * nnzb_bt + 4 * (n_v + 1) + 8 * m.n_p + 8 * m.n_u
    jac = 24 * m.n_u
    b = 28 * nnzb_b + 4 * (m.n_p + 1) + 8 * m.n_u + 8 * m.n_p
    return bt + jac + b


def device_mem_gb():
    """Device memory in use (hipMemGetInfo: total - free), GB."""
    import ctypes
    import dcp
    free, total = ctypes.c_size_t(0), ctypes.c_size_t(0)
    dcp.hip().hipMemGetInfo(ctypes.byref(free), ctypes.byref(total))
    return (total.value - free.value) / 1e9


def cpu_info():
    """Host CPU model and the cores this process may use (GPU box: read at run time)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return model, os.cpu_count(), max(1, min(usable, omp) if omp > 0 else usable)


class _SubMesh:
    """Cells [c0, c1) of a HostMesh with the whole mesh's dof numbering and
    constraints (the oracle's input for a bounded sample of its assembly)."""

    def __init__(self, m, c0, c1):
        self.n_cells = c1 - c0
        self.cell_nse_dofs = m.cell_nse_dofs[c0:c1]
        self.cell_T_dofs = m.cell_T_dofs[c0:c1]
        self.cell_geometry = m.cell_geometry[c0:c1]
        self.cell_diameter = m.cell_diameter[c0:c1]
        for k in ("n_u", "n_p", "n_T", "nse_constraints", "T_constraints", "T0"):
            setattr(self, k, getattr(m, k))


def cpu_baseline(ctx, m, refine, gpu_inner_per_s, gpu_full_asm_per_s, outer_refine=3,
                 outer_k=1):
    """The oracle (C++ restatement of the reference path) timed on bounded
    samples of the bench's own workload (refine 5) on this host, beside the GPU
    run:
    * "Assemble NSE system" (boussinesq_model.tpp:695): the full
      assemble_nse_system -- element matrices with the velocity block and
      AffineConstraints::distribute_local_to_global into CSR, WorkStream's
      result (threaded element work, copier in cell order) -- over a contiguous
      1/8 of the refine-5 cells in tree order (one 8-way partition's share) on
      all usable cores, and over 1/64 on one core; scaled to the whole mesh;
    * the inner Schur GMRES (block_schur_preconditioner.hpp:46-51): 28 steps
      (one restart cycle) of deal.II's SolverGMRES on the refine-5
      S = B D_A^-1 B^T, its blocks and the A-Jacobi exported from the GPU
      context (the parity tests hold them to the oracle's at 1e-12), on all
      usable cores (row-parallel CSR products) and on one core;
    * the outer FGMRES (:1139): the first outer iteration of the converging
      refine-3 step (the r=5 step never completes one; its inner solve fails).
    same_config_ratio: GPU / CPU at refine 5 for the full assembly (GPU
    assembly_with_velocity_block, the same output) and the inner Schur GMRES."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import dcp
    import oracle_py
    model, ncpu, threads = cpu_info()
    ph = dcp.classic_physics()
    n = m.n_u + m.n_p
    u = np.zeros(n)
    # 1. assembly samples
    oracle_py.set_threads(threads)
    c_all = m.n_cells // 8
    orc = oracle_py.Model(ph, _SubMesh(m, 0, c_all))
    t0 = time.perf_counter()
    orc.assemble_nse_system(u, m.T0)
    t_all = time.perf_counter() - t0
    del orc
    oracle_py.set_threads(1)
    c_one = m.n_cells // 64
    orc = oracle_py.Model(ph, _SubMesh(m, 0, c_one))
    t0 = time.perf_counter()
    orc.assemble_nse_system(u, m.T0)
    t_one = time.perf_counter() - t0
    del orc
    full_all = t_all * m.n_cells / c_all
    full_one = t_one * m.n_cells / c_one
    # 2. inner Schur GMRES sample on the refine-5 operator
    Bt, B = ctx.coupling_csr("Bt"), ctx.coupling_csr("B")
    a_diag, _ = ctx.precond_diagonals()
    a_inv = 1.0 / a_diag
    src = np.random.default_rng(20261015).uniform(-1, 1, m.n_p)
    src -= src.mean()
    k = 28
    sol = {}
    for cores in (threads, 1):
        oracle_py.set_threads(cores)
        sol[cores] = oracle_py.schur_gmres_sample(Bt, B, a_inv, src, k)[0]
    del Bt, B
    # 3. outer FGMRES sample on the converging refine-3 step
    m3 = dcp.HostMesh(refine=outer_refine)
    oracle_py.set_threads(threads)
    orc = oracle_py.Model(ph, m3)
    orc.assemble_nse_system(np.zeros(m3.n_u + m3.n_p), m3.T0)
    orc.build_nse_preconditioner()
    t0 = time.perf_counter()
    ko, its = orc.fgmres_outer(np.zeros(m3.n_u + m3.n_p), outer_k)
    ts = time.perf_counter() - t0
    oracle_py.set_threads(1)
    del orc
    out = {"value": n / full_all, "unit": "assembled DoFs/s", "cores": threads, "kind": "port",
           "cpu_model": model, "nproc": ncpu,
           "sample": f"full assemble_nse_system (element matrices incl. the velocity block + "
                     f"AffineConstraints distribute into CSR) over cells [0, {c_all}) of the "
                     f"refine-{refine} shell (1/8, tree order): {t_all:.2f} s on {threads} cores, "
                     f"scaled x{m.n_cells / c_all:g} to the {m.n_cells} cells / {n} NSE dofs",
           "one_core": {"value": n / full_one, "unit": "assembled DoFs/s", "cores": 1,
                        "sample": f"cells [0, {c_one}) (1/64): {t_one:.2f} s, scaled"},
           "solve": {"value": k / sol[threads], "unit": "inner Schur GMRES iter/s",
                     "cores": threads,
                     "sample": f"{k} steps of deal.II's SolverGMRES (MGS, restart 28) on the "
                               f"refine-{refine} S = B D_A^-1 B^T (n_p = {m.n_p}; blocks from the GPU "
                               f"context): {sol[threads]:.2f} s on {threads} cores",
                     "one_core": {"value": k / sol[1], "cores": 1, "seconds": sol[1]}},
           "outer": {"value": ko / ts, "unit": "FGMRES outer iter/s", "cores": threads,
                     "inner_iter_per_s": its / ts,
                     "sample": f"the first {ko} FGMRES outer iteration(s) of the converging "
                               f"refine-{outer_refine} step ({its} inner Schur GMRES "
                               f"iterations): {ts:.2f} s on {threads} cores"}}
    out["same_config_ratio"] = {
        "assembly_full": gpu_full_asm_per_s / out["value"] if gpu_full_asm_per_s else None,
        "inner_gmres": gpu_inner_per_s / out["solve"]["value"],
        "what": f"refine {refine}, GPU / CPU: the full assembly (GPU "
                "assembly_with_velocity_block: the same CSR output) and the inner Schur GMRES "
                "(the GPU's s-step cycles vs the CPU's deal.II GMRES sample)"}
    return out


def converging_leg(make_ctx, args, refine=3):
    """The BASELINE metric's GMRES half on a step whose solve converges: the
    classic prm at refine 3 (23 FGMRES outer / ~29 k inner iterations, the
    committed fixture tests/golden/shell_r3_step.npz), where every Krylov
    stage the r=5 headline step never reaches (FGMRES outer iterations, the
    matrix-free nse_matrix products inside it, the outer Gram-Schmidt) runs
    and is timed. One GPU; one warm-up step, then one timed step."""
    import dcp
    rp = dcp.load_prm(args.prm)
    ph = dcp.physics_from_params(rp)
    m = dcp.HostMesh(cuboid=False, refine=refine, R0=rp.R0, R1=rp.R1, length=rp.length,
                     temperature_degree=ph.temperature_degree)
    ctx = make_ctx()
    ctx.set_physics(ph)
    ctx.set_schur_explicit(args.schur == "explicit")
    ctx.set_gram_schmidt(args.gram_schmidt)
    ctx.upload_mesh(m)
    n = m.n_u + m.n_p
    ctx.set_state(dcp.OLD_NSE_SOLUTION, np.zeros(n))
    ctx.set_state(dcp.OLD_T_SOLUTION, m.T0)
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    recs = []
    for _ in range(2):
        hip.hipDeviceSynchronize()
        t0 = time.perf_counter()
        ctx.copy_state(dcp.NSE_SOLUTION, dcp.OLD_NSE_SOLUTION)
        ctx.copy_state(dcp.T_SOLUTION, dcp.OLD_T_SOLUTION)
        ctx.assemble_nse_system()
        ctx.build_nse_preconditioner()
        ctx.assemble_temperature_matrix()
        ctx.assemble_temperature_rhs()
        rc, outer, inner = ctx.solve_nse()
        ctx.solve_temperature()
        hip.hipDeviceSynchronize()
        recs.append((rc, outer, inner, ctx.timings(), time.perf_counter() - t0))
    ctx.close()
    rc, outer, inner, t, wall = recs[-1]
    solve_s = t["solve_nse_ms"] * 1e-3
    return {"workload": f"classic shell Q2/Q1 refine={refine}, one full time step "
                        f"({m.n_cells} cells, {n} NSE dofs)",
            "converged": rc == 0, "fgmres_outer_iterations": outer,
            "schur_gmres_inner_iterations": inner,
            "gmres_outer_iter_per_s": outer / solve_s, "gmres_inner_iter_per_s": inner / solve_s,
            "solve_nse_ms": t["solve_nse_ms"], "ms_per_step": wall * 1e3,
            "assembled_dofs_per_s": n / (t["assemble_nse_ms"] * 1e-3),
            "assemble_nse_ms": t["assemble_nse_ms"],
            "stokes_apply_ms_avg": t["stokes_apply_ms_avg"], "stokes_applies": t["stokes_applies"],
            "schur_apply_ms_avg": t["schur_apply_ms_avg"]}


def free_port():
    """A free TCP port on 127.0.0.1 for the ranks' rendezvous."""
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args):
    """`--gpus N` (N > 1) without a launcher: start the N rank processes here,
    one per GPU, as torch.distributed.run would (the reference's `mpirun -np N`
    of source/main.cxx:64-65, one MPI rank per p::d::Triangulation part,
    planet_geometry.tpp:13-20). The parent touches neither HIP nor torch: it
    only sets RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT for
    each child (the same script and arguments), lets them write to its own
    stdout / stderr (rank 0 prints the one JSON line), waits, and exits with the
    first non-zero child status. No exec: the children are new processes. A
    rank that fails leaves the others up to 120 s to finish before they are
    killed, so a rank stuck in a collective cannot hang the job."""
    import subprocess
    n = args.gpus
    port = str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n),
                    "LOCAL_WORLD_SIZE": str(n), "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                    "MASTER_PORT": port, "DCP_BENCH_CHILD": "1"})
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)]
                                      + sys.argv[1:], env=env))
    rc, failed_at = 0, None
    while any(p.poll() is None for p in procs):
        for p in procs:
            if p.returncode not in (None, 0) and rc == 0:
                rc, failed_at = p.returncode, time.monotonic()
        if failed_at is not None and time.monotonic() - failed_at > 120:
            for p in procs:
                if p.poll() is None:
                    p.kill()
        time.sleep(0.2)
    for p in procs:
        if p.returncode != 0 and rc == 0:
            rc = p.returncode
    if rc != 0:
        print(f"[bench] launch of {n} ranks failed: exit statuses "
              f"{[p.returncode for p in procs]}", file=sys.stderr, flush=True)
    return rc if rc > 0 else (1 if rc else 0)


def init_dist(args):
    """One process per GPU (torchrun env, or launch_ranks); the library's own
    RCCL communicator is created from rank 0's unique id broadcast through
    torch.distributed. dry: gloo and a random id, nothing touches a GPU."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dry = args.dry_launch
    host_only = args.shared_device or dry
    dist = None
    if args.shared_device:
        local_rank = 0
    if world > 1:
        import torch.distributed as dist  # noqa: F811
        import torch
        if not host_only:
            torch.cuda.set_device(local_rank)
        dist.init_process_group("gloo" if host_only else "nccl")
        assert dist.get_world_size() == world and dist.get_rank() == rank
    tdev = "cpu" if host_only else "cuda"
    nccl_id = None
    if world > 1:
        import torch
        idt = torch.zeros(128, dtype=torch.uint8, device=tdev)
        if rank == 0:
            raw = os.urandom(128) if dry else __import__("dcp").nccl_unique_id()
            idt.copy_(torch.frombuffer(bytearray(raw), dtype=torch.uint8))
        dist.broadcast(idt, 0)
        nccl_id = bytes(idt.cpu().numpy().tobytes())
    if dry:
        return world, rank, dist, tdev, nccl_id

    import dcp

    def make_ctx():
        return dcp.Context(device=local_rank, rank=rank, world_size=world, nccl_id=nccl_id)
    return world, rank, dist, tdev, make_ctx


def dry_launch(args):
    """--dry-launch: the N>1 launch up to the communicator id, no GPU. Every
    rank reports what it got; rank 0 prints them as one JSON line."""
    import hashlib
    world, rank, dist, _, nccl_id = init_dist(args)
    mine = {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
            "world_size": world, "pid": os.getpid(),
            "master": f"{os.environ.get('MASTER_ADDR')}:{os.environ.get('MASTER_PORT')}",
            "backend": dist.get_backend() if dist is not None else None,
            "nccl_id_sha": hashlib.sha256(nccl_id).hexdigest()[:16] if nccl_id else None,
            "gpu_touched": "dcp" in sys.modules or (
                "torch" in sys.modules and sys.modules["torch"].cuda.is_initialized())}
    gathered = [mine]
    if dist is not None:
        gathered = [None] * world
        dist.all_gather_object(gathered, mine)
    if rank == 0:
        print(json.dumps({"dry_launch": True, "n_gpus": args.gpus, "world_size": world,
                          "ranks": gathered}), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    if os.environ.get("DCP_BENCH_DRY_FAIL_RANK") == str(rank):
        sys.exit(3)  # test hook: a rank that fails after the rendezvous


def check_comm(ctx, args, world, rank, dist):
    """Every rank's communicator must span the N ranks with one device per
    rank (the reference's one MPI rank per process): a SCALE line that is
    really N single-GPU runs, or N ranks on one device, is refused."""
    info = ctx.comm_info()
    if world == 1:
        return [info]
    gathered = [None] * world
    dist.all_gather_object(gathered, info)
    counts = sorted({g["ranks"] for g in gathered})
    devices = [g["device"] for g in gathered]
    bad = []
    if counts != [world]:
        bad.append(f"communicator sizes {counts} != [{world}]")
    if [g["rank"] for g in gathered] != list(range(world)):
        bad.append(f"communicator ranks {[g['rank'] for g in gathered]}")
    if not args.shared_device and len(set(devices)) != world:
        bad.append(f"devices {devices} are not distinct")
    if bad:
        raise SystemExit(f"[bench rank {rank}] bad multi-GPU launch: " + "; ".join(bad))
    return gathered


def run_feec(args):
    """Config 4 (BASELINE.json configs[3]): the FEEC model's time step
    (ExteriorCalculus::BoussinesqModel<3>::run body, FEEC.tpp:2238-2300):
    assemble_nse_system, build_nse_preconditioner, temperature matrix/rhs,
    solve_NSE_block_preconditioned, solve_temperature; on N GPUs the p4est-style
    cell split with a ghost-DoF halo (configs[3] asks for 2)."""
    import ctypes
    world, rank, dist, tdev, make_ctx = init_dist(args)
    import dcp
    prm = args.prm if args.prm_set else os.path.join(ROOT, "configs",
                                                     "aqua_planet_shell_test_3d-feec.prm")
    rp = dcp.load_prm(prm)
    ph = dcp.physics_from_params(rp)
    refine = args.refine if args.refine_set else 4
    t_setup = time.perf_counter()
    m = dcp.HostMesh(cuboid=False, refine=refine, R0=rp.R0, R1=rp.R1, length=rp.length,
                     temperature_degree=ph.temperature_degree, feec=True)
    f = m.feec
    ctx = make_ctx()
    check_comm(ctx, args, world, rank, dist)
    ctx.set_physics(ph)
    ctx.upload_feec_mesh(m)
    ctx.set_feec_zero_mean(bool(rp.correct_pressure_to_zero_mean))
    ctx.set_state(dcp.OLD_NSE_SOLUTION, np.zeros(f.n))
    ctx.set_state(dcp.OLD_T_SOLUTION, m.T0)
    t_setup = time.perf_counter() - t_setup

    def step():
        ctx.copy_state(dcp.NSE_SOLUTION, dcp.OLD_NSE_SOLUTION)
        ctx.copy_state(dcp.T_SOLUTION, dcp.OLD_T_SOLUTION)
        ctx.cfl_number()
        ctx.max_velocity()
        ctx.feec_assemble_nse_system()
        ctx.feec_build_nse_preconditioner()
        ctx.assemble_temperature_matrix()
        ctx.assemble_temperature_rhs()
        rc, it = ctx.feec_solve_nse()
        rcT, itT, _ = ctx.solve_temperature()
        return rc, it, itT, ctx.timings()

    for _ in range(args.warmup):
        step()
    hip = ctypes.CDLL("libamdhip64.so")
    if dist is not None:
        dist.barrier()
    hip.hipDeviceSynchronize()
    t0 = time.perf_counter()
    recs = [step() for _ in range(args.steps)]
    hip.hipDeviceSynchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    asm_ms = float(np.mean([r[3]["assemble_nse_ms"] for r in recs]))
    solve_ms = float(np.mean([r[3]["solve_nse_ms"] for r in recs]))
    if dist is not None:
        import torch
        tt = torch.tensor([elapsed, asm_ms, solve_ms], dtype=torch.float64, device=tdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed, asm_ms, solve_ms = (float(v) for v in tt.tolist())
    its = recs[-1][1]
    out = {
        "metric": f"assembled DoFs/sec + GMRES iter/sec, 3D shell FEEC refine={refine} "
                  f"(config 4), {world} GPU",
        "value": f.n / (asm_ms * 1e-3), "unit": "assembled DoFs/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "strong",  # the global mesh is fixed whatever N
        "vs_baseline": None, "dtype": "f64",
        "data": "synthetic refined hypershell, reference initial state",
        "config": {"workload": f"FEEC shell Nedelec/RT/DGQ0 refine={refine}, one full time step",
                   "cells": f.n_cells, "nse_dofs": f.n, "n_w": f.n_w, "n_u": f.n_u,
                   "n_p": f.n_p, "T_dofs": m.n_T,
                   "parallelism": "single GPU" if world == 1 else
                   f"{world} GPUs: p4est-style cell partition, RCCL ghost halo + all-reduce"},
        "gmres_iterations": its, "gmres_iter_per_s": its / (solve_ms * 1e-3),
        "T_cg_iterations": recs[-1][2], "converged": all(r[0] == 0 for r in recs),
        "phase_ms": {k: float(np.mean([r[3][k] for r in recs])) for k in recs[0][3]
                     if k.endswith("_ms")},
        "setup_s": t_setup,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


def progress(msg):
    """One line per bench stage on stderr (long refine-6 runs stay visibly alive)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    if args.dry_launch:
        dry_launch(args)
        return
    if args.variant == "feec":
        run_feec(args)
        return
    world, rank, dist, tdev, make_ctx = init_dist(args)
    import dcp

    rp = dcp.load_prm(args.prm)
    ph = dcp.physics_from_params(rp)
    t_setup = time.perf_counter()
    m = dcp.HostMesh(cuboid=False, refine=args.refine, R0=rp.R0, R1=rp.R1, length=rp.length,
                     temperature_degree=ph.temperature_degree)
    progress(f"host mesh refine {args.refine}: {m.n_cells} cells")
    ctx = make_ctx()
    comm_seen = check_comm(ctx, args, world, rank, dist)
    ctx.set_physics(ph)
    ctx.set_schur_explicit(args.schur == "explicit")
    ctx.set_gram_schmidt(args.gram_schmidt)
    ctx.upload_mesh(m)
    progress("uploaded")
    u0 = np.zeros(m.n_u + m.n_p)
    for f, v in ((dcp.OLD_NSE_SOLUTION, u0), (dcp.OLD_T_SOLUTION, m.T0)):
        ctx.set_state(f, v)
    t_setup = time.perf_counter() - t_setup

    if args.probe_schur:
        # PMC probe: assemble once, then only Schur-complement applies (few dispatches)
        ctx.assemble_nse_system()
        ctx.build_nse_preconditioner()
        x = np.random.default_rng(20261015).uniform(-1, 1, m.n_p)
        x -= x.mean()
        with dcp.DeviceBuffer(m.n_p) as d_src, dcp.DeviceBuffer(m.n_p) as d_dst:
            d_src.upload(x)
            for _ in range(args.probe_schur):
                ctx._check(dcp.lib().dcp_schur_vmult(ctx._h, d_src.ptr, d_dst.ptr))
        print(json.dumps({"probe": "schur", "applies": args.probe_schur, "refine": args.refine}))
        ctx.close()
        return

    loud = args.refine >= 6   # minutes per step: a line per phase and a heartbeat
    if loud:
        import threading

        def heartbeat():
            while True:
                time.sleep(60)
                progress("running")
        threading.Thread(target=heartbeat, daemon=True).start()

    def step():
        ctx.copy_state(dcp.NSE_SOLUTION, dcp.OLD_NSE_SOLUTION)
        ctx.copy_state(dcp.T_SOLUTION, dcp.OLD_T_SOLUTION)
        ctx.cfl_number()
        ctx.max_velocity()
        ctx.assemble_nse_system()
        if loud:
            progress("assembled")
        ctx.build_nse_preconditioner()
        if loud:
            progress("preconditioner built")
        ctx.assemble_temperature_matrix()
        ctx.assemble_temperature_rhs()
        rc, outer, inner = ctx.solve_nse()
        rcT, itT, _ = ctx.solve_temperature()
        t = ctx.timings()
        progress(f"step: solve {t['solve_nse_ms']:.1f} ms, {outer} outer / {inner} inner")
        return rc, outer, inner, itT, t

    for _ in range(args.warmup):
        step()

    def barrier():
        if dist is not None:
            dist.barrier()

    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    barrier()
    hip.hipDeviceSynchronize()
    t0 = time.perf_counter()
    recs = [step() for _ in range(args.steps)]
    hip.hipDeviceSynchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    n_nse = m.n_u + m.n_p
    asm_ms = np.mean([r[4]["assemble_nse_ms"] for r in recs])
    solve_ms = np.mean([r[4]["solve_nse_ms"] for r in recs])
    if dist is not None:
        # slowest rank bounds the job (wall time, assembly, solve)
        import torch
        tt = torch.tensor([elapsed, asm_ms, solve_ms], dtype=torch.float64, device=tdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed, asm_ms, solve_ms = (float(v) for v in tt.tolist())
    outer = recs[-1][1]
    inner = recs[-1][2]
    schur_ms = np.mean([r[4]["schur_apply_ms_avg"] for r in recs])
    pcie = None
    if world == 1:
        # boundary hand-over from host buffers (PCIe-inclusive, not `value`):
        # old u / T in, assemble_nse_system, the assembled rhs back out
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            ctx.set_state(dcp.OLD_NSE_SOLUTION, u0)
            ctx.set_state(dcp.OLD_T_SOLUTION, m.T0)
            ctx.assemble_nse_system()
            ctx.get_state(dcp.NSE_RHS)
            ts.append(time.perf_counter() - t0)
        pcie = {"value": n_nse / min(ts), "unit": "assembled DoFs/s",
                "ms": min(ts) * 1e3,
                "what": "host u_old/T_old upload + assemble_nse_system + rhs download, host clock"}
    # one step with each other Gram-Schmidt variant of the inner Schur GMRES
    # (deal.II's modified Gram-Schmidt is the reference's); at refine >= 6
    # only the device-resident ones (the modified one reads every step back), and
    # on several GPUs likewise (d + 1 all-reduces per column: seconds per step)
    other = []
    for other_gs in ("modified", "classical2", "dcgs2", "sstep"):
        if args.no_other_gs:
            break
        if other_gs == args.gram_schmidt or (other_gs == "modified" and
                                             (args.refine >= 6 or world > 1)):
            continue
        ctx.set_gram_schmidt(other_gs)
        r_o = step()
        other.append({"gram_schmidt": other_gs, "fgmres_outer_iterations": r_o[1],
                      "schur_gmres_inner_iterations": r_o[2],
                      "solve_nse_ms": r_o[4]["solve_nse_ms"],
                      "gmres_inner_iter_per_s": r_o[2] / (r_o[4]["solve_nse_ms"] * 1e-3),
                      "converged": r_o[0] == 0})
    ctx.set_gram_schmidt(args.gram_schmidt)
    full_ms = mfma_ms = float("nan")
    if args.refine <= 5:
        # the same assembly with the velocity block scattered as well (the
        # reference's distribute_local_to_global output;
        # DCP_OPT_ASSEMBLE_VELOCITY_BLOCK; 58 GB of block values at refine 6)
        ctx.set_assemble_velocity_block(True)
        full_ms = []
        for _ in range(3):
            ctx.assemble_nse_system()
            full_ms.append(ctx.timings()["assemble_nse_ms"])
        # and with its node-pair sums on the matrix cores (DCP_OPT_ELEMENT_MFMA)
        ctx.set_element_mfma(True)
        mfma_ms = []
        for _ in range(3):
            ctx.assemble_nse_system()
            mfma_ms.append(ctx.timings()["assemble_nse_ms"])
        ctx.set_element_mfma(False)
        ctx.set_assemble_velocity_block(False)
        full_ms = float(np.min(full_ms))
        mfma_ms = float(np.min(mfma_ms))
    if dist is not None:
        import torch
        tt = torch.tensor([full_ms], dtype=torch.float64, device=tdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        full_ms = float(tt.item())
    full_matrix = None if args.refine > 5 else {"value": n_nse / (full_ms * 1e-3), "unit": "assembled DoFs/s", "ms": full_ms,
                   "what": "assemble_nse_system with the velocity block A scattered into "
                           "block-CSR as well (DCP_OPT_ASSEMBLE_VELOCITY_BLOCK=1); `value` "
                           "assembles nse_matrix in operator form (B^T, B, rhs, constrained "
                           "diagonal), every A product being matrix-free",
                   "element_mfma": {"value": n_nse / (mfma_ms * 1e-3), "ms": mfma_ms,
                                    "what": "the same with the node-pair Gram sums as "
                                            "v_mfma_f64_16x16x4_f64 tiles "
                                            "(DCP_OPT_ELEMENT_MFMA=1; DESIGN section 4e)"}}
    if full_matrix is not None and world == 1:
        # the element system's structural flops (0.884 MFLOP per
        # cell, geometry excluded) against the FP64 peak (78.6 TFLOP/s, vector =
        # matrix on gfx950) and its bytes (element matrix + rhs + indices out,
        # state and geometry in: 67.4 KB per cell) against HBM; bound = the larger
        # of the two times
        fl, by = 0.884e6 * m.n_cells, 67372.0 * m.n_cells
        t = full_ms * 1e-3
        full_matrix["roofline"] = {
            "bound": "mfma" if fl / 78.6e12 > by / 8e12 else "hbm",
            "achieved_tflops": fl / t / 1e12, "peak_tflops": 78.6,
            "frac_flops": fl / t / 78.6e12,
            "achieved_gbs": by / t / 1e9, "peak_gbs": HBM_PEAK_GBS,
            "frac_hbm": by / t / (HBM_PEAK_GBS * 1e9),
            "what": "the full element system (SURVEY 8(d) flops / bytes per cell), timed "
                    "as the velocity-block assembly leg"}
    pinfo = ctx.pattern_info()
    # this rank's own sizes (owned + ghost layers; the global mesh on one GPU)
    ls = ctx.local_sizes()
    if args.schur == "explicit":
        # fused SELL SpMV with the formed S: values + column indices per
        # nonzero (8 + 0 B with structured columns -- level-major rows, column
        # from the row's level and the L2-resident lateral neighbour table,
        # DESIGN section 10 --, 8 + 2 B with the 16-bit RCM layout, 8 + 4 B
        # otherwise), slice offsets (+ column bases), gathered x, y write,
        # scaled-basis write xs, v0 read
        lay = ctx.schur_layout()
        n_rows = ls["owned_p"]  # S rows of this rank (the owned pressure dofs)
        n_sl = (n_rows + 63) // 64
        cb = lay["col_bytes"]
        sbytes = (8 + cb) * pinfo["nnz_S"] + 8 * (n_sl + 1) + (4 * n_sl if cb == 2 else 0) \
            + 32 * n_rows
        kernel = ("explicit Schur complement SpMV S x, SELL-64 fused (k_sell_spmv<true>"
                  + {0: ", structured columns, level-major order)",
                     2: ", 16-bit columns, RCM order)"}.get(cb, ")"))
    else:
        sbytes = schur_bytes(m, pinfo["nnzb_Bt"], pinfo["nnzb_B"])
        kernel = "Schur complement apply B D_A^-1 B^T (3 kernels)"
    if world > 1:
        kernel += f" [rank {rank}'s apply of a {world}-way partition: its own rows' bytes]"
    achieved = sbytes / (schur_ms * 1e-3) / 1e9 if schur_ms > 0 else 0.0
    # whole-job rate: the global system assembled by all ranks together
    value = n_nse / (asm_ms * 1e-3)
    out = {
        "metric": "assembled DoFs/sec + GMRES iter/sec, 3D shell Q2/Q1 refine=5, 1/2/4/8 GPU"
        if args.refine == 5 else
        f"assembled DoFs/sec + GMRES iter/sec, 3D shell Q2/Q1 refine={args.refine}, {world} GPU",
        "value": value,
        "unit": "assembled DoFs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",  # the global refine-5 mesh is fixed whatever N
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic refined hypershell (hyper_shell + SphericalManifold refinement, "
                "MappingQ(3) as deal.II 9.2, deal.II no-normal-flux normals), reference "
                "initial state",
        "config": {"workload": f"classic shell Q2/Q1 refine={args.refine}, one full time step",
                   "cells": m.n_cells, "nse_dofs": n_nse, "T_dofs": m.n_T,
                   "parallelism": "single GPU" if world == 1 else
                   f"{world} GPUs: p4est-style cell partition, RCCL ghost halo + all-reduce"},
        "gmres_outer_iter_per_s": outer / (solve_ms * 1e-3),
        "gmres_inner_iter_per_s": inner / (solve_ms * 1e-3),
        "fgmres_outer_iterations": outer,
        "schur_gmres_inner_iterations": inner,
        "T_cg_iterations": recs[-1][3],
        "phase_ms": {k: float(np.mean([r[4][k] for r in recs])) for k in recs[0][4]
                     if k.endswith("_ms") or k.endswith("_avg")},
        "setup_s": t_setup,
        "converged": all(r[0] == 0 for r in recs),
        "nse_solve_status": "converged" if all(r[0] == 0 for r in recs) else
        "NoConvergence: the reference's inner Schur GMRES (5000 iterations, tol 1e-6, "
        "identity preconditioner) stagnates on the near-null constant pressure mode at the "
        "first preconditioner application of both FGMRES attempts; the reference throws "
        "here (DESIGN.md section 5, the config-3 fixture)",
        "patterns": pinfo,
        "schur_mode": args.schur,
        "gram_schmidt": args.gram_schmidt,
        "other_gram_schmidt": other,
        "device_mem_gb": device_mem_gb(),
        "pcie_inclusive": pcie,
        "assembly_with_velocity_block": full_matrix,
        # the temperature system's own assembled-DoFs rate
        "T_assembly": {"value": m.n_T / (1e-3 * (np.mean([r[4]["assemble_T_matrix_ms"] for r in recs])
                                                 + np.mean([r[4]["assemble_T_rhs_ms"] for r in recs]))),
                       "unit": "assembled T DoFs/s (assemble_temperature_matrix + _rhs)"},
        "roofline": {"kernel": kernel, "bound": "hbm",
                     "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "traffic": pmc_traffic(args.refine, args.schur, m.n_p)
                     if world == 1 else sbytes,
                     "bytes_per_apply": sbytes, "avg_apply_ms": schur_ms},
    }
    ceil = measured_ceilings()
    if ceil:
        # the SpMV streams S (read-dominated): against the measured read ceiling
        out["roofline"]["frac_measured_read_ceiling"] = achieved / ceil["read_GBps"]
        out["measured_ceilings"] = ceil
    # the metric's own kernel work (value): operator-form assemble_nse_system.
    # Algorithmic bytes = its outputs written once (B^T values 24 B per block,
    # the velocity rhs 8 B per dof) + the old state read once (u 8 B per velocity
    # dof, T 8 B per dof); index data and geometry tables excluded
    asm_bytes = 24.0 * pinfo["nnzb_Bt"] + 16.0 * ls["n_u"] + 8.0 * ls["n_T"]
    asm_ach = asm_bytes / (asm_ms * 1e-3) / 1e9
    out["roofline_assembly"] = {
        "kernel": "operator-form assemble_nse_system (B^T in Kronecker form: k_btk_lateral "
                  "+ k_btk_entries, constrained rows condensed in place; the rhs by the pencil "
                  "kernel + velocity gather; the constrained diagonals in Kronecker form, "
                  "k_cdk_diag)",
        "bound": "hbm", "achieved": asm_ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": asm_ach / HBM_PEAK_GBS, "bytes_per_assembly": asm_bytes, "ms": asm_ms,
        "frac_measured_copy_ceiling": asm_ach / ceil["copy_GBps"] if ceil else None,
        # HBM bytes per assembly, 2 x FETCH_SIZE + WRITE_SIZE (the gfx950
        # correction, as for every other roofline here); the counts as taken
        # in traffic_detail
        "traffic": None, "traffic_detail": None}
    if world == 1:
        t_asm = pmc_asm_traffic(args.refine)
        if t_asm:
            out["roofline_assembly"]["traffic"] = t_asm["two_fetch_plus_write"]
            out["roofline_assembly"]["traffic_detail"] = t_asm
            out["roofline_assembly"]["traffic_over_output"] = t_asm["two_fetch_plus_write"] / asm_bytes
    else:
        out["roofline_assembly"]["traffic"] = asm_bytes
    if args.schur == "explicit" and world == 1:
        out["roofline_chain"] = (chain_roofline_trace(args.refine, m.n_p, args.gram_schmidt)
                                 or chain_roofline(args.refine, m.n_p, args.gram_schmidt))
    # the headline roofline against the committed trace of the same step: the
    # S SpMV's average over its working launches there
    tk = trace_kernel(trace_summary(args.refine, args.gram_schmidt), "k_sell_spmv<true, 2>")
    if tk and world == 1 and args.schur == "explicit":
        t_ms = tk[1]["avg_ns_full"] * 1e-6
        out["roofline"]["trace_check"] = {
            "source": TRACE[(args.refine, args.gram_schmidt)], "kernel": tk[0].split("(")[0],
            "launches": tk[1]["full_calls"], "early_exits_dropped": tk[1]["early_exit_calls"],
            "avg_apply_ms": t_ms, "achieved": sbytes / (t_ms * 1e-3) / 1e9,
            "frac": sbytes / (t_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "line_over_trace": (achieved / (sbytes / (t_ms * 1e-3) / 1e9)) if t_ms > 0 else None}
    # matrix-free operator apply (north-star target, SURVEY §8d byte count):
    # src read + dst write per dof, int32 cell->dof map, J^-1 + JxW per point
    # (SURVEY's unit of work; the kernel recomputes the geometry instead of
    # streaming it, so "traffic" - the PMC bytes actually moved - is lower);
    # one apply = the cell-order pencil kernel + the dof gather
    st_ms = np.mean([r[4]["stokes_apply_ms_avg"] for r in recs])
    ve_ms = np.mean([r[4]["velocity_apply_ms_avg"] for r in recs])
    if st_ms > 0 or ve_ms > 0:
        nc = ls["cells"]  # the apply runs over every local cell (owned + ghost layers)
        st_bytes = 16 * (ls["n_u"] + ls["n_p"]) + 4 * 89 * nc + 80 * 27 * nc
        ve_bytes = 16 * ls["n_u"] + 4 * 27 * nc + 80 * 27 * nc
        mf_traffic, mf_traffic_why = pmc_mf_traffic(args.refine) if world == 1 else (st_bytes, None)
        mf = {"kernel": "matrix-free [A B^T; B 0] x (k_mf_pencil<true> cell-order sum "
                        "factorisation + k_mf_gather dof gather)",
              "bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s",
              "traffic": mf_traffic, "traffic_source": PMC_MF.get(args.refine, (None,))[0]
              if world == 1 else "per-rank byte model",
              "traffic_missing": mf_traffic_why,
              "bytes_per_apply": st_bytes, "avg_apply_ms": st_ms,
              "applies_per_step": recs[-1][4]["stokes_applies"],
              "achieved": st_bytes / (st_ms * 1e-3) / 1e9 if st_ms > 0 else None,
              "velocity_block": {"bytes_per_apply": ve_bytes, "avg_apply_ms": ve_ms,
                                 "applies_per_step": recs[-1][4]["velocity_applies"],
                                 "achieved": ve_bytes / (ve_ms * 1e-3) / 1e9 if ve_ms > 0
                                 else None}}
        mf["frac"] = mf["achieved"] / HBM_PEAK_GBS if mf["achieved"] else None
        # back-to-back applies (after the timed steps, outside them): one HIP
        # event pair per batch of 48 applies on the context's stream, the
        # sources rotating over 8 vectors (320 MB, more than the 256 MB
        # Infinity Cache: every source cold, as a solve's Krylov vectors are).
        # The in-step figure above is one event pair around every sampled
        # apply, whose own cost (~6 us of command-processor markers) it
        # includes: the kernel trace of the step puts pencil + gather at the
        # back-to-back time
        if world == 1 and not args.no_back_to_back:
            b2b = back_to_back_applies(ctx, ls)
            if b2b:
                mf["in_step_sampled"] = {"avg_apply_ms": st_ms, "achieved": mf["achieved"],
                                         "frac": mf["frac"]}
                mf["avg_apply_ms"] = b2b["nse_ms"]
                mf["achieved"] = st_bytes / (b2b["nse_ms"] * 1e-3) / 1e9
                mf["frac"] = mf["achieved"] / HBM_PEAK_GBS
                mf["velocity_block"]["in_step_avg_apply_ms"] = ve_ms
                mf["velocity_block"]["avg_apply_ms"] = b2b["velocity_ms"]
                mf["velocity_block"]["achieved"] = ve_bytes / (b2b["velocity_ms"] * 1e-3) / 1e9
                mf["timing"] = b2b["what"]
        if ceil and mf["achieved"]:
            mf["frac_measured_read_ceiling"] = mf["achieved"] / ceil["read_GBps"]
        tr = trace_summary(args.refine, args.gram_schmidt)
        tp, tg = trace_kernel(tr, "k_mf_pencil<true, true, false>"), trace_kernel(tr, "k_mf_gather<true>")
        if tp and tg and world == 1:
            t_ms = (tp[1]["avg_ns_full"] + tg[1]["avg_ns_full"]) * 1e-6
            mf["trace_check"] = {"source": tr["path"], "pencil_us": tp[1]["avg_ns_full"] * 1e-3,
                                 "gather_us": tg[1]["avg_ns_full"] * 1e-3,
                                 "avg_apply_ms": t_ms,
                                 "frac": st_bytes / (t_ms * 1e-3) / 1e9 / HBM_PEAK_GBS}
        # the bytes the apply actually moves (PMC; the geometry is recomputed,
        # not read) over the same apply time
        mf["frac_actual_traffic"] = (mf["traffic"] / (mf["avg_apply_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS
                                     if mf["traffic"] and mf["avg_apply_ms"] > 0 else None)
        out["roofline_matrix_free"] = mf
    t_last = recs[-1][4]
    out["handoff_timeouts"] = int(t_last.get("handoff_timeouts", 0))
    out["coop_launch"] = os.environ.get("DCP_COOP_LAUNCH", "0") == "1"
    if world > 1:
        # what each rank's communicator reports, its sizes and bytes per apply
        # (the traffic of N > 1 lines is this per-rank byte model: no PMC there)
        mine = {"rank": rank, "comm": ctx.comm_info(), "sizes": ls,
                "device_memory": ctx.device_memory(),
                "schur_bytes": sbytes, "schur_apply_ms": schur_ms,
                "assembly_bytes": asm_bytes, "assemble_ms": float(np.mean(
                    [r[4]["assemble_nse_ms"] for r in recs]))}
        gathered = [None] * world
        dist.all_gather_object(gathered, mine)
        out["ranks"] = gathered
        out["comm_ranks_reported"] = sorted({g["comm"]["ranks"] for g in gathered})
        out["comm_devices"] = [g["device"] for g in comm_seen]
        out["launcher"] = ("bench.py --gpus (launch_ranks)" if os.environ.get("DCP_BENCH_CHILD")
                           else "external (torch.distributed.run)")
        if out["comm_ranks_reported"] != [world]:
            raise SystemExit(f"comm_ranks_reported {out['comm_ranks_reported']} != [{world}]")
        # DESIGN.md section 6 "Cost at P=8, r=5": the expected strong-scaling
        # efficiency of each phase (budgeted, not measured)
        out["design_expectation"] = {
            "assembly_and_matrix_free": "~0.75 at P=8 (34 % ghost cells with two layers)",
            "inner_schur_gmres": "~0.27 at P=8 (2.2x: s-step + matrix powers; the block's two "
                                 "all-reduces and three launches dominate)",
            "source": "DESIGN.md section 6"}
    if world == 1 and not args.no_converging_leg:
        out["converging_step"] = converging_leg(make_ctx, args)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        progress("cpu baseline")
        out["cpu_baseline"] = cpu_baseline(
            ctx, m, args.refine, out["gmres_inner_iter_per_s"],
            full_matrix["value"] if full_matrix else None)
        cs = out.get("converging_step")
        if cs:
            out["cpu_baseline"]["same_config_ratio"]["outer_fgmres_refine3"] = (
                cs["gmres_outer_iter_per_s"] / out["cpu_baseline"]["outer"]["value"])
    if rank == 0:
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


def print_maps():
    """DCP_BENCH_MAPS=1: the executable mappings of this process on stderr, to
    place the frames of a crash at exit (their libraries) after the fact."""
    if os.environ.get("DCP_BENCH_MAPS") != "1":
        return
    with open("/proc/self/maps") as f:
        for line in f:
            parts = line.split()
            if len(parts) >= 6 and "x" in parts[1]:
                print("[maps] " + parts[0] + " " + parts[5], file=sys.stderr)
    sys.stderr.flush()


if __name__ == "__main__":
    main()
    print_maps()
