"""Worker of tests/test_peer_comm.py, run in its own process with
GPU_MAX_HW_QUEUES=32 (every in-process rank's streams on hardware queues of
their own, which PeerComm's polling all-reduce needs; the test process itself
keeps HIP's default of 4). Prints one JSON line with the comparisons."""
import json
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-dycoreplanet_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import dcp  # noqa: E402


def group_selftest(world, n, reps, peer):
    os.environ["DCP_PEER_COMM"] = "1" if peer else "0"
    g = dcp.Group(world)
    out, errors = [None] * world, []

    def run(rank):
        try:
            ctx = dcp.Context(rank=rank, world_size=world, group=g)
            vec = np.arange(n, dtype=np.float64) * (rank + 1) + 0.1 * rank
            s, ms = ctx.allreduce_selftest(vec, reps)
            out[rank] = (s, ms, ctx.comm_info()["transport"])
            ctx.close()
        except Exception as e:  # noqa: BLE001
            errors.append((rank, repr(e)))

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    g.close()
    if errors:
        raise RuntimeError(str(errors))
    return out


def selftests():
    res = []
    for world, n in ((2, 1), (3, 122), (8, 122), (8, 4096), (8, 5000)):
        peer = group_selftest(world, n, 200, True)
        local = group_selftest(world, n, 200, False)
        expect = np.zeros(n)
        for r in range(world):
            expect = expect + (np.arange(n, dtype=np.float64) * (r + 1) + 0.1 * r)
        res.append({"world": world, "n": n,
                    "transports": sorted({p[2] for p in peer} | {p[2] for p in local}),
                    "peer_equals_local": all(np.array_equal(peer[r][0], local[r][0])
                                             for r in range(world)),
                    "equals_expected": all(np.array_equal(peer[r][0], expect) for r in range(world)),
                    "peer_us": 1e3 * max(p[1] for p in peer),
                    "local_us": 1e3 * max(p[1] for p in local)})
    return res


def time_steps():
    from test_multi_rank import _group_run
    res = []
    cases = ((2, 2, "sstep", 0), (3, 2, "modified", 0), (3, 2, "classical2", 0),
             (8, 3, "sstep", 0), (8, 3, "dcgs2", 24))
    if os.environ.get("PEER_CASES"):
        cases = [c for c in cases if f"{c[0]}-{c[1]}-{c[2]}" in os.environ["PEER_CASES"].split(",")]
    for world, refine, gs, fixed in cases:
        m = dcp.HostMesh(refine=refine)
        ph = dcp.classic_physics()
        rng = np.random.default_rng(23)
        u = np.zeros(m.n_u + m.n_p)
        u[:m.n_u] = 0.05 * rng.uniform(-1, 1, m.n_u)
        T = m.T0.copy()

        def setup(ctx):
            ctx.set_gram_schmidt(gs)
            ctx.set_block_fixed_inner(fixed)
            if os.environ.get("WORKER_MP") == "0":  # diagnostics: per-SpMV halo exchanges
                ctx.set_matrix_powers(False)

        out = {}
        extra = {}
        for peer in (True, False):
            os.environ["DCP_PEER_COMM"] = "1" if peer else "0"
            if os.environ.get("PEER_VARIANTS") and peer:
                base_x = None
                for var in os.environ["PEER_VARIANTS"].split(";"):
                    for kv in var.split(","):
                        k_, v_ = kv.split("=")
                        os.environ[k_] = v_
                    runs = [_group_run(world, m, ph, u, T, setup, None) for _ in range(2)]
                    extra["var " + var] = [
                        all(np.array_equal(a["x"].view(np.int64), b["x"].view(np.int64))
                            for a, b in zip(runs[0], runs[1]))]
                    for kv in var.split(","):
                        os.environ.pop(kv.split("=")[0], None)
            if os.environ.get("PEER_TWICE") and peer:
                extra["again"] = _group_run(world, m, ph, u, T, setup,
                                            lambda c: [c.comm_info()["transport"],
                                                       c.timings()["solve_nse_ms"]])
            if os.environ.get("LOCAL_TWICE") and not peer:
                extra["local_again"] = _group_run(world, m, ph, u, T, setup, None)
            out[peer] = _group_run(world, m, ph, u, T, setup,
                                   lambda c: [c.comm_info()["transport"], c.timings()["solve_nse_ms"],
                                                       c.timings().get("handoff_timeouts", 0)])
        same = True
        diff = {}
        for r, (a, b) in enumerate(zip(out[True], out[False])):
            same &= tuple(a["nse"]) == tuple(b["nse"]) and a["T"][1] == b["T"][1]
            if tuple(a["nse"]) != tuple(b["nse"]) or a["T"][1] != b["T"][1]:
                diff[f"{r}:counts"] = [list(a["nse"]), list(b["nse"]), a["T"][1], b["T"][1]]
            for key in ("x", "Tx", "rhs", "T_rhs"):
                eq = bool(np.array_equal(a[key].view(np.int64), b[key].view(np.int64)))
                same &= eq
                if not eq:
                    diff[f"{r}:{key}"] = float(np.max(np.abs(a[key] - b[key])) /
                                              max(np.max(np.abs(b[key])), 1e-300))
            same &= a["cfl"] == b["cfl"] and a["vmax"] == b["vmax"]
            if a["cfl"] != b["cfl"] or a["vmax"] != b["vmax"]:
                diff[f"{r}:cfl/vmax"] = [a["cfl"], b["cfl"], a["vmax"], b["vmax"]]
        for key_ in [k_ for k_ in extra if k_.startswith("var ")]:
            diff[key_] = extra[key_]
        if "local_again" in extra:
            diff["local_vs_local_bitwise"] = all(
                np.array_equal(a["x"].view(np.int64), b["x"].view(np.int64))
                for a, b in zip(extra["local_again"], out[False]))
        if "again" in extra:
            diff["peer_vs_peer_bitwise"] = all(
                np.array_equal(a["x"].view(np.int64), b["x"].view(np.int64))
                for a, b in zip(extra["again"], out[True]))
        res.append({"world": world, "refine": refine, "gs": gs, "fixed_inner": fixed,
                    "transports": [out[True][0]["extra"][0], out[False][0]["extra"][0]],
                    "bitwise": bool(same), "nse": list(out[True][0]["nse"]), "diff": diff,
                    "handoff_timeouts": [sum(r["extra"][2] for r in out[True]),
                                         sum(r["extra"][2] for r in out[False])],
                    "solve_ms_peer": max(r["extra"][1] for r in out[True]),
                    "solve_ms_local": max(r["extra"][1] for r in out[False])})
    return res


if __name__ == "__main__":
    what = sys.argv[1]
    res = {what: selftests() if what == "selftests" else time_steps()}
    # a copy for the measurement record when run on the GPU box
    if os.path.isdir(os.path.join(ROOT, "gpurun_out")):
        with open(os.path.join(ROOT, "gpurun_out", f"peer_comm_{what}.json"), "w") as f:
            json.dump(res, f, indent=1)
    print(json.dumps(res), flush=True)
