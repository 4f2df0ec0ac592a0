"""bench.py --gpus N starts its own N rank processes (no external launcher),
checked on the CPU with --dry-launch: every child gets RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_ADDR / MASTER_PORT, joins the gloo rendezvous, receives
rank 0's communicator id through torch.distributed's broadcast (the path the
RCCL id takes on the GPU box) and stops before any GPU call. Reference: one
MPI rank per process, source/main.cxx:64-65, planet_geometry.tpp:13-20."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(args, extra_env=None, timeout=240):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(extra_env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=timeout, cwd=ROOT)


@pytest.mark.parametrize("n", [2, 8])
def test_gpus_n_spawns_n_ranks(n):
    out = run_bench(["--gpus", str(n), "--dry-launch"])
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["dry_launch"] and d["n_gpus"] == n and d["world_size"] == n
    ranks = d["ranks"]
    assert [r["rank"] for r in ranks] == list(range(n))
    assert [r["local_rank"] for r in ranks] == list(range(n))  # one device per rank
    assert all(r["world_size"] == n for r in ranks)
    assert len({r["pid"] for r in ranks}) == n  # separate processes
    assert len({r["master"] for r in ranks}) == 1
    assert all(r["master"].startswith("127.0.0.1:") for r in ranks)
    assert all(r["backend"] == "gloo" for r in ranks)
    # every rank holds rank 0's id
    assert len({r["nccl_id_sha"] for r in ranks}) == 1 and ranks[0]["nccl_id_sha"]
    assert not any(r["gpu_touched"] for r in ranks)


def test_single_gpu_runs_in_process():
    out = run_bench(["--gpus", "1", "--dry-launch"])
    assert out.returncode == 0, out.stderr[-3000:]
    d = json.loads(out.stdout.strip().splitlines()[-1])
    assert d["world_size"] == 1 and d["ranks"][0]["backend"] is None


def test_failing_rank_fails_the_launch():
    out = run_bench(["--gpus", "2", "--dry-launch"], {"DCP_BENCH_DRY_FAIL_RANK": "1"})
    assert out.returncode == 3, (out.returncode, out.stderr[-2000:])
    assert "launch of 2 ranks failed" in out.stderr


def test_driver_torchrun_command_is_not_respawned():
    """The driver's own N>1 command (torch.distributed.run sets WORLD_SIZE):
    bench.py is then one rank and must not start ranks of its own."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                          "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
                          "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                          "--gpus", "2", "--dry-launch"],
                         env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    assert d["world_size"] == 2 and [r["rank"] for r in d["ranks"]] == [0, 1]
    assert len({r["pid"] for r in d["ranks"]}) == 2
