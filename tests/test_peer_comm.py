"""Device-initiated all-reduce (PeerComm, comm.h / kernels/peer.hip) on
in-process groups: every rank's partial stored into every rank's mailbox,
tagged, polled and summed in rank order on the device, no host rendezvous.

Against LocalComm (host-barrier rendezvous + group_reduce) the sums are in
the same order, so the time step must agree BITWISE on every rank: the rhs,
the solution, iteration counts, the temperature and the CFL numbers. The
all-reduce latency on one GPU is printed. The checks run in a child process
with GPU_MAX_HW_QUEUES=32 (tests/_peer_comm_worker.py): in one process the
ranks' polling kernels need hardware queues of their own, which PeerComm
checks (it refuses to deadlock on shared queues). Reference: the
MPI_Allreduce behind every Trilinos dot of the inner Schur GMRES,
block_schur_preconditioner.hpp:46-51."""
import json
import os
import subprocess
import sys

import pytest

import dcp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _worker(what):
    env = dict(os.environ, GPU_MAX_HW_QUEUES="32")
    out = subprocess.run([sys.executable, "-u", os.path.join(HERE, "_peer_comm_worker.py"), what],
                         env=env, capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stderr[-3000:]
    return json.loads(out.stdout.strip().splitlines()[-1])[what]


def test_peer_allreduce_sums_in_rank_order():
    for r in _worker("selftests"):
        print(r)
        assert r["equals_expected"] and r["peer_equals_local"], r
        assert set(r["transports"]) == {"peer", "in-process"}, r


def test_peer_group_time_step_is_bitwise_local():
    """Bitwise on 2, 3 and 8 ranks. (The 8-rank s-step case found a race in
    the multi-launch s-step and DCGS2 steps: k_ss_final / k_dcgs_update tested
    st->status, which their block 0 sets when the cycle stops there, so blocks
    scheduled after it skipped their rows of the last basis vectors; they now
    test the copy the previous launch took, GmresDev::status_in. DESIGN 12b.)"""
    for r in _worker("time_steps"):
        print(r)
        assert r["transports"] == ["peer", "in-process"], r
        assert r["bitwise"], r


def test_peer_comm_refuses_shared_hardware_queues(monkeypatch):
    """In this process (HIP's default 4 hardware queues) an 8-rank peer group
    would share queues: context creation fails loudly instead of deadlocking."""
    import threading
    monkeypatch.setenv("DCP_PEER_COMM", "1")
    monkeypatch.delenv("GPU_MAX_HW_QUEUES", raising=False)
    g = dcp.Group(8)
    errors = []

    def run(rank):
        try:
            dcp.Context(rank=rank, world_size=8, group=g).close()
        except dcp.DcpError as e:
            errors.append(str(e))

    th = [threading.Thread(target=run, args=(r,)) for r in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=60)
    g.close()
    assert len(errors) == 8 and all("GPU_MAX_HW_QUEUES" in e for e in errors), errors
