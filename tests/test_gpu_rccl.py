"""The multi-shard path over real RCCL on a one-GPU box.

RCCL refuses two ranks on one device ("Duplicate GPU detected") unless they look like
different hosts: `bench.py --one-gpu` gives every rank its own NCCL_HOSTID, so two processes
on device 0 form a communicator whose exchange runs over RCCL's socket transport. Everything
the N-GPU run does then executes for real: the sharded APSP (row blocks broadcast over RCCL,
checked against a table built whole on every rank), per-round grouped ncclSend/ncclRecv of the
exchange slots and messages, k_import with the window advance, the graph-captured round
batches (SGN_GRAPH=1) or eager rounds (the default), and bench's shard_check, which re-runs all hosts
unsharded on rank 0 and compares every counter, the window and every host's digests bit for
bit. Timing from this transport means nothing; the driver's multi-GPU bench measures xGMI.
"""
import json
import os
import pathlib
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = pathlib.Path(__file__).resolve().parent.parent


# xsz: the exchange size the first rounds move per peer (SGN_XSZ_INIT); 16 runs make the
# early rounds exceed it, so they are held and completed with the whole slot (spill path)
# workload D: every host sends to a random peer every round (half of it to the other shard),
# through the LDS bucket minima of the PERIODIC kernel and a spill to a larger exchange size
# pools: a one-page-per-host CoDel pool, 16-run calendar slabs and a 64-run exchange slot, so
# rounds are held on both ranks alike (guards evaluated from the round-edge messages) while the
# pools and the slots grow over real RCCL
@pytest.mark.parametrize("graph,xsz,port,workload,pools", [("1", "", 29541, "C", False), ("0", "", 29542, "C", False),
                                                           ("1", "16", 29543, "C", False), ("0", "", 29544, "D", False),
                                                           ("0", "", 29545, "C", True)])
def test_rccl_two_ranks_one_gpu_match_unsharded(graph, xsz, port, workload, pools):
    env = dict(os.environ, SGN_GRAPH=graph, NCCL_DEBUG="WARN", TMPDIR="/tmp")
    if xsz:
        env["SGN_XSZ_INIT"] = xsz
    extra = []
    if pools:
        env["SGN_SLAB_CAP"] = "16"
        extra = ["--codel-cap", "1", "--exchange-slot", "64"]
    cmd = [sys.executable, "-u", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--one-gpu", "--hosts", "100000", "--rounds-per-step", "70",
           "--workload", workload] + extra
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-4000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2
    assert line["apsp_sharded"]["equal_on_all_ranks"] is True
    assert line["parity"] is True, line.get("parity_detail")
    # config C as BASELINE names it: 100k hosts in total, 2 x 50k (strong scaling)
    assert line["parity_detail"]["hosts_compared"] == 100_000
    assert line["config"]["hosts_total"] == 100_000 and line["scaling"] == "strong"
    assert line["rounds_timed"] == 140
    x = line["exchange"]
    assert x["hwm_runs"] > 0 and x["send_runs"] >= min(x["slot_runs"], x["hwm_runs"])
    if xsz:
        assert x["spills"] >= 1
    if pools:
        assert x["slot_runs"] > 64 and x["spills"] >= 1


@pytest.mark.parametrize("workload,port,launcher", [("C", 29548, False), ("D", 29549, True)])
def test_xpeer_two_processes_one_gpu_persistent(workload, port, launcher):
    """The N-GPU persistent path itself (k_rounds_x with peer-mapped inboxes): two processes on
    device 0 (SGN_XPEER_SHARED=1 lets the IPC mapping accept a peer on the same GPU; each grid
    is sized for half the GPU), every round's runs stored straight into the other process's
    inbox bins and slots, the messages (tagged 8-byte words, system-scope release and acquire)
    and the residency census across processes — against the unsharded run, bit for bit.
    Config C runs as the driver invokes the scaling bench without a launcher: `bench.py --gpus 2`
    starts its two ranks itself and the line says n_gpus 2."""
    env = dict(os.environ, SGN_GRAPH="0", NCCL_DEBUG="WARN", TMPDIR="/tmp", SGN_XPEER_SHARED="1")
    cmd = [sys.executable, "-u", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port)] if launcher else [sys.executable, "-u"]
    cmd += ["bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1", "--one-gpu", "--rounds-per-step", "70",
            "--workload", workload]
    if workload == "D":
        cmd += ["--hosts", "100000"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2
    assert line["exchange"]["mode"] == 2 and line["exchange"]["persistent_launches"] > 0, line["exchange"]
    assert line["roofline"]["kernel"] == "k_rounds_x"
    assert line["parity"] is True, line.get("parity_detail")


def test_xpeer_refusal_on_one_gpu_falls_back_everywhere():
    """a shard whose GPU cannot hold a resident k_rounds_x grid (forced on rank 1 by
    SGN_XREFUSE_RANK) must not leave its peers waiting in a launch it never joins: it launches
    one workgroup that tells them "not resident", and BOTH shards go on with per-round launches
    and the RCCL exchange — bit-exact against the unsharded run."""
    env = dict(os.environ, SGN_GRAPH="0", NCCL_DEBUG="WARN", TMPDIR="/tmp", SGN_XPEER_SHARED="1",
               SGN_XREFUSE_RANK="1")
    cmd = [sys.executable, "-u", "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "1", "--one-gpu",
           "--rounds-per-step", "40", "--hosts", "20000"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["exchange"]["mode"] == 1, line["exchange"]
    assert line["engine"]["persistent_fallbacks"] >= 1
    assert line["parity"] is True, line.get("parity_detail")


def test_rccl_eight_ranks_one_gpu_match_unsharded():
    """The driver's N = 8 configuration: config C's 100 k hosts over eight ranks (12.5 k each),
    every rank exchanging with seven peers each round, against one unsharded run."""
    env = dict(os.environ, NCCL_DEBUG="WARN", TMPDIR="/tmp")
    cmd = [sys.executable, "-u", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", "29546", "bench.py", "--gpus", "8",
           "--steps", "2", "--warmup", "1", "--one-gpu", "--hosts", "100000", "--rounds-per-step", "40"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-4000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 8 and line["config"]["hosts_per_gpu"] == 12_500
    assert line["apsp_sharded"]["equal_on_all_ranks"] is True
    assert line["parity"] is True, line.get("parity_detail")
    assert line["parity_detail"]["hosts_compared"] == 100_000
    assert line["rounds_timed"] == 80


def test_rccl_two_ranks_import_spill_hot_slabs():
    """Imported runs past their slab: workload H's servers sit in
    rank 0 and ~10 k clients of rank 1 fetch from them at the same instant, so k_import files thousands of
    runs into the servers' 16-run slabs (SGN_SLAB_CAP; SGN_SLAB_LIM keeps them small): they go
    past the slab into the spill area, the next round's gathers read them from there (the
    big-slab path), every rank holds the round after alike and the calendars are re-laid out
    with extensions. Eager 32-round batches over real RCCL, against the unsharded run."""
    env = dict(os.environ, SGN_GRAPH="0", NCCL_DEBUG="WARN", TMPDIR="/tmp", SGN_SLAB_CAP="16", SGN_SLAB_LIM="32")
    cmd = [sys.executable, "-u", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29547", "bench.py", "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--one-gpu", "--workload", "H", "--hosts", "20000",
           "--nodes", "50", "--rounds-per-step", "40"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["parity"] is True, line.get("parity_detail")
    assert line["parity_detail"]["hosts_compared"] == 20_000
    e = line["engine"]
    assert e["calendar_spill_runs"] > 0 and e["rounds_held"] >= 1 and e["slab_extensions"] >= 1, e
