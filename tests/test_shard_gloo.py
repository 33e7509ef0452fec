"""Multi-shard round-edge protocol on the CPU (world_size 2, gloo).

libsgn's multi-GPU path (shadow-gen_amd/csrc/comm.cpp) shards hosts into contiguous HostId
ranges and, every round: exchanges the events each shard produced for the other shards'
hosts, files them into the owners' queues, all-reduces {min next event time, min used
latency} and advances the window on every shard. This test rehearses exactly that protocol
with the oracle over torch.distributed/gloo and requires the sharded run to be identical
(per-host order-sensitive digests, counters, final window) to the unsharded run.
"""
import os
import pathlib
import sys

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent
INVALID = 0xFFFFFFFFFFFFFFFF
I64_INF = (1 << 63) - 1


def workload(kind):
    sys.path.insert(0, str(ROOT / "shadow-gen_amd"))
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle_py
    import sgn

    n, V = 240, 24
    g = sgn.tor_graph(V, seed=4) if kind in ("tgen", "bench_check", "bench_check_bad") else sgn.random_graph(V, seed=4)
    used = np.arange(V)
    lat, loss = oracle_py.routes(g, used)
    seeds = oracle_py.host_seeds(1, sgn.host_names(n))
    bw = np.where(np.arange(n) % 7 == 0, 100_000_000, 5_000_000).astype(np.uint64)
    hosts = sgn.HostArrays(sgn.assign_ips(n), (np.arange(n) * 5) % V, bw, bw, seeds)
    dyn = kind == "dynamic"
    cfg = sgn.make_config(400_000_000, runahead_ns=0 if dyn else 1_000_000, dynamic=dyn,
                          codel_cap=1 << 14)
    if kind in ("tgen", "bench_check", "bench_check_bad"):
        tr = sgn.make_traffic(sgn.TRAFFIC_TGEN, period_ns=60_000_000, period_jitter_ns=60_000_000,
                              start_jitter_ns=30_000_000, servers=np.arange(0, n, 8),
                              file_bytes=(20_000, 80_000, 200_000))
    else:
        tr = sgn.make_traffic(period_ns=2_000_000, start_jitter_ns=2_000_000,
                              unknown_dst_permille=20)
    return oracle_py, sgn, used, lat, loss, hosts, cfg, tr


def to_i64(x):
    return I64_INF if x == INVALID else int(x)


def from_i64(x):
    return INVALID if x == I64_INF else int(x)


def worker(rank, world, port, kind, q):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        oracle_py, sgn, used, lat, loss, hosts, cfg, tr = workload(kind)
        sim = oracle_py.Sim(used, lat, loss, hosts, cfg, tr)
        import ctypes as C
        lo, hi = C.c_uint32(), C.c_uint32()
        sgn.load().sgn_shard_range(hosts.n, rank, world, C.byref(lo), C.byref(hi))
        lo, hi = lo.value, hi.value
        sim.set_shard(lo, hi)
        rounds = 0
        while sim.window()[2]:
            ex = sim.shard_execute()  # rows: dst, time, src, eid, payload, tag
            # exchange: every shard sends the events of the other shards' hosts
            flat = torch.from_numpy(ex.astype(np.int64).ravel()) if len(ex) else torch.zeros(0, dtype=torch.int64)
            sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
            dist.all_gather(sizes, torch.tensor([flat.numel()], dtype=torch.int64))
            mx = max(int(s.item()) for s in sizes)
            pad = torch.zeros(mx, dtype=torch.int64)
            pad[: flat.numel()] = flat
            bufs = [torch.zeros(mx, dtype=torch.int64) for _ in range(world)]
            dist.all_gather(bufs, pad)
            for r in range(world):
                if r == rank:
                    continue
                recs = bufs[r][: int(sizes[r].item())].numpy().astype(np.uint64).reshape(-1, 6)
                mine = recs[(recs[:, 0] >= lo) & (recs[:, 0] < hi)]
                if len(mine):
                    sim.shard_import(mine)
            mn, mu = sim.shard_local_min()
            t = torch.tensor([to_i64(mn), to_i64(mu)], dtype=torch.int64)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            sim.shard_advance(from_i64(t[0].item()), from_i64(t[1].item()))
            rounds += 1
        if kind in ("bench_check", "bench_check_bad"):
            # bench.py's N > 1 verification, over this sharded run: rank 0 re-runs unsharded
            sys.path.insert(0, str(ROOT))
            import bench

            def unsharded():
                if kind == "bench_check_bad":  # a different run: the verdict must say so
                    seeds = hosts.seed.copy()
                    seeds[7] ^= 1
                    h2 = sgn.HostArrays(hosts.ip, hosts.node_id, hosts.bw_up, hosts.bw_down, seeds)
                    return oracle_py.Sim(used, lat, loss, h2, cfg, tr)
                return oracle_py.Sim(used, lat, loss, hosts, cfg, tr)

            out = bench.shard_check(sim, dist, rank, world, hosts.n, rounds, unsharded)
            q.put((rank, out))
            return
        q.put((rank, lo, hi, sim.digests(lo, hi), sim.stats(), sim.window(), rounds))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["periodic", "tgen", "dynamic"])
def test_two_shards_match_single(kind):
    import torch.multiprocessing as mp

    oracle_py, sgn, used, lat, loss, hosts, cfg, tr = workload(kind)
    ref = oracle_py.Sim(used, lat, loss, hosts, cfg, tr)
    ref.run()
    ref_d = ref.digests()
    ref_st = ref.stats()
    assert ref_st["packets_sent"] > 1000

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000)
    procs = [ctx.Process(target=worker, args=(r, 2, port, kind, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=600) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    total = {k: 0 for k in ref_st}
    for rank, lo, hi, d, st, win, rounds in res:
        for f in ("tx", "rx", "app", "rng", "next_event_id", "n_sent", "n_popped"):
            assert np.array_equal(d[f], ref_d[f][lo:hi]), (kind, rank, f)
        assert win == ref.window()
        assert rounds == ref_st["rounds"]
        for k in ("packets_sent", "packets_loss_dropped", "packet_events_popped", "delivered",
                  "codel_dropped", "local_events"):
            total[k] += st[k]
    for k in ("packets_sent", "packets_loss_dropped", "packet_events_popped", "delivered",
              "codel_dropped", "local_events"):
        assert total[k] == ref_st[k], k


@pytest.mark.parametrize("kind", ["bench_check", "bench_check_bad"])
def test_bench_shard_check_over_gloo(kind):
    """bench.py's multi-GPU parity verdict (shard_check: gather every shard's digests and
    counters, re-run unsharded on rank 0, compare) on two oracle shards over gloo; a
    reference run that differs in one host's seed must be reported."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 30500 + (os.getpid() % 1000)
    procs = [ctx.Process(target=worker, args=(r, 2, port, kind, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=600) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[1] is None
    v = res[0]
    assert v["hosts_compared"] == 240 and v["rounds_compared"] > 100
    if kind == "bench_check":
        assert v["ok"], v["mismatches"]
    else:
        assert not v["ok"] and any("HostId 7" in m for m in v["mismatches"]), v
