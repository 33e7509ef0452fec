"""Shared driver for the CPU-resident-application path (SGN_TRAFFIC_EXTERNAL): a CPU
controller that submits datagrams, moves the window to its own next send when that comes
first (sgn_set_window) and drains the datagrams' fates. Used against the oracle alone (CPU
tests) and against libsgn + the oracle in lockstep (GPU tests)."""
import numpy as np

import sgn

RUNAHEAD = 1_000_000


def external_world(n=60, V=20, seed=3, bw=2_000_000, fifo=4, stop_ns=400_000_000):
    g = sgn.random_graph(V, mean_degree=min(6, V - 1), seed=seed, loss_frac=0.5, loss_hi=0.05)
    used = np.arange(V)
    names = sgn.host_names(n)
    seeds = sgn.derive_seeds(11, names)
    bwv = np.full(n, bw, dtype=np.uint64)
    bwv[::7] = 200_000  # slow links: standing CoDel queues and drops
    hosts = sgn.HostArrays(sgn.assign_ips(n), (np.arange(n) * 5) % V, bwv, bwv, seeds)
    cfg = sgn.make_config(stop_ns, runahead_ns=RUNAHEAD, out_fifo_cap=fifo, codel_cap=4096,
                          event_capacity=1 << 18)
    tr = sgn.make_traffic(sgn.TRAFFIC_EXTERNAL)
    return g, used, hosts, cfg, tr


def datagrams(hosts, k=600, seed=5, span_ns=150_000_000):
    """k datagrams: random peers, some to unknown addresses or to the sender itself, bursts
    from a few hosts (send-queue blocking), times over [0, span)."""
    rng = np.random.default_rng(seed)
    n = hosts.n
    src = rng.integers(0, n, k).astype(np.uint32)
    src[: k // 4] = rng.integers(0, 3, k // 4)  # bursty senders
    dst = rng.integers(0, n, k)
    dip = hosts.ip[dst].astype(np.uint32)
    unk = rng.random(k) < 0.05
    dip[unk] = 0x0AFF0000 + rng.integers(1, 1000, unk.sum())  # 10.255/16: not registered
    me = rng.random(k) < 0.05
    dip[me] = hosts.ip[src[me]]
    pay = rng.integers(0, 1473, k).astype(np.uint32)
    pay[rng.random(k) < 0.1] = 0
    t = sgn.SIMULATION_START + np.sort(rng.integers(0, span_ns, k)).astype(np.uint64)
    t[: k // 4] = sgn.SIMULATION_START + np.sort(rng.integers(0, span_ns // 10, k // 4)).astype(np.uint64)
    order = np.argsort(t, kind="stable")
    handle = (np.arange(k, dtype=np.uint64) * 0x9E3779B97F4A7C15) & np.uint64(0xFFFFFFFFFFFFFFFF)
    # wire lengths: UDP (0 = implied, or payload + 28) and TCP segments from the CPU TCP stack
    # (payload + 40, + 44 with the window-scale option: network/packet.rs:617-635)
    kind = rng.integers(0, 4, k)
    wire = np.where(kind == 0, 0, pay + np.array([0, 28, 40, 44])[kind]).astype(np.uint32)
    return src[order], dip[order], pay[order], t[order], handle[order], wire[order]


def drive(sims, dg, rng_hosts=(1, 2), max_rounds=100_000, on_round=None):
    """Runs every sim in lockstep as a CPU controller would; returns the drain records of
    each (list of arrays) and the number of rounds."""
    src, dip, pay, t, handle, wire = dg
    nxt = 0
    drains = [[] for _ in sims]
    rounds = 0
    while rounds < max_rounds:
        wins = [s.window() for s in sims]
        assert all(w == wins[0] for w in wins), wins
        ws, we, active = wins[0]
        if nxt < len(t) and (not active or int(t[nxt]) < ws):
            ws, we = int(t[nxt]), int(t[nxt]) + RUNAHEAD
            for s in sims:
                s.set_window(ws, we)
            we = sims[0].window()[1]
        elif not active:
            break
        j = nxt
        while j < len(t) and int(t[j]) < we:
            j += 1
        if j > nxt:
            for s in sims:
                s.submit(src[nxt:j], dip[nxt:j], pay[nxt:j], t[nxt:j], handle[nxt:j], wire_len=wire[nxt:j])
            nxt = j
        mins = [s.round() for s in sims]
        assert all(m == mins[0] for m in mins), mins
        rounds += 1
        if rounds % 7 == 0:
            # CPU-side draws from the device-held host RNG (host_rngDouble / NextNBytes)
            h = rng_hosts[rounds % len(rng_hosts)]
            vals = [(s.rng_next_u64(h), s.rng_double(h), s.rng_fill_bytes(h, rounds % 13)) for s in sims]
            assert all(v == vals[0] for v in vals), vals
        if rounds % 5 == 0:
            half = 30
            for i, s in enumerate(sims):
                drains[i].append(s.drain(0, half))
                drains[i].append(s.drain(half, 1 << 32 - 1))
        if on_round:
            on_round(rounds)
    for i, s in enumerate(sims):
        drains[i].append(s.drain())
    return [np.concatenate(d) if d else np.zeros(0, sgn.DRAIN_DTYPE) for d in drains], rounds
