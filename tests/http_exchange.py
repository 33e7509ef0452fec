"""BASELINE.json configs[0], "getting_started_basic": the reference's own
`examples/docs/basic-file-transfer/shadow.yaml` (a python3 `http.server` on `server` and
`curl -s server` on `client1..3`, all on the built-in `1_gbit_switch` graph,
`core/configuration.rs:1367-1381`) through the packet core.

The real `http.server` and `curl` processes stay on the CPU side of Shadow (out of scope), so a
scripted stand-in plays their TCP conversation through the CPU-resident-application path
(SGN_TRAFFIC_EXTERNAL: `sgn_submit` / `sgn_drain` / `sgn_set_window`): at each client's process
start_time (5 s, from the yaml) a handshake (SYN and SYN-ACK carry the window-scale option:
44-B TCP header on the wire, the rest 40 B; network/packet.rs:617-635), a 78-B GET request, an
HTTP/1.0 response segmented at a 1460-B MSS and sent under a slow-start window (10 segments,
+1 per acknowledged segment), delayed ACKs every second segment, and the FIN exchange. Each
reply leaves when its trigger is delivered (drained), or at the window edge after it: the
application runs between rounds on the CPU (the window rules of sgn_set_window).

The same controller drives any number of simulations in lockstep (libsgn and the oracle), so
every drain record, counter, digest and interface capture can be compared bit for bit."""
import heapq
import json
import pathlib

import numpy as np

import sgn
import shadow_config as sc

GOLD = pathlib.Path(__file__).parent / "golden" / "reference_configs.json"
CONFIG = "examples/docs/basic-file-transfer/shadow.yaml"

SYN, SYNACK, ACK_HS, GET, DATA, ACK_DATA, FIN_S, FIN_C, LAST_ACK = range(9)
KIND_NAMES = ("SYN", "SYN-ACK", "ACK", "GET", "DATA", "ACK(data)", "FIN(server)", "FIN(client)", "ACK(last)")
MSS = 1460
GET_BYTES = len(b"GET / HTTP/1.1\r\nHost: server\r\nUser-Agent: curl/7.81.0\r\nAccept: */*\r\n\r\n")
HTTP_HEADER = 155   # "HTTP/1.0 200 OK" + Server/Date/Content-type/Content-Length lines
BODY = 20_000       # http.server's directory listing (bytes)
INIT_CWND = 10


def basic_file_transfer(argv=()):
    """SimSetup of the reference's basic-file-transfer shadow.yaml (from the committed corpus)."""
    corpus = json.loads(GOLD.read_text(encoding="utf-8"))["corpus"]
    return sc.sim_setup(sc.load(text=corpus[CONFIG]["text"], argv=list(argv)))


def handle_of(conn, kind, seq):
    return (conn << 40) | (kind << 32) | seq


def decode(h):
    h = int(h)
    return h >> 40, (h >> 32) & 0xFF, h & 0xFFFFFFFF


class Exchange:
    """The scripted http.server / curl conversation of one server and its clients."""

    def __init__(self, setup, server="server", clients=("client1", "client2", "client3"), body=BODY):
        self.ip = setup.hosts.ip
        self.server = setup.names.index(server)
        self.clients = [setup.names.index(c) for c in clients]
        self.total = -(-(HTTP_HEADER + body) // MSS)          # data segments per response
        self.last_pay = HTTP_HEADER + body - (self.total - 1) * MSS
        self.pending = []                                      # (time, seq, src, dst, pay, wire, handle)
        self.seq = 0
        self.conn = {}                                         # per client: server-side state
        for k, c in enumerate(self.clients):
            start = min(setup.process_start_ns[c])
            self.conn[k] = {"sent": 0, "acked": 0, "cwnd": INIT_CWND, "got": 0, "done": False}
            self.send(sgn.SIMULATION_START + start, c, self.server, 0, 44, k, SYN, 0)
        self.log = []

    def send(self, t, src, dst, pay, wire, conn, kind, seq):
        heapq.heappush(self.pending, (int(t), self.seq, src, dst, pay, wire, handle_of(conn, kind, seq)))
        self.seq += 1

    def _data(self, t, k):
        c = self.conn[k]
        cl = self.clients[k]
        while c["sent"] < self.total and c["sent"] - c["acked"] < c["cwnd"]:
            i = c["sent"]
            pay = MSS if i + 1 < self.total else self.last_pay
            self.send(t, self.server, cl, pay, pay + 40, k, DATA, i)
            c["sent"] += 1
        if c["sent"] == self.total and not c.get("fin"):
            c["fin"] = True  # HTTP/1.0: the server closes after the response
            self.send(t, self.server, cl, 0, 40, k, FIN_S, 0)

    def on_delivered(self, rec, t):
        """One delivered datagram (a drain record) at the application: its replies leave at t."""
        k, kind, seq = decode(rec["handle"])
        cl = self.clients[k]
        c = self.conn[k]
        self.log.append((int(rec["time"]), int(rec["host"]), KIND_NAMES[kind], seq))
        if kind == SYN:
            self.send(t, self.server, cl, 0, 44, k, SYNACK, 0)
        elif kind == SYNACK:
            self.send(t, cl, self.server, 0, 40, k, ACK_HS, 0)
            self.send(t, cl, self.server, GET_BYTES, GET_BYTES + 40, k, GET, 0)
        elif kind == GET:
            self.send(t, self.server, cl, 0, 40, k, ACK_HS, 1)
            self._data(t, k)
        elif kind == DATA:
            c["got"] += 1
            if c["got"] % 2 == 0 or c["got"] == self.total:   # delayed ACK
                self.send(t, cl, self.server, 0, 40, k, ACK_DATA, c["got"])
        elif kind == ACK_DATA:
            if seq > c["acked"]:
                c["cwnd"] += seq - c["acked"]
                c["acked"] = seq
            self._data(t, k)
        elif kind == FIN_S:
            self.send(t, cl, self.server, 0, 40, k, FIN_C, 0)
        elif kind == FIN_C:
            self.send(t, self.server, cl, 0, 40, k, LAST_ACK, 0)
        elif kind == LAST_ACK:
            c["done"] = True

    def finished(self):
        return all(c["done"] and c["got"] == self.total for c in self.conn.values())


def drive(sims, ex, runahead_ns, max_rounds=20_000):
    """Runs the simulations in lockstep under the exchange's controller; returns the drain
    records of each and the rounds run. Every round: the controller's own next send may open
    the window (sgn_set_window), its sends inside the window are submitted, one round runs,
    and the deliveries are drained and answered."""
    drains = [[] for _ in sims]
    rounds = 0
    while rounds < max_rounds:
        wins = [s.window() for s in sims]
        assert all(w == wins[0] for w in wins), wins
        ws, we, active = wins[0]
        if ex.pending and (not active or ex.pending[0][0] < ws):
            t = ex.pending[0][0]
            for s in sims:
                s.set_window(t, t + runahead_ns)
            ws, we, active = sims[0].window()
        elif not active:
            break
        batch = []
        while ex.pending and ex.pending[0][0] < we:
            batch.append(heapq.heappop(ex.pending))
        if batch:
            _, _, src, dst, pay, wire, handle = (np.array(x) for x in zip(*batch))
            for s in sims:
                s.submit(src.astype(np.uint32), ex.ip[dst].astype(np.uint32), pay.astype(np.uint32),
                         np.array([b[0] for b in batch], dtype=np.uint64), handle.astype(np.uint64),
                         wire_len=wire.astype(np.uint32))
        mins = [s.round() for s in sims]
        assert all(m == mins[0] for m in mins), mins
        rounds += 1
        got = [s.drain() for s in sims]
        for i, d in enumerate(got):
            drains[i].append(d)
        for rec in got[0]:  # (a reply cannot leave before the window that just ran ends)
            if rec["status"] == sgn.DRAIN_DELIVERED:
                ex.on_delivered(rec, max(int(rec["time"]), we))
    return [np.concatenate(d) if d else np.zeros(0, sgn.DRAIN_DTYPE) for d in drains], rounds
