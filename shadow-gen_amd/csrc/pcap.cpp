// pcap.cpp — packet capture of the path's packets, host side.
//
// * sgn_pcap_*: PcapWriter (utility/pcap_writer.rs): libpcap 2.4 global header in native
//   byte order, link type 101 (raw IP), then {ts_sec, ts_usec, captured, original} records.
// * sgn_packet_bytes: Packet::display_bytes (network/packet.rs:800-934) for IPv4 + UDP/TCP.
// * sgn_trace_pcap: one host's interface capture rebuilt from trace records: the capture
//   points are NetworkInterface::pop (a packet handed to relay_inet_out) and ::push (a packet
//   received, incl. a loopback packet pushed back by the relay), interface.rs:192-215,
//   relay/mod.rs:84-91; the record's time is Worker::current_time().to_abs_simtime().

#include <hip/hip_runtime.h>  // sgn_workload.h helpers are __host__ __device__

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

#include "sgn.h"
#include "sgn_workload.h"

struct sgn_pcap {
  FILE* f = nullptr;
  uint32_t capture_len = 0;
};

namespace {

template <typename T>
bool put(FILE* f, T v) {  // native byte order, like to_ne_bytes
  return std::fwrite(&v, sizeof(T), 1, f) == 1;
}

void be16(uint8_t* p, uint16_t v) {
  p[0] = (uint8_t)(v >> 8);
  p[1] = (uint8_t)v;
}
void be32(uint8_t* p, uint32_t v) {
  for (int i = 0; i < 4; i++) p[i] = (uint8_t)(v >> (24 - 8 * i));
}

}  // namespace

extern "C" {

int sgn_pcap_open(const char* path, uint32_t capture_len, sgn_pcap** out) {
  if (!path || !out) return SGN_EINVAL;
  *out = nullptr;
  FILE* f = std::fopen(path, "wb");
  if (!f) return SGN_ENOENT;
  bool ok = put<uint32_t>(f, 0xA1B2C3D4u) && put<uint16_t>(f, 2) && put<uint16_t>(f, 4) &&
            put<int32_t>(f, 0) && put<uint32_t>(f, 0) && put<uint32_t>(f, capture_len) &&
            put<uint32_t>(f, 101);
  if (!ok) {
    std::fclose(f);
    return SGN_EDEVICE;
  }
  sgn_pcap* p = new sgn_pcap();
  p->f = f;
  p->capture_len = capture_len;
  *out = p;
  return 0;
}

int sgn_pcap_write_packet(sgn_pcap* p, uint32_t ts_sec, uint32_t ts_usec, const uint8_t* bytes, uint32_t len) {
  if (!p || !p->f || (!bytes && len)) return SGN_EINVAL;
  const uint32_t cap = std::min(len, p->capture_len);
  bool ok = put(p->f, ts_sec) && put(p->f, ts_usec) && put(p->f, cap) && put(p->f, len);
  if (ok && cap) ok = std::fwrite(bytes, 1, cap, p->f) == cap;
  return ok ? 0 : SGN_EDEVICE;
}

int sgn_pcap_close(sgn_pcap* p) {
  if (!p) return SGN_EINVAL;
  int rc = p->f && std::fclose(p->f) == 0 ? 0 : SGN_EDEVICE;
  delete p;
  return rc;
}

uint32_t sgn_packet_bytes(uint32_t src_ip, uint32_t dst_ip, uint32_t payload_len, uint32_t tag, uint8_t* out,
                          uint32_t cap) {
  const uint32_t hdr = sgn_header_bytes(tag);  // 20 + 8 (UDP) / 20 (TCP) / 24 (TCP + window scale)
  const uint32_t total = hdr + payload_len;
  uint8_t h[44];
  std::memset(h, 0, sizeof(h));
  const uint32_t kind = (tag >> SGN_TAG_HDR_SHIFT) & 3u;
  h[0] = 0x45;                          // version 4, IHL 5
  be16(h + 2, (uint16_t)total);         // total length (Packet::len)
  be16(h + 6, 0x4000);                  // DF, fragment offset 0
  h[8] = 64;                            // TTL
  h[9] = kind == 0 ? 17 : 6;            // UDP / TCP
  be32(h + 12, src_ip);
  be32(h + 16, dst_ip);
  if (kind == 0) {
    be16(h + 24, (uint16_t)(8 + payload_len));  // UDP length; ports and checksum 0
  } else {
    const uint32_t tcp_len = hdr - 20;
    h[32] = (uint8_t)((tcp_len / 4) << 4);  // data offset in 32-bit words
    if (tcp_len == 24) {                    // window scale option (3, 3, ws) + 1 byte padding
      h[40] = 3;
      h[41] = 3;
    }
  }
  if (out) {
    const uint32_t n = std::min(cap, total);
    std::memcpy(out, h, std::min(n, hdr));
    if (n > hdr) std::memset(out + hdr, 0, n - hdr);  // payload bytes: none in the path
  }
  return total;
}

int64_t sgn_trace_pcap(const sgn_trace_rec* recs, uint64_t n, uint32_t host, const uint32_t* host_ip,
                       uint32_t n_hosts, const char* path, uint32_t capture_len) {
  if ((!recs && n) || !host_ip || host >= n_hosts) return SGN_EINVAL;
  std::vector<const sgn_trace_rec*> mine;
  for (uint64_t i = 0; i < n; i++)
    if (recs[i].host == host &&
        (recs[i].kind == SGN_TRACE_IF_POP || recs[i].kind == SGN_TRACE_DELIVER || recs[i].kind == SGN_TRACE_LOCAL))
      mine.push_back(&recs[i]);
  std::sort(mine.begin(), mine.end(), [](const sgn_trace_rec* a, const sgn_trace_rec* b) { return a->seq < b->seq; });
  sgn_pcap* p = nullptr;
  int rc = sgn_pcap_open(path, capture_len, &p);
  if (rc) return rc;
  std::vector<uint8_t> buf;
  const uint32_t me = host_ip[host];
  for (const sgn_trace_rec* r : mine) {
    const uint32_t payload = (uint32_t)r->b, tag = (uint32_t)(r->b >> 32);
    uint32_t src = me, dst = me;
    if (r->kind == SGN_TRACE_IF_POP) {
      if (r->peer != 0xFFFFFFFFu && r->peer >= n_hosts) { sgn_pcap_close(p); return SGN_EINVAL; }
      dst = r->peer == 0xFFFFFFFFu ? (uint32_t)r->c : host_ip[r->peer];
    } else if (r->kind == SGN_TRACE_DELIVER) {
      if (r->peer >= n_hosts) { sgn_pcap_close(p); return SGN_EINVAL; }
      src = host_ip[r->peer];
    }
    const uint32_t len = sgn_packet_bytes(src, dst, payload, tag, nullptr, 0);
    buf.resize(std::min(len, capture_len));
    sgn_packet_bytes(src, dst, payload, tag, buf.data(), (uint32_t)buf.size());
    // to_abs_simtime: seconds (saturating to u32) and the sub-second microseconds
    const uint64_t rel = r->a - SGN_SIMULATION_START;
    const uint64_t sec = rel / 1000000000ull;
    const uint32_t ts_sec = sec > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)sec;
    const uint32_t ts_usec = (uint32_t)((rel % 1000000000ull) / 1000ull);
    // write_packet_fmt writes min(len, capture_len) bytes of display_bytes
    const uint32_t cap = std::min(len, capture_len);
    bool ok = put(p->f, ts_sec) && put(p->f, ts_usec) && put(p->f, cap) && put(p->f, len);
    if (ok && cap) ok = std::fwrite(buf.data(), 1, cap, p->f) == cap;
    if (!ok) { sgn_pcap_close(p); return SGN_EDEVICE; }
  }
  rc = sgn_pcap_close(p);
  return rc ? rc : (int64_t)mine.size();
}

}  // extern "C"
