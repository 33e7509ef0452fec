// api.cpp — libsgn context, host registration and the CPU-side consumer entry points.
//
// Host registration restates the parts of SimConfig::new / Manager::run that the packet
// core depends on: DNS registration rules (network/dns.rs:97-131), the IP -> HostId map
// (dns.rs:174), IP -> node (IpAssignment, network/graph/mod.rs:348-418), and the seed
// derivation (core/sim_config.rs:50-54,220-242). The worker_* equivalents serve the CPU
// side of Shadow from the same tables (core/worker.rs:657-690).

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "sgn_internal.h"
#include "sgn_workload.h"

namespace sgn {

int set_error(sgn_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  return code;
}

int hip_fail(sgn_ctx* ctx, hipError_t e, const char* what) {
  return set_error(ctx, SGN_EDEVICE,
                   std::string("HIP error ") + hipGetErrorString(e) + " in " + what);
}

void* dev_alloc(sgn_ctx* ctx, size_t bytes, bool zero) {
  void* p = nullptr;
  if (bytes == 0) bytes = 16;
  if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
  if (zero && hipMemset(p, 0, bytes) != hipSuccess) {
    hipFree(p);
    return nullptr;
  }
  ctx->allocs.push_back(p);
  ctx->sim_bytes += bytes;
  return p;
}

// frees one dev_alloc'ed buffer before free_sim (a pool replaced by a larger one)
void dev_free(sgn_ctx* ctx, void* p, size_t bytes) {
  if (!p) return;
  auto it = std::find(ctx->allocs.begin(), ctx->allocs.end(), p);
  if (it == ctx->allocs.end()) return;
  ctx->allocs.erase(it);
  hipFree(p);
  if (bytes == 0) bytes = 16;
  ctx->sim_bytes -= std::min<uint64_t>(ctx->sim_bytes, bytes);
}

}  // namespace sgn

sgn_ctx::~sgn_ctx() {
  for (sgn_stage* st : stages) st->ctx = nullptr;  // the caller still owns (and destroys) them
  sgn::free_sim(this);
  if (d_lat) hipFree(d_lat);
  if (d_loss) hipFree(d_loss);
  for (auto& p : ev_pool) {
    hipEventDestroy(p.first);
    hipEventDestroy(p.second);
  }
  if (stream) hipStreamDestroy(stream);
}

using namespace sgn;

namespace {

thread_local std::string g_create_error;

inline uint64_t rotl(uint64_t x, int b) { return (x << b) | (x >> (64 - b)); }

// SipHash-1-3 with zero keys: Rust std's DefaultHasher (core::hash::sip::Sip13Rounds).
uint64_t sip13(const uint8_t* m, size_t n) {
  uint64_t v[4] = {0x736f6d6570736575ULL, 0x646f72616e646f6dULL, 0x6c7967656e657261ULL,
                   0x7465646279746573ULL};
  auto sipround = [&v]() {
    v[0] += v[1]; v[1] = rotl(v[1], 13) ^ v[0]; v[0] = rotl(v[0], 32);
    v[2] += v[3]; v[3] = rotl(v[3], 16) ^ v[2];
    v[0] += v[3]; v[3] = rotl(v[3], 21) ^ v[0];
    v[2] += v[1]; v[1] = rotl(v[1], 17) ^ v[2]; v[2] = rotl(v[2], 32);
  };
  const size_t full = n & ~(size_t)7;
  for (size_t off = 0; off < full; off += 8) {
    uint64_t w;
    std::memcpy(&w, m + off, 8);  // little-endian host
    v[3] ^= w;
    sipround();
    v[0] ^= w;
  }
  uint64_t tail = (uint64_t)(n & 0xff) << 56;
  for (size_t j = 0; j < (n & 7); j++) tail |= (uint64_t)m[full + j] << (8 * j);
  v[3] ^= tail;
  sipround();
  v[0] ^= tail;
  v[2] ^= 0xff;
  sipround();
  sipround();
  sipround();
  return v[0] ^ v[1] ^ v[2] ^ v[3];
}

inline uint64_t splitmix(uint64_t& s) {
  s += 0x9e3779b97f4a7c15ULL;
  uint64_t z = s;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

inline uint32_t dns_hash(uint32_t ip) { return ip * 0x9E3779B1u; }

}  // namespace

extern "C" {

int sgn_abi_version(void) { return SGN_ABI_VERSION; }

int sgn_create(sgn_ctx** out, const sgn_create_opts* opts) {
  if (!out) return SGN_EINVAL;
  *out = nullptr;
  sgn_create_opts o{};
  if (opts) o = *opts;
  if (o.shard_count == 0) o.shard_count = 1;
  if (o.shard_rank >= o.shard_count) {
    g_create_error = "shard_rank must be < shard_count";
    return SGN_EINVAL;
  }
  if (sgn::layout_sig_engine() != kLayoutSig || sgn::layout_sig_routes() != kLayoutSig ||
      sgn::layout_sig_comm() != kLayoutSig) {
    g_create_error = "libsgn's objects were compiled against different versions of sgn_internal.h (rebuild all of them)";
    return SGN_ESTATE;
  }
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev == 0) {
    g_create_error = std::string("no HIP device available: ") + hipGetErrorString(e);
    return SGN_EDEVICE;
  }
  if (o.device < 0 || o.device >= ndev) {
    g_create_error = "device ordinal out of range";
    return SGN_EINVAL;
  }
  if ((e = hipSetDevice(o.device)) != hipSuccess) {
    g_create_error = std::string("hipSetDevice: ") + hipGetErrorString(e);
    return SGN_EDEVICE;
  }
  sgn_ctx* c = new sgn_ctx();
  c->device = o.device;
  c->rank = o.shard_rank;
  c->nranks = o.shard_count;
  c->flags = o.flags;
  // experiment hook: no HIP-event timing at all (graph batches without event-record nodes)
  if (getenv("SGN_NO_TIMING")) c->flags &= ~(uint32_t)(SGN_CREATE_TIME_KERNELS | SGN_CREATE_TIME_EXECUTE);
  if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess) {
    g_create_error = std::string("hipStreamCreate: ") + hipGetErrorString(e);
    delete c;
    return SGN_EDEVICE;
  }
  *out = c;
  return 0;
}

void sgn_destroy(sgn_ctx* ctx) {
  if (!ctx) return;
  hipSetDevice(ctx->device);
  if (ctx->stream) hipStreamSynchronize(ctx->stream);
  // a captured batch holds RCCL work of the communicator: release it first (RCCL keeps the
  // communicator's captured resources alive until the graph is gone)
  drop_graph(ctx);
  comm_destroy(ctx);
  delete ctx;
}

const char* sgn_last_error(const sgn_ctx* ctx) {
  return ctx ? ctx->err.c_str() : g_create_error.c_str();
}

int sgn_shard_range(uint32_t n, uint32_t r, uint32_t k, uint32_t* lo, uint32_t* hi) {
  if (k == 0 || r >= k || !lo || !hi) return SGN_EINVAL;
  // contiguous HostId ranges, sizes differing by at most one
  const uint64_t base = n / k, rem = n % k;
  *lo = (uint32_t)(r * base + std::min<uint64_t>(r, rem));
  *hi = (uint32_t)(*lo + base + (r < rem ? 1 : 0));
  return 0;
}

int sgn_derive_host_seeds(uint32_t sim_seed, const char* const* names, uint32_t n,
                          uint64_t* out) {
  if ((!names || !out) && n) return SGN_EINVAL;
  // Xoshiro256PlusPlus::seed_from_u64(seed) then one next_u64 (sim_config.rs:51,54)
  uint64_t sm = sim_seed, s[4];
  for (int i = 0; i < 4; i++) s[i] = splitmix(sm);
  const uint64_t r = rotl(s[0] + s[3], 23) + s[0];
  for (uint32_t i = 0; i < n; i++) {
    if (!names[i]) return SGN_EINVAL;
    std::string b(names[i]);
    b.push_back((char)0xFF);  // str::hash terminator
    out[i] = r ^ sip13((const uint8_t*)b.data(), b.size());
  }
  return 0;
}

int sgn_hosts_set(sgn_ctx* ctx, const sgn_hosts* H) {
  if (!ctx || !H) return SGN_EINVAL;
  if (!ctx->routes_ready) return set_error(ctx, SGN_ESTATE, "sgn_routes_build must precede sgn_hosts_set");
  const uint32_t n = H->n_hosts;
  if (n == 0) return set_error(ctx, SGN_EINVAL, "The configuration did not contain any hosts");
  if (!H->ip || !H->node_id || !H->bw_up_bits || !H->bw_down_bits || !H->seed)
    return set_error(ctx, SGN_EINVAL, "null host array");
  std::unordered_map<uint32_t, uint32_t> unode;
  for (uint32_t i = 0; i < ctx->U; i++) unode[ctx->used_ids[i]] = i;
  ctx->ip.assign(H->ip, H->ip + n);
  ctx->node_id.assign(H->node_id, H->node_id + n);
  ctx->bw_up.assign(H->bw_up_bits, H->bw_up_bits + n);
  ctx->bw_down.assign(H->bw_down_bits, H->bw_down_bits + n);
  ctx->seed.assign(H->seed, H->seed + n);
  ctx->unode.resize(n);
  uint32_t cap = 16;
  while (cap < 2 * (uint64_t)n) cap <<= 1;
  ctx->dns_key.assign(cap, 0);
  ctx->dns_val.assign(cap, 0);
  ctx->dns_mask = cap - 1;
  for (uint32_t i = 0; i < n; i++) {
    auto it = unode.find(H->node_id[i]);
    if (it == unode.end())
      return set_error(ctx, SGN_EINVAL, "host " + std::to_string(i) + ": network node " +
                                            std::to_string(H->node_id[i]) + " is not a used node of the route table");
    ctx->unode[i] = it->second;
    const uint32_t a = H->ip[i];
    // DnsBuilder::register address rules (network/dns.rs:104-113)
    if (a == 0) return set_error(ctx, SGN_EINVAL, "unspecified address '0.0.0.0' is invalid in DNS");
    if ((a >> 24) == 127) return set_error(ctx, SGN_EINVAL, "loopback address is invalid in DNS");
    if (a == 0xFFFFFFFFu) return set_error(ctx, SGN_EINVAL, "broadcast address '255.255.255.255' is invalid in DNS");
    if ((a >> 28) == 0xE) return set_error(ctx, SGN_EINVAL, "multicast address is invalid in DNS");
    if ((a & 0xFFFF0000u) == SGN_UNKNOWN_IP_BASE)
      return set_error(ctx, SGN_EINVAL, "10.255.0.0/16 is reserved for unrouted synthetic traffic");
    uint32_t j = dns_hash(a) & ctx->dns_mask;
    while (ctx->dns_key[j] != 0) {
      if (ctx->dns_key[j] == a)
        return set_error(ctx, SGN_EINVAL, "a DNS registration record already exists for address " + std::to_string(a));
      j = (j + 1) & ctx->dns_mask;
    }
    ctx->dns_key[j] = a;
    ctx->dns_val[j] = i;
  }
  ctx->n_all = n;
  sgn_shard_range(n, ctx->rank, ctx->nranks, &ctx->lo, &ctx->hi);
  ctx->hosts_ready = true;
  if (ctx->sim_ready) free_sim(ctx);
  return 0;
}

int sgn_addr_to_host_id(sgn_ctx* ctx, uint32_t ip, uint32_t* host) {
  if (!ctx || !host) return SGN_EINVAL;
  if (!ctx->hosts_ready) return set_error(ctx, SGN_ESTATE, "no hosts registered");
  uint32_t j = dns_hash(ip) & ctx->dns_mask;
  while (ctx->dns_key[j] != 0) {
    if (ctx->dns_key[j] == ip) {
      *host = ctx->dns_val[j];
      return 0;
    }
    j = (j + 1) & ctx->dns_mask;
  }
  return SGN_ENOENT;
}

int sgn_route_get(sgn_ctx* ctx, uint32_t src, uint32_t dst, uint64_t* lat, float* loss) {
  if (!ctx) return SGN_EINVAL;
  if (!ctx->routes_ready) return set_error(ctx, SGN_ESTATE, "no route table");
  int si = -1, di = -1;
  for (uint32_t i = 0; i < ctx->U; i++) {
    if (ctx->used_ids[i] == src) si = (int)i;
    if (ctx->used_ids[i] == dst) di = (int)i;
  }
  if (si < 0 || di < 0) return SGN_ENOENT;
  if (int rc = sgn::ensure_host_routes(ctx)) return rc;
  const size_t k = (size_t)si * ctx->U + di;
  if (lat) *lat = ctx->h_lat[k];
  if (loss) *loss = ctx->h_loss[k];
  return 0;
}

int sgn_routes_copy(sgn_ctx* ctx, uint64_t* lat, float* loss) {
  if (!ctx) return SGN_EINVAL;
  if (!ctx->routes_ready) return set_error(ctx, SGN_ESTATE, "no route table");
  if (int rc = sgn::ensure_host_routes(ctx)) return rc;
  if (lat) std::memcpy(lat, ctx->h_lat.data(), ctx->h_lat.size() * 8);
  if (loss) std::memcpy(loss, ctx->h_loss.data(), ctx->h_loss.size() * 4);
  return 0;
}

int sgn_min_latency(sgn_ctx* ctx, uint64_t* out) {
  if (!ctx || !out) return SGN_EINVAL;
  if (!ctx->routes_ready) return set_error(ctx, SGN_ESTATE, "no route table");
  *out = ctx->lat_min;  // over every entry incl. self-loops (graph/mod.rs:472)
  return 0;
}

int sgn_routes_timing_get(sgn_ctx* ctx, sgn_routes_timing* out) {
  if (!ctx || !out) return SGN_EINVAL;
  *out = ctx->rt_timing;
  return 0;
}

static int route_index(sgn_ctx* ctx, uint32_t src_be, uint32_t dst_be, size_t* k) {
  uint32_t s, d;
  if (sgn_addr_to_host_id(ctx, __builtin_bswap32(src_be), &s) != 0) return -1;
  if (sgn_addr_to_host_id(ctx, __builtin_bswap32(dst_be), &d) != 0) return -1;
  *k = (size_t)ctx->unode[s] * ctx->U + ctx->unode[d];
  return 0;
}

uint64_t sgn_worker_get_latency(sgn_ctx* ctx, uint32_t src_be, uint32_t dst_be) {
  size_t k;
  if (!ctx || !ctx->hosts_ready || route_index(ctx, src_be, dst_be, &k)) return SGN_EMUTIME_INVALID;
  if (sgn::ensure_host_routes(ctx)) return SGN_EMUTIME_INVALID;
  return ctx->h_lat[k];
}

int32_t sgn_worker_is_routable(sgn_ctx* ctx, uint32_t src_be, uint32_t dst_be) {
  size_t k;
  if (!ctx || !ctx->hosts_ready) return 0;
  return route_index(ctx, src_be, dst_be, &k) == 0 ? 1 : 0;
}

uint64_t sgn_worker_get_bandwidth_up_bytes(sgn_ctx* ctx, uint32_t ip_be) {
  uint32_t h;
  if (!ctx || sgn_addr_to_host_id(ctx, __builtin_bswap32(ip_be), &h) != 0) return 0;
  return ctx->bw_up[h] / 8;
}

uint64_t sgn_worker_get_bandwidth_down_bytes(sgn_ctx* ctx, uint32_t ip_be) {
  uint32_t h;
  if (!ctx || sgn_addr_to_host_id(ctx, __builtin_bswap32(ip_be), &h) != 0) return 0;
  return ctx->bw_down[h] / 8;
}

}  // extern "C"

uint64_t sgn::layout_sig_api() { return kLayoutSig; }
