// oracle.cpp — CPU restatement of the reference hot path. TEST INFRASTRUCTURE ONLY.
//
// This file is the parity checker for libsgn (see oracle.h for who may load it). It
// restates, function by function, the reference code of iiins0mn1a/shadow-gen (a Shadow
// 3.3.0 fork; citations are paths relative to the reference's src/ directory). It is
// deliberately written the way the reference is structured — per-host binary-heap event
// queues, per-source Dijkstra, VecDeque CoDel queue, relay state machines — not the way
// the GPU engine is, so that the two implementations share no algorithmic code.
//
// Compiled with -ffp-contract=off: Rust never contracts a*b+c into an FMA, and the f32
// loss fold (network/graph/mod.rs:322) must round after every operation.

#include "oracle.h"

#include <algorithm>
#include <tuple>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <deque>
#include <atomic>
#include <map>
#include <memory>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <shared_mutex>
#include <thread>
#include <queue>
#include <string>
#include <unordered_map>
#include <vector>

#include "sgn_workload.h"

namespace {

constexpr uint64_t SIM_START = SGN_SIMULATION_START;  // emulated_time.rs:37
constexpr uint64_t EMU_MAX = SGN_EMUTIME_MAX;         // emulated_time.rs:30
constexpr uint64_t EMU_INVALID = SGN_EMUTIME_INVALID; // emulated_time.rs:29

void set_err(char* err, size_t len, const std::string& msg) {
  if (err && len) {
    std::snprintf(err, len, "%s", msg.c_str());
  }
}

// ------------------------------------------------------------------------------------
// RNG: rand_xoshiro 0.7.0 (src/Cargo.lock:2004-2012) Xoshiro256PlusPlus::seed_from_u64
// (SplitMix64 fill), next_u64; rand 0.9.2 StandardUniform f64 = (x >> 11) * 2^-53.
// Used at core/sim_config.rs:51,54 and host/host.rs:234, core/worker.rs:366.
// ------------------------------------------------------------------------------------
inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

uint64_t splitmix_next(uint64_t& state) {
  state += 0x9e3779b97f4a7c15ULL;
  uint64_t z = state;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

struct Xoshiro {
  uint64_t s[4];
  uint64_t pos = 0;  // draws so far: the stream position the trace reports
  static Xoshiro seed_from_u64(uint64_t seed) {
    Xoshiro x;
    uint64_t st = seed;
    for (int i = 0; i < 4; i++) x.s[i] = splitmix_next(st);
    return x;
  }
  uint64_t next_u64() {
    pos++;
    const uint64_t result = rotl(s[0] + s[3], 23) + s[0];
    const uint64_t t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl(s[3], 45);
    return result;
  }
  double next_f64() {
    const double scale = 1.0 / (double)(1ULL << 53);
    return (double)(next_u64() >> 11) * scale;
  }
};

// core::hash::sip::Hasher<Sip13Rounds> as used by std::hash::DefaultHasher (keys 0,0).
// `str::hash` writes the bytes then a 0xFF terminator (core::hash, write_str).
uint64_t siphash(int c, int d, uint64_t k0, uint64_t k1, const uint8_t* m, size_t len) {
  uint64_t v0 = k0 ^ 0x736f6d6570736575ULL;
  uint64_t v1 = k1 ^ 0x646f72616e646f6dULL;
  uint64_t v2 = k0 ^ 0x6c7967656e657261ULL;
  uint64_t v3 = k1 ^ 0x7465646279746573ULL;
  auto round = [&]() {
    v0 += v1; v1 = rotl(v1, 13); v1 ^= v0; v0 = rotl(v0, 32);
    v2 += v3; v3 = rotl(v3, 16); v3 ^= v2;
    v0 += v3; v3 = rotl(v3, 21); v3 ^= v0;
    v2 += v1; v1 = rotl(v1, 17); v1 ^= v2; v2 = rotl(v2, 32);
  };
  size_t i = 0;
  for (; i + 8 <= len; i += 8) {
    uint64_t w = 0;
    for (int b = 0; b < 8; b++) w |= (uint64_t)m[i + b] << (8 * b);
    v3 ^= w;
    for (int r = 0; r < c; r++) round();
    v0 ^= w;
  }
  uint64_t b = ((uint64_t)(len & 0xff)) << 56;
  for (size_t j = 0; i + j < len; j++) b |= (uint64_t)m[i + j] << (8 * j);
  v3 ^= b;
  for (int r = 0; r < c; r++) round();
  v0 ^= b;
  v2 ^= 0xff;
  for (int r = 0; r < d; r++) round();
  return v0 ^ v1 ^ v2 ^ v3;
}

// core/sim_config.rs:50-54 (G = seed_from_u64(seed as u64); r = G.random::<u64>()) and
// :220-242 (seed = r ^ DefaultHasher(hostname)).
uint64_t host_seed(uint64_t r, const char* name) {
  std::string bytes(name);
  bytes.push_back((char)0xFF);
  return r ^ siphash(1, 3, 0, 0, (const uint8_t*)bytes.data(), bytes.size());
}

// ------------------------------------------------------------------------------------
// units (utility/units.rs): FromStr at :406-440, convert() with checked_mul at :378-389.
// ------------------------------------------------------------------------------------
// kind 0 Time<TimePrefix> -> ns; 1 Bytes<SiPrefixUpper> -> bytes; 2 BitsPerSec -> bits.
int units_parse(int kind, const char* text, uint64_t* out) {
  std::string s(text);
  // regex ^([+-]?[0-9\.]*)\s*(.*)$ ('.' excludes '\n', '$' = end of text)
  size_t p = 0;
  if (p < s.size() && (s[p] == '+' || s[p] == '-')) p++;
  while (p < s.size() && ((s[p] >= '0' && s[p] <= '9') || s[p] == '.')) p++;
  std::string value = s.substr(0, p);
  size_t q = p;
  while (q < s.size() && (s[q] == ' ' || s[q] == '\t' || s[q] == '\n' || s[q] == '\r' ||
                          s[q] == '\f' || s[q] == '\v'))
    q++;
  std::string unit = s.substr(q);
  if (unit.find('\n') != std::string::npos) return SGN_EINVAL;
  auto trim = [](std::string x) {
    size_t a = 0, b = x.size();
    while (a < b && isspace((unsigned char)x[a])) a++;
    while (b > a && isspace((unsigned char)x[b - 1])) b--;
    return x.substr(a, b - a);
  };
  value = trim(value);
  unit = trim(unit);
  static const char* time_sfx[] = {""};
  static const char* bytes_sfx[] = {"B", "byte", "bytes"};
  static const char* bits_sfx[] = {"bit", "bits"};
  const char** sfx = kind == 0 ? time_sfx : (kind == 1 ? bytes_sfx : bits_sfx);
  int nsfx = kind == 0 ? 1 : (kind == 1 ? 3 : 2);
  std::string prefix = unit;
  for (int i = 0; i < nsfx; i++) {
    std::string sf = sfx[i];
    if (unit.size() >= sf.size() && unit.compare(unit.size() - sf.size(), sf.size(), sf) == 0) {
      prefix = unit.substr(0, unit.size() - sf.size());
      break;
    }
  }
  // magnitude relative to the base unit the value is converted to
  unsigned __int128 factor = 0;
  if (kind == 0) {
    // TimePrefix (units.rs:214-290), converted to Nano
    struct P { const char* n; uint64_t f; };
    static const P tp[] = {{"ns", 1}, {"nanosecond", 1}, {"nanoseconds", 1},
                           {"us", 1000}, {"\xce\xbcs", 1000}, {"microsecond", 1000},
                           {"microseconds", 1000}, {"ms", 1000000}, {"millisecond", 1000000},
                           {"milliseconds", 1000000}, {"s", 1000000000ULL},
                           {"sec", 1000000000ULL}, {"secs", 1000000000ULL},
                           {"second", 1000000000ULL}, {"seconds", 1000000000ULL},
                           {"m", 60000000000ULL}, {"min", 60000000000ULL},
                           {"mins", 60000000000ULL}, {"minute", 60000000000ULL},
                           {"minutes", 60000000000ULL}, {"h", 3600000000000ULL},
                           {"hr", 3600000000000ULL}, {"hrs", 3600000000000ULL},
                           {"hour", 3600000000000ULL}, {"hours", 3600000000000ULL}};
    if (prefix.empty()) factor = 1000000000ULL;  // default Sec
    for (const P& e : tp)
      if (prefix == e.n) factor = e.f;
  } else {
    // SiPrefixUpper (units.rs:140-205), converted to Base
    struct P { const char* n; uint64_t f; };
    static const P sp[] = {{"K", 1000ULL}, {"kilo", 1000ULL}, {"Ki", 1024ULL},
                           {"kibi", 1024ULL}, {"M", 1000000ULL}, {"mega", 1000000ULL},
                           {"Mi", 1048576ULL}, {"mebi", 1048576ULL},
                           {"G", 1000000000ULL}, {"giga", 1000000000ULL},
                           {"Gi", 1073741824ULL}, {"gibi", 1073741824ULL},
                           {"T", 1000000000000ULL}, {"tera", 1000000000000ULL},
                           {"Ti", 1099511627776ULL}, {"tebi", 1099511627776ULL}};
    if (prefix.empty()) factor = 1;
    for (const P& e : sp)
      if (prefix == e.n) factor = e.f;
  }
  if (factor == 0) return SGN_EINVAL;
  // u64::from_str: optional '+', digits only, non-empty, no overflow
  size_t i = 0;
  if (i < value.size() && value[i] == '+') i++;
  if (i >= value.size()) return SGN_EINVAL;
  unsigned __int128 v = 0;
  for (; i < value.size(); i++) {
    char ch = value[i];
    if (ch < '0' || ch > '9') return SGN_EINVAL;
    v = v * 10 + (unsigned)(ch - '0');
    if (v > UINT64_MAX) return SGN_EINVAL;
  }
  unsigned __int128 r = v * factor;  // checked_mul (units.rs:378-389)
  if (r > UINT64_MAX) return SGN_ERANGE;
  *out = (uint64_t)r;
  return 0;
}

// ------------------------------------------------------------------------------------
// GML (lib/gml-parser/src/parser.rs:43-301, gml.rs:99-103; network/graph/mod.rs:28-179)
// ------------------------------------------------------------------------------------
struct GVal {
  int type;  // 0 int(i32), 1 float(f32), 2 string
  int32_t i;
  float f;
  std::string s;
};

struct GNode {
  bool has_id = false;
  uint32_t id = 0;
  std::map<std::string, GVal> kv;
};

struct GEdge {
  uint32_t src = 0, dst = 0;
  std::map<std::string, GVal> kv;
};

struct GmlParser {
  const char* p;
  const char* e;
  std::string err;
  bool ws(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }
  bool sp(char c) { return c == ' ' || c == '\t'; }
  void space0() { while (p < e && sp(*p)) p++; }
  void multispace0() { while (p < e && ws(*p)) p++; }
  bool newline() {  // space0 multispace1 space0 (parser.rs:248-250)
    space0();
    if (p >= e || !ws(*p)) return false;
    multispace0();
    space0();
    return true;
  }
  bool tag(const char* t) {
    size_t n = std::strlen(t);
    if ((size_t)(e - p) < n || std::memcmp(p, t, n) != 0) return false;
    p += n;
    return true;
  }
  bool key(std::string& out) {  // parser.rs:43-49
    if (p >= e || !(isalpha((unsigned char)*p) || *p == '_')) return false;
    const char* s = p++;
    while (p < e && (isalnum((unsigned char)*p) || *p == '_')) p++;
    out.assign(s, p);
    return true;
  }
  // value: space0 then alt((int,newline),(float,newline),(string,newline)) (:212-219)
  bool value(GVal& v) {
    space0();
    const char* save = p;
    // int: digit1 parsed as i32
    {
      const char* q = p;
      while (q < e && *q >= '0' && *q <= '9') q++;
      if (q > p) {
        std::string digits(p, q);
        bool ok = digits.size() <= 10;
        long long x = ok ? std::stoll(digits) : 0;
        if (ok && x <= 2147483647LL) {
          const char* after = q;
          p = q;
          if (newline()) {
            v.type = 0;
            v.i = (int32_t)x;
            return true;
          }
          p = save;
          (void)after;
        }
      }
    }
    // float: nom recognize_float then str::parse::<f32>
    {
      const char* q = p;
      if (q < e && (*q == '+' || *q == '-')) q++;
      const char* ds = q;
      while (q < e && *q >= '0' && *q <= '9') q++;
      bool mant = false;
      if (q > ds) {
        mant = true;
        if (q < e && *q == '.') {
          q++;
          while (q < e && *q >= '0' && *q <= '9') q++;
        }
      } else if (q < e && *q == '.') {
        const char* d2 = q + 1;
        const char* r = d2;
        while (r < e && *r >= '0' && *r <= '9') r++;
        if (r > d2) {
          mant = true;
          q = r;
        }
      }
      if (mant) {
        if (q < e && (*q == 'e' || *q == 'E')) {
          const char* r = q + 1;
          if (r < e && (*r == '+' || *r == '-')) r++;
          const char* d3 = r;
          while (r < e && *r >= '0' && *r <= '9') r++;
          if (r == d3) {
            err = "invalid float exponent";
            return false;  // cut() makes this a failure
          }
          q = r;
        }
        std::string txt(p, q);
        char* endp = nullptr;
        float f = std::strtof(txt.c_str(), &endp);
        p = q;
        if (newline()) {
          v.type = 1;
          v.f = f;
          return true;
        }
        p = save;
      }
    }
    // string: '"' chars-until-'"' '"'
    if (p < e && *p == '"') {
      const char* q = p + 1;
      while (q < e && *q != '"') q++;
      if (q < e) {
        v.s.assign(p + 1, q);
        p = q + 1;
        if (newline()) {
          v.type = 2;
          return true;
        }
      }
    }
    p = save;
    return false;
  }
  bool kv_block(std::map<std::string, GVal>& kv) {
    space0();
    if (!tag("[")) return false;
    if (!newline()) return false;
    size_t count = 0;
    while (true) {
      if (tag("]")) break;
      std::string k;
      if (!key(k)) return false;
      GVal v;
      if (!value(v)) return false;
      kv[k] = v;
      count++;
    }
    if (kv.size() != count) {
      err = "Duplicate keys are not supported";
      return false;
    }
    if (!newline()) return false;
    return true;
  }
};

}  // namespace

struct ora_gml {
  bool directed = false;
  std::vector<uint32_t> node_id;
  std::vector<uint64_t> bw_up, bw_down;
  std::vector<int32_t> has_up, has_down;
  std::vector<uint32_t> esrc, edst;
  std::vector<uint64_t> elat;
  std::vector<float> eloss;
};

namespace {

int gml_parse(const char* text, size_t len, ora_gml** out, char* err, size_t err_len) {
  GmlParser P{text, text + len, ""};
  P.multispace0();
  if (!P.tag("graph")) { set_err(err, err_len, "expected 'graph'"); return SGN_EINVAL; }
  P.space0();
  if (!P.tag("[")) { set_err(err, err_len, "expected '['"); return SGN_EINVAL; }
  if (!P.newline()) { set_err(err, err_len, "expected newline"); return SGN_EINVAL; }
  std::vector<GNode> nodes;
  std::vector<GEdge> edges;
  int n_directed = 0;
  bool directed = false;
  std::vector<std::string> other_keys;
  while (true) {
    if (P.tag("]")) break;
    std::string k;
    if (!P.key(k)) { set_err(err, err_len, P.err.empty() ? "expected key" : P.err); return SGN_EINVAL; }
    if (k == "node") {
      GNode n;
      if (!P.kv_block(n.kv)) { set_err(err, err_len, P.err.empty() ? "bad node" : P.err); return SGN_EINVAL; }
      auto it = n.kv.find("id");
      if (it != n.kv.end()) {
        if (it->second.type != 0) { set_err(err, err_len, "Incorrect 'id' type"); return SGN_EINVAL; }
        n.has_id = true;
        n.id = (uint32_t)it->second.i;
        n.kv.erase(it);
      }
      nodes.push_back(n);
    } else if (k == "edge") {
      GEdge ed;
      if (!P.kv_block(ed.kv)) { set_err(err, err_len, P.err.empty() ? "bad edge" : P.err); return SGN_EINVAL; }
      for (const char* f : {"source", "target"}) {
        auto it = ed.kv.find(f);
        if (it == ed.kv.end()) { set_err(err, err_len, std::string("'") + f + "' doesn't exist"); return SGN_EINVAL; }
        if (it->second.type != 0) { set_err(err, err_len, std::string("Incorrect '") + f + "' type"); return SGN_EINVAL; }
        (std::strcmp(f, "source") == 0 ? ed.src : ed.dst) = (uint32_t)it->second.i;
        ed.kv.erase(it);
      }
      edges.push_back(ed);
    } else if (k == "directed") {
      GVal v;
      if (!P.value(v)) { set_err(err, err_len, "bad directed value"); return SGN_EINVAL; }
      if (v.type != 0) { set_err(err, err_len, "Value was not an integer"); return SGN_EINVAL; }
      if (v.i != 0 && v.i != 1) { set_err(err, err_len, "Bool must be 0 or 1"); return SGN_EINVAL; }
      directed = v.i == 1;
      n_directed++;
    } else {
      GVal v;
      if (!P.value(v)) { set_err(err, err_len, "bad value"); return SGN_EINVAL; }
      other_keys.push_back(k);
    }
  }
  if (n_directed > 1) { set_err(err, err_len, "The 'directed' key must only be specified once"); return SGN_EINVAL; }
  {
    std::vector<std::string> ks = other_keys;
    std::sort(ks.begin(), ks.end());
    if (std::unique(ks.begin(), ks.end()) != ks.end()) { set_err(err, err_len, "Duplicate keys are not supported"); return SGN_EINVAL; }
  }
  ora_gml* g = new ora_gml();
  g->directed = directed;
  // ShadowNode::try_from (graph/mod.rs:28-58)
  std::unordered_map<uint32_t, uint32_t> id_map;
  for (size_t i = 0; i < nodes.size(); i++) {
    GNode& n = nodes[i];
    if (!n.has_id) { delete g; set_err(err, err_len, "Node 'id' was not provided"); return SGN_EINVAL; }
    uint64_t up = 0, down = 0;
    int32_t hu = 0, hd = 0;
    for (int which = 0; which < 2; which++) {
      const char* name = which ? "host_bandwidth_up" : "host_bandwidth_down";
      auto it = n.kv.find(name);
      if (it == n.kv.end()) continue;
      if (it->second.type != 2) { delete g; set_err(err, err_len, std::string("Node '") + name + "' is not a string"); return SGN_EINVAL; }
      uint64_t bits = 0;
      if (units_parse(2, it->second.s.c_str(), &bits) != 0) { delete g; set_err(err, err_len, std::string("Node '") + name + "' is not a valid unit"); return SGN_EINVAL; }
      if (which) { up = bits; hu = 1; } else { down = bits; hd = 1; }
    }
    g->node_id.push_back(n.id);
    g->bw_up.push_back(up);
    g->bw_down.push_back(down);
    g->has_up.push_back(hu);
    g->has_down.push_back(hd);
    id_map[n.id] = (uint32_t)i;
  }
  // ShadowEdge::try_from (graph/mod.rs:70-109)
  for (GEdge& ed : edges) {
    auto it = ed.kv.find("latency");
    if (it == ed.kv.end()) { delete g; set_err(err, err_len, "Edge 'latency' was not provided"); return SGN_EINVAL; }
    if (it->second.type != 2) { delete g; set_err(err, err_len, "Edge 'latency' is not a string"); return SGN_EINVAL; }
    uint64_t lat_ns = 0;
    int rc = units_parse(0, it->second.s.c_str(), &lat_ns);
    if (rc == SGN_EINVAL) { delete g; set_err(err, err_len, "Edge 'latency' is not a valid unit"); return SGN_EINVAL; }
    if (rc != 0) { delete g; set_err(err, err_len, "Edge 'latency' overflows u64 ns"); return SGN_EINVAL; }
    auto jt = ed.kv.find("jitter");
    if (jt != ed.kv.end()) {
      uint64_t j = 0;
      if (jt->second.type != 2) { delete g; set_err(err, err_len, "Edge 'jitter' is not a string"); return SGN_EINVAL; }
      if (units_parse(0, jt->second.s.c_str(), &j) == SGN_EINVAL) { delete g; set_err(err, err_len, "Edge 'jitter' is not a valid unit"); return SGN_EINVAL; }
    }
    float loss = 0.0f;
    auto lt = ed.kv.find("packet_loss");
    if (lt != ed.kv.end()) {
      if (lt->second.type != 1) { delete g; set_err(err, err_len, "Edge 'packet_loss' is not a float"); return SGN_EINVAL; }
      loss = lt->second.f;
    }
    if (loss < 0.0f || loss > 1.0f) { delete g; set_err(err, err_len, "Edge 'packet_loss' is not in the range [0,1]"); return SGN_EINVAL; }
    if (lat_ns == 0) { delete g; set_err(err, err_len, "Edge 'latency' must not be 0"); return SGN_EINVAL; }
    if (!id_map.count(ed.src)) { delete g; set_err(err, err_len, "Edge source " + std::to_string(ed.src) + " doesn't exist"); return SGN_EINVAL; }
    if (!id_map.count(ed.dst)) { delete g; set_err(err, err_len, "Edge target " + std::to_string(ed.dst) + " doesn't exist"); return SGN_EINVAL; }
    g->esrc.push_back(ed.src);
    g->edst.push_back(ed.dst);
    g->elat.push_back(lat_ns);
    g->eloss.push_back(loss);
  }
  *out = g;
  return 0;
}

// ------------------------------------------------------------------------------------
// Routing: PathProperties (graph/mod.rs:291-334), compute_shortest_paths (:181-226) with
// petgraph 0.8.3 algo::dijkstra, get_direct_paths (:228-250), get_edge_weight (:254-287).
// ------------------------------------------------------------------------------------
struct PathProp {
  uint64_t lat;
  float loss;
};

// PartialOrd: latency, then loss (graph/mod.rs:299-307)
inline bool path_less(const PathProp& a, const PathProp& b) {
  if (a.lat != b.lat) return a.lat < b.lat;
  return a.loss < b.loss;
}

// Add: latency sum, loss = 1 - (1 - a)(1 - b) in f32, no contraction (graph/mod.rs:316-325)
inline PathProp path_add(const PathProp& a, const PathProp& e) {
  volatile float one_minus_a = 1.0f - a.loss;
  volatile float one_minus_e = 1.0f - e.loss;
  volatile float prod = one_minus_a * one_minus_e;
  PathProp r;
  r.lat = a.lat + e.lat;
  r.loss = 1.0f - prod;
  return r;
}

struct Adj {
  uint32_t to;
  uint32_t edge;
};

// Runs fn(t) for t in [0, threads) on threads (t = 0 on the caller) and joins them.
template <typename F>
void par_for_threads(int threads, F&& fn) {
  std::vector<std::thread> th;
  for (int t = 1; t < threads; t++) th.emplace_back(fn, t);
  fn(0);
  for (auto& x : th) x.join();
}

// compute_shortest_paths (graph/mod.rs:181-226) / get_direct_paths (:228-250) into a dense
// U x U table. Two restatements with identical results:
//  - faithful != 0: the reference's own data structures — per-source Dijkstra whose scores
//    are a hash map (petgraph 0.8.3 algo::dijkstra returns HashMap<NodeIndex, K>), the
//    `nodes.contains(dst)` linear filter, a HashMap<(src, dst), PathProperties> of U^2
//    entries per source merged into one (rayon flat_map + collect), the self-loop override,
//    and the to_ids re-collect into HashMap<(u32, u32), _> (core/sim_config.rs:423-445);
//  - faithful == 0: the same searches over dense arrays (CPU-optimised).
// Sources run on `threads` worker threads (rayon's into_par_iter over the used nodes).
int routes_mode(const sgn_graph* g, const uint32_t* used, uint32_t U, int shortest, int faithful,
                int threads, uint64_t* lat_out, float* loss_out, char* err, size_t err_len) {
  const uint32_t V = g->n_nodes;
  std::unordered_map<uint32_t, uint32_t> idx;  // GML id -> NodeIndex (last wins, mod.rs:159)
  for (uint32_t i = 0; i < V; i++) idx[g->node_id[i]] = i;
  std::vector<uint32_t> uidx(U);
  for (uint32_t i = 0; i < U; i++) {
    auto it = idx.find(used[i]);
    if (it == idx.end()) { set_err(err, err_len, "used node " + std::to_string(used[i]) + " not in graph"); return SGN_EINVAL; }
    uidx[i] = it->second;
  }
  std::vector<uint32_t> es(g->n_edges), ed(g->n_edges);
  for (uint32_t k = 0; k < g->n_edges; k++) {
    auto a = idx.find(g->edge_src[k]);
    auto b = idx.find(g->edge_dst[k]);
    if (a == idx.end() || b == idx.end()) { set_err(err, err_len, "edge endpoint not in graph"); return SGN_EINVAL; }
    es[k] = a->second;
    ed[k] = b->second;
  }
  // adjacency as petgraph iterates it: directed -> outgoing; undirected -> both, with
  // self-loops once
  std::vector<std::vector<Adj>> adj(V);
  for (uint32_t k = 0; k < g->n_edges; k++) {
    adj[es[k]].push_back({ed[k], k});
    if (!g->directed && es[k] != ed[k]) adj[ed[k]].push_back({es[k], k});
  }
  // get_edge_weight (:254-287): exactly one edge connecting a -> b (petgraph
  // Graph::edges_connecting walks a's edges; undirected: either orientation, a self-loop once)
  auto edge_weight = [&](uint32_t a, uint32_t b, PathProp* out) -> int {
    int count = 0;
    uint32_t found = 0;
    for (const Adj& x : adj[a]) {
      if (x.to == b) { if (count == 0) found = x.edge; count++; }
    }
    if (count == 0) return -1;
    if (count > 1) return -2;
    out->lat = g->edge_latency_ns[found];
    out->loss = g->edge_loss[found];
    return 0;
  };
  auto edge_err = [&](int rc, uint32_t a, uint32_t b) {
    std::string sa = std::to_string(g->node_id[a]), sb = std::to_string(g->node_id[b]);
    set_err(err, err_len, rc == -1 ? "No edge connecting node " + sa + " to " + sb
                                   : "More than one edge connecting node " + sa + " to " + sb);
    return SGN_EINVAL;
  };
  if (!shortest) {
    for (uint32_t i = 0; i < U; i++)
      for (uint32_t j = 0; j < U; j++) {
        PathProp p;
        int rc = edge_weight(uidx[i], uidx[j], &p);
        if (rc) return edge_err(rc, uidx[i], uidx[j]);
        lat_out[(size_t)i * U + j] = p.lat;
        loss_out[(size_t)i * U + j] = p.loss;
      }
    return 0;
  }
  threads = std::max(1, std::min<int>(threads, (int)std::max<uint32_t>(1, U)));
  struct HeapEnt {
    PathProp s;
    uint32_t node;
  };
  auto cmp = [](const HeapEnt& a, const HeapEnt& b) { return path_less(b.s, a.s); };
  std::atomic<uint32_t> next_src{0};
  std::atomic<int> disconnected{-1};  // a source with an unreachable used node
  std::mutex merge_mu;
  std::unordered_map<uint64_t, PathProp> paths;  // faithful: (src NodeIndex, dst NodeIndex)
  if (faithful) paths.reserve((size_t)U * U);
  auto worker = [&](int) {
    // dense per-thread buffers (CPU-optimised form)
    std::vector<PathProp> score(faithful ? 0 : V);
    std::vector<char> has(faithful ? 0 : V), visited(V);
    while (true) {
      const uint32_t si = next_src.fetch_add(1);
      if (si >= U || disconnected.load() >= 0) break;
      const uint32_t src = uidx[si];
      std::fill(visited.begin(), visited.end(), 0);
      std::priority_queue<HeapEnt, std::vector<HeapEnt>, decltype(cmp)> heap(cmp);
      if (faithful) {
        // petgraph::algo::dijkstra: scores in a HashMap, visited in a bit set
        std::unordered_map<uint32_t, PathProp> sc;
        sc[src] = {0, 0.0f};
        heap.push({{0, 0.0f}, src});
        while (!heap.empty()) {
          HeapEnt top = heap.top();
          heap.pop();
          const uint32_t node = top.node;
          if (visited[node]) continue;
          for (const Adj& a : adj[node]) {
            const uint32_t nx = a.to;
            if (visited[nx]) continue;
            const PathProp ns = path_add(top.s, {g->edge_latency_ns[a.edge], g->edge_loss[a.edge]});
            auto it = sc.find(nx);
            if (it != sc.end()) {
              if (path_less(ns, it->second)) {
                it->second = ns;
                heap.push({ns, nx});
              }
            } else {
              sc.emplace(nx, ns);
              heap.push({ns, nx});
            }
          }
          visited[node] = 1;
        }
        // .filter(|(dst, _)| nodes.contains(dst)).map(...).collect::<HashMap<_, _>>()
        std::unordered_map<uint64_t, PathProp> mine;
        for (const auto& kv : sc)
          if (std::find(uidx.begin(), uidx.end(), kv.first) != uidx.end())
            mine.emplace(((uint64_t)src << 32) | kv.first, kv.second);
        std::lock_guard<std::mutex> lk(merge_mu);  // rayon's collect of the flat_map
        paths.insert(mine.begin(), mine.end());
        continue;
      }
      score[src] = {0, 0.0f};
      std::fill(has.begin(), has.end(), 0);
      has[src] = 1;
      heap.push({score[src], src});
      while (!heap.empty()) {
        HeapEnt top = heap.top();
        heap.pop();
        const uint32_t node = top.node;
        if (visited[node]) continue;
        for (const Adj& a : adj[node]) {
          const uint32_t nx = a.to;
          if (visited[nx]) continue;
          const PathProp ns = path_add(top.s, {g->edge_latency_ns[a.edge], g->edge_loss[a.edge]});
          if (has[nx]) {
            if (path_less(ns, score[nx])) {
              score[nx] = ns;
              heap.push({ns, nx});
            }
          } else {
            has[nx] = 1;
            score[nx] = ns;
            heap.push({ns, nx});
          }
        }
        visited[node] = 1;
      }
      for (uint32_t dj = 0; dj < U; dj++) {
        const uint32_t dst = uidx[dj];
        if (!has[dst]) {
          int expect = -1;
          disconnected.compare_exchange_strong(expect, (int)si);
          break;
        }
        lat_out[(size_t)si * U + dj] = score[dst].lat;
        loss_out[(size_t)si * U + dj] = score[dst].loss;
      }
    }
  };
  par_for_threads(threads, worker);
  // assert_eq!(paths.len(), nodes.len().pow(2)) fails for a disconnected graph
  if (disconnected.load() >= 0 || (faithful && paths.size() != (size_t)U * U)) {
    // cold path: name the first (source, destination) pair in used-node order that has no path
    for (uint32_t si = 0; si < U; si++) {
      std::vector<char> seen(V, 0);
      std::vector<uint32_t> st{uidx[si]};
      seen[uidx[si]] = 1;
      while (!st.empty()) {
        const uint32_t x = st.back();
        st.pop_back();
        for (const Adj& e : adj[x])
          if (!seen[e.to]) { seen[e.to] = 1; st.push_back(e.to); }
      }
      for (uint32_t dj = 0; dj < U; dj++)
        if (!seen[uidx[dj]]) {
          set_err(err, err_len, "used nodes " + std::to_string(used[si]) + " -> " +
                                    std::to_string(used[dj]) + " are not connected");
          return SGN_EINVAL;
        }
    }
    set_err(err, err_len, "used nodes are not connected");
    return SGN_EINVAL;
  }
  // the self-loop replaces the zero-length path (graph/mod.rs:209-215)
  std::vector<PathProp> self(U);
  for (uint32_t i = 0; i < U; i++) {
    int rc = edge_weight(uidx[i], uidx[i], &self[i]);
    if (rc) return edge_err(rc, uidx[i], uidx[i]);
  }
  if (faithful) {
    for (uint32_t i = 0; i < U; i++) paths[((uint64_t)uidx[i] << 32) | uidx[i]] = self[i];
    // to_ids: NodeIndex -> GML id, re-collected (core/sim_config.rs:423-445)
    std::unordered_map<uint64_t, PathProp> by_id;
    by_id.reserve(paths.size());
    for (const auto& kv : paths)
      by_id.emplace(((uint64_t)g->node_id[kv.first >> 32] << 32) | g->node_id[(uint32_t)kv.first], kv.second);
    for (uint32_t i = 0; i < U; i++)
      for (uint32_t j = 0; j < U; j++) {
        const PathProp& p = by_id.at(((uint64_t)used[i] << 32) | used[j]);
        lat_out[(size_t)i * U + j] = p.lat;
        loss_out[(size_t)i * U + j] = p.loss;
      }
    return 0;
  }
  for (uint32_t i = 0; i < U; i++) {
    lat_out[(size_t)i * U + i] = self[i].lat;
    loss_out[(size_t)i * U + i] = self[i].loss;
  }
  return 0;
}

int routes(const sgn_graph* g, const uint32_t* used, uint32_t U, int shortest, uint64_t* lat_out,
           float* loss_out, char* err, size_t err_len) {
  return routes_mode(g, used, U, shortest, 0, 1, lat_out, loss_out, err, err_len);
}

// ------------------------------------------------------------------------------------
// TokenBucket (network/relay/token_bucket.rs:6-154)
// ------------------------------------------------------------------------------------
struct TB {
  uint64_t capacity, balance, refill_increment, refill_interval, last_refill;
  // lazy_refill (:124-154): returns the span to the next refill
  uint64_t lazy_refill(uint64_t now) {
    uint64_t span = now - last_refill;  // duration_since (panics if negative)
    if (span >= refill_interval) {
      uint64_t num_refills = span / refill_interval;
      unsigned __int128 nt = (unsigned __int128)refill_increment * num_refills;
      uint64_t num_tokens = nt > UINT64_MAX ? UINT64_MAX : (uint64_t)nt;  // saturating_mul
      uint64_t b = balance + num_tokens;
      if (b < balance) b = UINT64_MAX;  // saturating_add
      balance = b > capacity ? capacity : b;
      unsigned __int128 inc = (unsigned __int128)refill_interval * num_refills;
      uint64_t inc64 = inc > 17500059273709551614ULL ? 17500059273709551614ULL : (uint64_t)inc;
      // EmulatedTime::saturating_add -> MAX on overflow
      uint64_t lr = last_refill + inc64;
      last_refill = (lr < last_refill || lr > EMU_MAX) ? EMU_MAX : lr;
      span = now - last_refill;
    }
    return refill_interval - span;
  }
  // compute_conforming_duration (:91-117)
  uint64_t conforming_duration(uint64_t decrement, uint64_t next_refill_span) const {
    uint64_t req = decrement > balance ? decrement - balance : 0;
    uint64_t n = req / refill_increment + (req % refill_increment ? 1 : 0);
    if (n == 0) return 0;
    if (n == 1) return next_refill_span;
    unsigned __int128 m = (unsigned __int128)refill_interval * (n - 1);
    const uint64_t SIMTIME_MAX = 17500059273709551614ULL;
    uint64_t mm = m > SIMTIME_MAX ? SIMTIME_MAX : (uint64_t)m;
    uint64_t s = next_refill_span + mm;
    if (s < next_refill_span || s > SIMTIME_MAX) s = SIMTIME_MAX;
    return s;
  }
  // conforming_remove_inner (:72-83)
  bool remove(uint64_t decrement, uint64_t now, uint64_t* out) {
    uint64_t span = lazy_refill(now);
    if (decrement > balance) {
      *out = conforming_duration(decrement, span);
      return false;
    }
    balance -= decrement;
    *out = balance;
    return true;
  }
};

// create_token_bucket (network/relay/mod.rs:278-288): refill max(1, Bps/1000) per 1 ms,
// capacity = refill + CONFIG_MTU, starts full, last_refill = SIMULATION_START.
TB make_relay_bucket(uint64_t bytes_per_second) {
  TB t;
  t.refill_interval = 1000000ULL;
  t.refill_increment = std::max<uint64_t>(1, bytes_per_second / 1000);
  t.capacity = t.refill_increment + SGN_CONFIG_MTU;
  t.balance = t.capacity;
  t.last_refill = SIM_START;
  return t;
}

// ------------------------------------------------------------------------------------
// CoDel (network/router/codel_queue.rs:23-321)
// ------------------------------------------------------------------------------------
constexpr uint64_t CODEL_TARGET = 10000000ULL;     // :23
constexpr uint64_t CODEL_INTERVAL = 100000000ULL;  // :28

struct Pkt {
  uint32_t src_host;
  uint32_t dst_ip;
  uint32_t payload;
  uint32_t tag;
  uint64_t src_eid;
  // Packet::len (packet.rs:388-390): IPv4 20 + UDP 8, or + TCP 20 / 24 (window scale,
  // :617-635); the header kind rides in the tag (sgn_workload.h)
  uint32_t wire() const { return payload + sgn_header_bytes(tag); }
};

struct CoDelElem {
  Pkt pkt;
  uint64_t enqueue_ts;
};

// apply_control_law (:285-298)
uint64_t codel_control_law(uint64_t time, uint64_t count) {
  double interval = (double)CODEL_INTERVAL;
  double sq = count == 0 ? 1.0 : std::sqrt((double)count);
  double div = interval / sq;
  uint64_t inc = (uint64_t)std::round(div);  // f64::round: half away from zero
  uint64_t orig = time - SIM_START;
  const uint64_t SIMTIME_MAX = 17500059273709551614ULL;
  uint64_t adj = orig + inc;
  if (adj < orig || adj > SIMTIME_MAX) adj = SIMTIME_MAX;
  return SIM_START + adj;
}

struct CoDel {
  std::deque<CoDelElem> elems;
  uint64_t total_bytes = 0;
  int mode = 0;  // 0 Store, 1 Drop
  bool has_ie = false;
  uint64_t ie = 0;
  bool has_dn = false;
  uint64_t dn = 0;
  uint64_t cur = 0, prev = 0;
  uint64_t dropped_total = 0;
  std::vector<Pkt> dropped;  // drops of the current pop, in order

  static uint64_t sat_sub(uint64_t a, uint64_t b) { return a > b ? a - b : 0; }

  void push(const Pkt& p, uint64_t now) {  // :303-317 (LIMIT = usize::MAX)
    total_bytes += p.wire();
    elems.push_back({p, now});
  }
  // process_standing_delay (:231-262)
  bool process_standing_delay(uint64_t now, uint64_t sd) {
    if (sd < CODEL_TARGET || total_bytes <= SGN_CONFIG_MTU) {
      has_ie = false;
      return false;
    }
    if (has_ie) return now >= ie;
    has_ie = true;
    uint64_t x = now + CODEL_INTERVAL;
    ie = (x < now || x > EMU_MAX) ? EMU_MAX : x;
    return false;
  }
  // codel_pop (:204-227)
  bool codel_pop(uint64_t now, Pkt* out, bool* ok_to_drop) {
    if (elems.empty()) {
      has_ie = false;
      return false;
    }
    CoDelElem el = elems.front();
    elems.pop_front();
    total_bytes = sat_sub(total_bytes, el.pkt.wire());
    uint64_t sd = sat_sub(now, el.enqueue_ts);
    *ok_to_drop = process_standing_delay(now, sd);
    *out = el.pkt;
    return true;
  }
  bool should_drop(uint64_t now) const { return has_dn && now >= dn; }  // :265-270
  bool was_dropping_recently(uint64_t now) const {                      // :273-281
    if (!has_dn) return false;
    return sat_sub(now, dn) < CODEL_INTERVAL * 16;
  }
  void drop(const Pkt& p) {
    dropped.push_back(p);
    dropped_total++;
  }
  // pop (:125-148)
  bool pop(uint64_t now, Pkt* out) {
    Pkt p;
    bool okd;
    if (!codel_pop(now, &p, &okd)) {
      mode = 0;
      return false;
    }
    if (!okd) {
      mode = 0;
      *out = p;
      return true;
    }
    if (mode == 0) {
      // drop_from_store_mode (:150-170)
      drop(p);
      Pkt n;
      bool nok;
      bool has_n = codel_pop(now, &n, &nok);
      mode = 1;
      uint64_t delta = sat_sub(cur, prev);
      cur = (was_dropping_recently(now) && delta > 1) ? delta : 1;
      has_dn = true;
      dn = codel_control_law(now, cur);
      prev = cur;
      if (has_n) *out = n;
      return has_n;
    }
    // drop_from_drop_mode (:172-201)
    bool has_item = true;
    Pkt item = p;
    while (has_item && mode == 1 && should_drop(now)) {
      drop(item);
      cur += 1;
      bool iok = false;
      has_item = codel_pop(now, &item, &iok);
      if (has_item && iok) {
        dn = codel_control_law(dn, cur);
      } else {
        mode = 0;
      }
    }
    if (has_item) *out = item;
    return has_item;
  }
};

// ------------------------------------------------------------------------------------
// Events (core/work/event.rs:84-183) and the per-host EventQueue (event_queue.rs:11-90)
// ------------------------------------------------------------------------------------
enum { EV_PACKET = 0, EV_LOCAL = 1 };
enum { TASK_RELAY_OUT = 0, TASK_RELAY_IN = 1, TASK_APP = 2, TASK_SUBMIT = 3 };

struct Event {
  uint64_t time;
  int kind;
  uint32_t src_host;  // packets
  uint64_t eid;       // packets: src host's event id; locals: own event id
  int task;
  Pkt pkt;
  // reference-faithful mode: the destination's own heap copy of the packet
  // (PacketRc::new_copy_inner, worker.rs:397-398); unused by the optimised mode
  std::shared_ptr<Pkt> copy;
};

// Event ordering: time, then Packet < Local, then (src host, src event id) for packets or
// event id for locals.
struct EventGreater {
  bool operator()(const Event& a, const Event& b) const {
    if (a.time != b.time) return a.time > b.time;
    if (a.kind != b.kind) return a.kind > b.kind;
    if (a.kind == EV_PACKET) {
      if (a.src_host != b.src_host) return a.src_host > b.src_host;
      return a.eid > b.eid;
    }
    return a.eid > b.eid;
  }
};

enum { RELAY_IDLE = 0, RELAY_PENDING = 1, RELAY_FORWARDING = 2 };  // relay/mod.rs:68-77

struct Relay {
  bool limited = true;
  TB tb;
  int state = RELAY_IDLE;
  bool has_next = false;
  Pkt next;
};

struct FifoEnt {
  uint32_t dst_ip, payload, last_payload, count, tag;
};

struct Host {
  uint32_t id, ip, unode;
  Xoshiro rng;
  uint64_t eid_ctr = 0;  // host.rs:259,662-666
  std::priority_queue<Event, std::vector<Event>, EventGreater> q;
  uint64_t last_popped = SIM_START;
  Relay rout, rin;  // relay_inet_out / relay_inet_in (host.rs:284-291)
  CoDel codel;      // Router inbound queue (router/mod.rs:20)
  std::deque<FifoEnt> fifo;
  uint64_t app_k = 0;
  bool is_server = false;
  uint64_t d_tx = SGN_DIGEST_SEED, d_rx = SGN_DIGEST_SEED, d_app = SGN_DIGEST_SEED;
  sgn_drun r_tx = {0, 0, 0, 0}, r_rx = {0, 0, 0, 0}, r_app = {0, 0, 0, 0};  // pending runs
  uint64_t n_sent = 0, n_popped = 0, n_delivered = 0, n_codel_dropped = 0;
  uint64_t trace_seq = 0;
};

}  // namespace

// A persistent worker pool with one start/finish rendezvous per round, as the reference's
// thread-per-core scheduler (lib/scheduler/src/thread_per_core.rs:29-74,159-212: threads live
// for the whole simulation, spin briefly and then park between rounds). run(f) calls f(t)
// on every thread t (t = 0 on the caller) and returns when all have finished.
struct Pool {
  int n = 1;
  std::vector<std::thread> th;
  std::mutex mu;
  std::condition_variable cv;
  std::atomic<uint64_t> gen{0};
  std::atomic<int> pending{0};
  std::atomic<bool> stop{false};
  std::function<void(int)> job;

  explicit Pool(int nt) : n(nt) {
    for (int t = 1; t < n; t++) th.emplace_back([this, t] { loop(t); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(mu);
      stop = true;
      gen++;
    }
    cv.notify_all();
    for (auto& x : th) x.join();
  }
  void loop(int t) {
    uint64_t seen = 0;
    while (true) {
      for (int spin = 0; spin < 20000 && gen.load(std::memory_order_acquire) == seen; spin++)
        __builtin_ia32_pause();
      if (gen.load(std::memory_order_acquire) == seen) {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return gen.load() != seen; });
      }
      seen = gen.load(std::memory_order_acquire);
      if (stop.load()) return;
      job(t);
      pending.fetch_sub(1, std::memory_order_acq_rel);
    }
  }
  void run(const std::function<void(int)>& f) {
    job = f;
    pending.store(n - 1);
    {
      std::lock_guard<std::mutex> g(mu);
      gen.fetch_add(1, std::memory_order_acq_rel);
    }
    cv.notify_all();
    f(0);
    while (pending.load(std::memory_order_acquire) != 0) __builtin_ia32_pause();
  }
};

// Per-thread worker state, as the reference's thread-local Worker (core/worker.rs): the
// current time, this round's counters, trace records and exports, and the lowest used
// latency seen (Worker::update_lowest_used_latency); merged at the round barrier.
struct Wk {
  uint64_t now = 0;
  sgn_stats st{};
  std::vector<sgn_trace_rec> tr;
  std::vector<uint64_t> exports;
  std::vector<sgn_drain_rec> dr;  // EXTERNAL: datagram fates for the CPU-side apps
  bool min_set = false;
  uint64_t min_used = 0;
  // this round's minimum over the executed hosts' next event times and the deliveries this
  // thread produced (core/manager.rs:580-599, Worker::update_next_event_time)
  uint64_t next_min = EMU_INVALID;
};
static thread_local Wk* tl_wk = nullptr;

struct ora_sim {
  std::vector<uint32_t> used;
  uint32_t U = 0;
  std::vector<uint64_t> lat;
  std::vector<float> loss;
  std::vector<Host> hosts;
  std::unordered_map<uint32_t, uint32_t> dns;  // ip -> HostId (network/dns.rs:174)
  sgn_sim_config cfg;
  sgn_traffic traffic;
  std::vector<uint32_t> servers;
  uint64_t end_time = 0, bootstrap_end = 0;
  uint64_t min_possible_latency = 0;
  bool has_min_used = false;
  uint64_t min_used = 0;
  uint64_t ws = 0, we = 0;
  bool active = true;
  uint64_t round_end = 0;
  // worker threads (thread-per-core round, core/manager.rs:568-601): hosts are taken in
  // chunks from a shared counter (work stealing); pushes into another host's queue take that
  // host's mutex (Mutex<EventQueue>, core/worker.rs:603-613)
  int nthreads = 1;
  std::vector<Wk> wks = std::vector<Wk>(1);
  std::unique_ptr<std::mutex[]> qmu;
  std::unique_ptr<Pool> pool;
  uint64_t round_next_min = EMU_INVALID;  // min next event time after the last round
  // reference-faithful mode (CPU baseline): the reference's hash-map lookups per packet
  // (IpAssignment::get_node x6, RoutingInfo::path x2, Dns, the event-queue map), the global
  // packet-counter write lock (RoutingInfo::increment_packet_count, graph/mod.rs:450-458,
  // worker.rs:379), a heap copy of every packet and a lock around every queue operation.
  // Results are identical to the optimised mode (tests/test_oracle_threads.py).
  bool faithful = false;
  std::unordered_map<uint32_t, uint32_t> ip_node;         // IpAddr -> GML node id
  std::unordered_map<uint64_t, PathProp> route_map;       // (src node, dst node) -> path
  std::unordered_map<uint64_t, uint64_t> packet_counters; // (src node, dst node) -> packets
  std::shared_mutex counters_mu;
  std::unordered_map<uint32_t, std::mutex*> queue_map;    // HostId -> its queue's lock
  bool locked() const { return nthreads > 1 || faithful; }
  std::mutex& qlock(uint32_t host) { return faithful ? *queue_map.at(host) : qmu[host]; }
  Wk& W() { return *tl_wk; }
  sgn_stats st;
  bool trace = false;
  std::vector<sgn_trace_rec> tr;
  // sharding
  uint32_t lo = 0, hi = 0;
  std::vector<uint64_t> exports;
  bool local_min_used_set = false;
  uint64_t local_min_used = 0;
  // EXTERNAL traffic (CPU-resident applications): sgn_submit / sgn_drain / sgn_set_window
  uint64_t prev_we = SIM_START;           // end of the last executed window
  std::vector<uint64_t> handles;          // by submission slot
  std::vector<uint32_t> submit_seq;       // per host
  std::vector<sgn_drain_rec> drain_held;
  bool external() const { return traffic.kind == SGN_TRAFFIC_EXTERNAL; }
  void drain_rec(const Host& h, uint32_t status, uint32_t src, uint32_t dst, uint64_t seid,
                 uint32_t payload, uint32_t tag) {
    sgn_drain_rec r;
    r.time = W().now;
    r.src_eid = seid;
    r.handle = 0;
    r.host = h.id;
    r.src_host = src;
    r.dst_host = dst;
    r.status = status;
    r.payload_len = payload;
    r.tag = tag;
    W().dr.push_back(r);
  }

  // ---------------------------------------------------------------------------------
  void trace_rec(Host& h, uint32_t kind, uint32_t peer, uint32_t flags, uint64_t a, uint64_t b,
                 uint64_t c) {
    uint64_t seq = h.trace_seq++;
    if (!trace) return;
    sgn_trace_rec r;
    r.kind = kind;
    r.host = h.id;
    r.peer = peer;
    r.flags = flags;
    r.a = a;
    r.b = b;
    r.c = c;
    r.seq = seq;
    r.rng_pos = h.rng.pos;
    W().tr.push_back(r);
  }

  bool owned(uint32_t host) const { return host >= lo && host < hi; }

  // Runahead::get (core/runahead.rs:44-57)
  uint64_t runahead_get() const {
    uint64_t r = (cfg.use_dynamic_runahead && has_min_used) ? min_used : min_possible_latency;
    uint64_t c = cfg.runahead_ns;  // None -> ZERO
    return std::max(r, c);
  }

  // Host::push_local_event (host.rs:716-722) via schedule_task_at_emulated_time (:703-706);
  // Event::new_local consumes an event id first (event.rs:35-45).
  void schedule_task(Host& h, int task, uint64_t t) {
    Event ev;
    ev.time = t;
    ev.kind = EV_LOCAL;
    ev.src_host = h.id;
    ev.eid = h.eid_ctr++;
    ev.task = task;
    if (t >= end_time) return;
    if (locked()) {
      std::lock_guard<std::mutex> g(qlock(h.id));
      h.q.push(ev);
    } else {
      h.q.push(ev);
    }
  }

  // Relay::notify (relay/mod.rs:111-136)
  void relay_notify(Host& h, int which) {
    Relay& r = which == TASK_RELAY_OUT ? h.rout : h.rin;
    if (r.state == RELAY_IDLE) forward_later(h, which, 0);
  }

  // Relay::forward_later (relay/mod.rs:145-163)
  void forward_later(Host& h, int which, uint64_t delay) {
    Relay& r = which == TASK_RELAY_OUT ? h.rout : h.rin;
    r.state = RELAY_PENDING;
    schedule_task(h, which, W().now + delay);
  }

  // App-side delivery at the interface (NetworkInterface::push -> socket; synthetic sink).
  void deliver_to_app(Host& h, const Pkt& p, bool local) {
    if (local) {
      W().st.local_delivered++;
      trace_rec(h, SGN_TRACE_LOCAL, h.id, 0, W().now, (uint64_t)p.payload | ((uint64_t)p.tag << 32), 0);
      if (external()) drain_rec(h, SGN_DRAIN_LOCAL, h.id, h.id, 0, p.payload, p.tag);
      sgn_drun_flush_seq(&h.d_app, &h.r_app);  // a local delivery is a run of its own
      h.d_app = sgn_digest3(h.d_app, W().now, (uint64_t)p.src_host | (1ULL << 62) | (1ULL << 32),
                            p.payload);
      return;
    }
    W().st.delivered++;
    W().st.bytes_delivered += p.payload;
    h.n_delivered++;
    sgn_drun_add_seq(&h.d_app, &h.r_app, W().now, p.src_host, p.src_eid, 1);
    trace_rec(h, SGN_TRACE_DELIVER, p.src_host, 0, W().now, (uint64_t)p.payload | ((uint64_t)p.tag << 32),
              p.src_eid);
    if (external()) drain_rec(h, SGN_DRAIN_DELIVERED, p.src_host, h.id, p.src_eid, p.payload, p.tag);
    if (traffic.kind == SGN_TRAFFIC_TGEN && h.is_server && (p.tag & SGN_TAG_REQ)) {
      uint64_t size = traffic.file_bytes[p.tag & 3u];
      uint64_t n = (size + SGN_TGEN_MSS - 1) / SGN_TGEN_MSS;
      if (n == 0) return;
      uint32_t last = (uint32_t)(size - (n - 1) * SGN_TGEN_MSS);
      if (h.fifo.size() < cfg.out_fifo_cap) {
        h.fifo.push_back({hosts[p.src_host].ip, SGN_TGEN_MSS, last, (uint32_t)n, SGN_TAG_RESP});
        relay_notify(h, TASK_RELAY_OUT);
      } else {
        W().st.app_blocked++;
      }
    }
  }

  // Worker::send_packet (core/worker.rs:330-403)
  void send_packet(Host& h, Pkt p) {
    if (W().now >= end_time) return;  // is_completed (:334,338-341)
    bool bootstrapping = W().now < bootstrap_end;
    auto it = dns.find(p.dst_ip);  // resolve_ip_to_host_id (:347, dns.rs:174)
    if (it == dns.end()) {
      W().st.packets_unknown_dst++;
      sgn_drun_add_same(&h.d_tx, &h.r_tx, W().now, 0xFFFFFFFFULL | (2ULL << 32), 0, 1);
      trace_rec(h, SGN_TRACE_SEND, 0xFFFFFFFFu, 2, W().now, 0, 0);
      if (external()) drain_rec(h, SGN_DRAIN_UNKNOWN, h.id, 0xFFFFFFFFu, 0, p.payload, p.tag);
      return;
    }
    uint32_t dst = it->second;
    size_t ri = (size_t)h.unode * U + hosts[dst].unode;
    // reliability = 1.0f32 - loss, widened to f64 (:363-365, :532-537)
    float rel32;
    if (faithful) {  // WorkerShared::reliability: get_node x2 + RoutingInfo::path
      const uint32_t a = ip_node.at(h.ip), b = ip_node.at(p.dst_ip);
      rel32 = 1.0f - route_map.at(((uint64_t)a << 32) | b).loss;
    } else {
      rel32 = 1.0f - loss[ri];
    }
    double reliability = (double)rel32;
    double chance = h.rng.next_f64();  // :366
    if (!bootstrapping && chance >= reliability && p.payload > 0) {  // :371
      W().st.packets_loss_dropped++;
      sgn_drun_add_same(&h.d_tx, &h.r_tx, W().now, (uint64_t)dst | (1ULL << 32), 0, 1);
      trace_rec(h, SGN_TRACE_SEND, dst, 1, W().now, 0, 0);
      if (external()) drain_rec(h, SGN_DRAIN_LOSS, h.id, dst, 0, p.payload, p.tag);
      return;
    }
    uint64_t delay;
    if (faithful) {
      // WorkerShared::latency (:376): get_node x2 + path; increment_packet_count (:379):
      // get_node x2 + the global write lock (graph/mod.rs:450-458)
      const uint32_t a = ip_node.at(h.ip), b = ip_node.at(p.dst_ip);
      delay = route_map.at(((uint64_t)a << 32) | b).lat;
      const uint32_t c = ip_node.at(h.ip), d = ip_node.at(p.dst_ip);
      std::unique_lock<std::shared_mutex> g(counters_mu);
      uint64_t& cnt = packet_counters[((uint64_t)c << 32) | d];
      cnt = cnt == ~0ULL ? cnt : cnt + 1;
    } else {
      delay = lat[ri];  // :376
    }
    // Worker::update_lowest_used_latency -> Runahead (runahead.rs:61-107), dynamic only
    if (cfg.use_dynamic_runahead && (!W().min_set || delay < W().min_used)) {
      W().min_set = true;
      W().min_used = delay;
    }
    W().st.packets_sent++;
    h.n_sent++;
    uint64_t deliver = W().now + delay;  // :387-390
    if (deliver < round_end) deliver = round_end;
    W().next_min = std::min(W().next_min, deliver);  // Worker::update_next_event_time (:394)
    // push_packet_to_host (:603-613): Event::new_packet consumes the SOURCE host's id
    Event ev;
    ev.time = deliver;
    ev.kind = EV_PACKET;
    ev.src_host = h.id;
    ev.eid = h.eid_ctr++;
    ev.task = -1;
    p.src_eid = ev.eid;
    ev.pkt = p;
    sgn_drun_add_same(&h.d_tx, &h.r_tx, W().now, (uint64_t)dst, deliver, 1);
    trace_rec(h, SGN_TRACE_SEND, dst, 0, W().now, deliver, ev.eid);
    if (owned(dst)) {
      Host& d = hosts[dst];
      if (faithful) {
        ev.copy = std::make_shared<Pkt>(p);  // PacketRc::new_copy_inner (:397-398)
        std::lock_guard<std::mutex> g(*queue_map.at(dst));  // event_queues.get(dst).lock()
        if (ev.time < d.last_popped) std::abort();  // event_queue.rs:59
        d.q.push(std::move(ev));
      } else if (nthreads > 1) {
        std::lock_guard<std::mutex> g(qmu[dst]);
        if (ev.time < d.last_popped) std::abort();  // event_queue.rs:59
        d.q.push(ev);
      } else {
        if (ev.time < d.last_popped) std::abort();  // event_queue.rs:59
        d.q.push(ev);
      }
    } else {
      uint64_t rec[6] = {dst, ev.time, ev.src_host, ev.eid, p.payload, p.tag};
      W().exports.insert(W().exports.end(), rec, rec + 6);
    }
  }

  // source device pop for a relay (Host::get_packet_device, host.rs:946-954)
  bool relay_src_pop(Host& h, int which, Pkt* out) {
    if (which == TASK_RELAY_OUT) {
      // NetworkInterface::pop (interface.rs:224): the synthetic socket's send queue
      if (h.fifo.empty()) return false;
      FifoEnt& f = h.fifo.front();
      Pkt p;
      p.src_host = h.id;
      p.dst_ip = f.dst_ip;
      p.payload = f.count == 1 ? f.last_payload : f.payload;
      p.tag = f.tag;
      p.src_eid = 0;
      // the capture point of a sent packet (interface.rs:252-253)
      if (trace) {
        auto d = dns.find(p.dst_ip);
        const bool known = d != dns.end();
        trace_rec(h, SGN_TRACE_IF_POP, known ? d->second : 0xFFFFFFFFu, 0, W().now,
                  (uint64_t)p.payload | ((uint64_t)p.tag << 32), known ? 0 : p.dst_ip);
      }
      f.count--;
      if (f.count == 0) {
        h.fifo.pop_front();
      } else if (cfg.interface_qdisc == SGN_QDISC_ROUND_ROBIN) {
        // round-robin qdisc: the socket is popped, gives one packet and, having more, is
        // added back at the end of the queue (interface.rs:216-241, queuing.rs FirstInFirstOut)
        FifoEnt keep = f;
        h.fifo.pop_front();
        h.fifo.push_back(keep);
      }
      // (FIFO qdisc, queuing.rs MinPriority: the socket whose next packet was written first,
      // i.e. the front entry, keeps going)
      *out = p;
      return true;
    }
    // Router::pop -> CoDelQueue::pop(W().now) (router/mod.rs:65-68)
    bool got = h.codel.pop(W().now, out);
    for (const Pkt& d : h.codel.dropped) {
      W().st.codel_dropped++;
      h.n_codel_dropped++;
      sgn_drun_add_seq(&h.d_app, &h.r_app, W().now, (uint64_t)d.src_host | (1ULL << 63), d.src_eid, 1);
      trace_rec(h, SGN_TRACE_CODEL_DROP, d.src_host, 0, W().now, 0, d.src_eid);
      if (external()) drain_rec(h, SGN_DRAIN_CODEL, d.src_host, h.id, d.src_eid, d.payload, d.tag);
    }
    h.codel.dropped.clear();
    return got;
  }

  // Relay::forward_until_blocked (relay/mod.rs:201-273); returns true and *dur if blocked
  bool forward_until_blocked(Host& h, int which, uint64_t* dur) {
    Relay& r = which == TASK_RELAY_OUT ? h.rout : h.rin;
    bool bootstrapping = W().now < bootstrap_end;  // Worker::is_bootstrapping (worker.rs:482)
    r.state = RELAY_FORWARDING;
    // src device address: eth0 = host ip for inet_out, router = 0.0.0.0 for inet_in
    uint32_t src_addr = which == TASK_RELAY_OUT ? h.ip : 0u;
    while (true) {
      Pkt p;
      if (r.has_next) {
        p = r.next;
        r.has_next = false;
      } else if (!relay_src_pop(h, which, &p)) {
        r.state = RELAY_IDLE;
        return false;
      }
      bool is_local = src_addr == p.dst_ip;
      if (!bootstrapping && !is_local && r.limited) {
        uint64_t out;
        if (!r.tb.remove(p.wire(), W().now, &out)) {
          r.next = p;
          r.has_next = true;
          r.state = RELAY_IDLE;
          *dur = out;
          return true;
        }
      }
      if (is_local) {
        deliver_to_app(h, p, true);  // src.push(packet): loopback through eth0
      } else if (which == TASK_RELAY_OUT) {
        send_packet(h, p);  // Router::push -> route_outgoing_packet (router/mod.rs:48-73)
      } else {
        deliver_to_app(h, p, false);  // eth0 push for the host's own address
      }
    }
  }

  // run_forward_task + forward_now (relay/mod.rs:166-187)
  void run_forward_task(Host& h, int which) {
    Relay& r = which == TASK_RELAY_OUT ? h.rout : h.rin;
    r.state = RELAY_IDLE;
    uint64_t dur;
    if (forward_until_blocked(h, which, &dur)) forward_later(h, which, dur);
  }

  void app_task(Host& h) {
    uint64_t k = h.app_k++;
    uint32_t dst_ip;
    uint32_t payload, tag;
    uint64_t next_delay;
    if (traffic.kind == SGN_TRAFFIC_PERIODIC) {
      uint32_t peer = 0, uip = 0;
      if (sgn_periodic_dst(traffic.flow_seed, h.id, k, (uint32_t)hosts.size(),
                           traffic.unknown_dst_permille, &peer, &uip))
        dst_ip = hosts[peer].ip;
      else
        dst_ip = uip;
      payload = traffic.payload_len;
      tag = SGN_TAG_DATA;
      next_delay = traffic.period_ns;
    } else {
      uint32_t si = 0, cls = 0;
      sgn_tgen_fetch(traffic.flow_seed, h.id, k, (uint32_t)servers.size(), &si, &cls);
      dst_ip = hosts[servers[si]].ip;
      payload = traffic.req_payload;
      tag = SGN_TAG_REQ | cls;
      next_delay =
          sgn_tgen_think(traffic.flow_seed, h.id, k, traffic.period_ns, traffic.period_jitter_ns);
    }
    if (h.fifo.size() < cfg.out_fifo_cap) {
      h.fifo.push_back({dst_ip, payload, payload, 1, tag});
      relay_notify(h, TASK_RELAY_OUT);  // Host::notify_socket_has_packets (host.rs:969-983)
    } else {
      W().st.app_blocked++;
    }
    schedule_task(h, TASK_APP, W().now + next_delay);
  }

  // EXTERNAL traffic: a CPU application's datagram (sgn_submit) at its send time enters the
  // socket send queue and notifies relay_inet_out (Host::notify_socket_has_packets,
  // host.rs:969-983), as app_task does for the synthetic apps.
  void app_submit(Host& h, const Pkt& p) {
    if (h.fifo.size() < cfg.out_fifo_cap) {
      h.fifo.push_back({p.dst_ip, p.payload, p.payload, 1, p.tag});
      relay_notify(h, TASK_RELAY_OUT);
    } else {
      W().st.app_blocked++;
      drain_rec(h, SGN_DRAIN_BLOCKED, h.id, 0xFFFFFFFFu, 0, p.payload, p.tag);
    }
  }

  // Host::execute (host.rs:762-830)
  void execute(Host& h, uint64_t until) {
    // (pop under the host's own queue lock in threaded mode: other hosts push into it)
    auto pop_due = [&](Event* out) {
      std::unique_lock<std::mutex> g;
      if (locked()) g = std::unique_lock<std::mutex>(qlock(h.id));
      if (h.q.empty() || h.q.top().time >= until) return false;
      *out = h.q.top();
      h.q.pop();
      return true;
    };
    bool first = true;
    Event ev;
    while (pop_due(&ev)) {
      if (first) W().st.host_executions++;
      first = false;
      if (ev.time < h.last_popped) std::abort();  // event_queue.rs:75
      h.last_popped = ev.time;
      W().now = ev.time;  // Worker::set_current_time
      if (ev.kind == EV_PACKET && ev.task == TASK_SUBMIT) {
        app_submit(h, ev.pkt);
      } else if (ev.kind == EV_PACKET) {
        W().st.packet_events_popped++;
        h.n_popped++;
        sgn_drun_add_seq(&h.d_rx, &h.r_rx, ev.time, ev.src_host, ev.eid, 1);
        trace_rec(h, SGN_TRACE_POP, ev.src_host, 0, ev.time, 0, ev.eid);
        h.codel.push(ev.pkt, W().now);            // Router::route_incoming_packet (router/mod.rs:55)
        relay_notify(h, TASK_RELAY_IN);       // notify_router_has_packets (host.rs:958)
        W().st.max_codel_len = std::max<uint64_t>(W().st.max_codel_len, h.codel.elems.size());
      } else {
        W().st.local_events++;
        if (ev.task == TASK_APP)
          app_task(h);
        else
          run_forward_task(h, ev.task);
      }
    }
    // digests are run-encoded (sgn_workload.h): close the pending runs
    sgn_drun_flush_same(&h.d_tx, &h.r_tx);
    sgn_drun_flush_seq(&h.d_rx, &h.r_rx);
    sgn_drun_flush_seq(&h.d_app, &h.r_app);
  }

  uint64_t local_min_next() const {
    uint64_t m = EMU_INVALID;
    for (uint32_t i = lo; i < hi; i++)
      if (!hosts[i].q.empty()) m = std::min(m, hosts[i].q.top().time);
    return m;
  }

  // Controller::manager_finished_current_round (controller.rs:88-112)
  void advance(uint64_t min_next) {
    uint64_t runahead = runahead_get();
    uint64_t new_start = min_next;
    uint64_t new_end;
    uint64_t x = new_start + runahead;
    if (x < new_start || x > EMU_MAX)
      new_end = EMU_MAX;
    else
      new_end = x;
    new_end = std::min(new_end, end_time);
    active = new_start < new_end;
    prev_we = we;
    ws = new_start;
    we = new_end;
    st.rounds++;
  }

  // Host::next_event_time (host.rs:832-834), under the queue's lock when others may push
  uint64_t host_next(Host& h) {
    std::unique_lock<std::mutex> g;
    if (locked()) g = std::unique_lock<std::mutex>(qlock(h.id));
    return h.q.empty() ? EMU_INVALID : h.q.top().time;
  }

  // One round on the worker threads (core/manager.rs:568-601): each thread executes hosts
  // (taken in chunks from a shared counter) and keeps the minimum of their next event times
  // and of the deliveries it produced; the minima are reduced after the barrier (:623-628).
  void execute_round() {
    round_end = we;  // Worker::set_round_end_time (manager.rs:578)
    std::atomic<uint32_t> next{lo};
    auto worker = [&](int t) {
      tl_wk = &wks[t];
      Wk& w = wks[t];
      w.next_min = EMU_INVALID;  // Worker::reset_next_event_time (worker.rs:310)
      while (true) {
        const uint32_t a = next.fetch_add(256);
        if (a >= hi) break;
        const uint32_t e = std::min<uint32_t>(hi, a + 256);
        for (uint32_t i = a; i < e; i++) {
          execute(hosts[i], we);
          w.next_min = std::min(w.next_min, host_next(hosts[i]));
        }
      }
    };
    if (nthreads <= 1) {
      worker(0);
    } else {
      if (!pool || pool->n != nthreads) pool.reset(new Pool(nthreads));
      pool->run(worker);
      tl_wk = &wks[0];
    }
    merge_workers();
  }

  // the round barrier (manager.rs:623-628): fold the workers' counters and minima
  void merge_workers() {
    round_next_min = EMU_INVALID;
    for (Wk& w : wks) {
      round_next_min = std::min(round_next_min, w.next_min);
      st.packets_sent += w.st.packets_sent;
      st.packets_loss_dropped += w.st.packets_loss_dropped;
      st.packets_unknown_dst += w.st.packets_unknown_dst;
      st.packet_events_popped += w.st.packet_events_popped;
      st.codel_dropped += w.st.codel_dropped;
      st.delivered += w.st.delivered;
      st.local_delivered += w.st.local_delivered;
      st.app_blocked += w.st.app_blocked;
      st.local_events += w.st.local_events;
      st.bytes_delivered += w.st.bytes_delivered;
      st.host_executions += w.st.host_executions;
      st.max_codel_len = std::max(st.max_codel_len, w.st.max_codel_len);
      w.st = sgn_stats{};
      if (!w.tr.empty()) {
        tr.insert(tr.end(), w.tr.begin(), w.tr.end());
        w.tr.clear();
      }
      if (!w.exports.empty()) {
        exports.insert(exports.end(), w.exports.begin(), w.exports.end());
        w.exports.clear();
      }
      if (!w.dr.empty()) {
        drain_held.insert(drain_held.end(), w.dr.begin(), w.dr.end());
        w.dr.clear();
      }
      if (w.min_set) {
        if (!local_min_used_set || w.min_used < local_min_used) {
          local_min_used_set = true;
          local_min_used = w.min_used;
        }
        if (!has_min_used || w.min_used < min_used) {
          has_min_used = true;
          min_used = w.min_used;
        }
        w.min_set = false;
      }
    }
  }
};

// ====================================================================================
// extern "C"
// ====================================================================================
extern "C" {

uint64_t ora_siphash(int c, int d, uint64_t k0, uint64_t k1, const uint8_t* msg, size_t len) {
  return siphash(c, d, k0, k1, msg, len);
}
void ora_xoshiro_seed_from_u64(uint64_t seed, uint64_t st[4]) {
  Xoshiro x = Xoshiro::seed_from_u64(seed);
  std::memcpy(st, x.s, sizeof(x.s));
}
uint64_t ora_xoshiro_next_u64(uint64_t st[4]) {
  Xoshiro x;
  std::memcpy(x.s, st, sizeof(x.s));
  uint64_t r = x.next_u64();
  std::memcpy(st, x.s, sizeof(x.s));
  return r;
}
double ora_xoshiro_next_f64(uint64_t st[4]) {
  Xoshiro x;
  std::memcpy(x.s, st, sizeof(x.s));
  double r = x.next_f64();
  std::memcpy(st, x.s, sizeof(x.s));
  return r;
}
uint64_t ora_splitmix_next(uint64_t* state) { return splitmix_next(*state); }
void ora_host_seeds(uint32_t sim_seed, const char* const* names, uint32_t n, uint64_t* out) {
  Xoshiro g = Xoshiro::seed_from_u64((uint64_t)sim_seed);
  uint64_t r = g.next_u64();
  for (uint32_t i = 0; i < n; i++) out[i] = host_seed(r, names[i]);
}

int ora_units_parse(int kind, const char* text, uint64_t* value_base) {
  return units_parse(kind, text, value_base);
}

int ora_tb_new(uint64_t capacity, uint64_t inc, uint64_t interval, uint64_t last, ora_tb* out) {
  // TokenBucket::new_inner (token_bucket.rs:37-57)
  if (!(capacity > 0 && inc > 0 && interval != 0)) return SGN_EINVAL;
  out->capacity = capacity;
  out->balance = capacity;
  out->refill_increment = inc;
  out->refill_interval = interval;
  out->last_refill = last;
  return 0;
}
int ora_tb_remove(ora_tb* t, uint64_t dec, uint64_t now, uint64_t* out) {
  TB b{t->capacity, t->balance, t->refill_increment, t->refill_interval, t->last_refill};
  bool ok = b.remove(dec, now, out);
  t->balance = b.balance;
  t->last_refill = b.last_refill;
  return ok ? 1 : 0;
}
uint64_t ora_codel_control_law(uint64_t time, uint64_t count) {
  return codel_control_law(time, count);
}
struct ora_codel {
  CoDel q;
};
ora_codel* ora_codel_new(void) { return new ora_codel(); }
void ora_codel_free(ora_codel* q) { delete q; }
void ora_codel_push(ora_codel* q, uint32_t wire_len, uint64_t now) {
  Pkt p{0, 0, wire_len - SGN_UDP_HEADER_BYTES, 0, 0};
  q->q.push(p, now);
}
int ora_codel_pop(ora_codel* q, uint64_t now, uint32_t* wire_len) {
  Pkt p;
  bool got = q->q.pop(now, &p);
  q->q.dropped.clear();
  if (got && wire_len) *wire_len = p.wire();
  return got ? 1 : 0;
}
int ora_codel_process_standing_delay(ora_codel* q, uint64_t now, uint64_t sd) {
  return q->q.process_standing_delay(now, sd) ? 1 : 0;
}
void ora_codel_get(const ora_codel* q, ora_codel_state* o) {
  o->len = q->q.elems.size();
  o->total_bytes = q->q.total_bytes;
  o->mode = (uint64_t)q->q.mode;
  o->has_interval_end = q->q.has_ie;
  o->interval_end = q->q.ie;
  o->has_drop_next = q->q.has_dn;
  o->drop_next = q->q.dn;
  o->current_drop_count = q->q.cur;
  o->previous_drop_count = q->q.prev;
  o->dropped_total = q->q.dropped_total;
}
void ora_codel_set_mode(ora_codel* q, int drop_mode) { q->q.mode = drop_mode ? 1 : 0; }
int ora_codel_was_dropping_recently(const ora_codel* q, uint64_t now) {
  return q->q.was_dropping_recently(now) ? 1 : 0;
}
int ora_codel_should_drop(const ora_codel* q, uint64_t now) { return q->q.should_drop(now) ? 1 : 0; }

// IpAssignment (graph/mod.rs:348-418) as used by assign_ips (sim_config.rs:386-407)
int ora_assign_ips(uint32_t n, const uint8_t* explicit_flags, uint32_t* ips) {
  std::unordered_map<uint32_t, int> taken;
  for (uint32_t i = 0; i < n; i++)
    if (explicit_flags[i]) {
      if (taken.count(ips[i])) return SGN_EINVAL;
      taken[ips[i]] = 1;
    }
  uint32_t last = (11u << 24);  // 11.0.0.0
  for (uint32_t i = 0; i < n; i++) {
    if (explicit_flags[i]) continue;
    while (true) {
      uint32_t inc = 1;
      uint32_t next;
      while (true) {
        next = last + inc;
        uint32_t o = next & 0xff;
        if (o == 0 || o == 255)
          inc++;
        else
          break;
      }
      last = next;
      if (!taken.count(next)) {
        taken[next] = 1;
        ips[i] = next;
        break;
      }
    }
  }
  return 0;
}

int ora_gml_parse(const char* text, size_t len, ora_gml** out, char* err, size_t err_len) {
  return gml_parse(text, len, out, err, err_len);
}
void ora_gml_free(ora_gml* g) { delete g; }
int ora_gml_graph(const ora_gml* g, sgn_graph* o) {
  o->n_nodes = (uint32_t)g->node_id.size();
  o->node_id = g->node_id.data();
  o->n_edges = (uint32_t)g->esrc.size();
  o->edge_src = g->esrc.data();
  o->edge_dst = g->edst.data();
  o->edge_latency_ns = g->elat.data();
  o->edge_loss = g->eloss.data();
  o->directed = g->directed ? 1 : 0;
  return 0;
}
int ora_gml_node_bandwidth(const ora_gml* g, uint32_t i, uint64_t* up, int32_t* hu,
                           uint64_t* down, int32_t* hd) {
  if (i >= g->node_id.size()) return SGN_EINVAL;
  *up = g->bw_up[i];
  *hu = g->has_up[i];
  *down = g->bw_down[i];
  *hd = g->has_down[i];
  return 0;
}

int ora_routes(const sgn_graph* g, const uint32_t* used, uint32_t U, int shortest,
               uint64_t* lat, float* loss, char* err, size_t err_len) {
  return routes(g, used, U, shortest, lat, loss, err, err_len);
}

int ora_sim_create(const uint32_t* used, uint32_t U, const uint64_t* lat, const float* loss,
                   const sgn_hosts* H, const sgn_sim_config* cfg, const sgn_traffic* tr,
                   int trace, ora_sim** out, char* err, size_t err_len) {
  ora_sim* s = new ora_sim();
  s->U = U;
  s->used.assign(used, used + U);
  s->lat.assign(lat, lat + (size_t)U * U);
  s->loss.assign(loss, loss + (size_t)U * U);
  s->cfg = *cfg;
  s->traffic = *tr;
  if (tr->kind == SGN_TRAFFIC_TGEN) s->servers.assign(tr->server_hosts, tr->server_hosts + tr->n_servers);
  s->traffic.server_hosts = nullptr;
  s->trace = trace != 0;
  std::memset(&s->st, 0, sizeof(s->st));
  s->end_time = SIM_START + cfg->stop_time_ns;
  s->bootstrap_end = SIM_START + cfg->bootstrap_end_ns;
  s->min_possible_latency = *std::min_element(s->lat.begin(), s->lat.end());
  std::unordered_map<uint32_t, uint32_t> unode;
  for (uint32_t i = 0; i < U; i++) unode[used[i]] = i;
  s->hosts.resize(H->n_hosts);
  for (uint32_t i = 0; i < H->n_hosts; i++) {
    Host& h = s->hosts[i];
    h.id = i;
    h.ip = H->ip[i];
    auto it = unode.find(H->node_id[i]);
    if (it == unode.end()) { delete s; set_err(err, err_len, "host node not a used node"); return SGN_EINVAL; }
    h.unode = it->second;
    h.rng = Xoshiro::seed_from_u64(H->seed[i]);  // host.rs:234
    h.rout.tb = make_relay_bucket(H->bw_up_bits[i] / 8);    // host.rs:284-287
    h.rin.tb = make_relay_bucket(H->bw_down_bits[i] / 8);   // host.rs:288-291
    if (s->dns.count(h.ip)) { delete s; set_err(err, err_len, "duplicate host address"); return SGN_EINVAL; }
    s->dns[h.ip] = i;
  }
  for (uint32_t sv : s->servers) s->hosts[sv].is_server = true;
  s->submit_seq.assign(H->n_hosts, 0u);
  s->lo = 0;
  s->hi = H->n_hosts;
  // the initial window (manager.rs:506-509)
  s->ws = SIM_START;
  s->we = SIM_START + 1;
  s->active = true;
  // each app's first event (a process start is a local task, host.rs:703-706)
  for (uint32_t i = 0; i < H->n_hosts; i++) {
    Host& h = s->hosts[i];
    bool has_app = tr->kind == SGN_TRAFFIC_PERIODIC || (tr->kind == SGN_TRAFFIC_TGEN && !h.is_server);
    if (!has_app) continue;
    uint64_t t = SIM_START + sgn_app_start_rel(tr->flow_seed, i, tr->start_ns, tr->start_jitter_ns);
    tl_wk = &s->wks[0];
    s->wks[0].now = SIM_START;
    s->schedule_task(h, TASK_APP, t);
  }
  *out = s;
  return 0;
}

void ora_sim_free(ora_sim* s) { delete s; }

// ---- CPU-resident applications (SGN_TRAFFIC_EXTERNAL): the same contract as libsgn's
//      sgn_submit / sgn_drain / sgn_set_window (include/sgn.h) ----
int ora_sim_submit(ora_sim* s, const sgn_pkt_soa* b) {
  if (!s->external()) return SGN_ESTATE;
  std::vector<Event> evs;
  std::vector<uint32_t> seq = s->submit_seq;
  for (uint64_t i = 0; i < b->n; i++) {
    const uint32_t src = b->src_host[i];
    const uint64_t t = b->send_time[i];
    const uint32_t pay = b->payload_len[i];
    if (src < s->lo || src >= s->hi || t < s->ws || t >= s->end_time || pay > 0xFFFFu) return SGN_EINVAL;
    uint32_t hdr = 0;
    if (b->wire_len && b->wire_len[i] != 0) {
      const uint32_t w = b->wire_len[i];
      if (w == pay + SGN_UDP_HEADER_BYTES) hdr = 0;
      else if (w == pay + SGN_TCP_HEADER_BYTES) hdr = SGN_TAG_HDR_TCP;
      else if (w == pay + SGN_TCP_WS_HEADER_BYTES) hdr = SGN_TAG_HDR_TCPWS;
      else return SGN_EINVAL;
    }
    Event ev;
    ev.time = t;
    ev.kind = EV_PACKET;  // ordered with the host's packet events: (time, src = itself, order)
    ev.src_host = src;
    ev.eid = ((uint64_t)seq[src]++ << 32) | b->dst_ip[i];
    ev.task = TASK_SUBMIT;
    ev.pkt.src_host = src;
    ev.pkt.dst_ip = b->dst_ip[i];
    ev.pkt.payload = pay;
    ev.pkt.tag = SGN_TAG_EXT | hdr | (uint32_t)(s->handles.size() + i);
    ev.pkt.src_eid = 0;
    evs.push_back(ev);
  }
  for (const Event& ev : evs) s->hosts[ev.src_host].q.push(ev);
  for (uint64_t i = 0; i < b->n; i++) s->handles.push_back(b->handle ? b->handle[i] : 0);
  s->submit_seq.swap(seq);
  return 0;
}

int ora_sim_drain(ora_sim* s, uint32_t lo, uint32_t hi, sgn_drain_rec* out, uint64_t cap, uint64_t* n_out) {
  if (!s->external()) return SGN_ESTATE;
  for (sgn_drain_rec& r : s->drain_held) {
    const uint32_t slot = r.tag & SGN_TAG_SLOT_MASK;
    r.handle = ((r.tag & SGN_TAG_EXT) && slot < s->handles.size()) ? s->handles[slot] : 0;
  }
  std::vector<sgn_drain_rec> sel, keep;
  for (const sgn_drain_rec& r : s->drain_held) (r.host >= lo && r.host < hi ? sel : keep).push_back(r);
  auto key = [](const sgn_drain_rec& r) {
    return std::make_tuple(r.host, r.time, r.src_host, r.src_eid, r.tag, r.status);
  };
  std::sort(sel.begin(), sel.end(), [&](const sgn_drain_rec& a, const sgn_drain_rec& c) { return key(a) < key(c); });
  const uint64_t k = std::min<uint64_t>(cap, sel.size());
  if (k) std::memcpy(out, sel.data(), k * sizeof(sgn_drain_rec));
  keep.insert(keep.end(), sel.begin() + k, sel.end());
  s->drain_held.swap(keep);
  if (n_out) *n_out = k;
  return 0;
}

int ora_sim_set_window(ora_sim* s, uint64_t start, uint64_t end) {
  // Controller with CPU-side hosts (controller.rs:88-112): the caller's window must not skip
  // an event (start <= the next event time) nor go back (start >= the last window's end)
  if (start < s->prev_we || start > s->ws || end <= start) return SGN_EINVAL;
  end = std::min(end, s->end_time);
  if (end <= start) return SGN_EINVAL;
  s->ws = start;
  s->we = end;
  s->active = true;
  return 0;
}

// The host RNG (host/host.rs:1324-1336: host_rngDouble, host_rngNextNBytes)
int ora_sim_rng_next_u64(ora_sim* s, uint32_t host, uint64_t* out) {
  if (host >= s->hosts.size()) return SGN_EINVAL;
  *out = s->hosts[host].rng.next_u64();
  return 0;
}
int ora_sim_rng_double(ora_sim* s, uint32_t host, double* out) {
  if (host >= s->hosts.size()) return SGN_EINVAL;
  *out = s->hosts[host].rng.next_f64();  // rand 0.9 StandardUniform f64
  return 0;
}
int ora_sim_rng_fill_bytes(ora_sim* s, uint32_t host, uint8_t* buf, size_t len) {
  // rand_core 0.9.3 impls::fill_bytes_via_next (RngCore::fill_bytes of rand_xoshiro 0.7's
  // Xoshiro256PlusPlus; its next_u32 is the upper half of next_u64)
  if (host >= s->hosts.size()) return SGN_EINVAL;
  Xoshiro& x = s->hosts[host].rng;
  size_t i = 0;
  while (len - i >= 8) {
    const uint64_t v = x.next_u64();
    for (int k = 0; k < 8; k++) buf[i + k] = (uint8_t)(v >> (8 * k));
    i += 8;
  }
  const size_t n = len - i;
  if (n > 4) {
    const uint64_t v = x.next_u64();
    for (size_t k = 0; k < n; k++) buf[i + k] = (uint8_t)(v >> (8 * k));
  } else if (n > 0) {
    const uint32_t v = (uint32_t)(x.next_u64() >> 32);
    for (size_t k = 0; k < n; k++) buf[i + k] = (uint8_t)(v >> (8 * k));
  }
  return 0;
}

// Worker threads for the round loop (1 = sequential). Results do not depend on it.
int ora_sim_set_threads(ora_sim* s, int n) {
  if (n < 1 || n > 1024) return SGN_EINVAL;
  s->nthreads = n;
  s->wks.assign(n, Wk());
  s->pool.reset();
  if (n > 1 && !s->qmu) s->qmu.reset(new std::mutex[s->hosts.size()]);
  return 0;
}

// Reference-faithful (1) or CPU-optimised (0) data structures; results are identical.
int ora_sim_set_faithful(ora_sim* s, int on) {
  s->faithful = on != 0;
  if (!s->faithful) return 0;
  if (!s->qmu) s->qmu.reset(new std::mutex[s->hosts.size()]);
  s->ip_node.clear();
  s->route_map.clear();
  s->queue_map.clear();
  for (const Host& h : s->hosts) {
    s->ip_node[h.ip] = s->used[h.unode];            // IpAssignment (graph/mod.rs:348-418)
    s->queue_map[h.id] = &s->qmu[h.id];             // WorkerShared::event_queues
  }
  for (uint32_t i = 0; i < s->U; i++)              // RoutingInfo::paths (graph/mod.rs:430)
    for (uint32_t j = 0; j < s->U; j++)
      s->route_map[((uint64_t)s->used[i] << 32) | s->used[j]] = {s->lat[(size_t)i * s->U + j],
                                                                s->loss[(size_t)i * s->U + j]};
  return 0;
}

int ora_routes_mode(const sgn_graph* g, const uint32_t* used, uint32_t U, int shortest, int faithful,
                    int threads, uint64_t* lat, float* loss, char* err, size_t err_len) {
  return routes_mode(g, used, U, shortest, faithful, threads, lat, loss, err, err_len);
}

int ora_sim_window(const ora_sim* s, uint64_t* start, uint64_t* end, int32_t* active) {
  *start = s->ws;
  *end = s->we;
  *active = s->active ? 1 : 0;
  return 0;
}

int ora_sim_round(ora_sim* s, uint64_t* min_next) {
  if (!s->active) return SGN_ESTATE;
  s->execute_round();
  // the threads' minima (manager.rs:623-628); sharded runs use the shard protocol instead
  uint64_t m = s->round_next_min;
  if (m == EMU_INVALID) m = EMU_MAX;  // unwrap_or(EmulatedTime::MAX) (manager.rs:628)
  if (min_next) *min_next = m;
  s->advance(m);
  return 0;
}

int ora_sim_run(ora_sim* s, uint64_t max_rounds, uint64_t* done) {
  uint64_t n = 0;
  while (s->active && n < max_rounds) {
    ora_sim_round(s, nullptr);
    n++;
  }
  if (done) *done = n;
  return 0;
}

int ora_sim_stats(const ora_sim* s, sgn_stats* out) {
  *out = s->st;
  out->min_used_latency_ns = s->has_min_used ? s->min_used : EMU_INVALID;
  return 0;
}

int ora_sim_host_digests(const ora_sim* s, uint32_t lo, uint32_t hi, sgn_host_digest* out) {
  if (hi > s->hosts.size() || lo > hi) return SGN_EINVAL;
  for (uint32_t i = lo; i < hi; i++) {
    const Host& h = s->hosts[i];
    sgn_host_digest& d = out[i - lo];
    d.tx = h.d_tx;
    d.rx = h.d_rx;
    d.app = h.d_app;
    std::memcpy(d.rng, h.rng.s, sizeof(d.rng));
    d.next_event_id = h.eid_ctr;
    d.n_sent = h.n_sent;
    d.n_popped = h.n_popped;
    d.n_delivered = h.n_delivered;
    d.n_codel_dropped = h.n_codel_dropped;
  }
  return 0;
}

uint64_t ora_sim_trace_count(const ora_sim* s) { return s->tr.size(); }
uint64_t ora_sim_trace_read(const ora_sim* s, sgn_trace_rec* out, uint64_t cap) {
  uint64_t n = std::min<uint64_t>(cap, s->tr.size());
  std::memcpy(out, s->tr.data(), n * sizeof(sgn_trace_rec));
  return n;
}

int ora_sim_host_next_event_time(const ora_sim* s, uint32_t host, uint64_t* t) {
  if (host >= s->hosts.size()) return SGN_EINVAL;
  *t = s->hosts[host].q.empty() ? EMU_INVALID : s->hosts[host].q.top().time;
  return 0;
}

int ora_sim_set_shard(ora_sim* s, uint32_t lo, uint32_t hi) {
  if (lo > hi || hi > s->hosts.size()) return SGN_EINVAL;
  // hosts outside the shard must not hold events
  for (uint32_t i = 0; i < s->hosts.size(); i++)
    if (i < lo || i >= hi)
      while (!s->hosts[i].q.empty()) s->hosts[i].q.pop();
  s->lo = lo;
  s->hi = hi;
  return 0;
}

int ora_sim_shard_execute(ora_sim* s, uint64_t* n_exported) {
  if (!s->active) return SGN_ESTATE;
  s->exports.clear();
  s->local_min_used_set = false;
  s->execute_round();
  if (n_exported) *n_exported = s->exports.size() / 6;
  return 0;
}

uint64_t ora_sim_shard_take_exports(ora_sim* s, uint64_t* out, uint64_t cap) {
  uint64_t n = std::min<uint64_t>(cap, s->exports.size() / 6);
  std::memcpy(out, s->exports.data(), n * 6 * sizeof(uint64_t));
  return n;
}

int ora_sim_shard_import(ora_sim* s, const uint64_t* r, uint64_t n) {
  for (uint64_t i = 0; i < n; i++) {
    const uint64_t* x = r + 6 * i;
    uint32_t dst = (uint32_t)x[0];
    if (!s->owned(dst)) return SGN_EINVAL;
    Event ev;
    ev.time = x[1];
    ev.kind = EV_PACKET;
    ev.src_host = (uint32_t)x[2];
    ev.eid = x[3];
    ev.task = -1;
    ev.pkt.src_host = ev.src_host;
    ev.pkt.dst_ip = s->hosts[dst].ip;
    ev.pkt.payload = (uint32_t)x[4];
    ev.pkt.tag = (uint32_t)x[5];
    ev.pkt.src_eid = ev.eid;
    s->hosts[dst].q.push(ev);
  }
  return 0;
}

int ora_sim_shard_local_min(const ora_sim* s, uint64_t* min_next, uint64_t* min_used_lat) {
  *min_next = s->local_min_next();
  *min_used_lat = s->local_min_used_set ? s->local_min_used : EMU_INVALID;
  return 0;
}

int ora_sim_shard_advance(ora_sim* s, uint64_t gmin, uint64_t gmin_used) {
  if (gmin_used != EMU_INVALID && s->cfg.use_dynamic_runahead) {
    if (!s->has_min_used || gmin_used < s->min_used) {
      s->has_min_used = true;
      s->min_used = gmin_used;
    }
  }
  s->advance(gmin == EMU_INVALID ? EMU_MAX : gmin);
  return 0;
}

}  // extern "C"
