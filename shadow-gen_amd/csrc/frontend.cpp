// frontend.cpp — drop-in graph ingest: GML text -> sgn_graph, and unit strings.
//
// Grammar of gml_parser (lib/gml-parser/src/parser.rs):
//   gml      := ms0 "graph" sp0 "[" nl item* "]" ms0 (trailing text ignored, lib.rs:55-60)
//   item     := key ( node | edge | "directed" value(int 0|1) | value )
//   node/edge:= sp0 "[" nl (key value)* "]" nl          (duplicate keys rejected)
//   value    := sp0 ( int nl | float nl | string nl )   (int = digit1 as i32; float =
//               nom recognize_float parsed as f32; string = '"' [^"]* '"')
//   nl       := sp0 ms1 sp0
// and NetworkGraph::parse / ShadowNode / ShadowEdge (network/graph/mod.rs:28-179):
//   node id (Int) required; host_bandwidth_{up,down} strings -> BitsPerSec;
//   edge latency (string, non-zero), jitter (string, ignored), packet_loss (Float in [0,1]).
// Units: utility/units.rs FromStr (:406-440) and convert() with checked_mul (:378-389).

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "sgn.h"

struct sgn_gml {
  int directed = 0;
  std::vector<uint32_t> node_id;
  std::vector<uint64_t> up, down;
  std::vector<int32_t> has_up, has_down;
  std::vector<uint32_t> src, dst;
  std::vector<uint64_t> lat;
  std::vector<float> loss;
};

namespace {

struct Unit {
  const char* name;
  uint64_t factor;
};

// TimePrefix (units.rs:214-262) in nanoseconds
const Unit kTime[] = {
    {"ns", 1ULL}, {"nanosecond", 1ULL}, {"nanoseconds", 1ULL},
    {"us", 1000ULL}, {"\xce\xbcs", 1000ULL}, {"microsecond", 1000ULL}, {"microseconds", 1000ULL},
    {"ms", 1000000ULL}, {"millisecond", 1000000ULL}, {"milliseconds", 1000000ULL},
    {"s", 1000000000ULL}, {"sec", 1000000000ULL}, {"secs", 1000000000ULL},
    {"second", 1000000000ULL}, {"seconds", 1000000000ULL},
    {"m", 60000000000ULL}, {"min", 60000000000ULL}, {"mins", 60000000000ULL},
    {"minute", 60000000000ULL}, {"minutes", 60000000000ULL},
    {"h", 3600000000000ULL}, {"hr", 3600000000000ULL}, {"hrs", 3600000000000ULL},
    {"hour", 3600000000000ULL}, {"hours", 3600000000000ULL},
};
// SiPrefixUpper (units.rs:159-205)
const Unit kSi[] = {
    {"K", 1000ULL}, {"kilo", 1000ULL}, {"Ki", 1024ULL}, {"kibi", 1024ULL},
    {"M", 1000000ULL}, {"mega", 1000000ULL}, {"Mi", 1048576ULL}, {"mebi", 1048576ULL},
    {"G", 1000000000ULL}, {"giga", 1000000000ULL}, {"Gi", 1073741824ULL}, {"gibi", 1073741824ULL},
    {"T", 1000000000000ULL}, {"tera", 1000000000000ULL}, {"Ti", 1099511627776ULL},
    {"tebi", 1099511627776ULL},
};

bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\f' || c == '\v'; }

int parse_unit(int kind, const std::string& in, uint64_t* out) {
  // ^([+-]?[0-9\.]*)\s*(.*)$
  size_t i = 0, n = in.size();
  if (i < n && (in[i] == '+' || in[i] == '-')) i++;
  while (i < n && (isdigit((unsigned char)in[i]) || in[i] == '.')) i++;
  std::string num = in.substr(0, i);
  while (i < n && is_ws(in[i])) i++;
  std::string rest = in.substr(i);
  if (rest.find('\n') != std::string::npos) return SGN_EINVAL;  // '.' never matches '\n'
  auto strip = [](std::string s) {
    while (!s.empty() && is_ws(s.back())) s.pop_back();
    size_t a = 0;
    while (a < s.size() && is_ws(s[a])) a++;
    return s.substr(a);
  };
  num = strip(num);
  rest = strip(rest);
  std::vector<std::string> suffixes;
  if (kind == 0) suffixes = {""};
  else if (kind == 1) suffixes = {"B", "byte", "bytes"};
  else suffixes = {"bit", "bits"};
  std::string prefix = rest;
  for (const std::string& sfx : suffixes) {
    if (rest.size() >= sfx.size() && rest.compare(rest.size() - sfx.size(), sfx.size(), sfx) == 0) {
      prefix = rest.substr(0, rest.size() - sfx.size());
      break;
    }
  }
  uint64_t factor = 0;
  if (prefix.empty()) {
    factor = kind == 0 ? 1000000000ULL : 1ULL;  // TimePrefix::Sec / SiPrefixUpper::Base
  } else if (kind == 0) {
    for (const Unit& u : kTime) if (prefix == u.name) factor = u.factor;
  } else {
    for (const Unit& u : kSi) if (prefix == u.name) factor = u.factor;
  }
  if (!factor) return SGN_EINVAL;
  // <u64 as FromStr>: optional '+', at least one digit, digits only, no overflow
  const char* p = num.c_str();
  if (*p == '+') p++;
  if (!*p) return SGN_EINVAL;
  uint64_t v = 0;
  for (; *p; p++) {
    if (*p < '0' || *p > '9') return SGN_EINVAL;
    const uint64_t d = (uint64_t)(*p - '0');
    if (v > (UINT64_MAX - d) / 10) return SGN_EINVAL;
    v = v * 10 + d;
  }
  if (v != 0 && factor > UINT64_MAX / v) return SGN_ERANGE;  // checked_mul
  *out = v * factor;
  return 0;
}

enum VType { V_INT, V_FLOAT, V_STR };
struct Val {
  VType t;
  int32_t i = 0;
  float f = 0;
  std::string s;
};

class Cursor {
 public:
  Cursor(const char* b, const char* e) : p_(b), e_(e) {}
  std::string error;

  void sp0() { while (p_ < e_ && (*p_ == ' ' || *p_ == '\t')) p_++; }
  void ms0() { while (p_ < e_ && (*p_ == ' ' || *p_ == '\t' || *p_ == '\n' || *p_ == '\r')) p_++; }
  bool nl() {
    sp0();
    const char* s = p_;
    ms0();
    if (p_ == s) return false;
    sp0();
    return true;
  }
  bool lit(const char* t) {
    const size_t n = std::strlen(t);
    if ((size_t)(e_ - p_) < n || std::strncmp(p_, t, n) != 0) return false;
    p_ += n;
    return true;
  }
  bool key(std::string* k) {
    if (p_ >= e_ || !(isalpha((unsigned char)*p_) || *p_ == '_')) return false;
    const char* s = p_;
    while (p_ < e_ && (isalnum((unsigned char)*p_) || *p_ == '_')) p_++;
    k->assign(s, p_);
    return true;
  }
  bool value(Val* v) {
    sp0();
    const char* start = p_;
    if (try_int(v)) return true;
    p_ = start;
    if (!error.empty()) return false;
    if (try_float(v)) return true;
    p_ = start;
    if (!error.empty()) return false;
    if (try_str(v)) return true;
    p_ = start;
    return false;
  }
  bool block(std::map<std::string, Val>* kv) {
    sp0();
    if (!lit("[") || !nl()) return false;
    size_t count = 0;
    while (!lit("]")) {
      std::string k;
      Val v;
      if (!key(&k) || !value(&v)) return false;
      (*kv)[k] = v;
      count++;
    }
    if (kv->size() != count) {
      error = "Duplicate keys are not supported";
      return false;
    }
    return nl();
  }

 private:
  bool try_int(Val* v) {
    const char* s = p_;
    while (p_ < e_ && isdigit((unsigned char)*p_)) p_++;
    if (p_ == s || p_ - s > 10) return false;
    const long long x = std::strtoll(std::string(s, p_).c_str(), nullptr, 10);
    if (x > 2147483647LL) return false;  // i32 parse error -> next alternative
    if (!nl()) return false;
    v->t = V_INT;
    v->i = (int32_t)x;
    return true;
  }
  bool try_float(Val* v) {
    const char* s = p_;
    if (p_ < e_ && (*p_ == '+' || *p_ == '-')) p_++;
    const char* d = p_;
    while (p_ < e_ && isdigit((unsigned char)*p_)) p_++;
    if (p_ > d) {
      if (p_ < e_ && *p_ == '.') {
        p_++;
        while (p_ < e_ && isdigit((unsigned char)*p_)) p_++;
      }
    } else {
      if (!(p_ < e_ && *p_ == '.')) return false;
      p_++;
      const char* f = p_;
      while (p_ < e_ && isdigit((unsigned char)*p_)) p_++;
      if (p_ == f) return false;
    }
    if (p_ < e_ && (*p_ == 'e' || *p_ == 'E')) {
      p_++;
      if (p_ < e_ && (*p_ == '+' || *p_ == '-')) p_++;
      const char* x = p_;
      while (p_ < e_ && isdigit((unsigned char)*p_)) p_++;
      if (p_ == x) {
        error = "invalid float exponent";  // nom cut(): a hard failure
        return false;
      }
    }
    const std::string txt(s, p_);
    const float f = std::strtof(txt.c_str(), nullptr);  // correctly rounded, like Rust
    if (!nl()) return false;
    v->t = V_FLOAT;
    v->f = f;
    return true;
  }
  bool try_str(Val* v) {
    if (!lit("\"")) return false;
    const char* s = p_;
    while (p_ < e_ && *p_ != '"') p_++;
    if (p_ >= e_) return false;
    v->s.assign(s, p_);
    p_++;
    if (!nl()) return false;
    v->t = V_STR;
    return true;
  }
  const char* p_;
  const char* e_;
};

int fail(char* err, size_t n, const std::string& m) {
  if (err && n) std::snprintf(err, n, "%s", m.c_str());
  return SGN_EINVAL;
}

}  // namespace

extern "C" {

int sgn_units_parse(int32_t kind, const char* text, uint64_t* value_base) {
  if (!text || !value_base || kind < 0 || kind > 2) return SGN_EINVAL;
  return parse_unit(kind, text, value_base);
}

int sgn_gml_parse(const char* text, size_t len, sgn_gml** out, char* err, size_t err_len) {
  if (!text || !out) return SGN_EINVAL;
  *out = nullptr;
  Cursor c(text, text + len);
  c.ms0();
  if (!c.lit("graph")) return fail(err, err_len, "expected 'graph'");
  c.sp0();
  if (!c.lit("[") || !c.nl()) return fail(err, err_len, "expected '[' and a newline after 'graph'");
  struct RawNode { std::map<std::string, Val> kv; };
  std::vector<RawNode> nodes, edges;
  int n_directed = 0, directed = 0;
  std::map<std::string, int> others;
  size_t n_others = 0;
  while (!c.lit("]")) {
    std::string k;
    if (!c.key(&k)) return fail(err, err_len, c.error.empty() ? "expected a key" : c.error);
    if (k == "node" || k == "edge") {
      RawNode r;
      if (!c.block(&r.kv)) return fail(err, err_len, c.error.empty() ? "malformed " + k : c.error);
      (k == "node" ? nodes : edges).push_back(r);
    } else {
      Val v;
      if (!c.value(&v)) return fail(err, err_len, c.error.empty() ? "malformed value for " + k : c.error);
      if (k == "directed") {
        if (v.t != V_INT) return fail(err, err_len, "Value was not an integer");
        if (v.i != 0 && v.i != 1) return fail(err, err_len, "Bool must be 0 or 1");
        directed = v.i;
        n_directed++;
      } else {
        others[k]++;
        n_others++;
      }
    }
  }
  if (n_directed > 1) return fail(err, err_len, "The 'directed' key must only be specified once");
  if (others.size() != n_others) return fail(err, err_len, "Duplicate keys are not supported");
  sgn_gml* g = new sgn_gml();
  g->directed = directed;
  std::unordered_map<uint32_t, bool> ids;
  for (RawNode& n : nodes) {
    auto it = n.kv.find("id");
    if (it != n.kv.end() && it->second.t != V_INT) { delete g; return fail(err, err_len, "Incorrect 'id' type"); }
    if (it == n.kv.end()) { delete g; return fail(err, err_len, "Node 'id' was not provided"); }
    const uint32_t id = (uint32_t)it->second.i;
    uint64_t bw[2] = {0, 0};
    int32_t has[2] = {0, 0};
    const char* names[2] = {"host_bandwidth_up", "host_bandwidth_down"};
    for (int w = 0; w < 2; w++) {
      auto b = n.kv.find(names[w]);
      if (b == n.kv.end()) continue;
      if (b->second.t != V_STR) { delete g; return fail(err, err_len, std::string("Node '") + names[w] + "' is not a string"); }
      if (parse_unit(2, b->second.s, &bw[w]) != 0) { delete g; return fail(err, err_len, std::string("Node '") + names[w] + "' is not a valid unit"); }
      has[w] = 1;
    }
    g->node_id.push_back(id);
    g->up.push_back(bw[0]);
    g->down.push_back(bw[1]);
    g->has_up.push_back(has[0]);
    g->has_down.push_back(has[1]);
    ids[id] = true;
  }
  for (RawNode& e : edges) {
    uint32_t st[2];
    const char* ends[2] = {"source", "target"};
    for (int w = 0; w < 2; w++) {
      auto it = e.kv.find(ends[w]);
      if (it == e.kv.end()) { delete g; return fail(err, err_len, std::string("'") + ends[w] + "' doesn't exist"); }
      if (it->second.t != V_INT) { delete g; return fail(err, err_len, std::string("Incorrect '") + ends[w] + "' type"); }
      st[w] = (uint32_t)it->second.i;
    }
    auto l = e.kv.find("latency");
    if (l == e.kv.end()) { delete g; return fail(err, err_len, "Edge 'latency' was not provided"); }
    if (l->second.t != V_STR) { delete g; return fail(err, err_len, "Edge 'latency' is not a string"); }
    uint64_t ns = 0;
    int rc = parse_unit(0, l->second.s, &ns);
    if (rc == SGN_EINVAL) { delete g; return fail(err, err_len, "Edge 'latency' is not a valid unit"); }
    if (rc) { delete g; return fail(err, err_len, "Edge 'latency' overflows u64 nanoseconds"); }
    auto j = e.kv.find("jitter");
    if (j != e.kv.end()) {
      uint64_t jn;
      if (j->second.t != V_STR) { delete g; return fail(err, err_len, "Edge 'jitter' is not a string"); }
      if (parse_unit(0, j->second.s, &jn) == SGN_EINVAL) { delete g; return fail(err, err_len, "Edge 'jitter' is not a valid unit"); }
    }
    float p = 0.0f;
    auto lo = e.kv.find("packet_loss");
    if (lo != e.kv.end()) {
      if (lo->second.t != V_FLOAT) { delete g; return fail(err, err_len, "Edge 'packet_loss' is not a float"); }
      p = lo->second.f;
    }
    if (p < 0.0f || p > 1.0f) { delete g; return fail(err, err_len, "Edge 'packet_loss' is not in the range [0,1]"); }
    if (ns == 0) { delete g; return fail(err, err_len, "Edge 'latency' must not be 0"); }
    if (!ids.count(st[0])) { delete g; return fail(err, err_len, "Edge source " + std::to_string(st[0]) + " doesn't exist"); }
    if (!ids.count(st[1])) { delete g; return fail(err, err_len, "Edge target " + std::to_string(st[1]) + " doesn't exist"); }
    g->src.push_back(st[0]);
    g->dst.push_back(st[1]);
    g->lat.push_back(ns);
    g->loss.push_back(p);
  }
  *out = g;
  return 0;
}

void sgn_gml_free(sgn_gml* g) { delete g; }

int sgn_gml_graph(const sgn_gml* g, sgn_graph* o) {
  if (!g || !o) return SGN_EINVAL;
  o->n_nodes = (uint32_t)g->node_id.size();
  o->node_id = g->node_id.data();
  o->n_edges = (uint32_t)g->src.size();
  o->edge_src = g->src.data();
  o->edge_dst = g->dst.data();
  o->edge_latency_ns = g->lat.data();
  o->edge_loss = g->loss.data();
  o->directed = g->directed;
  return 0;
}

int sgn_assign_ips(uint32_t n, const uint8_t* explicit_ip, uint32_t* ips, uint32_t* bad_host) {
  if (n && (!ips || !explicit_ip)) return SGN_EINVAL;
  // Configured addresses first, in HostId order; a repeat is IpPreviouslyAssignedError.
  std::vector<std::pair<uint32_t, uint32_t>> fixed;  // (address, host)
  for (uint32_t i = 0; i < n; i++)
    if (explicit_ip[i]) fixed.emplace_back(ips[i], i);
  std::sort(fixed.begin(), fixed.end());
  // Registration stops at the first host (in HostId order) whose address is taken: in each
  // group of equal addresses that is the group's second-lowest host.
  uint32_t first_bad = UINT32_MAX;
  for (size_t k = 1; k < fixed.size(); k++)
    if (fixed[k].first == fixed[k - 1].first && (k < 2 || fixed[k - 2].first != fixed[k].first))
      first_bad = std::min(first_bad, fixed[k].second);
  if (first_bad != UINT32_MAX) {
    if (bad_host) *bad_host = first_bad;
    return SGN_EINVAL;
  }
  // The dynamic cursor only moves up, so one pass over the sorted configured addresses
  // finds the collisions that IpAssignment::assign's vacancy loop skips.
  uint64_t last = 11ull << 24;  // 11.0.0.0
  size_t f = 0;
  for (uint32_t i = 0; i < n; i++) {
    if (explicit_ip[i]) continue;
    for (;;) {
      uint64_t next = last + 1;
      while ((next & 0xFF) == 0 || (next & 0xFF) == 255) next++;
      if (next > 0xFFFFFFFFull) {
        if (bad_host) *bad_host = i;
        return SGN_ERANGE;  // the reference's u32 addition would overflow here
      }
      last = next;
      while (f < fixed.size() && fixed[f].first < next) f++;
      if (f < fixed.size() && fixed[f].first == next) continue;
      ips[i] = (uint32_t)next;
      break;
    }
  }
  return 0;
}

int sgn_gml_node_bandwidth(const sgn_gml* g, uint32_t i, uint64_t* up, int32_t* has_up,
                           uint64_t* down, int32_t* has_down) {
  if (!g || i >= g->node_id.size()) return SGN_EINVAL;
  if (up) *up = g->up[i];
  if (has_up) *has_up = g->has_up[i];
  if (down) *down = g->down[i];
  if (has_down) *has_down = g->has_down[i];
  return 0;
}

}  // extern "C"
