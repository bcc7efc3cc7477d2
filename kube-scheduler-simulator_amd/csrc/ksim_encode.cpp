// ksim_encode.cpp — the native host snapshot encoder (SURVEY §2.3 "Host
// snapshot encoder", ABI 10; include/ksim_engine.h "native snapshot encoder").
//
// v1.Node / v1.Pod objects, handed over as one flat pool, become the engine's
// inputs: the node table in nodeTree order with the NodeInfo aggregates of the
// bound pods ([upstream] internal/cache snapshot + NodeInfo.AddPod), the taint
// and label vocabularies, and the queue's compiled pods (the PreFilter /
// PreScore precomputation of NodeResourcesFit, TaintToleration, NodeAffinity,
// NodePorts, ImageLocality, PodTopologySpread, InterPodAffinity and the
// simulator's NetworkBandwidth plugin).
//
// It restates ksim/encode.py and ksim/topology.py function by function (the
// names below are theirs), in the same order of operations, so that every
// output array is byte-equal to the Python compile's (tests/test_native_encode.py):
// label columns are created in the order the pods first reference their keys,
// count classes in the order the Python registry creates them.  Strings stay
// on the host; the device only sees integer ids.  Host code only: no HIP call.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <iterator>
#include <memory>
#include <new>
#include <stdexcept>
#include <string>
#include <string_view>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

#include "../../include/ksim_engine.h"

namespace {

using std::string;
using std::string_view;
using std::vector;
using Labels = vector<std::pair<string, string>>;

struct EncError {
  int code;
  string msg;
};

[[noreturn]] void fail(const string& m, int code = KSIM_E_INVALID) { throw EncError{code, m}; }

constexpr int64_t kDefaultMilliCPU = 100;                // schedutil.DefaultMilliCPURequest
constexpr int64_t kDefaultMemory = 200LL * 1024 * 1024;  // schedutil.DefaultMemoryRequest
constexpr int64_t kMB = 1024 * 1024;
constexpr int64_t kImageMin = 23 * kMB;                  // imagelocality minThreshold
constexpr int64_t kImageMaxContainer = 1000 * kMB;       // imagelocality maxContainerThreshold
const char* const kHostname = "kubernetes.io/hostname";
const char* const kZone = "topology.kubernetes.io/zone";
const char* const kRegion = "topology.kubernetes.io/region";
const char* const kZoneBeta = "failure-domain.beta.kubernetes.io/zone";
const char* const kRegionBeta = "failure-domain.beta.kubernetes.io/region";
const char* const kTaintUnschedulable = "node.kubernetes.io/unschedulable";
const char* const kBindAll = "0.0.0.0";                  // DefaultBindAllHostIP
const char* const kIngressBandwidth = "kubernetes.io/ingress-bandwidth";   // networkbandwidth/plugin.go:21
const char* const kEgressBandwidth = "kubernetes.io/egress-bandwidth";     // plugin.go:22

bool is_native_resource(string_view k) {
  return k == "cpu" || k == "memory" || k == "ephemeral-storage" || k == "pods";
}

const string* lookup(const Labels& m, string_view k) {
  for (const auto& kv : m)
    if (kv.first == k) return &kv.second;
  return nullptr;
}

// ---- the input pool -----------------------------------------------------------
struct PoolView {
  const ksim_k8s_pool& p;

  explicit PoolView(const ksim_k8s_pool& q) : p(q) {
    if (p.n_strings < 0 || (p.n_strings > 0 && !p.str_off)) fail("pool: bad string table");
    if (p.n_strings > 0) {
      if (p.str_off[0] < 0) fail("pool: bad string offsets");
      for (int64_t i = 0; i < p.n_strings; i++)
        if (p.str_off[i + 1] < p.str_off[i]) fail("pool: string offsets decrease");
      if (p.str_off[p.n_strings] > 0 && !p.strings) fail("pool: no string bytes");
    }
  }
  string_view str(int32_t id) const {
    if (id < 0 || id >= p.n_strings) fail("pool: string id out of range");
    return string_view(p.strings + p.str_off[id], (size_t)(p.str_off[id + 1] - p.str_off[id]));
  }
  template <class T>
  const T* at(const T* arr, int64_t n, int32_t first, int32_t count, const char* what) const {
    if (count == 0) return arr;
    if (first < 0 || count < 0 || (int64_t)first + count > n || !arr) fail(string("pool: range out of ") + what);
    return arr + first;
  }
  template <class T>
  const T& one(const T* arr, int64_t n, int32_t i, const char* what) const {
    if (i < 0 || i >= n || !arr) fail(string("pool: index out of ") + what);
    return arr[i];
  }
  Labels kv(int32_t first, int32_t count) const {
    Labels out;
    const ksim_k8s_kv* x = at(p.kv, p.n_kv, first, count, "kv");
    out.reserve(count > 0 ? count : 0);
    for (int32_t i = 0; i < count; i++) out.emplace_back(string(str(x[i].key)), string(str(x[i].value)));
    return out;
  }
  vector<string> strs(int32_t first, int32_t count) const {
    vector<string> out;
    const int32_t* x = at(p.str_list, p.n_str_list, first, count, "str_list");
    for (int32_t i = 0; i < count; i++) out.emplace_back(str(x[i]));
    return out;
  }
};

// ---- resource.Quantity -----------------------------------------------------------
// The exact value sign * digits * 10^e10 * 2^e2 of a Quantity string, by the
// grammar ksim/model.py (and ksim/netbw.py) parse:
//   [+-]?(\d+\.?\d*|\.\d+)((Ki|Mi|Gi|Ti|Pi|Ei|[numkMGTPE])|[eE][+-]?\d+)?
struct Dec {
  bool neg = false;
  string digits;      // mantissa digits, no point
  int64_t e10 = 0;
  int e2 = 0;
};

bool parse_quantity_text(string_view s, Dec& q) {
  size_t i = 0;
  q = Dec{};
  if (i < s.size() && (s[i] == '+' || s[i] == '-')) q.neg = s[i++] == '-';
  size_t a = i;
  while (i < s.size() && s[i] >= '0' && s[i] <= '9') i++;
  const size_t nint = i - a;
  q.digits.assign(s.substr(a, nint));
  size_t nfrac = 0;
  if (i < s.size() && s[i] == '.') {
    i++;
    const size_t b = i;
    while (i < s.size() && s[i] >= '0' && s[i] <= '9') i++;
    nfrac = i - b;
    q.digits.append(s.substr(b, nfrac));
    if (nint == 0 && nfrac == 0) return false;
  } else if (nint == 0) {
    return false;
  }
  q.e10 = -(int64_t)nfrac;
  const string_view suf = s.substr(i);
  if (suf.empty()) return true;
  static const char* const kBin[] = {"Ki", "Mi", "Gi", "Ti", "Pi", "Ei"};
  for (int k = 0; k < 6; k++)
    if (suf == kBin[k]) {
      q.e2 = 10 * (k + 1);
      return true;
    }
  if (suf.size() == 1) {
    static const char* const kDecSuf = "numkMGTPE";
    static const int kDecExp[] = {-9, -6, -3, 3, 6, 9, 12, 15, 18};
    const char* f = std::strchr(kDecSuf, suf[0]);
    if (f && suf[0]) {
      q.e10 += kDecExp[f - kDecSuf];
      return true;
    }
  }
  if (suf[0] != 'e' && suf[0] != 'E') return false;
  size_t j = 1;
  bool eneg = false;
  if (j < suf.size() && (suf[j] == '+' || suf[j] == '-')) eneg = suf[j++] == '-';
  if (j >= suf.size()) return false;
  int64_t e = 0;
  for (; j < suf.size(); j++) {
    if (suf[j] < '0' || suf[j] > '9') return false;
    e = e * 10 + (suf[j] - '0');
    if (e > 100000) fail("quantity exponent out of range");
  }
  q.e10 += eneg ? -e : e;
  return true;
}

// value * 10^extra as (|quotient|, exact) of the truncated magnitude; false
// when the magnitude does not fit in an unsigned 64-bit word.
bool scaled_magnitude(const Dec& q, int extra, uint64_t& mag, bool& exact) {
  vector<uint32_t> big;                       // little-endian base 2^32
  auto mul_add = [&](uint32_t m, uint32_t add) {
    uint64_t carry = add;
    for (auto& w : big) {
      const uint64_t t = (uint64_t)w * m + carry;
      w = (uint32_t)t;
      carry = t >> 32;
    }
    if (carry) big.push_back((uint32_t)carry);
  };
  for (char c : q.digits) mul_add(10, (uint32_t)(c - '0'));
  int64_t e = q.e10 + extra;
  for (int k = 0; k < q.e2; k++) mul_add(2, 0);
  auto is_zero = [&]() {
    for (auto w : big)
      if (w) return false;
    return true;
  };
  exact = true;
  if (is_zero()) {
    mag = 0;
    return true;
  }
  while (e > 0) {
    mul_add(10, 0);
    e--;
    if (big.size() > 4) return false;
  }
  while (e < 0 && !is_zero()) {
    uint64_t rem = 0;
    for (size_t k = big.size(); k-- > 0;) {
      const uint64_t cur = (rem << 32) | big[k];
      big[k] = (uint32_t)(cur / 10);
      rem = cur % 10;
    }
    if (rem) exact = false;
    e++;
  }
  if (e < 0) exact = false;                   // a non-zero value divided to zero
  while (!big.empty() && big.back() == 0) big.pop_back();
  if (big.size() > 2) return false;
  mag = big.empty() ? 0 : (big.size() == 1 ? big[0] : ((uint64_t)big[1] << 32) | big[0]);
  return true;
}

// math.ceil(value * 10^extra) as an int64 (quantity_value / quantity_milli_value)
int64_t quantity_ceil(string_view raw, int extra) {
  string_view s = raw;
  auto ws = [](char c) { return c == ' ' || (c >= '\t' && c <= '\r') || (c >= '\x1c' && c <= '\x1f'); };
  while (!s.empty() && ws(s.front())) s.remove_prefix(1);
  while (!s.empty() && ws(s.back())) s.remove_suffix(1);
  Dec q;
  if (!parse_quantity_text(s, q)) fail("invalid quantity '" + string(raw) + "'");
  uint64_t mag;
  bool exact;
  if (!scaled_magnitude(q, extra, mag, exact)) fail("quantity '" + string(raw) + "' out of the int64 range");
  if (!q.neg) {
    if (!exact) mag += 1;
    if (mag > (uint64_t)INT64_MAX) fail("quantity '" + string(raw) + "' out of the int64 range");
    return (int64_t)mag;
  }
  if (mag > (uint64_t)INT64_MAX + 1) fail("quantity '" + string(raw) + "' out of the int64 range");
  return mag == (uint64_t)INT64_MAX + 1 ? INT64_MIN : -(int64_t)mag;   // ceil of a negative: truncation
}

// ksim/netbw.py milli: resource.ParseQuantity in milli-units; false when the
// string does not parse; fails (QuantityError) for a finer fraction or a value
// outside (-2^63, 2^63 / 1024).
bool netbw_milli(string_view s, int64_t& out) {
  Dec q;
  if (!parse_quantity_text(s, q)) return false;
  uint64_t mag;
  bool exact;
  const bool fits = scaled_magnitude(q, 3, mag, exact);
  if (fits && !exact) fail("quantity '" + string(s) + "' is finer than 1m");
  const uint64_t lim = ((uint64_t)1 << 63) / 1024;
  if (!fits || (q.neg ? mag >= ((uint64_t)1 << 63) : mag >= lim))
    fail("quantity '" + string(s) + "' out of the engine's range");
  out = q.neg ? -(int64_t)mag : (int64_t)mag;
  return true;
}

// strconv.ParseInt(s, 10, 64) as encode.py _parse_int64 restates it
bool parse_int64(const string& s, int64_t& v) {
  size_t i = (!s.empty() && (s[0] == '+' || s[0] == '-')) ? 1 : 0;
  if (i >= s.size()) return false;
  for (size_t k = i; k < s.size(); k++)
    if (s[k] < '0' || s[k] > '9') return false;
  const bool neg = s[0] == '-';
  unsigned __int128 m = 0;
  for (size_t k = i; k < s.size(); k++) {
    m = m * 10 + (unsigned)(s[k] - '0');
    if (m > ((unsigned __int128)1 << 64)) return false;
  }
  if (!neg && m > (unsigned __int128)INT64_MAX) return false;
  if (neg && m > (unsigned __int128)INT64_MAX + 1) return false;
  v = neg ? (m == (unsigned __int128)INT64_MAX + 1 ? INT64_MIN : -(int64_t)m) : (int64_t)m;
  return true;
}

// ---- Kubernetes objects, as the compile reads them --------------------------------
struct Req {                    // NodeSelectorRequirement / LabelSelectorRequirement
  string key, op;
  vector<string> values;
};

struct SelTerm {                // NodeSelectorTerm
  vector<Req> exprs, fields;
};

// metav1.LabelSelector in canonical form (LabelSelector.key(): matchLabels
// and requirements sorted; a selector is a pure conjunction, so matching the
// canonical form is matching the object)
struct Selector {
  Labels labels;
  vector<Req> exprs;            // values sorted
  string key;

  bool empty() const { return labels.empty() && exprs.empty(); }
  // LabelSelector.matches (an invalid requirement matches nothing)
  bool matches(const Labels& l) const {
    for (const auto& kv : labels) {
      const string* v = lookup(l, kv.first);
      if (!v || *v != kv.second) return false;
    }
    for (const auto& r : exprs) {
      const string* v = lookup(l, r.key);
      if (r.op == "In") {
        if (r.values.empty() || !v || !std::binary_search(r.values.begin(), r.values.end(), *v)) return false;
      } else if (r.op == "NotIn") {
        if (r.values.empty()) return false;
        if (v && std::binary_search(r.values.begin(), r.values.end(), *v)) return false;
      } else if (r.op == "Exists") {
        if (!r.values.empty() || !v) return false;
      } else if (r.op == "DoesNotExist") {
        if (!r.values.empty() || v) return false;
      } else {
        return false;
      }
    }
    return true;
  }
};

Selector make_selector(Labels labels, vector<Req> exprs) {
  Selector s;
  std::sort(labels.begin(), labels.end());
  // matchLabels is a map: one entry per key (the last wins, as a dict's update)
  Labels uniq;
  for (auto& kv : labels) {
    if (!uniq.empty() && uniq.back().first == kv.first) uniq.back().second = kv.second;
    else uniq.push_back(kv);
  }
  s.labels = std::move(uniq);
  for (auto& r : exprs) std::sort(r.values.begin(), r.values.end());
  std::sort(exprs.begin(), exprs.end(), [](const Req& a, const Req& b) {
    if (a.key != b.key) return a.key < b.key;
    if (a.op != b.op) return a.op < b.op;
    return a.values < b.values;
  });
  s.exprs = std::move(exprs);
  string k;
  for (const auto& kv : s.labels) k += kv.first + '\x1f' + kv.second + '\x1e';
  k += '\x1d';
  for (const auto& r : s.exprs) {
    k += r.key + '\x1f' + r.op;
    for (const auto& v : r.values) k += '\x1f' + v;
    k += '\x1e';
  }
  s.key = std::move(k);
  return s;
}

// topology.py _validate_selector
void validate_selector(const Selector& s) {
  for (const auto& r : s.exprs) {
    if ((r.op == "In" || r.op == "NotIn") && r.values.empty())
      fail("selector requirement " + r.key + " " + r.op + " needs values");
    if ((r.op == "Exists" || r.op == "DoesNotExist") && !r.values.empty())
      fail("selector requirement " + r.key + " " + r.op + " must not have values");
    if (r.op != "In" && r.op != "NotIn" && r.op != "Exists" && r.op != "DoesNotExist")
      fail("selector operator " + r.op + " not supported");
  }
}

struct PodTerm {                // PodAffinityTerm (+ weight)
  string topology_key;
  std::shared_ptr<Selector> selector;      // null: nil
  vector<string> namespaces;
  std::shared_ptr<Selector> ns_selector;   // null: nil
  int32_t weight = 0;
  string ckey;                  // the term's pool content (memo key of Topo::term_matcher)
};

struct Spread {                 // TopologySpreadConstraint
  int32_t max_skew = 1;
  string topology_key, when;
  std::shared_ptr<Selector> selector;
  bool naff_set = false, ntaint_set = false;
  string naff, ntaint;
};

struct HostPort {
  string ip, proto;
  int32_t port;
  bool operator==(const HostPort& o) const { return port == o.port && ip == o.ip && proto == o.proto; }
};

struct Container {
  Labels requests;
  vector<HostPort> ports;       // hostPort > 0 only
  string image;
};

struct Toleration {
  string key, op, value, effect;
};

struct Taint {
  string key, value, effect;
};

// k8s.io/api core/v1 Toleration.ToleratesTaint (ksim/model.py Toleration.tolerates)
bool tolerates(const Toleration& t, const Taint& x) {
  if (!t.effect.empty() && t.effect != x.effect) return false;
  if (!t.key.empty() && t.key != x.key) return false;
  if (t.op.empty() || t.op == "Equal") return t.value == x.value;
  return t.op == "Exists";
}

struct ReqMemo {                // a pod's resource sums (pod_requests, pod_nonzero_requests)
  vector<std::pair<string, int64_t>> requests;
  std::pair<int64_t, int64_t> nonzero;
};

struct Pod {
  string name, ns;
  Labels labels, annotations, overhead, node_selector;
  vector<Container> containers, init_containers;
  bool has_required = false;
  vector<SelTerm> required;
  vector<std::pair<int32_t, SelTerm>> preferred;
  vector<Toleration> tolerations;
  vector<Spread> spread;
  vector<PodTerm> aff_req, aff_pref, anti_req, anti_pref;
  string node_name;
  bool has_owner = false;
  string owner_api, owner_kind, owner_name;
  int32_t volumes = KSIM_K8S_VOLUMES_NONE;
  vector<vector<SelTerm>> vb, vz;
  int32_t vb_bound = 0;
  int sig = -1;                 // (namespace, labels) signature id (Topo::sig_of)
  string sig_key, req_key;      // pool content of (namespace, labels) and of the resource lists
  const ReqMemo* req = nullptr; // its resource sums (read_pod)
};

struct Node {
  string name;
  bool unschedulable = false;
  Labels labels, alloc, annotations;
  vector<Taint> taints;
  vector<std::pair<vector<string>, int64_t>> images;
};

struct Service {
  string ns;
  bool has_selector = false;
  Labels selector;
};

struct Controller {
  string kind, ns, name;
  bool rc_set = false;
  Labels rc_selector;
  std::shared_ptr<Selector> selector;      // ReplicaSet / StatefulSet (null: nil)
};

// ---- reading the pool ---------------------------------------------------------------
// raw bytes of pool ids: memo keys (pool string ids are unique per string)
inline void put(string& k, int32_t x) { k.append(reinterpret_cast<const char*>(&x), sizeof x); }

struct Reader {
  const PoolView& v;
  // selectors by pool content: pods that repeat a selector share its canonical form
  mutable std::unordered_map<string, std::shared_ptr<Selector>> sel_cache;

  void put_kv(string& k, int32_t first, int32_t count) const {
    const ksim_k8s_kv* x = v.at(v.p.kv, v.p.n_kv, first, count, "kv");
    put(k, count);
    for (int32_t i = 0; i < count; i++) {
      v.str(x[i].key);
      v.str(x[i].value);
      put(k, x[i].key);
      put(k, x[i].value);
    }
  }
  void put_reqs(string& k, int32_t first, int32_t count) const {
    const ksim_k8s_requirement* x = v.at(v.p.reqs, v.p.n_reqs, first, count, "reqs");
    put(k, count);
    for (int32_t i = 0; i < count; i++) {
      put(k, x[i].key);
      put(k, x[i].op);
      put(k, x[i].values_count);
      const int32_t* vals = v.at(v.p.str_list, v.p.n_str_list, x[i].values_first, x[i].values_count, "str_list");
      for (int32_t j = 0; j < x[i].values_count; j++) put(k, vals[j]);
    }
  }
  string selector_key(int32_t i) const {
    string k;
    if (i < 0) {
      put(k, -1);
      return k;
    }
    const ksim_k8s_label_selector& s = v.one(v.p.selectors, v.p.n_selectors, i, "selectors");
    put_kv(k, s.labels_first, s.labels_count);
    put_reqs(k, s.exprs_first, s.exprs_count);
    return k;
  }

  Req req(const ksim_k8s_requirement& r) const {
    return Req{string(v.str(r.key)), string(v.str(r.op)), v.strs(r.values_first, r.values_count)};
  }
  vector<Req> reqs(int32_t first, int32_t count) const {
    vector<Req> out;
    const ksim_k8s_requirement* x = v.at(v.p.reqs, v.p.n_reqs, first, count, "reqs");
    for (int32_t i = 0; i < count; i++) out.push_back(req(x[i]));
    return out;
  }
  SelTerm term(int32_t i) const {
    const ksim_k8s_selector_term& t = v.one(v.p.terms, v.p.n_terms, i, "terms");
    return SelTerm{reqs(t.exprs_first, t.exprs_count), reqs(t.fields_first, t.fields_count)};
  }
  vector<SelTerm> terms(int32_t first, int32_t count) const {
    vector<SelTerm> out;
    v.at(v.p.terms, v.p.n_terms, first, count, "terms");
    for (int32_t i = 0; i < count; i++) out.push_back(term(first + i));
    return out;
  }
  std::shared_ptr<Selector> selector(int32_t i) const {
    if (i < 0) return nullptr;
    string key = selector_key(i);
    auto it = sel_cache.find(key);
    if (it != sel_cache.end()) return it->second;
    const ksim_k8s_label_selector& s = v.one(v.p.selectors, v.p.n_selectors, i, "selectors");
    auto sel = std::make_shared<Selector>(make_selector(v.kv(s.labels_first, s.labels_count),
                                                        reqs(s.exprs_first, s.exprs_count)));
    sel_cache.emplace(std::move(key), sel);
    return sel;
  }
  vector<PodTerm> pod_terms(int32_t first, int32_t count) const {
    vector<PodTerm> out;
    const ksim_k8s_pod_term* x = v.at(v.p.pod_terms, v.p.n_pod_terms, first, count, "pod_terms");
    for (int32_t i = 0; i < count; i++) {
      PodTerm t;
      t.topology_key = string(v.str(x[i].topology_key));
      t.selector = selector(x[i].selector);
      t.namespaces = v.strs(x[i].ns_first, x[i].ns_count);
      t.ns_selector = selector(x[i].ns_selector);
      t.weight = x[i].weight;
      put(t.ckey, x[i].topology_key);
      t.ckey += selector_key(x[i].selector);
      put(t.ckey, x[i].ns_count);
      const int32_t* ns = v.at(v.p.str_list, v.p.n_str_list, x[i].ns_first, x[i].ns_count, "str_list");
      for (int32_t j = 0; j < x[i].ns_count; j++) put(t.ckey, ns[j]);
      out.push_back(std::move(t));
    }
    return out;
  }
  Spread spread(const ksim_k8s_spread& c) const {
    Spread s;
    s.max_skew = c.max_skew;
    s.topology_key = string(v.str(c.topology_key));
    s.when = string(v.str(c.when_unsatisfiable));
    s.selector = selector(c.selector);
    if (c.node_affinity_policy >= 0) {
      s.naff_set = true;
      s.naff = string(v.str(c.node_affinity_policy));
    }
    if (c.node_taints_policy >= 0) {
      s.ntaint_set = true;
      s.ntaint = string(v.str(c.node_taints_policy));
    }
    return s;
  }
  vector<Spread> spreads(int32_t first, int32_t count) const {
    vector<Spread> out;
    const ksim_k8s_spread* x = v.at(v.p.spread, v.p.n_spread, first, count, "spread");
    for (int32_t i = 0; i < count; i++) out.push_back(spread(x[i]));
    return out;
  }
  vector<Container> containers(int32_t first, int32_t count, bool requests = true, bool image = true) const {
    vector<Container> out;
    const ksim_k8s_container* x = v.at(v.p.containers, v.p.n_containers, first, count, "containers");
    for (int32_t i = 0; i < count; i++) {
      Container c;
      if (requests) c.requests = v.kv(x[i].requests_first, x[i].requests_count);
      const ksim_k8s_port* pt = v.at(v.p.ports, v.p.n_ports, x[i].ports_first, x[i].ports_count, "ports");
      for (int32_t k = 0; k < x[i].ports_count; k++)
        if (pt[k].host_port > 0) {    // topology.py pod_host_ports: "" -> 0.0.0.0 / TCP
          string ip(v.str(pt[k].host_ip)), proto(v.str(pt[k].protocol));
          c.ports.push_back(HostPort{ip.empty() ? kBindAll : ip, proto.empty() ? "TCP" : proto, pt[k].host_port});
        }
      if (image) c.image = string(v.str(x[i].image));
      out.push_back(std::move(c));
    }
    return out;
  }
  vector<vector<SelTerm>> groups(int32_t first, int32_t count) const {
    vector<vector<SelTerm>> out;
    const ksim_k8s_volume_group* g = v.at(v.p.volume_groups, v.p.n_volume_groups, first, count, "volume_groups");
    for (int32_t i = 0; i < count; i++) out.push_back(terms(g[i].terms_first, g[i].terms_count));
    return out;
  }
  Node node(const ksim_k8s_node& x) const {
    Node n;
    n.name = string(v.str(x.name));
    n.unschedulable = x.unschedulable != 0;
    n.labels = v.kv(x.labels_first, x.labels_count);
    n.alloc = v.kv(x.alloc_first, x.alloc_count);
    n.annotations = v.kv(x.annotations_first, x.annotations_count);
    const ksim_k8s_taint* t = v.at(v.p.taints, v.p.n_taints, x.taints_first, x.taints_count, "taints");
    for (int32_t i = 0; i < x.taints_count; i++)
      n.taints.push_back(Taint{string(v.str(t[i].key)), string(v.str(t[i].value)), string(v.str(t[i].effect))});
    const ksim_k8s_image* im = v.at(v.p.images, v.p.n_images, x.images_first, x.images_count, "images");
    for (int32_t i = 0; i < x.images_count; i++)
      n.images.emplace_back(v.strs(im[i].names_first, im[i].names_count), im[i].size_bytes);
    return n;
  }
};

// ---- quantities of objects ------------------------------------------------------------
struct Quantities {
  std::unordered_map<string, int64_t> value, milli;   // memoized, as model.py's lru caches
  int64_t get(const string& q, bool is_milli) {
    auto& m = is_milli ? milli : value;
    auto it = m.find(q);
    if (it != m.end()) return it->second;
    const int64_t x = quantity_ceil(q, is_milli ? 3 : 0);
    m.emplace(q, x);
    return x;
  }
  // encode.py _res
  int64_t res(const Labels& requests, const string& name) {
    const string* q = lookup(requests, name);
    if (!q) return 0;
    return get(*q, name == "cpu");
  }
};

// encode.py pod_requests: sum containers, max init containers, + overhead ("pods" excluded)
vector<std::pair<string, int64_t>> pod_requests(Quantities& qs, const Pod& p) {
  vector<string> names;
  auto note = [&](const Labels& m) {
    for (const auto& kv : m)
      if (std::find(names.begin(), names.end(), kv.first) == names.end()) names.push_back(kv.first);
  };
  for (const auto& c : p.containers) note(c.requests);
  for (const auto& c : p.init_containers) note(c.requests);
  note(p.overhead);
  vector<std::pair<string, int64_t>> out;
  for (const auto& n : names) {
    if (n == "pods") continue;
    int64_t v = 0;
    for (const auto& c : p.containers) v += qs.res(c.requests, n);
    for (const auto& c : p.init_containers) v = std::max(v, qs.res(c.requests, n));
    v += qs.res(p.overhead, n);
    out.emplace_back(n, v);
  }
  return out;
}

int64_t req_of(const vector<std::pair<string, int64_t>>& r, const char* name) {
  for (const auto& x : r)
    if (x.first == name) return x.second;
  return 0;
}

// encode.py pod_nonzero_requests (schedutil.GetNonzeroRequests per container)
std::pair<int64_t, int64_t> pod_nonzero_requests(Quantities& qs, const Pod& p) {
  auto nz = [&](const Labels& r) {
    const int64_t cpu = lookup(r, "cpu") ? qs.res(r, "cpu") : kDefaultMilliCPU;
    const int64_t mem = lookup(r, "memory") ? qs.res(r, "memory") : kDefaultMemory;
    return std::make_pair(cpu, mem);
  };
  int64_t cpu = 0, mem = 0;
  for (const auto& c : p.containers) {
    const auto x = nz(c.requests);
    cpu += x.first;
    mem += x.second;
  }
  for (const auto& c : p.init_containers) {
    const auto x = nz(c.requests);
    cpu = std::max(cpu, x.first);
    mem = std::max(mem, x.second);
  }
  if (lookup(p.overhead, "cpu")) cpu += qs.res(p.overhead, "cpu");
  if (lookup(p.overhead, "memory")) mem += qs.res(p.overhead, "memory");
  return {cpu, mem};
}

// ---- NetworkBandwidth (ksim/netbw.py) ----------------------------------------------------
struct NbArgs {
  string node_limit = "node.kubernetes.io/network-limit";
  string egress = "kubernetes.io/egress-request";
  string ingress = "kubernetes.io/ingress-request";
};

int64_t nb_pod_allocated(const Labels& ann, const NbArgs& a) {
  int64_t total = 0;
  for (const string* key : {&a.ingress, &a.egress}) {
    const string* s = lookup(ann, *key);
    int64_t q;
    if (s && netbw_milli(*s, q)) total += q;
  }
  return total;
}

// ---- count classes (ksim/topology.py TopologyIndex) -----------------------------------
struct Matcher {                // topology.py Matcher
  vector<string> namespaces;    // sorted, unique
  bool all = false;
  int sel = -1;                 // Topo::selectors index, -1: nil selector
  string key;
};

enum ClassKind { kSel, kCarry, kPort, kImage };

struct Cls {
  ClassKind kind;
  int matcher = -1;             // kSel (single), kCarry
  vector<int> all;              // kSel ("all", (m1, m2, ...)): podMatchesAllAffinityTerms
  bool is_all = false;
  string carry_kind, tk;        // kCarry
  string ip, proto;             // kPort
  int32_t port = 0;
  vector<string> names;         // kImage
  vector<int32_t> counts;
};

const char* const kReqAnti = "req_anti";
const char* const kReqAff = "req_aff";
const char* const kPrefAff = "pref_aff";
const char* const kPrefAnti = "pref_anti";

struct Use {
  int32_t cls, arg;
  uint16_t col;
  uint8_t kind, flags;
};

struct Encoder;

struct Topo {
  int n = 0;
  vector<std::pair<string, Labels>> ns_labels;   // a dict: insertion order
  std::unordered_map<string, size_t> ns_index;
  vector<Selector> selectors;
  std::unordered_map<string, int> selector_ids;
  vector<Matcher> matchers;
  std::unordered_map<string, int> matcher_ids;
  vector<Cls> classes;
  std::unordered_map<string, int> class_ids;
  vector<int> sel_ids, carry_ids, port_ids, image_ids;
  struct ImageState {
    int64_t size;
    vector<uint8_t> mask;
  };
  std::unordered_map<string, ImageState> images;
  vector<std::pair<int, HostPort>> bound_ports;
  // signatures: (namespace, sorted labels)
  vector<std::pair<string, Labels>> sigs;
  std::unordered_map<string, int> sig_ids;
  std::unordered_map<int, vector<int32_t>> bound_sigs;   // signature -> node positions of bound pods
  vector<int> bound_sig_order;
  std::unordered_map<uint64_t, bool> match_cache;       // (signature, matcher) -> match
  std::unordered_map<uint64_t, vector<Use>> carry_uses; // (signature, carried classes) -> uses
  // per-call memos keyed by pool content (cleared by begin_call: pool ids are per pool)
  std::unordered_map<string, int> term_memo, sig_memo;
  std::unordered_map<int, int> sel_memo;                // matcher -> its selector class
  std::unordered_map<string, int> tk_ids;               // topology keys of carried classes
  std::unordered_map<uint64_t, int> carry_memo;         // (kind, matcher, topology key) -> class

  void begin_call() {
    term_memo.clear();
    sig_memo.clear();
  }

  int sig_of_pod(const string& key, const string& ns, const Labels& labels) {
    auto it = sig_memo.find(key);
    if (it != sig_memo.end()) return it->second;
    const int id = sig_of(ns, labels);
    sig_memo.emplace(key, id);
    return id;
  }

  void note_namespace(const string& ns) {
    if (!ns_index.count(ns)) {
      ns_index[ns] = ns_labels.size();
      ns_labels.emplace_back(ns, Labels{});
    }
  }

  int sig_of(const string& ns, const Labels& labels) {
    Labels s = labels;
    std::sort(s.begin(), s.end());
    string k = ns + '\x1d';
    for (const auto& kv : s) k += kv.first + '\x1f' + kv.second + '\x1e';
    auto it = sig_ids.find(k);
    if (it != sig_ids.end()) return it->second;
    const int id = (int)sigs.size();
    sigs.emplace_back(ns, std::move(s));
    sig_ids.emplace(std::move(k), id);
    return id;
  }

  // _sel_key: validated, interned by its canonical key (the first object wins)
  int sel_key(const std::shared_ptr<Selector>& s) {
    if (!s) return -1;
    validate_selector(*s);
    auto it = selector_ids.find(s->key);
    if (it != selector_ids.end()) return it->second;
    const int id = (int)selectors.size();
    selectors.push_back(*s);
    selector_ids.emplace(s->key, id);
    return id;
  }

  int intern_matcher(vector<string> names, bool all, int sel) {
    std::sort(names.begin(), names.end());
    names.erase(std::unique(names.begin(), names.end()), names.end());
    string k = all ? "A" : "N";
    for (const auto& x : names) k += x + '\x1f';
    k += '\x1d';
    k += sel < 0 ? string("\x01nil") : selectors[sel].key;
    auto it = matcher_ids.find(k);
    if (it != matcher_ids.end()) return it->second;
    const int id = (int)matchers.size();
    matchers.push_back(Matcher{std::move(names), all, sel, k});
    matcher_ids.emplace(std::move(k), id);
    return id;
  }

  // term_matcher: newAffinityTerm + getNamespacesFromPodAffinityTerm, a
  // non-empty namespaceSelector resolved over the known namespaces
  int term_matcher(const string& owner_ns, const PodTerm& t) {
    if (!t.ns_selector) {                  // a pure function of the term and its owner's namespace
      string k = owner_ns;
      k += '\0';
      k += t.ckey;
      auto it = term_memo.find(k);
      if (it != term_memo.end()) return it->second;
      const int m = term_matcher_impl(owner_ns, t);
      term_memo.emplace(std::move(k), m);
      return m;
    }
    return term_matcher_impl(owner_ns, t);
  }

  int term_matcher_impl(const string& owner_ns, const PodTerm& t) {
    vector<string> names = t.namespaces;
    bool all = false;
    if (t.namespaces.empty() && !t.ns_selector) names.push_back(owner_ns);
    if (t.ns_selector) {
      validate_selector(*t.ns_selector);
      if (t.ns_selector->empty()) {
        all = true;
      } else {
        for (const auto& x : ns_labels)
          if (t.ns_selector->matches(x.second)) names.push_back(x.first);
      }
    }
    return intern_matcher(std::move(names), all, sel_key(t.selector));
  }

  bool matches(int m, const string& ns, const Labels& labels) const {
    const Matcher& x = matchers[m];
    if (!x.all && !std::binary_search(x.namespaces.begin(), x.namespaces.end(), ns)) return false;
    return x.sel >= 0 && selectors[x.sel].matches(labels);
  }

  bool sig_matches_one(int m, int sig) {
    const uint64_t k = ((uint64_t)(uint32_t)sig << 32) | (uint32_t)m;
    auto it = match_cache.find(k);
    if (it != match_cache.end()) return it->second;
    const bool v = matches(m, sigs[sig].first, sigs[sig].second);
    match_cache.emplace(k, v);
    return v;
  }

  bool class_matches(const Cls& c, int sig) {
    if (c.is_all) {
      for (int m : c.all)
        if (!sig_matches_one(m, sig)) return false;
      return true;
    }
    return sig_matches_one(c.matcher, sig);
  }

  int new_class(const string& key, Cls c) {
    const int cid = (int)classes.size();
    if (cid >= KSIM_MAX_CLASSES) fail("too many count classes");
    class_ids.emplace(key, cid);
    switch (c.kind) {
      case kSel: sel_ids.push_back(cid); break;
      case kCarry: carry_ids.push_back(cid); break;
      case kPort: port_ids.push_back(cid); break;
      case kImage: image_ids.push_back(cid); break;
    }
    classes.push_back(std::move(c));
    return cid;
  }

  // ---- NodePorts: HostPortInfo as count classes ----
  int port_class(const string& ip, const string& proto, int32_t port) {
    const string key = "P" + ip + '\x1f' + proto + '\x1f' + std::to_string(port);
    auto it = class_ids.find(key);
    if (it != class_ids.end()) return it->second;
    Cls c;
    c.kind = kPort;
    c.ip = ip;
    c.proto = proto;
    c.port = port;
    c.counts.assign(n, 0);
    for (const auto& bp : bound_ports)
      if (bp.second.proto == proto && bp.second.port == port && (ip == "*" || ip == bp.second.ip))
        c.counts[bp.first] += 1;
    return new_class(key, std::move(c));
  }

  vector<int> port_check_classes(const Pod& p) {
    vector<int> out;
    for (const auto& c : p.containers)
      for (const auto& hp : c.ports) {
        vector<std::pair<string, string>> keys;
        if (hp.ip == kBindAll) keys = {{"*", hp.proto}};
        else keys = {{kBindAll, hp.proto}, {hp.ip, hp.proto}};
        for (const auto& k : keys) {
          const int cid = port_class(k.first, k.second, hp.port);
          if (std::find(out.begin(), out.end(), cid) == out.end()) out.push_back(cid);
        }
      }
    return out;
  }

  // port_adds: UsedPorts.Add of each host port on the registered classes
  vector<std::pair<int, int32_t>> port_adds(const Pod& p) const {
    vector<std::pair<int, int32_t>> out;   // a dict: insertion order
    auto add = [&](int cid) {
      for (auto& x : out)
        if (x.first == cid) {
          x.second += 1;
          return;
        }
      out.emplace_back(cid, 1);
    };
    for (const auto& c : p.containers)
      for (const auto& hp : c.ports)
        for (const string& ip : {string("*"), hp.ip}) {
          auto it = class_ids.find("P" + ip + '\x1f' + hp.proto + '\x1f' + std::to_string(hp.port));
          if (it != class_ids.end()) add(it->second);
        }
    return out;
  }

  // ---- ImageLocality ----
  void set_images(const vector<Node>& nodes_in_add_order, const std::unordered_map<string, int32_t>& pos_of) {
    for (const auto& nd : nodes_in_add_order)
      for (const auto& im : nd.images)
        for (const auto& name : im.first) {
          auto it = images.find(name);
          if (it == images.end()) it = images.emplace(name, ImageState{im.second, vector<uint8_t>(n, 0)}).first;
          it->second.mask[pos_of.at(nd.name)] = 1;
        }
  }

  static string normalized_image_name(const string& name) {
    const auto c = name.rfind(':'), s = name.rfind('/');
    const long ci = c == string::npos ? -1 : (long)c, si = s == string::npos ? -1 : (long)s;
    return ci <= si ? name + ":latest" : name;
  }

  int image_class_of(const vector<string>& names) {
    string key = "I";
    for (const auto& x : names) key += x + '\x1f';
    auto it = class_ids.find(key);
    if (it != class_ids.end()) return it->second;
    Cls c;
    c.kind = kImage;
    c.names = names;
    c.counts = image_counts(names);
    return new_class(key, std::move(c));
  }

  // ImageLocality's per-node score of a container image list (scaledImageScore
  // over the snapshot's image states)
  vector<int32_t> image_counts(const vector<string>& names) const {
    vector<int64_t> total(n, 0);
    for (const auto& nm : names) {
      auto st = images.find(nm);
      if (st == images.end()) continue;
      int64_t cnt = 0;
      for (uint8_t b : st->second.mask) cnt += b;
      const double spread = (double)cnt / (double)n;            // float64(NumNodes) / float64(totalNumNodes)
      const int64_t add = (int64_t)((double)st->second.size * spread);
      for (int i = 0; i < n; i++)
        if (st->second.mask[i]) total[i] += add;
    }
    const int64_t max_t = kImageMaxContainer * (int64_t)names.size();
    vector<int32_t> counts(n);
    for (int i = 0; i < n; i++) {
      const int64_t s = std::min(std::max(total[i], kImageMin), max_t);
      counts[i] = (int32_t)((100 * (s - kImageMin)) / (max_t - kImageMin));
    }
    return counts;
  }

  int image_class(const Pod& p) {
    vector<string> names;
    bool any = false;
    for (const auto& c : p.containers) {
      names.push_back(normalized_image_name(c.image));
      any = any || images.count(names.back());
    }
    if (!any) return -1;
    return image_class_of(names);
  }

  // ---- selector / carried classes ----
  static string sel_class_key(int m) { return "S" + std::to_string(m); }
  static string all_class_key(const vector<int>& ms) {
    string k = "A";
    for (int m : ms) k += std::to_string(m) + ',';
    return k;
  }

  int selector_class_impl(const string& key, Cls c) {
    auto it = class_ids.find(key);
    if (it != class_ids.end()) return it->second;
    c.kind = kSel;
    c.counts.assign(n, 0);
    for (int sig : bound_sig_order)
      if (class_matches(c, sig))
        for (int32_t pos : bound_sigs[sig]) c.counts[pos] += 1;
    return new_class(key, std::move(c));
  }
  int selector_class(int m) {
    auto it = sel_memo.find(m);
    if (it != sel_memo.end()) return it->second;
    Cls c;
    c.matcher = m;
    const int cid = selector_class_impl(sel_class_key(m), std::move(c));
    sel_memo.emplace(m, cid);
    return cid;
  }
  int selector_class_all(const vector<int>& ms) {
    Cls c;
    c.is_all = true;
    c.all = ms;
    return selector_class_impl(all_class_key(ms), std::move(c));
  }

  int carried_class(const string& kind, int m, const string& tk) {
    auto ti = tk_ids.find(tk);
    if (ti == tk_ids.end()) ti = tk_ids.emplace(tk, (int)tk_ids.size()).first;
    const uint64_t kind_i = kind == kReqAnti ? 0 : kind == kReqAff ? 1 : kind == kPrefAff ? 2 : 3;
    const uint64_t mk = (kind_i << 62) | ((uint64_t)(uint32_t)m << 24) | (uint64_t)ti->second;
    auto mi = carry_memo.find(mk);
    if (mi != carry_memo.end()) return mi->second;
    const string key = "C" + kind + '\x1f' + std::to_string(m) + '\x1f' + tk;
    auto it = class_ids.find(key);
    if (it != class_ids.end()) {
      carry_memo.emplace(mk, it->second);
      return it->second;
    }
    Cls c;
    c.kind = kCarry;
    c.matcher = m;
    c.carry_kind = kind;
    c.tk = tk;
    c.counts.assign(n, 0);
    const int cid = new_class(key, std::move(c));
    carry_memo.emplace(mk, cid);
    return cid;
  }

  // carried_terms: (class, multiplicity) of the terms the pod carries once bound
  vector<std::pair<int, int32_t>> carried_terms(const Pod& p) {
    vector<std::pair<int, int32_t>> out;
    auto add = [&](int cid, int32_t k) {
      for (auto& x : out)
        if (x.first == cid) {
          x.second += k;
          return;
        }
      out.emplace_back(cid, k);
    };
    for (const auto& t : p.anti_req) add(carried_class(kReqAnti, term_matcher(p.ns, t), t.topology_key), 1);
    for (const auto& t : p.aff_req) add(carried_class(kReqAff, term_matcher(p.ns, t), t.topology_key), 1);
    for (const auto& w : p.aff_pref) add(carried_class(kPrefAff, term_matcher(p.ns, w), w.topology_key), w.weight);
    for (const auto& w : p.anti_pref) add(carried_class(kPrefAnti, term_matcher(p.ns, w), w.topology_key), w.weight);
    std::sort(out.begin(), out.end());
    return out;
  }

  // add_bound: an existing pod bound at node position pos (NodeInfo.AddPod)
  void add_bound(const Pod& p, int32_t pos, const vector<std::pair<int, int32_t>>& carried) {
    note_namespace(p.ns);
    for (const auto& c : carried) classes[c.first].counts[pos] += c.second;
    for (int cid : sel_ids)
      if (class_matches(classes[cid], p.sig)) classes[cid].counts[pos] += 1;
    for (const auto& c : port_adds(p)) classes[c.first].counts[pos] += c.second;
    vector<HostPort> ports;
    for (const auto& c : p.containers)
      for (const auto& hp : c.ports) ports.push_back(hp);
    add_member(p.sig, ports, pos);
  }

  // The snapshot's membership (ABI 11 deltas): which signatures and host
  // ports sit on which node.  A class registered later counts its bound pods
  // from it; the class rows of registered classes stay the snapshot's (the
  // device adds the binds made since, ksim_upsert_nodes' replay).
  void add_member(int sig, const vector<HostPort>& ports, int32_t pos) {
    for (const auto& hp : ports) bound_ports.emplace_back(pos, hp);
    auto it = bound_sigs.find(sig);
    if (it == bound_sigs.end()) {
      bound_sig_order.push_back(sig);
      bound_sigs[sig].push_back(pos);
    } else {
      it->second.push_back(pos);
    }
  }

  void drop_member(int sig, const vector<HostPort>& ports, int32_t pos) {
    for (const auto& hp : ports)
      for (size_t i = 0; i < bound_ports.size(); i++)
        if (bound_ports[i].first == pos && bound_ports[i].second == hp) {
          bound_ports.erase(bound_ports.begin() + (long)i);
          break;
        }
    auto it = bound_sigs.find(sig);
    if (it == bound_sigs.end()) fail("encoder membership: signature not bound");
    auto at = std::find(it->second.begin(), it->second.end(), pos);
    if (at == it->second.end()) fail("encoder membership: pod not on its node");
    it->second.erase(at);
  }

  // node positions moved (a node delta): new_of[old] = new position, -1 = the
  // node left the snapshot with its pods
  void remap_members(const vector<int32_t>& new_of) {
    vector<std::pair<int, HostPort>> ports;
    for (auto& bp : bound_ports)
      if (new_of[bp.first] >= 0) ports.emplace_back(new_of[bp.first], std::move(bp.second));
    bound_ports = std::move(ports);
    for (auto& s : bound_sigs) {
      vector<int32_t> v;
      for (int32_t q : s.second)
        if (new_of[q] >= 0) v.push_back(new_of[q]);
      s.second = std::move(v);
    }
  }

  // adds: the pod's carried terms plus every selector class it matches, plus ports
  vector<std::pair<int, int32_t>> adds(const Pod& p) {
    vector<std::pair<int, int32_t>> out = carried_terms(p);
    auto add = [&](int cid, int32_t k) {
      for (auto& x : out)
        if (x.first == cid) {
          x.second += k;
          return;
        }
      out.emplace_back(cid, k);
    };
    for (int cid : sig_sel_classes(p.sig)) add(cid, 1);
    for (const auto& c : port_adds(p)) add(c.first, c.second);
    std::sort(out.begin(), out.end());
    return out;
  }

  // the selector classes a signature matches (topology.py _sig_sel), valid
  // while no selector class is added
  std::unordered_map<int, std::pair<size_t, vector<int>>> sig_sel;
  const vector<int>& sig_sel_classes(int sig) {
    auto& e = sig_sel[sig];
    if (e.first != sel_ids.size() || (e.second.empty() && e.first == 0)) {
      e.second.clear();
      for (int cid : sel_ids)
        if (class_matches(classes[cid], sig)) e.second.push_back(cid);
      e.first = sel_ids.size();
    }
    return e.second;
  }
};

// ---- the encoder --------------------------------------------------------------------------
// a pod bound in the snapshot (the scheduler cache's view): its node and
// what the count classes registered after its bind read of it
struct Member {
  int32_t pos = -1;
  int sig = -1;
  vector<HostPort> ports;
};

struct Cluster {
  int32_t n = 0, n_scalar = 0;
  vector<int64_t> alloc_cpu, alloc_mem, alloc_eph, alloc_scalar, req_cpu, req_mem, req_eph, req_scalar, nz_cpu,
      nz_mem, nb_limit, nb_alloc;
  vector<int32_t> alloc_pods, num_pods, order;
  vector<uint32_t> flags;
  vector<uint16_t> taints;              // [8][N]
  vector<uint32_t> labels;              // [L][N]
  vector<uint8_t> taint_effect;
  vector<int32_t> label_col_offset;
  vector<int64_t> label_num;
  vector<uint8_t> label_num_ok;
  vector<double> topo_log;
  vector<int32_t> class_count;          // [C][N], materialized
  vector<string> node_names, scalar_names, label_keys;
  vector<vector<string>> label_values;
  vector<std::unordered_map<string, int32_t>> value_index;   // first index of a value in its column
  vector<Taint> taint_vocab;            // [0] unused
  vector<Labels> node_labels;
  std::unordered_map<string, int32_t> pos_of;
  NbArgs nb;
};

}  // namespace

struct ksim_encoder {
  Cluster c;
  Topo topo;
  Quantities qs;
  std::unordered_map<string, ReqMemo> req_memo;   // per call: resource lists by pool content
  bool has_cluster = false;
  // snapshot deltas (ABI 11): the nodes in informer add order, the bound pods
  // by namespace / name, the current pod set's membership records (bind), the
  // last node delta's old positions
  vector<Node> nodes;
  vector<string> extra_scalar;
  std::unordered_map<string, Member> members;
  std::unordered_set<string> dup_keys;      // bound twice in one snapshot: not unbindable
  vector<std::pair<string, Member>> queue_members;
  vector<int32_t> old_pos;
  bool in_place = false;                    // the last node delta only updated rows (ksim_encoder_changed_rows)
  vector<int32_t> changed;
  // the pod set
  vector<ksim_pod> pods;
  vector<ksim_label_expr> exprs;
  vector<ksim_term> terms;
  vector<ksim_topo_use> uses;
  vector<ksim_class_add> adds;
  vector<int32_t> nn;
  string err;
};

namespace {

// a pod's resource sums (pod_requests, pod_nonzero_requests), memoized by the
// pool content of its resource lists
const ReqMemo& requests_of(ksim_encoder*, const Pod& p) { return *p.req; }

// A pod of the pool.  Memoized by pool content: the (namespace, labels)
// signature (labels are read only for a new signature, or for a queue pod,
// whose labels the topology compile reads) and the resource sums.  A bound
// pod (bound = true) reads only what NodeInfo.AddPod and the count classes use.
Pod read_pod(const Reader& rd, const ksim_k8s_pod& x, Topo& t, std::unordered_map<string, ReqMemo>& rm,
             Quantities& qs, bool bound) {
  const PoolView& v = rd.v;
  Pod p;
  p.ns = string(v.str(x.namespace_));
  put(p.sig_key, x.namespace_);
  rd.put_kv(p.sig_key, x.labels_first, x.labels_count);
  auto si = t.sig_memo.find(p.sig_key);
  if (!bound || si == t.sig_memo.end()) p.labels = v.kv(x.labels_first, x.labels_count);
  p.sig = si != t.sig_memo.end() ? si->second : t.sig_of_pod(p.sig_key, p.ns, p.labels);
  const ksim_k8s_container* cs = v.at(v.p.containers, v.p.n_containers, x.containers_first, x.containers_count,
                                      "containers");
  const ksim_k8s_container* is = v.at(v.p.containers, v.p.n_containers, x.init_first, x.init_count, "containers");
  for (int32_t i = 0; i < x.containers_count; i++) rd.put_kv(p.req_key, cs[i].requests_first, cs[i].requests_count);
  put(p.req_key, -1);
  for (int32_t i = 0; i < x.init_count; i++) rd.put_kv(p.req_key, is[i].requests_first, is[i].requests_count);
  put(p.req_key, -1);
  rd.put_kv(p.req_key, x.overhead_first, x.overhead_count);
  auto ri = rm.find(p.req_key);
  const bool need_req = ri == rm.end();
  p.containers = rd.containers(x.containers_first, x.containers_count, need_req, !bound);
  if (need_req) {
    p.init_containers = rd.containers(x.init_first, x.init_count, true, false);
    p.overhead = v.kv(x.overhead_first, x.overhead_count);
    ReqMemo m{pod_requests(qs, p), pod_nonzero_requests(qs, p)};
    ri = rm.emplace(p.req_key, std::move(m)).first;
  }
  p.req = &ri->second;
  if (x.annotations_count) p.annotations = v.kv(x.annotations_first, x.annotations_count);
  if (bound) return p;                  // its terms: encode_nodes' first pass
  p.aff_req = rd.pod_terms(x.aff_req_first, x.aff_req_count);
  p.aff_pref = rd.pod_terms(x.aff_pref_first, x.aff_pref_count);
  p.anti_req = rd.pod_terms(x.anti_req_first, x.anti_req_count);
  p.anti_pref = rd.pod_terms(x.anti_pref_first, x.anti_pref_count);
  p.node_name = string(v.str(x.node_name));
  p.name = string(v.str(x.name));
  p.node_selector = v.kv(x.selector_first, x.selector_count);
  p.has_required = x.required_first >= 0;
  if (p.has_required) p.required = rd.terms(x.required_first, x.required_count);
  const ksim_k8s_preferred_term* pr =
      v.at(v.p.preferred, v.p.n_preferred, x.preferred_first, x.preferred_count, "preferred");
  for (int32_t i = 0; i < x.preferred_count; i++) p.preferred.emplace_back(pr[i].weight, rd.term(pr[i].term));
  const ksim_k8s_toleration* tl =
      v.at(v.p.tolerations, v.p.n_tolerations, x.tolerations_first, x.tolerations_count, "tolerations");
  for (int32_t i = 0; i < x.tolerations_count; i++)
    p.tolerations.push_back(Toleration{string(v.str(tl[i].key)), string(v.str(tl[i].op)), string(v.str(tl[i].value)),
                                       string(v.str(tl[i].effect))});
  p.spread = rd.spreads(x.spread_first, x.spread_count);
  if (x.owner_kind >= 0) {
    p.has_owner = true;
    p.owner_api = string(v.str(x.owner_api_version));
    p.owner_kind = string(v.str(x.owner_kind));
    p.owner_name = string(v.str(x.owner_name));
  }
  p.volumes = x.volumes;
  if (p.volumes == KSIM_K8S_VOLUMES_GROUPS) {
    p.vb = rd.groups(x.vb_first, x.vb_count);
    p.vb_bound = x.vb_bound;
    p.vz = rd.groups(x.vz_first, x.vz_count);
  } else if (p.volumes != KSIM_K8S_VOLUMES_NONE && p.volumes != KSIM_K8S_VOLUMES_REFUSE) {
    fail("pod " + p.name + ": unknown volumes mode");
  }
  return p;
}

// ---- label columns (encode.py EncodedCluster.label_col / value_id) -------------------------
int label_col(ksim_encoder* e, const string& key, bool force = false) {
  Cluster& c = e->c;
  for (size_t i = 0; i < c.label_keys.size(); i++)
    if (c.label_keys[i] == key) return (int)i;
  bool any = force;
  for (const auto& lb : c.node_labels) {
    if (any) break;
    if (lookup(lb, key)) any = true;
  }
  if (!any) return -1;
  if ((int)c.label_keys.size() >= KSIM_MAX_LABEL_COLS)
    fail("more than " + std::to_string(KSIM_MAX_LABEL_COLS) + " referenced label keys");
  vector<string> values{""};
  std::unordered_map<string, int32_t> index;
  const size_t base = c.labels.size();
  c.labels.resize(base + c.n, 0);
  for (int32_t pos = 0; pos < c.n; pos++) {
    const string* v = lookup(c.node_labels[pos], key);
    if (!v) continue;
    auto it = index.find(*v);
    int32_t vid;
    if (it == index.end()) {
      vid = (int32_t)values.size();
      index.emplace(*v, vid);
      values.push_back(*v);
    } else {
      vid = it->second;
    }
    c.labels[base + pos] = (uint32_t)vid;
  }
  c.label_col_offset.push_back((int32_t)c.label_num.size());
  for (const auto& v : values) {
    int64_t x = 0;
    const bool ok = !v.empty() && parse_int64(v, x);
    c.label_num.push_back(ok ? x : 0);
    c.label_num_ok.push_back(ok ? 1 : 0);
  }
  std::unordered_map<string, int32_t> first;
  for (size_t i = 0; i < values.size(); i++) first.emplace(values[i], (int32_t)i);
  c.value_index.push_back(std::move(first));
  c.label_keys.push_back(key);
  c.label_values.push_back(std::move(values));
  return (int)c.label_keys.size() - 1;
}

int32_t value_id(const ksim_encoder* e, int col, const string& value) {
  if (col < 0) return 0;
  const auto& m = e->c.value_index[col];
  auto it = m.find(value);
  return it == m.end() ? 0 : it->second;
}

uint16_t col_or_none(ksim_encoder* e, const string& key) {
  const int c = label_col(e, key);
  return c < 0 ? (uint16_t)KSIM_COL_NONE : (uint16_t)c;
}

// ---- encode_cluster ---------------------------------------------------------------------------
string zone_key(const Labels& l) {
  const string* z = lookup(l, kZone);
  if (!z) z = lookup(l, kZoneBeta);
  const string* r = lookup(l, kRegion);
  if (!r) r = lookup(l, kRegionBeta);
  const string zone = z ? *z : "", region = r ? *r : "";
  if (region.empty() && zone.empty()) return "";
  return region + string(":\0:", 3) + zone;
}

// node_tree.go nodeTree.list(): round-robin over zones (zone insertion order),
// insertion order inside each zone
vector<int32_t> node_tree_order(const vector<string>& zone_keys) {
  vector<string> zones;
  std::unordered_map<string, vector<int32_t>> tree;
  for (size_t i = 0; i < zone_keys.size(); i++) {
    auto it = tree.find(zone_keys[i]);
    if (it == tree.end()) {
      zones.push_back(zone_keys[i]);
      it = tree.emplace(zone_keys[i], vector<int32_t>{}).first;
    }
    it->second.push_back((int32_t)i);
  }
  vector<int32_t> out;
  out.reserve(zone_keys.size());
  for (size_t idx = 0; out.size() < zone_keys.size(); idx++)
    for (const auto& z : zones) {
      const auto& lst = tree[z];
      if (idx < lst.size()) out.push_back(lst[idx]);
    }
  return out;
}

uint8_t effect_id(const string& e) {
  if (e == "NoSchedule") return KSIM_EFFECT_NO_SCHEDULE;
  if (e == "PreferNoSchedule") return KSIM_EFFECT_PREFER_NO_SCHEDULE;
  if (e == "NoExecute") return KSIM_EFFECT_NO_EXECUTE;
  return KSIM_EFFECT_NONE;
}

// class_count [C][N] from the classes' rows.  A queue compile only appends
// classes (a pending pod's adds never change a count), so only the new rows
// are copied (from = the classes materialized before).
void materialize_classes(ksim_encoder* e, size_t from = 0) {
  Cluster& c = e->c;
  c.class_count.resize((size_t)e->topo.classes.size() * c.n);
  for (size_t k = from; k < e->topo.classes.size(); k++)
    std::copy(e->topo.classes[k].counts.begin(), e->topo.classes[k].counts.end(),
              c.class_count.begin() + k * (size_t)c.n);
}

// The node half of a snapshot (encode.py encode_cluster up to the bound pods):
// nodeTree order over `nodes` (informer add order), scalar columns (`prev`'s
// first when given), the taint vocabulary (`prev`'s ids first when
// keep_taints), the static columns, zeroed dynamic columns, names, labels,
// positions.  c.nb must be set.
void node_columns(Cluster& c, const vector<Node>& nodes, Quantities& qs, const Cluster* prev, bool keep_taints,
                  const vector<string>& extra_scalar) {
  vector<string> zk;
  zk.reserve(nodes.size());
  for (const auto& nd : nodes) zk.push_back(zone_key(nd.labels));
  c.order = node_tree_order(zk);
  const int32_t N = (int32_t)nodes.size();
  if (N > KSIM_MAX_NODES) fail("too many nodes");
  c.n = N;
  // scalar resources: every non-native allocatable name
  if (prev) c.scalar_names = prev->scalar_names;
  for (int32_t pos = 0; pos < N; pos++)
    for (const auto& kv : nodes[c.order[pos]].alloc)
      if (!is_native_resource(kv.first) &&
          std::find(c.scalar_names.begin(), c.scalar_names.end(), kv.first) == c.scalar_names.end())
        c.scalar_names.push_back(kv.first);
  for (const auto& s : extra_scalar)
    if (std::find(c.scalar_names.begin(), c.scalar_names.end(), s) == c.scalar_names.end()) c.scalar_names.push_back(s);
  if ((int)c.scalar_names.size() > KSIM_MAX_SCALAR) fail("too many scalar resources");
  const int32_t S = (int32_t)c.scalar_names.size();
  c.n_scalar = S;
  // taints
  std::unordered_map<string, int> tindex;
  if (keep_taints && prev && !prev->taint_vocab.empty()) {
    c.taint_vocab = prev->taint_vocab;
    for (size_t t = 1; t < c.taint_vocab.size(); t++) {
      const Taint& x = c.taint_vocab[t];
      tindex.emplace(x.key + '\x1f' + x.value + '\x1f' + x.effect, (int)t);
    }
  } else {
    c.taint_vocab.push_back(Taint{});
  }
  c.taints.assign((size_t)KSIM_MAX_NODE_TAINTS * N, 0);
  for (int32_t pos = 0; pos < N; pos++) {
    const Node& nd = nodes[c.order[pos]];
    if ((int)nd.taints.size() > KSIM_MAX_NODE_TAINTS)
      fail("node " + nd.name + ": more than " + std::to_string(KSIM_MAX_NODE_TAINTS) + " taints");
    for (size_t k = 0; k < nd.taints.size(); k++) {
      const Taint& t = nd.taints[k];
      const string key = t.key + '\x1f' + t.value + '\x1f' + t.effect;
      auto it = tindex.find(key);
      int tid;
      if (it == tindex.end()) {
        tid = (int)c.taint_vocab.size();
        c.taint_vocab.push_back(t);
        tindex.emplace(key, tid);
      } else {
        tid = it->second;
      }
      c.taints[k * N + pos] = (uint16_t)tid;
    }
  }
  if ((int)c.taint_vocab.size() > 64 * KSIM_TAINT_WORDS) fail("taint vocabulary too large");
  c.taint_effect.push_back(0);
  for (size_t t = 1; t < c.taint_vocab.size(); t++) c.taint_effect.push_back(effect_id(c.taint_vocab[t].effect));
  // allocatable columns
  c.alloc_cpu.resize(N);
  c.alloc_mem.resize(N);
  c.alloc_eph.resize(N);
  c.alloc_pods.resize(N);
  c.alloc_scalar.resize((size_t)S * N);
  c.flags.assign(N, 0);
  c.nb_limit.assign(N, 0);
  for (int32_t pos = 0; pos < N; pos++) {
    const Node& nd = nodes[c.order[pos]];
    c.alloc_cpu[pos] = qs.res(nd.alloc, "cpu");
    c.alloc_mem[pos] = qs.res(nd.alloc, "memory");
    c.alloc_eph[pos] = qs.res(nd.alloc, "ephemeral-storage");
    const int64_t pods = qs.res(nd.alloc, "pods");
    if (pods < INT32_MIN || pods > INT32_MAX) fail("node " + nd.name + ": allocatable pods out of the int32 range");
    c.alloc_pods[pos] = (int32_t)pods;
    for (int32_t k = 0; k < S; k++) c.alloc_scalar[(size_t)k * N + pos] = qs.res(nd.alloc, c.scalar_names[k]);
    c.flags[pos] = nd.unschedulable ? KSIM_NODE_UNSCHEDULABLE : 0;
    const string* lim = lookup(nd.annotations, c.nb.node_limit);   // netbw.node_limit
    if (lim) {
      int64_t q;
      if (netbw_milli(*lim, q)) {
        c.flags[pos] |= KSIM_NODE_NB_LIMIT;
        c.nb_limit[pos] = q;
      } else {
        c.flags[pos] |= KSIM_NODE_NB_LIMIT | KSIM_NODE_NB_LIMIT_BAD;
      }
    }
  }
  c.req_cpu.assign(N, 0);
  c.req_mem.assign(N, 0);
  c.req_eph.assign(N, 0);
  c.req_scalar.assign((size_t)S * N, 0);
  c.nz_cpu.assign(N, 0);
  c.nz_mem.assign(N, 0);
  c.num_pods.assign(N, 0);
  c.nb_alloc.assign(N, 0);
  for (int32_t pos = 0; pos < N; pos++) {
    c.node_names.push_back(nodes[c.order[pos]].name);
    c.node_labels.push_back(nodes[c.order[pos]].labels);
  }
  for (int32_t pos = 0; pos < N; pos++) c.pos_of[c.node_names[pos]] = pos;
  c.topo_log.resize((size_t)N + 1);
  for (int32_t s = 0; s <= N; s++) c.topo_log[s] = std::log((double)(s + 2));
}

void read_namespaces(Topo& t, const PoolView& pv) {
  const ksim_k8s_pool& pool = pv.p;
  if (pool.n_namespaces < 0 || (pool.n_namespaces > 0 && !pool.namespaces)) fail("pool: bad namespace list");
  for (int64_t i = 0; i < pool.n_namespaces; i++) {
    const ksim_k8s_namespace& ns = pool.namespaces[i];
    const string name(pv.str(ns.name));
    Labels lb = pv.kv(ns.labels_first, ns.labels_count);
    auto it = t.ns_index.find(name);
    if (it == t.ns_index.end()) {
      t.ns_index[name] = t.ns_labels.size();
      t.ns_labels.emplace_back(name, std::move(lb));
    } else {
      t.ns_labels[it->second].second = std::move(lb);
    }
  }
}

string member_key(string_view ns, string_view name) {
  string k(ns);
  k += '\x1f';
  k += name;
  return k;
}

vector<HostPort> host_ports(const Pod& p) {
  vector<HostPort> out;
  for (const auto& c : p.containers)
    for (const auto& hp : c.ports) out.push_back(hp);
  return out;
}

void encode_nodes(ksim_encoder* e, const ksim_k8s_pool& pool, const ksim_encode_nodes_opts& o) {
  PoolView pv(pool);
  Reader rd{pv};
  Cluster prev = std::move(e->c);
  Topo prev_topo = std::move(e->topo);
  const bool keep = o.keep_previous && e->has_cluster;
  e->has_cluster = false;
  e->c = Cluster{};
  e->topo = Topo{};
  e->pods.clear();
  e->exprs.clear();
  e->terms.clear();
  e->uses.clear();
  e->adds.clear();
  e->nn.clear();
  e->members.clear();
  e->dup_keys.clear();
  e->queue_members.clear();
  e->old_pos.clear();
  e->in_place = false;
  Cluster& c = e->c;
  e->req_memo.clear();
  if (o.nb_node_limit >= 0) c.nb.node_limit = string(pv.str(o.nb_node_limit));
  if (o.nb_egress_request >= 0) c.nb.egress = string(pv.str(o.nb_egress_request));
  if (o.nb_ingress_request >= 0) c.nb.ingress = string(pv.str(o.nb_ingress_request));
  if (pool.n_nodes < 0 || (pool.n_nodes > 0 && !pool.nodes)) fail("pool: bad node list");
  vector<Node> nodes;
  nodes.reserve(pool.n_nodes);
  for (int64_t i = 0; i < pool.n_nodes; i++) nodes.push_back(rd.node(pool.nodes[i]));
  e->extra_scalar = pv.strs(o.extra_scalar_first, o.extra_scalar_count);
  Quantities& qs = e->qs;
  node_columns(c, nodes, qs, keep ? &prev : nullptr, false, e->extra_scalar);
  const int32_t N = c.n;
  const int32_t S = c.n_scalar;
  // count classes
  Topo& t = e->topo;
  t.n = N;
  read_namespaces(t, pv);
  t.set_images(nodes, c.pos_of);
  if (keep) {                                // TopologyIndex.preregister
    t.selectors = prev_topo.selectors;
    t.selector_ids = prev_topo.selector_ids;
    t.matchers = prev_topo.matchers;
    t.matcher_ids = prev_topo.matcher_ids;
    for (const auto& pc : prev_topo.classes) {
      switch (pc.kind) {
        case kCarry: t.carried_class(pc.carry_kind, pc.matcher, pc.tk); break;
        case kSel: pc.is_all ? t.selector_class_all(pc.all) : t.selector_class(pc.matcher); break;
        case kPort: t.port_class(pc.ip, pc.proto, pc.port); break;
        case kImage: t.image_class_of(pc.names); break;
      }
    }
  }
  if (pool.n_pods < 0 || (pool.n_pods > 0 && !pool.pods)) fail("pool: bad pod list");
  // pass 1: every carried class exists before any bound pod is added (the
  // bound pods' terms see only the snapshot's namespaces, as upstream's
  // NodeInfo.AddPod builds each PodInfo's terms independently)
  const int64_t NB = pool.n_pods;
  vector<int32_t> bpos((size_t)NB, -1);
  std::unordered_map<string, int> carry_fast;
  vector<vector<std::pair<int, int32_t>>> carried((size_t)NB);
  Pod tmp;
  for (int64_t i = 0; i < NB; i++) {
    const ksim_k8s_pod& x = pool.pods[i];
    auto it = c.pos_of.find(string(pv.str(x.node_name)));
    if (it == c.pos_of.end()) continue;                 // a pod naming no node of the snapshot
    bpos[i] = it->second;
    if (!(x.aff_req_count | x.aff_pref_count | x.anti_req_count | x.anti_pref_count)) continue;
    // fast path: every term without a namespaceSelector is a pure function of
    // its pool content and the owner's namespace (memo of its carried class)
    {
      bool fast = true;
      vector<std::pair<int, int32_t>>& out = carried[i];
      auto add = [&](int cid, int32_t k) {
        for (auto& y : out)
          if (y.first == cid) {
            y.second += k;
            return;
          }
        out.emplace_back(cid, k);
      };
      const struct {
        int32_t first, count;
        const char* kind;
        bool weighted;
      } lists[4] = {{x.anti_req_first, x.anti_req_count, kReqAnti, false},
                    {x.aff_req_first, x.aff_req_count, kReqAff, false},
                    {x.aff_pref_first, x.aff_pref_count, kPrefAff, true},
                    {x.anti_pref_first, x.anti_pref_count, kPrefAnti, true}};
      string key;
      for (int l = 0; l < 4 && fast; l++) {
        const ksim_k8s_pod_term* pt = pv.at(pool.pod_terms, pool.n_pod_terms, lists[l].first, lists[l].count, "pod_terms");
        for (int32_t k = 0; k < lists[l].count && fast; k++) {
          if (pt[k].ns_selector >= 0) {
            fast = false;
            break;
          }
          key.clear();
          put(key, l);
          put(key, x.namespace_);
          put(key, pt[k].topology_key);
          key += rd.selector_key(pt[k].selector);
          put(key, pt[k].ns_count);
          const int32_t* ns = pv.at(pool.str_list, pool.n_str_list, pt[k].ns_first, pt[k].ns_count, "str_list");
          for (int32_t j = 0; j < pt[k].ns_count; j++) put(key, ns[j]);
          auto mi = carry_fast.find(key);
          int cid;
          if (mi != carry_fast.end()) {
            cid = mi->second;
          } else {
            const vector<PodTerm> one = rd.pod_terms(lists[l].first + k, 1);
            cid = t.carried_class(lists[l].kind, t.term_matcher(string(pv.str(x.namespace_)), one[0]),
                                  one[0].topology_key);
            carry_fast.emplace(key, cid);
          }
          add(cid, lists[l].weighted ? pt[k].weight : 1);
        }
      }
      if (fast) {
        std::sort(out.begin(), out.end());
        continue;
      }
      out.clear();
    }
    tmp.ns = string(pv.str(x.namespace_));
    tmp.aff_req = rd.pod_terms(x.aff_req_first, x.aff_req_count);
    tmp.aff_pref = rd.pod_terms(x.aff_pref_first, x.aff_pref_count);
    tmp.anti_req = rd.pod_terms(x.anti_req_first, x.anti_req_count);
    tmp.anti_pref = rd.pod_terms(x.anti_pref_first, x.anti_pref_count);
    carried[i] = t.carried_terms(tmp);
  }
  // pass 2: NodeInfo.AddPod of each bound pod
  for (int64_t i = 0; i < NB; i++) {
    if (bpos[i] < 0) continue;
    const Pod p = read_pod(rd, pool.pods[i], t, e->req_memo, qs, true);
    const int32_t pos = bpos[i];
    t.add_bound(p, pos, carried[i]);
    const ksim_k8s_pod& x = pool.pods[i];
    string key = member_key(pv.str(x.namespace_), pv.str(x.name));
    auto [mi, fresh] = e->members.emplace(std::move(key), Member{pos, p.sig, host_ports(p)});
    if (!fresh) e->dup_keys.insert(mi->first);
    const ReqMemo& rm = requests_of(e, p);
    const auto& r = rm.requests;
    const auto& nz = rm.nonzero;
    c.req_cpu[pos] += req_of(r, "cpu");
    c.req_mem[pos] += req_of(r, "memory");
    c.req_eph[pos] += req_of(r, "ephemeral-storage");
    for (int32_t k = 0; k < S; k++) c.req_scalar[(size_t)k * N + pos] += req_of(r, c.scalar_names[k].c_str());
    c.nz_cpu[pos] += nz.first;
    c.nz_mem[pos] += nz.second;
    c.num_pods[pos] += 1;
    if (!p.annotations.empty()) c.nb_alloc[pos] += nb_pod_allocated(p.annotations, c.nb);
  }
  materialize_classes(e);
  e->nodes = std::move(nodes);
  e->has_cluster = true;
}

// ---- encode_pods --------------------------------------------------------------------------
struct PodBuilder {
  ksim_encoder* e;

  void expr(int col = 0, uint8_t op = KSIM_OP_FALSE, const vector<uint32_t>& vals = {}, int64_t num = 0) {
    if ((int)vals.size() > KSIM_EXPR_VALS) fail("requirement has too many values after vocabulary filtering");
    ksim_label_expr x{};
    x.col = (uint16_t)std::max(col, 0);
    x.op = op;
    x.nvals = (uint8_t)vals.size();
    for (size_t i = 0; i < vals.size(); i++) x.vals[i] = vals[i];
    x.num = num;
    e->exprs.push_back(x);
  }

  // nodeSelectorRequirementsAsSelector, compiled to ids (invalid -> OP_FALSE)
  void requirement(const Req& r) {
    const int col = label_col(e, r.key);
    const string& op = r.op;
    if (op == "In" || op == "NotIn") {
      if (r.values.empty()) return expr();
      vector<uint32_t> vids;
      for (const auto& v : r.values) {
        const int32_t id = value_id(e, col, v);
        if (id) vids.push_back((uint32_t)id);
      }
      std::sort(vids.begin(), vids.end());
      vids.erase(std::unique(vids.begin(), vids.end()), vids.end());
      if (op == "In") return vids.empty() ? expr() : expr(col, KSIM_OP_IN, vids);
      if (vids.empty()) return expr(0, KSIM_OP_TRUE);
      return expr(col, KSIM_OP_NOT_IN, vids);
    }
    if (op == "Exists" || op == "DoesNotExist") {
      if (!r.values.empty()) return expr();
      if (col < 0) return op == "Exists" ? expr() : expr(0, KSIM_OP_TRUE);
      return expr(col, op == "Exists" ? KSIM_OP_EXISTS : KSIM_OP_DOES_NOT_EXIST);
    }
    if (op == "Gt" || op == "Lt") {
      if (r.values.size() != 1) return expr();
      int64_t v;
      if (!parse_int64(r.values[0], v) || col < 0) return expr();
      return expr(col, op == "Gt" ? KSIM_OP_GT : KSIM_OP_LT, {}, v);
    }
    expr();
  }

  // nodeSelectorRequirementsAsFieldSelector: metadata.name In/NotIn, one value
  void field_requirement(const Req& r) {
    if (r.op == "__true__") return expr(0, KSIM_OP_TRUE);
    if (r.op == "__false__") return expr();
    if (r.key != "metadata.name" || (r.op != "In" && r.op != "NotIn") || r.values.size() != 1) return expr();
    auto it = e->c.pos_of.find(r.values[0]);
    const bool known = it != e->c.pos_of.end();
    vector<uint32_t> pos;
    if (known) pos.push_back((uint32_t)it->second);
    if (r.op == "In") return known ? expr(0, KSIM_OP_FIELD_IN, pos) : expr();
    known ? expr(0, KSIM_OP_FIELD_NOT_IN, pos) : expr(0, KSIM_OP_TRUE);
  }

  void term(const SelTerm& t, int32_t weight = 0) {
    const int32_t first = (int32_t)e->exprs.size();
    for (const auto& r : t.exprs) requirement(r);
    for (const auto& r : t.fields) field_requirement(r);
    e->terms.push_back(ksim_term{first, (int32_t)e->exprs.size() - first, weight, 0});
  }
};

// nodeaffinity.PreFilter's PreFilterResult.NodeNames (encode.py prefilter_node_names):
// false = every node; true with the sorted names otherwise
bool prefilter_node_names(const Pod& p, vector<string>& names) {
  if (!p.has_required || p.required.empty()) return false;
  std::vector<string> acc;
  for (const auto& t : p.required) {
    bool have = false;
    vector<string> tn;
    for (const auto& r : t.fields) {
      if (r.key != "metadata.name" || r.op != "In") continue;
      vector<string> vals = r.values;
      std::sort(vals.begin(), vals.end());
      vals.erase(std::unique(vals.begin(), vals.end()), vals.end());
      if (!have) {
        tn = vals;
        have = true;
      } else {
        vector<string> x;
        std::set_intersection(tn.begin(), tn.end(), vals.begin(), vals.end(), std::back_inserter(x));
        tn = std::move(x);
      }
    }
    if (!have) return false;
    acc.insert(acc.end(), tn.begin(), tn.end());
  }
  std::sort(acc.begin(), acc.end());
  acc.erase(std::unique(acc.begin(), acc.end()), acc.end());
  names = std::move(acc);
  return true;
}

void tol_bits(const vector<Toleration>& tols, const vector<Taint>& vocab, uint64_t* w, bool prefer_only) {
  for (int k = 0; k < KSIM_TAINT_WORDS; k++) w[k] = 0;
  for (size_t tid = 1; tid < vocab.size(); tid++)
    for (const auto& t : tols) {
      if (prefer_only && !(t.effect.empty() || t.effect == "PreferNoSchedule")) continue;
      if (tolerates(t, vocab[tid])) {
        w[tid >> 6] |= (uint64_t)1 << (tid & 63);
        break;
      }
    }
}

// topology.py SpreadDefaults
struct SpreadDefaults {
  bool active = false, system = false;
  vector<Spread> defaults;
  std::unordered_map<string, vector<Service>> services;   // by namespace, list order
  std::unordered_map<string, Controller> controllers;     // kind \x1f ns \x1f name

  // helper.DefaultSelector (null when Empty())
  std::shared_ptr<Selector> default_selector(const Pod& p) const {
    Labels label_set;                        // a dict updated in order
    auto update = [&](const Labels& m) {
      for (const auto& kv : m) {
        bool found = false;
        for (auto& x : label_set)
          if (x.first == kv.first) {
            x.second = kv.second;
            found = true;
          }
        if (!found) label_set.push_back(kv);
      }
    };
    auto sv = services.find(p.ns);
    if (sv != services.end())
      for (const auto& s : sv->second) {
        if (!s.has_selector) continue;       // nil selectors match nothing
        bool all = true;
        for (const auto& kv : s.selector) {
          const string* v = lookup(p.labels, kv.first);
          if (!v || *v != kv.second) {
            all = false;
            break;
          }
        }
        if (all) update(s.selector);
      }
    vector<Req> extra;
    if (p.has_owner) {
      if (p.owner_api == "v1" && p.owner_kind == "ReplicationController") {
        auto it = controllers.find("ReplicationController\x1f" + p.ns + '\x1f' + p.owner_name);
        if (it != controllers.end() && it->second.rc_set && !it->second.rc_selector.empty())
          update(it->second.rc_selector);
      } else if (p.owner_api == "apps/v1" && (p.owner_kind == "ReplicaSet" || p.owner_kind == "StatefulSet")) {
        auto it = controllers.find(p.owner_kind + '\x1f' + p.ns + '\x1f' + p.owner_name);
        if (it != controllers.end() && it->second.selector) {
          const Selector& s = *it->second.selector;
          validate_selector(s);
          for (const auto& kv : s.labels) extra.push_back(Req{kv.first, "In", {kv.second}});   // sorted items
          for (const auto& r : s.exprs) extra.push_back(r);
        }
      }
    }
    if (label_set.empty() && extra.empty()) return nullptr;
    return std::make_shared<Selector>(make_selector(label_set, extra));
  }

  // constraints(pod) -> (constraints, system defaults); pod_spread with spread None when !active
  vector<Spread> constraints(const Pod& p, bool& sysdef) const {
    sysdef = false;
    if (!active || !p.spread.empty()) return p.spread;
    if (defaults.empty()) return {};
    auto sel = default_selector(p);
    if (!sel) return {};
    vector<Spread> out = defaults;
    for (auto& c : out) c.selector = sel;
    sysdef = system;
    return out;
  }
};

// pass 1: every class the pod uses or carries exists before any pod's adds
void register_pod_classes(Topo& t, const Pod& p, const SpreadDefaults& sd) {
  t.note_namespace(p.ns);
  t.carried_terms(p);
  bool sysdef;
  for (const auto& c : sd.constraints(p, sysdef)) {
    if (c.selector) validate_selector(*c.selector);
    if (c.selector && !c.selector->empty()) t.selector_class(t.intern_matcher({p.ns}, false, t.sel_key(c.selector)));
  }
  if (!p.aff_req.empty()) {
    vector<int> ms;
    for (const auto& x : p.aff_req) ms.push_back(t.term_matcher(p.ns, x));
    t.selector_class_all(ms);
  }
  for (const auto& x : p.anti_req) t.selector_class(t.term_matcher(p.ns, x));
  for (const auto& w : p.aff_pref) t.selector_class(t.term_matcher(p.ns, w));
  for (const auto& w : p.anti_pref) t.selector_class(t.term_matcher(p.ns, w));
  t.port_check_classes(p);
  t.image_class(p);
}

Use use(uint8_t kind, int32_t cls, uint16_t col, int32_t arg = 0, uint8_t flags = 0) {
  return Use{cls, arg, col, kind, flags};
}

// carried_uses: uses of the carried classes whose term matches the pod
vector<Use> carried_uses(ksim_encoder* e, const Pod& p) {
  Topo& t = e->topo;
  const uint64_t ck = ((uint64_t)(uint32_t)p.sig << 32) | (uint32_t)t.carry_ids.size();
  auto hit = t.carry_uses.find(ck);
  if (hit != t.carry_uses.end()) return hit->second;
  vector<Use> out;
  for (int cid : t.carry_ids) {
    const Cls& c = t.classes[cid];
    if (!t.sig_matches_one(c.matcher, p.sig)) continue;
    const uint16_t col = col_or_none(e, c.tk);
    if (c.carry_kind == kReqAnti) out.push_back(use(KSIM_USE_IPA_EXISTING_ANTI, cid, col));
    else if (c.carry_kind == kReqAff) out.push_back(use(KSIM_USE_IPA_SCORE_HARD, cid, col, 1));
    else if (c.carry_kind == kPrefAff) out.push_back(use(KSIM_USE_IPA_SCORE, cid, col, 1));
    else out.push_back(use(KSIM_USE_IPA_SCORE, cid, col, -1));
  }
  t.carry_uses.emplace(ck, out);
  return out;
}

// pass 2: the pod's uses and topo flags (topology.py pod_uses)
vector<Use> pod_uses(ksim_encoder* e, const Pod& p, const SpreadDefaults& sd, uint32_t& flags) {
  Topo& t = e->topo;
  vector<Use> uses;
  flags = 0;
  vector<string> seen_dns, seen_sa;
  bool sysdef;
  const vector<Spread> cons = sd.constraints(p, sysdef);
  if (sysdef && !cons.empty()) flags |= KSIM_POD_PTS_SYSTEM_DEFAULT;
  for (const auto& c : cons) {
    vector<string>* seen = c.when == "DoNotSchedule" ? &seen_dns : c.when == "ScheduleAnyway" ? &seen_sa : nullptr;
    if (!seen) fail("whenUnsatisfiable " + c.when + " not supported");
    if (std::find(seen->begin(), seen->end(), c.topology_key) != seen->end())
      fail("duplicate topologyKey/whenUnsatisfiable (rejected by API validation)");
    seen->push_back(c.topology_key);
    if (c.max_skew < 1) fail("maxSkew must be >= 1");
    int32_t cls = -1;
    if (c.selector && !c.selector->empty())
      cls = t.selector_class(t.intern_matcher({p.ns}, false, t.sel_key(c.selector)));
    uint8_t f = 0;
    if (c.selector && c.selector->matches(p.labels)) f |= KSIM_USEF_SELF_MATCH;
    if ((c.naff_set && !c.naff.empty() ? c.naff : string("Honor")) == "Honor") f |= KSIM_USEF_HONOR_AFFINITY;
    if ((c.ntaint_set && !c.ntaint.empty() ? c.ntaint : string("Ignore")) == "Honor") f |= KSIM_USEF_HONOR_TAINTS;
    if (c.topology_key == kHostname) f |= KSIM_USEF_HOSTNAME;
    const uint8_t kind = c.when == "DoNotSchedule" ? KSIM_USE_PTS_HARD : KSIM_USE_PTS_SOFT;
    uses.push_back(use(kind, cls, col_or_none(e, c.topology_key), c.max_skew, f));
  }
  if (!p.aff_req.empty()) {
    vector<int> ms;
    for (const auto& x : p.aff_req) ms.push_back(t.term_matcher(p.ns, x));
    const int cls = t.selector_class_all(ms);
    for (const auto& x : p.aff_req) uses.push_back(use(KSIM_USE_IPA_AFFINITY, cls, col_or_none(e, x.topology_key)));
    bool self = true;
    for (int m : ms) self = self && t.matches(m, p.ns, p.labels);
    if (self) flags |= KSIM_POD_IPA_SELF_AFFINITY;
  }
  for (const auto& x : p.anti_req) {
    const int cls = t.selector_class(t.term_matcher(p.ns, x));
    uses.push_back(use(KSIM_USE_IPA_ANTI, cls, col_or_none(e, x.topology_key)));
  }
  for (const auto& u : carried_uses(e, p)) uses.push_back(u);
  for (const auto& w : p.aff_pref) {
    const int cls = t.selector_class(t.term_matcher(p.ns, w));
    uses.push_back(use(KSIM_USE_IPA_SCORE, cls, col_or_none(e, w.topology_key), w.weight));
  }
  for (const auto& w : p.anti_pref) {
    const int cls = t.selector_class(t.term_matcher(p.ns, w));
    uses.push_back(use(KSIM_USE_IPA_SCORE, cls, col_or_none(e, w.topology_key), -w.weight));
  }
  const int ic = t.image_class(p);
  if (ic >= 0) uses.push_back(use(KSIM_USE_IMAGE, ic, (uint16_t)KSIM_COL_NONE));
  for (int cls : t.port_check_classes(p)) uses.push_back(use(KSIM_USE_NODE_PORT, cls, (uint16_t)KSIM_COL_NONE));
  if ((int)uses.size() > KSIM_MAX_USES)
    fail("pod " + p.name + ": " + std::to_string(uses.size()) + " topology uses > " + std::to_string(KSIM_MAX_USES));
  return uses;
}

void encode_pods(ksim_encoder* e, const ksim_k8s_pool& pool, const ksim_encode_pods_opts& o) {
  if (!e->has_cluster) fail("ksim_encode_pods before ksim_encode_nodes");
  PoolView pv(pool);
  Reader rd{pv};
  Cluster& c = e->c;
  Topo& t = e->topo;
  t.begin_call();
  e->req_memo.clear();
  e->pods.clear();
  e->exprs.clear();
  e->terms.clear();
  e->uses.clear();
  e->adds.clear();
  e->nn.clear();
  PodBuilder b{e};
  // NodeAffinityArgs.addedAffinity
  int32_t added_first = 0, added_count = 0;
  vector<std::pair<int32_t, SelTerm>> added_pref;
  if (o.added_required_first >= 0) {
    added_first = (int32_t)e->terms.size();
    for (const auto& x : rd.terms(o.added_required_first, o.added_required_count)) b.term(x);
    added_count = (int32_t)e->terms.size() - added_first;
  }
  {
    const ksim_k8s_preferred_term* pr =
        pv.at(pool.preferred, pool.n_preferred, o.added_preferred_first, o.added_preferred_count, "preferred");
    for (int32_t i = 0; i < o.added_preferred_count; i++)
      if (pr[i].weight) added_pref.emplace_back(pr[i].weight, rd.term(pr[i].term));
  }
  // PodTopologySpreadArgs defaults
  SpreadDefaults sd;
  if (o.spread_defaults == KSIM_SPREAD_DEFAULTS_SYSTEM || o.spread_defaults == KSIM_SPREAD_DEFAULTS_LIST) {
    sd.active = true;
    sd.system = o.spread_defaults == KSIM_SPREAD_DEFAULTS_SYSTEM;
    if (sd.system) {
      Spread h;
      h.max_skew = 3;
      h.topology_key = kHostname;
      h.when = "ScheduleAnyway";
      Spread z = h;
      z.max_skew = 5;
      z.topology_key = kZone;
      sd.defaults = {h, z};
    } else {
      sd.defaults = rd.spreads(o.spread_first, o.spread_count);
    }
    for (int64_t i = 0; i < pool.n_services; i++) {
      const ksim_k8s_service& s = pool.services[i];
      Service x;
      x.ns = string(pv.str(s.namespace_));
      x.has_selector = s.selector_first >= 0;
      if (x.has_selector) x.selector = pv.kv(s.selector_first, s.selector_count);
      sd.services[x.ns].push_back(std::move(x));
    }
    for (int64_t i = 0; i < pool.n_controllers; i++) {
      const ksim_k8s_controller& k = pool.controllers[i];
      Controller x;
      x.kind = string(pv.str(k.kind));
      x.ns = string(pv.str(k.namespace_));
      x.name = string(pv.str(k.name));
      x.rc_set = k.rc_selector_first >= 0;
      if (x.rc_set) x.rc_selector = pv.kv(k.rc_selector_first, k.rc_selector_count);
      x.selector = rd.selector(k.selector);
      sd.controllers[x.kind + '\x1f' + x.ns + '\x1f' + x.name] = std::move(x);
    }
  } else if (o.spread_defaults != KSIM_SPREAD_DEFAULTS_NONE) {
    fail("unknown spread_defaults");
  }
  if (pool.n_pods < 0 || (pool.n_pods > 0 && !pool.pods)) fail("pool: bad pod list");
  vector<Pod> pods;
  pods.reserve(pool.n_pods);
  for (int64_t i = 0; i < pool.n_pods; i++) {
    pods.push_back(read_pod(rd, pool.pods[i], t, e->req_memo, e->qs, false));
  }
  const size_t classes_before = t.classes.size();
  for (const auto& p : pods) register_pod_classes(t, p, sd);   // pass 1
  vector<Taint> unsched_vocab{Taint{}, Taint{kTaintUnschedulable, "", "NoSchedule"}};
  e->pods.resize(pods.size());
  e->queue_members.clear();
  e->queue_members.reserve(pods.size());
  for (size_t i = 0; i < pods.size(); i++) {
    const Pod& p = pods[i];
    e->queue_members.emplace_back(member_key(p.ns, p.name), Member{-1, p.sig, host_ports(p)});
    ksim_pod& rec = e->pods[i];
    rec = ksim_pod{};
    const ReqMemo& rm = requests_of(e, p);
    const auto& r = rm.requests;
    const auto& nz = rm.nonzero;
    rec.req_cpu = req_of(r, "cpu");
    rec.req_mem = req_of(r, "memory");
    rec.req_eph = req_of(r, "ephemeral-storage");
    rec.nz_cpu = nz.first;
    rec.nz_mem = nz.second;
    uint32_t flags = 0;
    for (const auto& x : r) {
      if (is_native_resource(x.first)) continue;
      flags |= KSIM_POD_HAS_SCALAR;
      auto it = std::find(c.scalar_names.begin(), c.scalar_names.end(), x.first);
      if (it == c.scalar_names.end())
        fail("scalar resource " + x.first + " unknown to the cluster encoder (pass extra_scalar)");
      rec.scalar_req[it - c.scalar_names.begin()] = x.second;
    }
    tol_bits(p.tolerations, c.taint_vocab, rec.tol_filter, false);
    tol_bits(p.tolerations, c.taint_vocab, rec.tol_prefer, true);
    for (const auto& x : p.tolerations)
      if (tolerates(x, unsched_vocab[1])) {
        flags |= KSIM_POD_TOLERATES_UNSCHEDULABLE;
        break;
      }
    if (!p.node_name.empty()) {
      auto it = c.pos_of.find(p.node_name);
      rec.node_name = it == c.pos_of.end() ? -2 : it->second;
    } else {
      rec.node_name = -1;
    }
    // spec.nodeSelector -> Equals requirements
    rec.sel_first = (int32_t)e->exprs.size();
    for (const auto& kv : p.node_selector) {
      const int col = label_col(e, kv.first);
      const int32_t vid = value_id(e, col, kv.second);
      if (vid) b.expr(col, KSIM_OP_IN, {(uint32_t)vid});
      else b.expr();
    }
    rec.sel_count = (int32_t)e->exprs.size() - rec.sel_first;
    if (p.has_required) {
      flags |= KSIM_POD_HAS_REQUIRED_AFFINITY;
      rec.req_term_first = (int32_t)e->terms.size();
      for (const auto& x : p.required) b.term(x);
      rec.req_term_count = (int32_t)e->terms.size() - rec.req_term_first;
    }
    rec.pref_term_first = (int32_t)e->terms.size();
    for (const auto& w : p.preferred)
      if (w.first != 0) b.term(w.second, w.first);
    for (const auto& w : added_pref) b.term(w.second, w.first);
    rec.pref_term_count = (int32_t)e->terms.size() - rec.pref_term_first;
    if (added_count) {
      flags |= KSIM_POD_ADDED_AFFINITY;
      rec.added_term_first = added_first;
      rec.added_term_count = added_count;
    }
    if (p.volumes == KSIM_K8S_VOLUMES_REFUSE) {
      flags |= KSIM_POD_HAS_VOLUMES;
    } else if (p.volumes == KSIM_K8S_VOLUMES_GROUPS) {
      rec.vb_first = (int32_t)e->terms.size();
      for (size_t g = 0; g < p.vb.size(); g++) {
        const int32_t gid = (int32_t)g < p.vb_bound ? (int32_t)g : ((int32_t)g | KSIM_VB_UNBOUND_GROUP);
        for (const auto& x : p.vb[g]) b.term(x, gid);
      }
      rec.vb_count = (int32_t)e->terms.size() - rec.vb_first;
      rec.vz_first = (int32_t)e->terms.size();
      for (size_t g = 0; g < p.vz.size(); g++)
        for (const auto& x : p.vz[g]) b.term(x, (int32_t)g);
      rec.vz_count = (int32_t)e->terms.size() - rec.vz_first;
    }
    vector<string> pf;
    if (prefilter_node_names(p, pf)) {       // findNodesThatFitPod scans only these nodes
      flags |= KSIM_POD_NODE_NAMES;
      vector<int32_t> known;
      for (const auto& nm : pf) {
        auto it = c.pos_of.find(nm);
        if (it != c.pos_of.end()) known.push_back(it->second);
      }
      std::sort(known.begin(), known.end());
      if (known.size() < pf.size()) flags |= KSIM_POD_NODE_NAMES_UNKNOWN;
      rec.nn_first = (int32_t)e->nn.size();
      rec.nn_count = (int32_t)known.size();
      e->nn.insert(e->nn.end(), known.begin(), known.end());
    }
    rec.flags = flags;
    uint32_t tflags = 0;
    const vector<Use> u = pod_uses(e, p, sd, tflags);
    rec.use_first = (int32_t)e->uses.size();
    rec.use_count = (int32_t)u.size();
    for (const auto& x : u) e->uses.push_back(ksim_topo_use{x.cls, x.arg, x.col, x.kind, x.flags, 0});
    const auto a = t.adds(p);
    rec.add_first = (int32_t)e->adds.size();
    rec.add_count = (int32_t)a.size();
    for (const auto& x : a) e->adds.push_back(ksim_class_add{x.first, x.second});
    rec.topo_flags = tflags;
    // NetworkBandwidth: the Filter request (each request annotation falling
    // back to the *-bandwidth one) and the pod's share once bound
    {
      int64_t total = 0;
      uint32_t nbf = 0;
      const std::pair<const string*, const char*> keys[2] = {{&c.nb.ingress, kIngressBandwidth},
                                                             {&c.nb.egress, kEgressBandwidth}};
      const uint32_t bad[2] = {KSIM_POD_NB_INGRESS_BAD, KSIM_POD_NB_EGRESS_BAD};
      for (int k = 0; k < 2; k++) {
        const string* s = lookup(p.annotations, *keys[k].first);
        if (!s) s = lookup(p.annotations, keys[k].second);
        if (!s) continue;
        int64_t q;
        try {
          if (netbw_milli(*s, q)) total += q;
          else nbf |= bad[k];
        } catch (const EncError& x) {
          fail("pod " + p.ns + "/" + p.name + ": " + x.msg);
        }
      }
      rec.nb_flags = nbf;
      rec.nb_req = total;
      try {
        rec.nb_add = nb_pod_allocated(p.annotations, c.nb);
      } catch (const EncError& x) {
        fail("pod " + p.ns + "/" + p.name + ": " + x.msg);
      }
    }
  }
  materialize_classes(e, classes_before);
}

// ---- snapshot deltas (ABI 11) ---------------------------------------------------------------
// Node informer deltas on the encoder's snapshot ([upstream] internal/cache
// cache.go AddNode / UpdateNode / RemoveNode, node_tree.go): pool.nodes are
// added (a new name) or updated (a known name) nodes, removed[] string ids of
// the pool naming nodes that leave.  The node table is rebuilt over the nodes
// in add order -- an update that changes the node's zone re-adds it at the end,
// as nodeTree.updateNode does -- with the previous scalar columns, taint ids,
// label columns and count classes kept.  A kept node's dynamic columns and
// class rows stay the snapshot's (the device replays the binds made since on
// them, ksim_upsert_nodes); an added node starts empty; a removed node's bound
// pods leave the snapshot.  ImageLocality's rows are recomputed (they read
// every node's images and the node count).
// Node updates that move no node and need no new vocabulary (same zone, same
// images, scalar resources, taints and label values the snapshot already
// has): the rows' static columns in place.  False (nothing changed) otherwise.
bool update_rows_in_place(ksim_encoder* e, const vector<Node>& upd) {
  Cluster& c = e->c;
  std::unordered_map<string, size_t> at;
  for (size_t i = 0; i < e->nodes.size(); i++) at.emplace(e->nodes[i].name, i);
  std::unordered_map<string, int> tid;
  for (size_t t = 1; t < c.taint_vocab.size(); t++) {
    const Taint& x = c.taint_vocab[t];
    tid.emplace(x.key + '\x1f' + x.value + '\x1f' + x.effect, (int)t);
  }
  std::unordered_set<string> seen;
  for (const Node& nd : upd) {
    auto it = at.find(nd.name);
    if (it == at.end() || !seen.insert(nd.name).second) return false;
    const Node& old = e->nodes[it->second];
    if (zone_key(old.labels) != zone_key(nd.labels) || old.images != nd.images) return false;
    if ((int)nd.taints.size() > KSIM_MAX_NODE_TAINTS) return false;
    for (const auto& kv : nd.alloc)
      if (!is_native_resource(kv.first) &&
          std::find(c.scalar_names.begin(), c.scalar_names.end(), kv.first) == c.scalar_names.end())
        return false;
    for (const Taint& x : nd.taints)
      if (!tid.count(x.key + '\x1f' + x.value + '\x1f' + x.effect)) return false;
    for (size_t k = 0; k < c.label_keys.size(); k++) {
      const string* v = lookup(nd.labels, c.label_keys[k]);
      if (v && !c.value_index[k].count(*v)) return false;
    }
  }
  const int32_t N = c.n;
  Quantities& qs = e->qs;
  e->changed.clear();
  for (const Node& nd : upd) {
    const int32_t pos = c.pos_of.at(nd.name);
    c.alloc_cpu[pos] = qs.res(nd.alloc, "cpu");
    c.alloc_mem[pos] = qs.res(nd.alloc, "memory");
    c.alloc_eph[pos] = qs.res(nd.alloc, "ephemeral-storage");
    const int64_t pods = qs.res(nd.alloc, "pods");
    if (pods < INT32_MIN || pods > INT32_MAX) fail("node " + nd.name + ": allocatable pods out of the int32 range");
    c.alloc_pods[pos] = (int32_t)pods;
    for (int32_t k = 0; k < c.n_scalar; k++) c.alloc_scalar[(size_t)k * N + pos] = qs.res(nd.alloc, c.scalar_names[k]);
    c.flags[pos] = nd.unschedulable ? KSIM_NODE_UNSCHEDULABLE : 0;
    c.nb_limit[pos] = 0;
    if (const string* lim = lookup(nd.annotations, c.nb.node_limit)) {
      int64_t q;
      if (netbw_milli(*lim, q)) {
        c.flags[pos] |= KSIM_NODE_NB_LIMIT;
        c.nb_limit[pos] = q;
      } else {
        c.flags[pos] |= KSIM_NODE_NB_LIMIT | KSIM_NODE_NB_LIMIT_BAD;
      }
    }
    for (int k = 0; k < KSIM_MAX_NODE_TAINTS; k++) c.taints[(size_t)k * N + pos] = 0;
    for (size_t k = 0; k < nd.taints.size(); k++) {
      const Taint& x = nd.taints[k];
      c.taints[k * N + pos] = (uint16_t)tid.at(x.key + '\x1f' + x.value + '\x1f' + x.effect);
    }
    for (size_t k = 0; k < c.label_keys.size(); k++) {
      const string* v = lookup(nd.labels, c.label_keys[k]);
      c.labels[k * N + pos] = v ? (uint32_t)c.value_index[k].at(*v) : 0u;
    }
    c.node_labels[pos] = nd.labels;
    e->nodes[at.at(nd.name)] = nd;
    e->changed.push_back(pos);
  }
  e->old_pos.resize(N);
  for (int32_t p = 0; p < N; p++) e->old_pos[p] = p;
  e->in_place = true;
  e->pods.clear();
  e->exprs.clear();
  e->terms.clear();
  e->uses.clear();
  e->adds.clear();
  e->nn.clear();
  e->queue_members.clear();
  return true;
}

void update_nodes(ksim_encoder* e, const ksim_k8s_pool& pool, const int32_t* removed, int32_t n_removed) {
  if (!e->has_cluster) fail("ksim_encoder_update_nodes before ksim_encode_nodes");
  if (n_removed < 0 || (n_removed > 0 && !removed)) fail("bad removed-node list");
  PoolView pv(pool);
  Reader rd{pv};
  if (pool.n_nodes < 0 || (pool.n_nodes > 0 && !pool.nodes)) fail("pool: bad node list");
  e->in_place = false;
  if (n_removed == 0) {
    vector<Node> upd;
    for (int64_t i = 0; i < pool.n_nodes; i++) upd.push_back(rd.node(pool.nodes[i]));
    read_namespaces(e->topo, pv);
    if (update_rows_in_place(e, upd)) return;
  }
  const size_t M = e->nodes.size();
  std::unordered_map<string, size_t> at;     // name -> index in the add order
  for (size_t i = 0; i < M; i++) at.emplace(e->nodes[i].name, i);
  vector<char> gone(M, 0);
  for (int32_t r = 0; r < n_removed; r++) {
    auto it = at.find(string(pv.str(removed[r])));
    if (it == at.end()) fail("remove of a node not in the snapshot: " + string(pv.str(removed[r])));
    gone[it->second] = 1;
  }
  struct Entry {
    Node node;
    int32_t old;                               // position in the current snapshot, -1: new
  };
  vector<Entry> head, tail;                    // kept in place; re-added or added (delta order)
  vector<std::pair<bool, Node>> upd(M);
  std::unordered_set<string> seen;
  for (int64_t i = 0; i < pool.n_nodes; i++) {
    Node nd = rd.node(pool.nodes[i]);
    if (!seen.insert(nd.name).second) fail("node " + nd.name + " twice in one delta");
    auto it = at.find(nd.name);
    if (it == at.end() || gone[it->second]) {  // added (a removed name added again starts empty)
      tail.push_back(Entry{std::move(nd), -1});
      continue;
    }
    const size_t k = it->second;
    if (zone_key(e->nodes[k].labels) != zone_key(nd.labels)) {
      tail.push_back(Entry{std::move(nd), e->c.pos_of.at(e->nodes[k].name)});
      gone[k] = 2;                             // moved: out of its place, identity kept
    } else {
      upd[k] = {true, std::move(nd)};
    }
  }
  for (size_t k = 0; k < M; k++) {
    if (gone[k]) continue;
    const int32_t old = e->c.pos_of.at(e->nodes[k].name);
    head.push_back(Entry{upd[k].first ? std::move(upd[k].second) : std::move(e->nodes[k]), old});
  }
  for (auto& x : tail) head.push_back(std::move(x));
  vector<Node> nodes;
  vector<int32_t> entry_old;
  nodes.reserve(head.size());
  for (auto& x : head) {
    entry_old.push_back(x.old);
    nodes.push_back(std::move(x.node));
  }
  Cluster oc = std::move(e->c);
  e->c = Cluster{};
  Cluster& c = e->c;
  c.nb = oc.nb;
  node_columns(c, nodes, e->qs, &oc, true, e->extra_scalar);
  const int32_t N = c.n, oN = oc.n;
  vector<int32_t> old_pos(N), new_of(oN, -1);
  for (int32_t p = 0; p < N; p++) {
    old_pos[p] = entry_old[c.order[p]];
    if (old_pos[p] >= 0) new_of[old_pos[p]] = p;
  }
  // the snapshot's dynamic columns on kept nodes
  for (int32_t p = 0; p < N; p++) {
    const int32_t o = old_pos[p];
    if (o < 0) continue;
    c.req_cpu[p] = oc.req_cpu[o];
    c.req_mem[p] = oc.req_mem[o];
    c.req_eph[p] = oc.req_eph[o];
    c.nz_cpu[p] = oc.nz_cpu[o];
    c.nz_mem[p] = oc.nz_mem[o];
    c.num_pods[p] = oc.num_pods[o];
    c.nb_alloc[p] = oc.nb_alloc[o];
    for (int32_t k = 0; k < oc.n_scalar; k++) c.req_scalar[(size_t)k * N + p] = oc.req_scalar[(size_t)k * oN + o];
  }
  // the same label columns, in the same order (value ids renumbered over the new nodes)
  for (const auto& key : oc.label_keys) label_col(e, key, true);
  // count classes: membership moves with its nodes, rows too
  Topo& t = e->topo;
  t.n = N;
  read_namespaces(t, pv);
  for (auto it = e->members.begin(); it != e->members.end();) {
    const int32_t np = new_of[it->second.pos];
    if (np < 0) {
      e->dup_keys.erase(it->first);
      it = e->members.erase(it);
    } else {
      it->second.pos = np;
      ++it;
    }
  }
  t.remap_members(new_of);
  t.images.clear();
  t.set_images(nodes, c.pos_of);
  for (auto& cls : t.classes) {
    if (cls.kind == kImage) {
      cls.counts = t.image_counts(cls.names);
      continue;
    }
    vector<int32_t> row(N, 0);
    for (int32_t p = 0; p < N; p++)
      if (old_pos[p] >= 0) row[p] = cls.counts[old_pos[p]];
    cls.counts = std::move(row);
  }
  materialize_classes(e);
  e->nodes = std::move(nodes);
  e->old_pos = std::move(old_pos);
  // pod sets compiled against the old positions are gone
  e->pods.clear();
  e->exprs.clear();
  e->terms.clear();
  e->uses.clear();
  e->adds.clear();
  e->nn.clear();
  e->queue_members.clear();
}

// Pod `pod_index` of the current pod set is bound at node position `node` in
// the snapshot: the scheduler cache's AssumePod / an informer AddPod of a
// bound pod.  Membership only: the device takes the pod's adds through
// ksim_assume, and the count classes registered from now on count it.
void bind_pod(ksim_encoder* e, int32_t pod_index, int32_t node) {
  if (!e->has_cluster) fail("ksim_encoder_bind before ksim_encode_nodes");
  if (pod_index < 0 || pod_index >= (int32_t)e->queue_members.size()) fail("bind: pod index out of the pod set");
  if (node < 0 || node >= e->c.n) fail("bind: node position out of range");
  const auto& q = e->queue_members[pod_index];
  if (e->members.count(q.first)) fail("bind: the pod is already bound in the snapshot");
  Member m = q.second;
  m.pos = node;
  e->topo.note_namespace(q.first.substr(0, q.first.find('\x1f')));
  e->topo.add_member(m.sig, m.ports, node);
  e->members.emplace(q.first, std::move(m));
}

// The bound pod namespace/name leaves the snapshot (ForgetPod / RemovePod).
int32_t unbind_pod(ksim_encoder* e, const char* ns, const char* name) {
  if (!e->has_cluster) fail("ksim_encoder_unbind before ksim_encode_nodes");
  if (!ns || !name) fail("unbind: null name");
  const string key = member_key(ns, name);
  auto it = e->members.find(key);
  if (it == e->members.end()) fail("unbind: " + string(ns) + "/" + name + " is not bound in the snapshot");
  if (e->dup_keys.count(key)) fail("unbind: " + string(ns) + "/" + name + " is bound twice in the snapshot");
  const int32_t pos = it->second.pos;
  e->topo.drop_member(it->second.sig, it->second.ports, pos);
  e->members.erase(it);
  return pos;
}

template <class F>
int guarded(ksim_encoder* e, F&& f) {
  if (!e) return KSIM_E_INVALID;
  try {
    f();
    e->err.clear();
    return KSIM_OK;
  } catch (const EncError& x) {
    e->err = x.msg;
    return x.code;
  } catch (const std::bad_alloc&) {
    e->err = "out of memory";
    return KSIM_E_OOM;
  } catch (const std::exception& x) {
    e->err = x.what();
    return KSIM_E_INVALID;
  }
}

}  // namespace

extern "C" {

int ksim_encoder_create(ksim_encoder** out) {
  if (!out) return KSIM_E_INVALID;
  try {
    *out = new ksim_encoder();
  } catch (...) {
    return KSIM_E_OOM;
  }
  return KSIM_OK;
}

void ksim_encoder_destroy(ksim_encoder* e) { delete e; }

const char* ksim_encoder_last_error(const ksim_encoder* e) { return e ? e->err.c_str() : "null encoder"; }

int ksim_encode_nodes(ksim_encoder* e, const ksim_k8s_pool* pool, const ksim_encode_nodes_opts* opts) {
  return guarded(e, [&] {
    if (!pool) fail("pool is null");
    ksim_encode_nodes_opts o{-1, -1, -1, 0, 0, 0};
    if (opts) o = *opts;
    encode_nodes(e, *pool, o);
  });
}

int ksim_encode_pods(ksim_encoder* e, const ksim_k8s_pool* pool, const ksim_encode_pods_opts* opts) {
  return guarded(e, [&] {
    if (!pool) fail("pool is null");
    ksim_encode_pods_opts o{-1, 0, 0, 0, KSIM_SPREAD_DEFAULTS_NONE, 0, 0, 0};
    if (opts) o = *opts;
    encode_pods(e, *pool, o);
  });
}

int ksim_encoder_cluster(const ksim_encoder* e, ksim_node_table* t, ksim_vocab* v) {
  if (!e || !e->has_cluster) return KSIM_E_INVALID;
  const Cluster& c = e->c;
  auto p = [](const auto& vec) { return vec.empty() ? nullptr : vec.data(); };
  if (t) {
    *t = ksim_node_table{};
    t->n_nodes = c.n;
    t->n_scalar = c.n_scalar;
    t->n_label_cols = (int32_t)c.label_keys.size();
    t->alloc_cpu = p(c.alloc_cpu);
    t->alloc_mem = p(c.alloc_mem);
    t->alloc_eph = p(c.alloc_eph);
    t->alloc_pods = p(c.alloc_pods);
    t->alloc_scalar = p(c.alloc_scalar);
    t->req_cpu = p(c.req_cpu);
    t->req_mem = p(c.req_mem);
    t->req_eph = p(c.req_eph);
    t->req_scalar = p(c.req_scalar);
    t->nz_cpu = p(c.nz_cpu);
    t->nz_mem = p(c.nz_mem);
    t->num_pods = p(c.num_pods);
    t->flags = p(c.flags);
    t->taints = p(c.taints);
    t->labels = p(c.labels);
    t->n_classes = (int32_t)e->topo.classes.size();
    t->class_count = p(c.class_count);
    t->nb_limit = p(c.nb_limit);
    t->nb_alloc = p(c.nb_alloc);
  }
  if (v) {
    *v = ksim_vocab{};
    v->n_taints = (int32_t)c.taint_effect.size();
    v->n_label_values = (int32_t)c.label_num.size();
    v->taint_effect = p(c.taint_effect);
    v->label_col_offset = p(c.label_col_offset);
    v->label_num = p(c.label_num);
    v->label_num_ok = p(c.label_num_ok);
    v->n_topo_log = (int32_t)c.topo_log.size();
    v->topo_log = p(c.topo_log);
  }
  return KSIM_OK;
}

int ksim_encoder_pods(const ksim_encoder* e, ksim_pod_set* s) {
  if (!e || !e->has_cluster || !s) return KSIM_E_INVALID;
  auto p = [](const auto& vec) { return vec.empty() ? nullptr : vec.data(); };
  *s = ksim_pod_set{};
  s->n_pods = (int32_t)e->pods.size();
  s->n_exprs = (int32_t)e->exprs.size();
  s->n_terms = (int32_t)e->terms.size();
  s->pods = p(e->pods);
  s->exprs = p(e->exprs);
  s->terms = p(e->terms);
  s->n_uses = (int32_t)e->uses.size();
  s->n_adds = (int32_t)e->adds.size();
  s->uses = p(e->uses);
  s->adds = p(e->adds);
  s->n_nn = (int32_t)e->nn.size();
  s->nn = p(e->nn);
  return KSIM_OK;
}

int ksim_encoder_get_info(const ksim_encoder* e, ksim_encoder_info* out) {
  if (!e || !out) return KSIM_E_INVALID;
  *out = ksim_encoder_info{};
  out->n_nodes = e->c.n;
  out->n_scalar = e->c.n_scalar;
  out->n_label_cols = (int32_t)e->c.label_keys.size();
  out->n_taints = (int32_t)e->c.taint_vocab.size();
  out->n_classes = (int32_t)e->topo.classes.size();
  out->n_pods = (int32_t)e->pods.size();
  out->n_exprs = (int32_t)e->exprs.size();
  out->n_terms = (int32_t)e->terms.size();
  out->n_uses = (int32_t)e->uses.size();
  out->n_adds = (int32_t)e->adds.size();
  out->n_nn = (int32_t)e->nn.size();
  out->n_members = (int32_t)e->members.size();
  return KSIM_OK;
}

int ksim_encoder_update_nodes(ksim_encoder* e, const ksim_k8s_pool* pool, const int32_t* removed,
                              int32_t n_removed) {
  return guarded(e, [&] {
    if (!pool) fail("pool is null");
    update_nodes(e, *pool, removed, n_removed);
  });
}

int ksim_encoder_old_pos(const ksim_encoder* e, int32_t* old_pos) {
  if (!e || !e->has_cluster || (!old_pos && e->c.n > 0)) return KSIM_E_INVALID;
  if ((int32_t)e->old_pos.size() != e->c.n) return KSIM_E_INVALID;   // no node delta since the snapshot
  std::copy(e->old_pos.begin(), e->old_pos.end(), old_pos);
  return KSIM_OK;
}

int ksim_encoder_changed_rows(const ksim_encoder* e, int32_t* rows, int32_t cap) {
  if (!e || !e->has_cluster || cap < 0 || (cap > 0 && !rows)) return KSIM_E_INVALID;
  if (!e->in_place) return -1;
  const int32_t n = (int32_t)e->changed.size();
  for (int32_t i = 0; i < n && i < cap; i++) rows[i] = e->changed[i];
  return n;
}

int ksim_encoder_bind(ksim_encoder* e, int32_t pod_index, int32_t node) {
  return guarded(e, [&] { bind_pod(e, pod_index, node); });
}

int ksim_encoder_unbind(ksim_encoder* e, const char* namespace_, const char* name, int32_t* node) {
  return guarded(e, [&] {
    const int32_t pos = unbind_pod(e, namespace_, name);
    if (node) *node = pos;
  });
}

int ksim_encoder_bound_node(const ksim_encoder* e, const char* namespace_, const char* name, int32_t* node) {
  if (!e || !e->has_cluster || !namespace_ || !name || !node) return KSIM_E_INVALID;
  auto it = e->members.find(member_key(namespace_, name));
  *node = it == e->members.end() ? -1 : it->second.pos;
  return KSIM_OK;
}

int ksim_encoder_node_order(const ksim_encoder* e, int32_t* order) {
  if (!e || !e->has_cluster || (!order && e->c.n > 0)) return KSIM_E_INVALID;
  std::copy(e->c.order.begin(), e->c.order.end(), order);
  return KSIM_OK;
}

const char* ksim_encoder_string(const ksim_encoder* e, int32_t what, int32_t i, int32_t j) {
  if (!e || i < 0) return nullptr;
  const Cluster& c = e->c;
  switch (what) {
    case KSIM_ENC_STR_LABEL_KEY:
      return (size_t)i < c.label_keys.size() ? c.label_keys[i].c_str() : nullptr;
    case KSIM_ENC_STR_LABEL_VALUE:
      return ((size_t)i < c.label_values.size() && j >= 0 && (size_t)j < c.label_values[i].size())
                 ? c.label_values[i][j].c_str()
                 : nullptr;
    case KSIM_ENC_STR_SCALAR:
      return (size_t)i < c.scalar_names.size() ? c.scalar_names[i].c_str() : nullptr;
    case KSIM_ENC_STR_TAINT_KEY:
    case KSIM_ENC_STR_TAINT_VALUE:
    case KSIM_ENC_STR_TAINT_EFFECT:
      if (i < 1 || (size_t)i >= c.taint_vocab.size()) return nullptr;
      return what == KSIM_ENC_STR_TAINT_KEY     ? c.taint_vocab[i].key.c_str()
             : what == KSIM_ENC_STR_TAINT_VALUE ? c.taint_vocab[i].value.c_str()
                                                : c.taint_vocab[i].effect.c_str();
    case KSIM_ENC_STR_NODE_NAME:
      return (size_t)i < c.node_names.size() ? c.node_names[i].c_str() : nullptr;
  }
  return nullptr;
}

}  // extern "C"
