// ksim_emit.cpp — result emission: one cycle's per-node
// filter codes and score matrices -> the three large annotation values the
// simulator writes for every scheduled pod, encoded as Go's encoding/json
// encodes the result store's maps (sorted keys, compact, HTML-escaped).
//
// In the reference each (node, plugin) pair is a map insert under the store's
// global mutex (resultstore/store.go:418-502, called from the wrapped plugins,
// wrappedplugin.go:388-516) followed by json.Marshal of nested maps
// (AddStoredResultToPod, store.go:129-190).  Here the maps never exist: the
// JSON text is written straight from the arrays in one pass per annotation,
// with node and plugin names sorted once.  Host code only (no device work).
#include <algorithm>
#include <cinttypes>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ksim_engine.h"

namespace {

// encoding/json string encoding: quotes, backslash, control characters as
// \u00XX (\n \r \t short forms), and <, >, & and U+2028 / U+2029 escaped.
bool plain(const char* s, size_t& n) {
  n = 0;
  for (const unsigned char* p = (const unsigned char*)s; *p; p++, n++)
    if (*p < 0x20 || *p == '"' || *p == '\\' || *p == '<' || *p == '>' || *p == '&' || *p >= 0x80) return false;
  return true;
}

void put_string(std::string& o, const char* s) {
  static const char* hex = "0123456789abcdef";
  size_t n;
  if (plain(s, n)) {                                  // the common case: nothing to escape
    o.push_back('"');
    o.append(s, n);
    o.push_back('"');
    return;
  }
  o.push_back('"');
  for (const unsigned char* p = (const unsigned char*)s; *p; p++) {
    const unsigned char c = *p;
    switch (c) {
      case '"': o += "\\\""; continue;
      case '\\': o += "\\\\"; continue;
      case '\n': o += "\\n"; continue;
      case '\r': o += "\\r"; continue;
      case '\t': o += "\\t"; continue;
      case '<': case '>': case '&':
        o += "\\u00";
        o.push_back(hex[c >> 4]);
        o.push_back(hex[c & 15]);
        continue;
      default: break;
    }
    if (c < 0x20) {
      o += "\\u00";
      o.push_back(hex[c >> 4]);
      o.push_back(hex[c & 15]);
    } else if (c == 0xE2 && p[1] == 0x80 && (p[2] == 0xA8 || p[2] == 0xA9)) {
      o += p[2] == 0xA8 ? "\\u2028" : "\\u2029";
      p += 2;
    } else {
      o.push_back((char)c);
    }
  }
  o.push_back('"');
}

void put_int(std::string& o, int64_t v) {              // strconv.FormatInt, as a JSON string
  char b[24];
  int n = 0;
  uint64_t u = v < 0 ? 0 - (uint64_t)v : (uint64_t)v;
  do {
    b[n++] = (char)('0' + u % 10);
    u /= 10;
  } while (u);
  o.push_back('"');
  if (v < 0) o.push_back('-');
  while (n) o.push_back(b[--n]);
  o.push_back('"');
}

std::vector<int32_t> sorted_order(int32_t n, const char* const* names) {
  std::vector<int32_t> idx((size_t)n);
  for (int32_t i = 0; i < n; i++) idx[i] = i;
  std::sort(idx.begin(), idx.end(), [&](int32_t a, int32_t b) { return strcmp(names[a], names[b]) < 0; });
  return idx;
}

int copy_out(const std::string& s, char* dst, int64_t cap, int64_t* len) {
  *len = (int64_t)s.size();
  if (!dst || cap < (int64_t)s.size() + 1) return KSIM_E_INVALID;
  memcpy(dst, s.data(), s.size());
  dst[s.size()] = 0;
  return KSIM_OK;
}

}  // namespace

extern "C" int ksim_emit_cycle_json(const ksim_emit_input* in, char* filter_json, int64_t filter_cap,
                                    char* score_json, int64_t score_cap, char* final_json, int64_t final_cap,
                                    int64_t* lens) {
  if (!in || !lens || in->n_nodes < 0 || in->n_filter < 0 || in->n_filter > KSIM_MAX_FILTER || in->n_score < 0 ||
      in->n_score > KSIM_MAX_SCORE || (in->n_nodes && (!in->node_names || !in->fail_plugin)))
    return KSIM_E_INVALID;
  const int32_t N = in->n_nodes, F = in->n_filter, S = in->n_score;
  for (int32_t i = 0; i < N; i++) {
    const uint8_t f = in->fail_plugin[i];
    if (!in->node_names[i]) return KSIM_E_INVALID;
    if (f != KSIM_PASSED && f != KSIM_NOT_EVALUATED &&
        (f >= F || !in->msg_id || in->msg_id[i] < 0 || in->msg_id[i] >= in->n_messages))
      return KSIM_E_INVALID;
  }
  for (int32_t k = 0; k < F; k++)
    if (!in->filter_names || !in->filter_names[k]) return KSIM_E_INVALID;
  for (int32_t k = 0; k < S; k++)
    if (!in->score_names || !in->score_names[k]) return KSIM_E_INVALID;
  const std::vector<int32_t> nodes = sorted_order(N, in->node_names);
  const std::vector<int32_t> fsort = sorted_order(F, in->filter_names);
  const std::vector<int32_t> ssort = sorted_order(S, in->score_names);

  // filter-result: node -> {plugin -> "passed" | reason} for the plugins run
  // (RunFilterPlugins stops at the first failure); nodes never evaluated are absent.
  std::string fj = "{";
  fj.reserve((size_t)N * (size_t)(24 + 40 * F));
  bool first_node = true;
  for (const int32_t i : nodes) {
    const uint8_t f = in->fail_plugin[i];
    if (f == KSIM_NOT_EVALUATED) continue;
    const int32_t ran = f == KSIM_PASSED ? F : f + 1;
    if (!first_node) fj.push_back(',');
    first_node = false;
    put_string(fj, in->node_names[i]);
    fj += ":{";
    bool first = true;
    for (const int32_t k : fsort) {
      if (k >= ran) continue;
      if (!first) fj.push_back(',');
      first = false;
      put_string(fj, in->filter_names[k]);
      fj.push_back(':');
      put_string(fj, k == f ? in->messages[in->msg_id[i]] : "passed");
    }
    fj.push_back('}');
  }
  fj.push_back('}');

  // score-result: node -> {plugin -> raw}; finalscore-result: node -> {plugin ->
  // weight x (normalized if the plugin normalizes, else raw)} (applyWeightOnScore
  // with the registry-default weight, store.go:476-502).  Scored nodes only.
  std::string sj = "{", gj = "{";
  sj.reserve((size_t)N * (size_t)(24 + 40 * S));
  gj.reserve((size_t)N * (size_t)(24 + 40 * S));
  first_node = true;
  if (S > 0 && in->scored) {
    for (const int32_t i : nodes) {
      if (!in->scored[i]) continue;
      if (!first_node) {
        sj.push_back(',');
        gj.push_back(',');
      }
      first_node = false;
      put_string(sj, in->node_names[i]);
      put_string(gj, in->node_names[i]);
      sj += ":{";
      gj += ":{";
      bool first = true;
      for (const int32_t k : ssort) {
        if (!first) {
          sj.push_back(',');
          gj.push_back(',');
        }
        first = false;
        const int64_t raw = in->raw[(size_t)k * N + i];
        const int64_t v = (in->has_normalize && in->has_normalize[k]) ? in->norm[(size_t)k * N + i] : raw;
        put_string(sj, in->score_names[k]);
        sj.push_back(':');
        put_int(sj, raw);
        put_string(gj, in->score_names[k]);
        gj.push_back(':');
        put_int(gj, v * (in->score_weight ? in->score_weight[k] : 0));
      }
      sj.push_back('}');
      gj.push_back('}');
    }
  }
  sj.push_back('}');
  gj.push_back('}');
  int rc = KSIM_OK, r;
  if ((r = copy_out(fj, filter_json, filter_cap, &lens[0]))) rc = r;
  if ((r = copy_out(sj, score_json, score_cap, &lens[1]))) rc = r;
  if ((r = copy_out(gj, final_json, final_cap, &lens[2]))) rc = r;
  return rc;
}
