// oracle/cpu_nfa.cpp — CPU BASELINE / TEST INFRASTRUCTURE ONLY.
//
// An optimized CPU matcher: the second CPU figure of bench.py's cpu_baseline
// leg ("optionally add an optimized CPU hash-NFA for honesty").
// emqx_oracle.cpp restates the reference's data structures (an ordered key
// table, fresh prefix strings per step, emqx_trie.erl:255-333); this file
// computes the same emqx_router:match_routes/1 result set (emqx_router.erl:
// 128-145) the way a tuned CPU program would: a level trie over flat
// open-addressing tables, words resolved once per topic, the frontier walked
// level by level, T threads over contiguous slices of the batch.  Like the
// rest of oracle/, the product (emqx_amd/, libemqx_gpu_match.so) never links,
// loads or calls it; tests/test_oracle_props.py checks it against the
// faithful restatement.
//
// Semantics (the faithful restatement's, see emqx_oracle.cpp): the row of a
// topic T is {T, if T is a route} ∪ {the wildcard filters matching T, unless T
// itself holds a wildcard}; '+' matches one word (the empty word too), '#'
// matches the rest including none (so "a/#" matches "a"); a topic whose first
// word starts with '$' skips the root's '+' and '#' (emqx_trie.erl:271-278).
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint64_t kEmpty = ~0ull;

uint64_t mix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}
uint64_t hash_bytes(const uint8_t* p, size_t n) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ n;
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t c;
    std::memcpy(&c, p + i, 8);
    h = mix64(h ^ c);
  }
  uint64_t c = 0;
  std::memcpy(&c, p + i, n - i);
  return mix64(h ^ c ^ 0x5bd1e995ull);
}
size_t pow2_at_least(size_t n) {
  size_t c = 16;
  while (c < n) c <<= 1;
  return c;
}

// byte strings (words or filters) -> dense id, open addressing
struct StrTable {
  std::vector<uint64_t> hs;    // hash per slot (kEmpty: free)
  std::vector<uint32_t> ids;   // id per slot
  std::vector<uint64_t> off;   // id -> [off[id], off[id+1]) in bytes
  std::vector<uint8_t> bytes;
  uint64_t mask = 0;
  void init(size_t n) {
    const size_t cap = pow2_at_least(n * 2 + 16);
    hs.assign(cap, kEmpty);
    ids.assign(cap, kNone);
    mask = cap - 1;
    off.assign(1, 0);
  }
  uint32_t find(const uint8_t* p, size_t n, uint64_t h) const {
    for (uint64_t s = h & mask;; s = (s + 1) & mask) {
      if (hs[s] == kEmpty) return kNone;
      if (hs[s] == h) {
        const uint32_t id = ids[s];
        if (off[id + 1] - off[id] == n && std::memcmp(bytes.data() + off[id], p, n) == 0) return id;
      }
    }
  }
  uint32_t find(const uint8_t* p, size_t n) const { return find(p, n, hash_bytes(p, n)); }
  uint32_t add(const uint8_t* p, size_t n) {  // the id of an existing entry, else a new one
    const uint64_t h = hash_bytes(p, n);
    const uint32_t f = find(p, n, h);
    if (f != kNone) return f;
    uint64_t s = h & mask;
    while (hs[s] != kEmpty) s = (s + 1) & mask;
    const uint32_t id = uint32_t(off.size() - 1);
    hs[s] = h;
    ids[s] = id;
    bytes.insert(bytes.end(), p, p + n);
    off.push_back(bytes.size());
    return id;
  }
};

struct Node {
  uint32_t plus = kNone;    // child through '+'
  uint32_t hash_f = kNone;  // filter id of "<node>/#"
  uint32_t end_f = kNone;   // wildcard filter id ending here
};

struct Nfa {
  StrTable words;    // distinct filter words
  StrTable routes;   // every filter (exact route lookup), id = rank
  std::vector<Node> nodes;
  std::vector<uint64_t> ekey;  // (parent << 32 | word) per slot, kEmpty: free
  std::vector<uint32_t> echild;
  uint64_t emask = 0;
  uint32_t plus_w = kNone, hash_w = kNone;

  uint32_t child(uint32_t parent, uint32_t w) const {
    const uint64_t key = (uint64_t(parent) << 32) | w;
    for (uint64_t s = mix64(key) & emask;; s = (s + 1) & emask) {
      if (ekey[s] == key) return echild[s];
      if (ekey[s] == kEmpty) return kNone;
    }
  }
  uint32_t add_child(uint32_t parent, uint32_t w) {
    const uint64_t key = (uint64_t(parent) << 32) | w;
    uint64_t s = mix64(key) & emask;
    for (; ekey[s] != kEmpty; s = (s + 1) & emask)
      if (ekey[s] == key) return echild[s];
    ekey[s] = key;
    echild[s] = uint32_t(nodes.size());
    nodes.emplace_back();
    return echild[s];
  }
};

template <class F>
void split(const uint8_t* p, size_t n, F&& f) {  // emqx_topic:tokens/1: n '/' give n + 1 words
  size_t a = 0;
  for (size_t i = 0; i <= n; ++i)
    if (i == n || p[i] == '/') {
      f(p + a, i - a);
      a = i + 1;
    }
}

struct NfaRows {  // a batch's CSR (orc_nfa_rows_* read it)
  std::vector<uint64_t> row_off;
  std::vector<uint32_t> ids;
};

}  // namespace

extern "C" {

// Build over n filters (duplicates allowed); ids = rank among the sorted unique filters.
void* orc_nfa_new(const uint8_t* fb, const uint64_t* fo, uint64_t n) {
  std::vector<std::string> fs;
  fs.reserve(n);
  for (uint64_t i = 0; i < n; ++i) fs.emplace_back(reinterpret_cast<const char*>(fb + fo[i]), fo[i + 1] - fo[i]);
  std::sort(fs.begin(), fs.end());  // unsigned bytewise = Erlang binary order
  fs.erase(std::unique(fs.begin(), fs.end()), fs.end());
  auto* x = new Nfa;
  size_t levels = 0;
  for (auto& f : fs) levels += 1 + size_t(std::count(f.begin(), f.end(), '/'));
  x->routes.init(fs.size());
  x->words.init(levels + 2);  // at most one word per level
  for (auto& f : fs) x->routes.add(reinterpret_cast<const uint8_t*>(f.data()), f.size());
  const size_t cap = pow2_at_least(levels * 2 + 16);
  x->ekey.assign(cap, kEmpty);
  x->echild.assign(cap, kNone);
  x->emask = cap - 1;
  x->nodes.emplace_back();  // root
  x->plus_w = x->words.add(reinterpret_cast<const uint8_t*>("+"), 1);
  x->hash_w = x->words.add(reinterpret_cast<const uint8_t*>("#"), 1);
  std::vector<uint32_t> ws;
  for (uint32_t id = 0; id < fs.size(); ++id) {
    const auto* p = reinterpret_cast<const uint8_t*>(fs[id].data());
    ws.clear();
    split(p, fs[id].size(), [&](const uint8_t* w, size_t l) { ws.push_back(x->words.add(w, l)); });
    bool wild = false;
    for (uint32_t w : ws) wild |= (w == x->plus_w || w == x->hash_w);
    if (!wild) continue;  // exact filters are routes only (emqx_router.erl:112-125)
    uint32_t node = 0;
    for (size_t k = 0; k < ws.size(); ++k) {
      if (ws[k] == x->hash_w && k + 1 == ws.size()) {  // '#' last: the parent's "<node>/#"
        x->nodes[node].hash_f = id;
        node = kNone;
        break;
      }
      if (ws[k] == x->plus_w) {
        if (x->nodes[node].plus == kNone) {
          const uint32_t c = uint32_t(x->nodes.size());
          x->nodes.emplace_back();
          x->nodes[node].plus = c;
        }
        node = x->nodes[node].plus;
      } else {
        node = x->add_child(node, ws[k]);  // ('#' inside a filter is an ordinary word here, as in the trie)
      }
    }
    if (node != kNone) x->nodes[node].end_f = id;
  }
  return x;
}

void orc_nfa_free(void* h) { delete static_cast<Nfa*>(h); }

// Match a batch on nthreads threads; want_ids = 0: row lengths only (the
// baseline's timed form).  Rows sorted by filter id.  Returns a CSR handle
// (orc_nfa_rows_* below).
void* orc_nfa_match(void* h, const uint8_t* tb, const uint64_t* to, uint64_t n, int nthreads, int want_ids) {
  const Nfa& x = *static_cast<const Nfa*>(h);
  if (nthreads < 1) nthreads = 1;
  std::vector<uint64_t> cnt(n);
  std::vector<std::vector<uint32_t>> rows(want_ids ? n : 0);
  auto work = [&](uint64_t lo, uint64_t hi) {
    std::vector<uint32_t> ws, cur, nxt, out;
    for (uint64_t i = lo; i < hi; ++i) {
      const uint8_t* p = tb + to[i];
      const size_t len = to[i + 1] - to[i];
      out.clear();
      const uint32_t lit = x.routes.find(p, len);  // lookup_routes(T)
      if (lit != kNone) out.push_back(lit);
      ws.clear();
      bool wild = false;
      split(p, len, [&](const uint8_t* w, size_t l) {
        wild |= (l == 1 && (w[0] == '+' || w[0] == '#'));
        ws.push_back(x.words.find(w, l));
      });
      if (!wild) {
        const bool dollar = len > 0 && p[0] == '$';
        cur.assign(1, 0u);
        for (size_t k = 0; k < ws.size() && !cur.empty(); ++k) {
          nxt.clear();
          for (uint32_t nd : cur) {
            const Node& N = x.nodes[nd];
            const bool skip = dollar && nd == 0;  // '$' topics: no root '+' / '#'
            if (N.hash_f != kNone && !skip) out.push_back(N.hash_f);
            if (ws[k] != kNone) {
              const uint32_t c = x.child(nd, ws[k]);
              if (c != kNone) nxt.push_back(c);
            }
            if (N.plus != kNone && !skip) nxt.push_back(N.plus);
          }
          cur.swap(nxt);
        }
        for (uint32_t nd : cur) {  // every word consumed: filters ending here and "<node>/#"
          const Node& N = x.nodes[nd];
          if (N.end_f != kNone) out.push_back(N.end_f);
          if (N.hash_f != kNone) out.push_back(N.hash_f);
        }
      }
      cnt[i] = out.size();
      if (want_ids) {
        std::sort(out.begin(), out.end());
        rows[i] = out;
      }
    }
  };
  std::vector<std::thread> th;
  const uint64_t per = (n + nthreads - 1) / nthreads;
  for (int k = 0; k < nthreads; ++k) {
    const uint64_t lo = std::min<uint64_t>(n, k * per), hi = std::min<uint64_t>(n, lo + per);
    th.emplace_back(work, lo, hi);
  }
  for (auto& t : th) t.join();
  auto* c = new NfaRows;
  c->row_off.resize(n + 1);
  c->row_off[0] = 0;
  for (uint64_t i = 0; i < n; ++i) c->row_off[i + 1] = c->row_off[i] + cnt[i];
  if (want_ids) {
    c->ids.reserve(c->row_off[n]);
    for (auto& r : rows) c->ids.insert(c->ids.end(), r.begin(), r.end());
  }
  return c;
}

uint64_t orc_nfa_rows_n(void* c) { return static_cast<NfaRows*>(c)->row_off.size() - 1; }
uint64_t orc_nfa_rows_nnz(void* c) { return static_cast<NfaRows*>(c)->ids.size(); }
const uint64_t* orc_nfa_rows_off(void* c) { return static_cast<NfaRows*>(c)->row_off.data(); }
const uint32_t* orc_nfa_rows_ids(void* c) { return static_cast<NfaRows*>(c)->ids.data(); }
void orc_nfa_rows_free(void* c) { delete static_cast<NfaRows*>(c); }

}  // extern "C"
