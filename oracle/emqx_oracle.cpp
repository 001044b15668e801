// oracle/emqx_oracle.cpp — TEST INFRASTRUCTURE ONLY.
//
// This file is the CPU oracle for the emqx-gpu-match hot path.  It is a
// faithful C++ restatement of the reference Erlang algorithm and is used ONLY
// as a checker: by tests/, by __graft_entry__.smoke() and by bench.py's
// cpu_baseline leg.  The product path (emqx_amd/, libemqx_gpu_match.so) never
// links, loads or calls it.
//
// Parity is pinned by the reference's own test vectors (tests/golden/
// suite_vectors.json, ported from apps/emqx/test/emqx_trie_SUITE.erl,
// emqx_topic_SUITE.erl, emqx_router_SUITE.erl, emqx_broker_SUITE.erl and the
// EUnit block of apps/emqx/src/emqx_trie.erl) and, at scale, by agreement of
// two independent restatements: the trie walk below and the brute-force
// emqx_topic:match/2 predicate (orc_bruteforce_batch).  The Erlang reference
// itself cannot run here (no erl/erlc/rebar3).
//
// Reference files restated (paths relative to /root/reference):
//   apps/emqx/src/emqx_topic.erl   words/1 :157-164, wildcard/1 :52-62,
//                                  match/2 :65-87, join/1 :183-195,
//                                  validate/2 :96-127
//   apps/emqx/src/emqx_trie.erl    insert/2 :114-119, delete/2 :131-136,
//                                  make_keys :191-193, do_compact :207-221,
//                                  make_prefixes :223-232, insert_key :234-241,
//                                  delete_key :243-251, lookup_topic :255-262,
//                                  has_prefix :264-269, do_match :271-286,
//                                  match_no_compact :288-312,
//                                  match_compact :314-329, 'match_#' :331-333,
//                                  empty/1 :170
//   apps/emqx/src/emqx_router.erl  do_add_route :112-125, match_routes :128-134,
//                                  match_trie :137-141, lookup_routes :144-145,
//                                  do_delete_route :164-172
//   apps/emqx/src/emqx_router_utils.erl insert_trie_route :33-38,
//                                  delete_trie_route :53-70
//   apps/emqx/src/emqx_broker.erl  do_subscribe :147-165, handle_call
//                                  {subscribe,T,I} :445-454, do_dispatch
//                                  :506-530, subscribers/1 :319-322
//   apps/emqx/src/emqx_broker_helper.erl get_sub_shard :82-86 (SHARD=1024 :54)
//
// Synthetic workload generator: SURVEY.md §8d (spec restated in DESIGN.md
// "Workload generator"); emqx_amd/csrc/workload.cpp is the product's own
// independent implementation of the same spec and tests check they agree.

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

namespace {

// ---------------------------------------------------------------------------
// emqx_topic
// ---------------------------------------------------------------------------

// A word: emqx_topic:word/1 maps <<>> -> '', <<"+">> -> '+', <<"#">> -> '#'.
enum WordKind { W_BIN = 0, W_EMPTY = 1, W_PLUS = 2, W_HASH = 3 };
struct Word {
  WordKind kind;
  std::string bin;  // only for W_BIN
};

// emqx_topic:tokens/1 (binary:split(T, <<"/">>, [global])) + word/1.
std::vector<Word> words(const std::string& t) {
  std::vector<Word> out;
  size_t start = 0;
  for (;;) {
    size_t p = t.find('/', start);
    std::string tok = t.substr(start, p == std::string::npos ? std::string::npos : p - start);
    Word w;
    if (tok.empty()) w.kind = W_EMPTY;
    else if (tok == "+") w.kind = W_PLUS;
    else if (tok == "#") w.kind = W_HASH;
    else { w.kind = W_BIN; w.bin = tok; }
    out.push_back(std::move(w));
    if (p == std::string::npos) break;
    start = p + 1;
  }
  return out;
}

// emqx_topic:bin/1
std::string bin(const Word& w) {
  switch (w.kind) {
    case W_EMPTY: return std::string();
    case W_PLUS: return "+";
    case W_HASH: return "#";
    default: return w.bin;
  }
}

// emqx_topic:wildcard/1
bool wildcard(const std::vector<Word>& ws) {
  for (auto& w : ws)
    if (w.kind == W_PLUS || w.kind == W_HASH) return true;
  return false;
}

// emqx_topic:join/1
std::string join_words(const std::vector<std::string>& parts) {
  std::string out;
  for (size_t i = 0; i < parts.size(); ++i) {
    if (i) out.push_back('/');
    out += parts[i];
  }
  return out;
}

bool word_eq(const Word& a, const Word& b) {
  return a.kind == b.kind && (a.kind != W_BIN || a.bin == b.bin);
}

// emqx_topic:match/2 on word lists (:74-87).
bool match_words(const std::vector<Word>& n, size_t i, const std::vector<Word>& f, size_t j) {
  for (;;) {
    if (i == n.size() && j == f.size()) return true;          // match([], [])
    if (i < n.size() && j < f.size() && word_eq(n[i], f[j])) { ++i; ++j; continue; }
    if (i < n.size() && j < f.size() && f[j].kind == W_PLUS) { ++i; ++j; continue; }
    if (j + 1 == f.size() && f[j].kind == W_HASH) return true; // match(_, ['#'])
    return false;
  }
}

// emqx_topic:match/2 (:65-73) with the '$' rule on the raw binaries.
bool topic_match(const std::string& name, const std::string& filter) {
  if (!name.empty() && name[0] == '$' && !filter.empty() && (filter[0] == '+' || filter[0] == '#'))
    return false;
  return match_words(words(name), 0, words(filter), 0);
}

// ---------------------------------------------------------------------------
// emqx_trie: ordered_set of {Key, 0|1} -> count.  A Prefix is either the atom
// `empty` (virtual root) or a binary; join/2 (:217-221) builds a fresh binary
// at every step exactly like the reference.
// ---------------------------------------------------------------------------

struct Prefix {
  bool empty_atom;
  std::string s;
};

Prefix join2(const Prefix& p, const Word& w) {
  if (p.empty_atom) return Prefix{false, bin(w)};  // join(empty, W)
  std::string s;
  s.reserve(p.s.size() + 1 + w.bin.size() + 1);
  s = p.s;
  s.push_back('/');
  s += bin(w);
  return Prefix{false, std::move(s)};               // emqx_topic:join([Prefix, Word])
}

// A segment for do_compact is a binary or the atom `empty`.
std::vector<std::string> do_compact(const std::vector<Word>& ws) {
  std::vector<std::string> acc;
  Prefix seg{true, {}};
  for (auto& w : ws) {
    if (w.kind == W_PLUS || w.kind == W_HASH) {
      acc.push_back(join2(seg, w).s);
      seg = Prefix{true, {}};
    } else {
      seg = join2(seg, w);
    }
  }
  if (!seg.empty_atom) acc.push_back(seg.s);
  return acc;
}

// Per-thread lookup counter (no shared cache line between baseline threads).
thread_local unsigned long long tl_lookups = 0;

struct Trie {
  bool compact;
  std::map<std::pair<std::string, int>, long long> tab;  // ETS ordered_set

  explicit Trie(bool c) : compact(c) {}

  // make_prefixes/1 (:223-232): all strict prefixes of the (compacted)
  // segment list, longest first, each joined by emqx_topic:join/1.
  std::vector<std::string> make_prefixes(const std::vector<Word>& ws) const {
    std::vector<std::string> segs;
    if (compact) segs = do_compact(ws);
    else for (auto& w : ws) segs.push_back(bin(w));
    std::vector<std::string> out;
    for (size_t k = segs.size(); k-- > 1;) {
      std::vector<std::string> pre(segs.begin(), segs.begin() + k);
      out.push_back(join_words(pre));
    }
    return out;
  }

  void insert_key(const std::pair<std::string, int>& k) { tab[k] += 1; }
  void delete_key(const std::pair<std::string, int>& k) {
    auto it = tab.find(k);
    if (it == tab.end()) return;
    if (it->second > 1) it->second -= 1;
    else tab.erase(it);
  }

  void insert(const std::string& topic) {  // insert/2 (:114-119)
    std::pair<std::string, int> tk{topic, 1};
    if (tab.count(tk)) return;
    insert_key(tk);
    for (auto& p : make_prefixes(words(topic))) insert_key({p, 0});
  }
  void erase(const std::string& topic) {   // delete/2 (:131-136)
    std::pair<std::string, int> tk{topic, 1};
    if (!tab.count(tk)) return;
    delete_key(tk);
    for (auto& p : make_prefixes(words(topic))) delete_key({p, 0});
  }
  bool empty() const { return tab.empty(); }

  void lookup_topic(const std::string& t, std::vector<std::string>& acc) {
    ++tl_lookups;
    auto it = tab.find({t, 1});
    if (it != tab.end() && it->second > 0) acc.push_back(t);
  }
  bool has_prefix(const Prefix& p) {
    if (p.empty_atom) return true;
    ++tl_lookups;
    auto it = tab.find({p.s, 0});
    return it != tab.end() && it->second > 0;
  }
  void match_hash(const Prefix& p, std::vector<std::string>& acc) {  // 'match_#'
    lookup_topic(join2(p, Word{W_HASH, {}}).s, acc);
  }

  void match_compact(const std::vector<Word>& ws, size_t i, const Prefix& p, bool isw,
                     std::vector<std::string>& acc) {
    if (i == ws.size()) {
      match_hash(p, acc);
      if (isw) lookup_topic(p.s, acc);
      return;
    }
    match_hash(p, acc);
    match_compact(ws, i + 1, join2(p, ws[i]), isw, acc);
    Prefix wp = join2(p, Word{W_PLUS, {}});
    if (i + 1 == ws.size() || has_prefix(wp)) match_compact(ws, i + 1, wp, true, acc);
  }

  void match_no_compact(const std::vector<Word>& ws, size_t i, const Prefix& p, bool isw,
                        std::vector<std::string>& acc) {
    if (i == ws.size()) {
      match_hash(p, acc);
      if (isw) lookup_topic(p.s, acc);
      return;
    }
    if (!has_prefix(p)) return;
    match_hash(p, acc);
    match_no_compact(ws, i + 1, join2(p, Word{W_PLUS, {}}), true, acc);
    match_no_compact(ws, i + 1, join2(p, ws[i]), isw, acc);
  }

  void do_match_from(const std::vector<Word>& ws, size_t i, const Prefix& p,
                     std::vector<std::string>& acc) {
    if (compact) match_compact(ws, i, p, false, acc);
    else match_no_compact(ws, i, p, false, acc);
  }

  // match/2 (:147-161) + do_match/2 (:271-280)
  std::vector<std::string> match(const std::string& topic) {
    std::vector<std::string> acc;
    std::vector<Word> ws = words(topic);
    if (wildcard(ws)) return acc;
    if (ws[0].kind == W_BIN && !ws[0].bin.empty() && ws[0].bin[0] == '$') {
      if (ws.size() == 1) lookup_topic(ws[0].bin, acc);
      do_match_from(ws, 1, Prefix{false, ws[0].bin}, acc);
    } else {
      do_match_from(ws, 0, Prefix{true, {}}, acc);
    }
    return acc;
  }
};

// ---------------------------------------------------------------------------
// emqx_router: emqx_route is a bag of #route{topic, dest}.
// ---------------------------------------------------------------------------

struct Router {
  Trie trie;
  std::map<std::string, std::vector<std::string>> routes;  // topic -> dests (set semantics)
  explicit Router(bool compact) : trie(compact) {}

  void add_route(const std::string& topic, const std::string& dest) {  // do_add_route/2
    auto& ds = routes[topic];
    if (std::find(ds.begin(), ds.end(), dest) != ds.end()) return;
    if (wildcard(words(topic)) && ds.empty()) trie.insert(topic);  // insert_trie_route
    ds.push_back(dest);
  }
  void delete_route(const std::string& topic, const std::string& dest) {  // do_delete_route/2
    auto it = routes.find(topic);
    if (it == routes.end()) return;
    auto& ds = it->second;
    auto d = std::find(ds.begin(), ds.end(), dest);
    if (d == ds.end()) return;
    ds.erase(d);
    if (ds.empty()) {
      routes.erase(it);
      if (wildcard(words(topic))) trie.erase(topic);  // delete_trie_route
    }
  }
  // lookup_routes/1 -> list of filters having routes, with their dests.
  void lookup_routes(const std::string& t, std::vector<std::pair<std::string, std::string>>& out) const {
    auto it = routes.find(t);
    if (it == routes.end()) return;
    for (auto& d : it->second) out.push_back({t, d});
  }
  std::vector<std::string> match_trie(const std::string& topic) {  // :137-141
    if (trie.empty()) return {};
    return trie.match(topic);
  }
  std::vector<std::pair<std::string, std::string>> match_routes(const std::string& topic) {
    std::vector<std::pair<std::string, std::string>> out;
    std::vector<std::string> m = match_trie(topic);
    lookup_routes(topic, out);
    for (auto& f : m) lookup_routes(f, out);
    return out;
  }
  // Distinct filters having at least one route in match_routes(T).
  std::vector<std::string> match_route_filters(const std::string& topic) {
    std::vector<std::string> out;
    std::vector<std::string> m = match_trie(topic);
    if (routes.count(topic)) out.push_back(topic);
    for (auto& f : m)
      if (routes.count(f)) out.push_back(f);
    return out;
  }
};

// ---------------------------------------------------------------------------
// emqx_broker subscriber table with the shard indirection.
// ---------------------------------------------------------------------------

struct SubEntry {  // a pid or {shard, I}
  bool shard;
  uint64_t v;
};

struct Broker {
  Router router;
  int shards_num;
  std::map<std::string, std::vector<SubEntry>> subscriber;              // Topic -> [pid | {shard,I}]
  std::map<std::pair<std::string, int>, std::vector<uint64_t>> shard_subs;  // {shard,Topic,I} -> [pid]
  std::set<std::pair<uint64_t, std::string>> suboption;                 // {SubPid, Topic}
  std::map<std::string, long long> seq;                                 // emqx_subseq
  std::set<std::pair<std::string, int>> shard_put;                      // broker pool process dict

  Broker(bool compact, int schedulers) : router(compact), shards_num(schedulers * 32) {}

  // erlang:phash2(SubPid, N) stand-in: the delivered multiset does not depend
  // on which shard a subscriber lands in (dispatch folds over all shards).
  int phash(uint64_t pid) const {
    uint64_t z = pid * 0x9E3779B97F4A7C15ull;
    z ^= z >> 29;
    return int(z % uint64_t(shards_num));
  }

  void subscribe(const std::string& topic, uint64_t pid) {  // subscribe/3 + do_subscribe/4
    if (suboption.count({pid, topic})) return;               // existed
    suboption.insert({pid, topic});
    long long s = ++seq[topic];                               // get_sub_shard/2
    if (s <= 1024) {
      subscriber[topic].push_back(SubEntry{false, pid});
      router.add_route(topic, "node");
    } else {
      int I = phash(pid) + 1;
      shard_subs[{topic, I}].push_back(pid);
      if (!shard_put.count({topic, I})) {                     // handle_call({subscribe,T,I})
        shard_put.insert({topic, I});
        subscriber[topic].push_back(SubEntry{true, uint64_t(I)});
      }
      router.add_route(topic, "node");
    }
  }

  // do_dispatch/2 (:506-530): one delivery per live subscriber pid.
  void dispatch(const std::string& filter, std::vector<uint64_t>& out) const {
    auto it = subscriber.find(filter);
    if (it == subscriber.end()) return;
    for (auto& e : it->second) {
      if (!e.shard) { out.push_back(e.v); continue; }
      auto s = shard_subs.find({filter, int(e.v)});
      if (s == shard_subs.end()) continue;
      for (auto p : s->second) out.push_back(p);
    }
  }

  // publish/1: match_routes -> aggre -> route -> dispatch (local node only).
  std::vector<uint64_t> publish(const std::string& topic) {
    std::vector<uint64_t> out;
    for (auto& r : router.match_routes(topic)) dispatch(r.first, out);
    return out;
  }
};

// ---------------------------------------------------------------------------
// Result containers exposed to ctypes.
// ---------------------------------------------------------------------------

struct StrList { std::vector<std::string> v; };
struct U64List { std::vector<uint64_t> v; };
struct Csr {
  std::vector<uint64_t> row_off;
  std::vector<uint32_t> ids;
  std::vector<uint64_t> aux;  // per-row lookup counts (trie walk)
};

std::vector<std::string> unpack(const uint8_t* bytes, const uint64_t* off, uint64_t n) {
  std::vector<std::string> out(n);
  for (uint64_t i = 0; i < n; ++i)
    out[i].assign(reinterpret_cast<const char*>(bytes + off[i]), off[i + 1] - off[i]);
  return out;
}

// ---------------------------------------------------------------------------
// Synthetic workload (spec in DESIGN.md "Workload generator").
// ---------------------------------------------------------------------------

const int kLevels = 5;
const int kVocab[kLevels] = {64, 1024, 1024, 64, 16};
const int16_t C_PLUS = -1, C_HASH = -2, C_END = -3;

struct SplitMix {
  uint64_t s;
  uint64_t next() {
    s += 0x9E3779B97F4A7C15ull;
    uint64_t z = s;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
};
uint64_t mix64(uint64_t x) { SplitMix m{x}; return m.next(); }

void gen_filter_codes(uint64_t seed, uint64_t n, int wildcard_only, int16_t* codes) {
  SplitMix r{mix64(seed ^ 0xF17E5ull)};
  std::unordered_set<uint64_t> seen;
  seen.reserve(n * 2);
  uint64_t got = 0;
  while (got < n) {
    int16_t c[kLevels];
    for (int l = 0; l < kLevels; ++l) c[l] = C_END;
    uint64_t kind = wildcard_only ? 20 + r.next() % 80 : r.next() % 100;
    if (kind < 20) {
      for (int l = 0; l < kLevels; ++l) c[l] = int16_t(r.next() % kVocab[l]);
    } else if (kind < 60) {
      for (int l = 0; l < kLevels; ++l) c[l] = int16_t(r.next() % kVocab[l]);
      c[r.next() % kLevels] = C_PLUS;
    } else if (kind < 90) {
      int k = 2 + int(r.next() % 3);
      for (int l = 0; l < k; ++l) c[l] = int16_t(r.next() % kVocab[l]);
      c[k] = C_HASH;
    } else {
      int p = 1 + int(r.next() % 3);
      for (int l = 0; l < p; ++l) c[l] = int16_t(r.next() % kVocab[l]);
      c[p] = C_PLUS;
      c[p + 1] = C_HASH;
    }
    uint64_t key = 0;
    for (int l = 0; l < kLevels; ++l) key = key * 1031 + uint64_t(c[l] + 3);
    if (!seen.insert(key).second) continue;
    std::memcpy(codes + got * kLevels, c, sizeof(c));
    ++got;
  }
}

std::string code_string(const int16_t* c) {
  std::string s;
  for (int l = 0; l < kLevels && c[l] != C_END; ++l) {
    if (l) s.push_back('/');
    if (c[l] == C_PLUS) s += "+";
    else if (c[l] == C_HASH) s += "#";
    else { s += "l" + std::to_string(l) + "w" + std::to_string(c[l]); }
  }
  return s;
}

void gen_topic_codes(uint64_t seed, uint64_t idx, const int16_t* fcodes, uint64_t nf, int16_t* out) {
  SplitMix r{mix64(mix64(seed ^ 0x70C1Cull) ^ (idx * 0xD1B54A32D192ED03ull))};
  if (nf == 0 || (r.next() & 1) == 0) {
    for (int l = 0; l < kLevels; ++l) out[l] = int16_t(r.next() % kVocab[l]);
    return;
  }
  const int16_t* c = fcodes + (r.next() % nf) * kLevels;
  for (int l = 0; l < kLevels; ++l) {
    if (c[l] >= 0) out[l] = c[l];
    else if (c[l] == C_PLUS) out[l] = int16_t(r.next() % kVocab[l]);
    else {  // '#': extend to 5 levels
      for (int m = l; m < kLevels; ++m) out[m] = int16_t(r.next() % kVocab[m]);
      break;
    }
  }
}

}  // namespace

// ===========================================================================
// extern "C" API (ctypes; oracle/oracle.py)
// ===========================================================================
extern "C" {

// ---- result lists ----
int64_t orc_strlist_len(StrList* l) { return int64_t(l->v.size()); }
const char* orc_strlist_get(StrList* l, int64_t i, uint64_t* len) {
  *len = l->v[i].size();
  return l->v[i].data();
}
void orc_strlist_free(StrList* l) { delete l; }
int64_t orc_u64list_len(U64List* l) { return int64_t(l->v.size()); }
const uint64_t* orc_u64list_data(U64List* l) { return l->v.data(); }
void orc_u64list_free(U64List* l) { delete l; }
uint64_t orc_csr_rows(Csr* c) { return c->row_off.size() - 1; }
uint64_t orc_csr_nnz(Csr* c) { return c->ids.size(); }
const uint64_t* orc_csr_row_off(Csr* c) { return c->row_off.data(); }
const uint32_t* orc_csr_ids(Csr* c) { return c->ids.data(); }
const uint64_t* orc_csr_aux(Csr* c) { return c->aux.data(); }
void orc_csr_free(Csr* c) { delete c; }

// ---- emqx_topic ----
int orc_topic_match(const char* n, uint64_t nl, const char* f, uint64_t fl) {
  return topic_match(std::string(n, nl), std::string(f, fl)) ? 1 : 0;
}
int orc_topic_wildcard(const char* t, uint64_t tl) { return wildcard(words(std::string(t, tl))) ? 1 : 0; }
// words/1 rendered as strings; '' -> "", '+' -> "+", '#' -> "#".  kinds[i]
// receives the WordKind so callers can tell '' (atom) from a literal.
StrList* orc_topic_words(const char* t, uint64_t tl, int32_t* kinds, int64_t kcap) {
  auto ws = words(std::string(t, tl));
  auto* l = new StrList;
  for (size_t i = 0; i < ws.size(); ++i) {
    l->v.push_back(bin(ws[i]));
    if (int64_t(i) < kcap) kinds[i] = ws[i].kind;
  }
  return l;
}

// ---- emqx_trie ----
void* orc_trie_new(int compact) { return new Trie(compact != 0); }
void orc_trie_free(void* t) { delete static_cast<Trie*>(t); }
void orc_trie_insert(void* t, const char* s, uint64_t n) { static_cast<Trie*>(t)->insert(std::string(s, n)); }
void orc_trie_delete(void* t, const char* s, uint64_t n) { static_cast<Trie*>(t)->erase(std::string(s, n)); }
int orc_trie_empty(void* t) { return static_cast<Trie*>(t)->empty() ? 1 : 0; }
StrList* orc_trie_match(void* t, const char* s, uint64_t n, uint64_t* lookups) {
  auto* tr = static_cast<Trie*>(t);
  uint64_t before = tl_lookups;
  auto* l = new StrList{tr->match(std::string(s, n))};
  if (lookups) *lookups = tl_lookups - before;
  return l;
}
// Table dump (key bytes, kind 0|1, count), in ordered_set order.
StrList* orc_trie_keys(void* t, int64_t* kinds, int64_t* counts, int64_t cap) {
  auto* tr = static_cast<Trie*>(t);
  auto* l = new StrList;
  int64_t i = 0;
  for (auto& kv : tr->tab) {
    if (i < cap) { kinds[i] = kv.first.second; counts[i] = kv.second; }
    l->v.push_back(kv.first.first);
    ++i;
  }
  return l;
}
StrList* orc_trie_make_prefixes(int compact, const char* s, uint64_t n) {
  Trie tmp(compact != 0);
  return new StrList{tmp.make_prefixes(words(std::string(s, n)))};
}
StrList* orc_do_compact(const char* s, uint64_t n) { return new StrList{do_compact(words(std::string(s, n)))}; }

// ---- emqx_router ----
void* orc_router_new(int compact) { return new Router(compact != 0); }
void orc_router_free(void* r) { delete static_cast<Router*>(r); }
void orc_router_add_route(void* r, const char* t, uint64_t tl, const char* d, uint64_t dl) {
  static_cast<Router*>(r)->add_route(std::string(t, tl), std::string(d, dl));
}
// add_route/1 for each of n packed filters (dest "node"): the same
// do_add_route/2 as above, without a foreign call per filter (large configs).
void orc_router_add_routes(void* r, const uint8_t* fb, const uint64_t* fo, uint64_t n) {
  auto* rt = static_cast<Router*>(r);
  const std::string node("node");
  for (uint64_t i = 0; i < n; ++i)
    rt->add_route(std::string(reinterpret_cast<const char*>(fb + fo[i]), fo[i + 1] - fo[i]), node);
}
void orc_router_delete_route(void* r, const char* t, uint64_t tl, const char* d, uint64_t dl) {
  static_cast<Router*>(r)->delete_route(std::string(t, tl), std::string(d, dl));
}
void* orc_router_trie(void* r) { return &static_cast<Router*>(r)->trie; }
// match_routes/1: items alternate topic, dest.
StrList* orc_router_match_routes(void* r, const char* t, uint64_t tl) {
  auto* l = new StrList;
  for (auto& kv : static_cast<Router*>(r)->match_routes(std::string(t, tl))) {
    l->v.push_back(kv.first);
    l->v.push_back(kv.second);
  }
  return l;
}
StrList* orc_router_topics(void* r) {
  auto* l = new StrList;
  for (auto& kv : static_cast<Router*>(r)->routes) l->v.push_back(kv.first);
  return l;
}

// ---- emqx_broker ----
void* orc_broker_new(int compact, int schedulers) { return new Broker(compact != 0, schedulers); }
void orc_broker_free(void* b) { delete static_cast<Broker*>(b); }
void* orc_broker_router(void* b) { return &static_cast<Broker*>(b)->router; }
void orc_broker_subscribe(void* b, const char* t, uint64_t tl, uint64_t pid) {
  static_cast<Broker*>(b)->subscribe(std::string(t, tl), pid);
}
U64List* orc_broker_subscribers(void* b, const char* t, uint64_t tl) {
  auto* l = new U64List;
  static_cast<Broker*>(b)->dispatch(std::string(t, tl), l->v);
  return l;
}
int64_t orc_broker_shard_entries(void* b, const char* t, uint64_t tl) {
  auto* br = static_cast<Broker*>(b);
  auto it = br->subscriber.find(std::string(t, tl));
  if (it == br->subscriber.end()) return 0;
  int64_t n = 0;
  for (auto& e : it->second) n += e.shard;
  return n;
}
U64List* orc_broker_publish(void* b, const char* t, uint64_t tl) {
  return new U64List{static_cast<Broker*>(b)->publish(std::string(t, tl))};
}

// ---- batch matching (trie walk; multi-threaded CPU baseline) ----
// mode 0 = emqx_trie:match/1 result set; mode 1 = match_routes/1 filter set.
// Filters are ranked by `ranked` (sorted unique filter strings = the id space).
// Filter string -> id (its rank among the sorted unique filters), built once
// and reused by many batches (orc_match_batch_ranked).
struct Ranker {
  std::unordered_map<std::string, uint32_t> rank;
};
void* orc_ranker_new(const uint8_t* fb, const uint64_t* foff, uint64_t nf) {
  auto* k = new Ranker;
  k->rank.reserve(nf * 2);
  for (uint64_t i = 0; i < nf; ++i)
    k->rank.emplace(std::string(reinterpret_cast<const char*>(fb + foff[i]), foff[i + 1] - foff[i]), uint32_t(i));
  return k;
}
void orc_ranker_free(void* k) { delete static_cast<Ranker*>(k); }

Csr* orc_match_batch_ranked(void* router, int mode, const uint8_t* tb, const uint64_t* toff, uint64_t n,
                            const void* ranker, int nthreads);

Csr* orc_match_batch(void* router, int mode, const uint8_t* tb, const uint64_t* toff, uint64_t n,
                     const uint8_t* fb, const uint64_t* foff, uint64_t nf, int nthreads, int want_ids) {
  Ranker* k = want_ids ? static_cast<Ranker*>(orc_ranker_new(fb, foff, nf)) : nullptr;
  Csr* c = orc_match_batch_ranked(router, mode, tb, toff, n, k, nthreads);
  delete k;
  return c;
}

// ranker == nullptr: counts (and lookup counts) only, no ids (the CPU baseline).
Csr* orc_match_batch_ranked(void* router, int mode, const uint8_t* tb, const uint64_t* toff, uint64_t n,
                            const void* ranker, int nthreads) {
  auto* r = static_cast<Router*>(router);
  const bool want_ids = ranker != nullptr;
  static const std::unordered_map<std::string, uint32_t> no_rank;
  const auto& rank = want_ids ? static_cast<const Ranker*>(ranker)->rank : no_rank;
  if (nthreads < 1) nthreads = 1;
  std::vector<std::vector<uint32_t>> rows(n);
  std::vector<uint64_t> cnt(n), lk(n);
  auto work = [&](uint64_t lo, uint64_t hi) {
    for (uint64_t i = lo; i < hi; ++i) {
      std::string t(reinterpret_cast<const char*>(tb + toff[i]), toff[i + 1] - toff[i]);
      std::vector<std::string> m;
      uint64_t before = tl_lookups;
      if (mode == 0) m = r->trie.empty() ? std::vector<std::string>() : r->trie.match(t);
      else m = r->match_route_filters(t);
      lk[i] = tl_lookups - before;
      cnt[i] = m.size();
      if (want_ids) {
        auto& row = rows[i];
        for (auto& f : m) {
          auto it = rank.find(f);
          row.push_back(it == rank.end() ? 0xFFFFFFFFu : it->second);
        }
        std::sort(row.begin(), row.end());
      }
    }
  };
  std::vector<std::thread> th;
  uint64_t per = (n + nthreads - 1) / nthreads;
  for (int k = 0; k < nthreads; ++k) {
    uint64_t lo = std::min<uint64_t>(n, k * per), hi = std::min<uint64_t>(n, lo + per);
    th.emplace_back(work, lo, hi);
  }
  for (auto& t : th) t.join();
  auto* c = new Csr;
  c->row_off.resize(n + 1);
  c->row_off[0] = 0;
  for (uint64_t i = 0; i < n; ++i) c->row_off[i + 1] = c->row_off[i] + cnt[i];
  c->aux = std::move(lk);
  if (want_ids) {
    c->ids.reserve(c->row_off[n]);
    for (auto& row : rows) c->ids.insert(c->ids.end(), row.begin(), row.end());
  }
  return c;
}

// ---- brute force over emqx_topic:match/2 (independent second restatement) ----
// filters: sorted unique filter strings (id = index).  in_trie[i] marks which
// filters the trie holds (mode 0); mode 1 uses route semantics (all filters).
Csr* orc_bruteforce_batch(int mode, const uint8_t* tb, const uint64_t* toff, uint64_t n,
                          const uint8_t* fb, const uint64_t* foff, uint64_t nf, const uint8_t* in_trie) {
  std::vector<std::string> fs = unpack(fb, foff, nf);
  std::vector<std::vector<Word>> fw(nf);
  std::vector<char> fwild(nf);
  for (uint64_t j = 0; j < nf; ++j) { fw[j] = words(fs[j]); fwild[j] = wildcard(fw[j]); }
  auto* c = new Csr;
  c->row_off.push_back(0);
  for (uint64_t i = 0; i < n; ++i) {
    std::string t(reinterpret_cast<const char*>(tb + toff[i]), toff[i + 1] - toff[i]);
    std::vector<Word> tw = words(t);
    bool twild = wildcard(tw);
    bool dollar = !t.empty() && t[0] == '$';
    for (uint64_t j = 0; j < nf; ++j) {
      bool hit;
      if (mode == 1) {
        // match_routes: exact route lookup of T itself (also for a wildcard
        // T), plus the wildcard filters the trie returns.
        hit = (fs[j] == t) || (!twild && fwild[j] && topic_match(t, fs[j]));
      } else {
        if (!in_trie[j] || twild) hit = false;
        else if (fwild[j]) hit = topic_match(t, fs[j]);
        else hit = dollar && tw.size() == 1 && fs[j] == t;  // do_match/2 :271-278
      }
      if (hit) c->ids.push_back(uint32_t(j));
    }
    c->row_off.push_back(c->ids.size());
  }
  return c;
}

// ---- fan-out (do_dispatch fold over the matched filters) ----
// matches: CSR of filter ids per topic; subs: CSR of subscriber ids per filter.
Csr* orc_fanout(const uint64_t* m_off, const uint32_t* m_ids, uint64_t n,
                const uint64_t* s_off, const uint32_t* s_ids) {
  auto* c = new Csr;
  c->row_off.push_back(0);
  for (uint64_t i = 0; i < n; ++i) {
    for (uint64_t k = m_off[i]; k < m_off[i + 1]; ++k) {
      uint32_t f = m_ids[k];
      for (uint64_t s = s_off[f]; s < s_off[f + 1]; ++s) c->ids.push_back(s_ids[s]);
    }
    c->row_off.push_back(c->ids.size());
  }
  return c;
}

// ---- workload generator ----
void orc_gen_filter_codes(uint64_t seed, uint64_t n, int wildcard_only, int16_t* codes) {
  gen_filter_codes(seed, n, wildcard_only, codes);
}
void orc_gen_topic_codes(uint64_t seed, uint64_t start, uint64_t n, const int16_t* fcodes, uint64_t nf,
                         int16_t* out) {
  for (uint64_t i = 0; i < n; ++i) gen_topic_codes(seed, start + i, fcodes, nf, out + i * kLevels);
}
// Render codes (n x 5) to bytes + offsets; returns total bytes.  Two-call:
// pass bytes == nullptr to size.
uint64_t orc_render_codes(const int16_t* codes, uint64_t n, uint8_t* bytes, uint64_t* off) {
  uint64_t pos = 0;
  for (uint64_t i = 0; i < n; ++i) {
    std::string s = code_string(codes + i * kLevels);
    if (off) off[i] = pos;
    if (bytes) std::memcpy(bytes + pos, s.data(), s.size());
    pos += s.size();
  }
  if (off) off[n] = pos;
  return pos;
}

}  // extern "C"
