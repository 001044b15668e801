// tests/asan/asan_host_compiler.cpp — TEST ONLY: the host index compiler
// (emqx_amd/csrc/gm_index.cpp), the overlay id mapping and the in-place
// update (gm_overlay.cpp) built with AddressSanitizer + UBSan
// and fed untrusted filter bytes: random bytes (NUL, '/', '+', '#', 0xFF),
// empty sets and empty filters, 65,535-byte filters, 5,000-level filters,
// duplicates; then random insert/delete sequences patched into a host-only
// index (its mirror is the index) with every table invariant checked after
// each update.  Never touches a device.  Built and run by
// tests/test_host_cpu.py::test_host_compiler_under_asan (`make -C
// emqx_amd/csrc asan`).
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <random>
#include <set>
#include <string>
#include <vector>

#include "../../emqx_amd/csrc/gm_internal.h"

namespace gm {
int set_err(emqx_gm_ctx*, int code, const std::string&) { return code; }  // gm_api.cpp's, minus the thread-local
// gm_match.hip's device step of an in-place update: never reached here (no
// context, so no snapshot keeps a mirror)
int apply_patch_device(emqx_gm_ctx*, void*, const void*, size_t, const std::vector<std::pair<uint64_t, uint32_t>>&,
                       const uint8_t*, const IndexView&, uint64_t, uint64_t, uint64_t, const IdShift&,
                       const std::vector<std::pair<uint64_t, uint32_t>>&) {
  return EMQX_GM_EDEVICE;
}
// gm_multi.cpp's replica helpers: a host-only index has no replicas
thread_local emqx_gm_update_stats tl_ustats{};
double now_ms() { return 0.0; }
int run_all(int K, const std::function<int(int)>& f) {
  for (int k = 0; k < K; ++k)
    if (const int rc = f(k)) return rc;
  return 0;
}
std::vector<RepTarget> rep_targets(emqx_gm_ctx*, emqx_gm_index*) { return {}; }
emqx_gm_index* replica_shell(emqx_gm_ctx*, const emqx_gm_index*) { return nullptr; }
int attach_replicas(emqx_gm_index*, std::vector<RepTarget>&, int rc) { return rc; }
void free_route(emqx_gm_route*) {}  // (gm_route.hip's: no host-only index has a route)
}

static int compile(const std::vector<std::string>& fs) {
  std::vector<uint8_t> b;
  std::vector<uint64_t> o{0};
  for (auto& f : fs) {
    b.insert(b.end(), f.begin(), f.end());
    o.push_back(b.size());
  }
  b.resize(b.size() + 64, 0);
  std::vector<uint32_t> perm(fs.size() + 1);
  emqx_gm_index_info_t info{};
  const int rc = gm::build_index(nullptr, b.data(), o.data(), fs.size(), nullptr, nullptr, perm.data(), nullptr,
                                 &info);
  if (rc) return rc;
  // ids are ranks of the unique filters: perm is a valid id for every input
  for (size_t i = 0; i < fs.size(); ++i)
    if (perm[i] >= info.n_filters) return -100;
  return 0;
}

// ---- in-place update: random sequences on a host-only index ---------------
namespace {
using namespace gm;

std::vector<std::string> split_words(const std::string& f) {
  std::vector<std::string> w;
  size_t a = 0;
  for (size_t i = 0; i <= f.size(); ++i)
    if (i == f.size() || f[i] == '/') {
      w.push_back(f.substr(a, i - a));
      a = i + 1;
    }
  return w;
}
uint32_t v_dict_find(const IndexView& v, const std::string& w) {
  const uint8_t* p = reinterpret_cast<const uint8_t*>(w.data());
  const uint64_t head = word_head_host(p, w.size());
  for (uint64_t s = dict_slot(dict_hash_host(p, w.size()), v.dict_mask);; s = (s + 1) & v.dict_mask) {
    const DictSlot& d = v.dict[s];
    if (d.len == DICT_EMPTY_LEN) return NONE;
    if (d.len == w.size() && d.head == head &&
        (w.size() <= 8 || std::memcmp(v.arena + d.word + 8, p + 8, w.size() - 8) == 0))
      return d.word;
  }
}
uint32_t v_edge_get(const IndexView& v, uint32_t depth, uint32_t parent, uint32_t wid) {
  const int d = edge_depth(depth);
  const EdgeSlot* tab = v.edges + v.etab_off[d];
  const uint64_t key = edge_key(parent, wid), mask = v.etab_mask[d];
  for (uint64_t s = edge_slot(key, mask);; s = (s + 1) & mask) {
    if (tab[s].key == key) return tab[s].child;
    if (tab[s].key == EDGE_EMPTY) return NONE;
  }
}
// the device lookup (gm_match.hip hot_resolve): with rh, an absent key stops
// at the first resident nearer its own home than the probe
uint32_t v_hot_lookup(const IndexView& v, int t, uint64_t key, bool rh) {
  const uint64_t cap = v.hot_cap[t];
  if (!cap) return NONE;
  if (v.mph_cap[t]) return hot_lookup_host(v, v.hot, v.mph_word, t, key);  // a perfect-hash table
  const HotSlot* tab = v.hot + v.hot_off[t];
  uint64_t s = hot_slot(key, cap), dist = 0;
  for (uint64_t step = 0; step < cap; ++step) {
    if (tab[s].key == key) return uint32_t(s);
    if (tab[s].key == EDGE_EMPTY) return NONE;
    if (rh) {
      const uint64_t h = hot_slot(tab[s].key, cap);
      if ((s >= h ? s - h : s + cap - h) < dist) return NONE;
    }
    s = s + 1 == cap ? 0 : s + 1;
    ++dist;
  }
  return NONE;
}
bool is_wild(const std::vector<std::string>& ws) {
  for (auto& w : ws)
    if (w == "+" || w == "#") return true;
  return false;
}

// Every table invariant of a (patched) index against the filter set it holds.
int verify(const emqx_gm_index* idx, const std::set<std::string>& cur, const char* what) {
  const IndexView& v = idx->view;
  int bad = 0;
  auto fail = [&](const std::string& m) {
    if (bad++ < 5) std::fprintf(stderr, "patch verify (%s): %s\n", what, m.c_str());
  };
  if (idx->info.n_filters != cur.size()) fail("n_filters");
  uint32_t f = 0;
  for (const std::string& flt : cur) {
    uint64_t gl;
    const uint8_t* gp = idx->ft.at(f, &gl);
    const std::string got(reinterpret_cast<const char*>(gp), gl);
    if (got != flt) fail("filter bytes of id " + std::to_string(f));
    const auto ws = split_words(flt);
    const bool wild = is_wild(ws);
    // the level trie (slow path, literal lookups)
    uint32_t node = 0;
    for (size_t i = 0; i < ws.size(); ++i) {
      const uint32_t wid = v_dict_find(v, ws[i]);
      const uint32_t ch = wid == NONE ? NONE : v_edge_get(v, uint32_t(i), node, wid);
      if (ch == NONE) {
        fail("v1 path of " + flt);
        node = NONE;
        break;
      }
      if (i + 1 == ws.size() && ws[i] == "#") {
        if (v.nodes[node].hash_filter != f || v.nodes[ch & REF_MASK].end_filter != f) fail("v1 '#' of " + flt);
        node = NONE;
        break;
      }
      node = ch & REF_MASK;
    }
    if (node != NONE && v.nodes[node].end_filter != f) fail("v1 end of " + flt);
    // the hot path (walk kernels)
    uint32_t kind = 0, slot = 0;  // 0 root, 1 slot, 2 inline
    int table = 0;
    for (size_t i = 0; i < ws.size(); ++i) {
      const HotSlot* P = kind ? &v.hot[v.hot_off[table] + slot] : nullptr;
      const uint32_t hf = kind == 1 ? P->hf : kind == 2 ? P->p_hf : 0u;
      const uint32_t sig = kind == 0 ? v.root_sig : kind == 1 ? hot_sig(P->hf, P->sig) : P->p_sig;
      if (kind == 1 && (hf & HOT_CHAIN) && !(i + 1 == ws.size() && ws[i] == "#")) {
        // a chain node: a filter through it is its own '#' filter or its one tail (s1 [s2] then F)
        const uint32_t lc = P->p_sig == NONE ? 1u : 2u;
        if (ws.size() - i != lc || v_dict_find(v, ws[i]) != P->sig ||
            (lc == 2 && v_dict_find(v, ws[i + 1]) != P->p_sig) || P->p_end != (f | (wild ? END_WILD : 0u)) ||
            (P->hf & HOT_PLUS))
          fail("chain node on the path of " + flt);
      }
      if (i + 1 == ws.size() && ws[i] == "#") {
        const uint32_t id = kind == 0 ? v.root_hash : (hf & HF_MASK);
        if (id != f) fail("hot '#' of " + flt);
        kind = 9;
        break;
      }
      const uint32_t wid = v_dict_find(v, ws[i]);
      const bool plus = ws[i] == "+";
      const bool pflag = kind == 0 ? (v.root_flags & HOT_PLUS) != 0 : (hf & HOT_PLUS) != 0;
      if (plus && !pflag) fail("HOT_PLUS on the parent in " + flt);
      if (plus && plus_inline(uint32_t(i), kind == 1)) {
        kind = 2;
        continue;
      }
      if (!plus && !(sig & sig_bit(wid))) fail("sig bit in " + flt);
      const uint32_t hid = kind == 0 ? 0u : kind == 1 ? slot : (slot | HOT_INLINE);
      const int t = hot_table(uint32_t(i + 1));
      const uint64_t key = hot_key(hid, wid, uint32_t(i));
      if (!plus && v.efilt_mask[t]) {
        const uint32_t fh = edge_filter_hash(key), fb = edge_filter_bits(fh);
        if ((v.efilt[v.efilt_off[t] + edge_filter_word(fh, v.efilt_mask[t])] & fb) != fb) fail("efilt in " + flt);
      }
      const uint32_t s = v_hot_lookup(v, t, key, false);
      if (s == NONE) {
        fail("hot slot of " + flt);
        kind = 9;
        break;
      }
      if (((v.rh_mask >> t) & 1u) && v_hot_lookup(v, t, key, true) != s) fail("Robin Hood exit loses " + flt);
      kind = 1;
      slot = s;
      table = t;
    }
    if (kind == 1 || kind == 2) {
      const HotSlot& H = v.hot[v.hot_off[table] + slot];
      const uint32_t e = kind == 1 ? H.end_filter : H.p_end;
      if (e != (f | (wild ? END_WILD : 0u))) fail("hot end of " + flt);
    }
    ++f;
  }
  // REF_X: an edge / '+' reference carries its child's has-exact flag
  for (int d = 0; d < EDGE_DEPTHS; ++d)
    for (uint64_t s = 0; s <= v.etab_mask[d]; ++s) {
      const EdgeSlot& e = v.edges[v.etab_off[d] + s];
      if (e.key == EDGE_EMPTY) continue;
      const bool x = (v.nodes[e.child & REF_MASK].flags & NF_HAS_EXACT) != 0;
      if (((e.child & REF_X) != 0) != x) fail("edge REF_X");
    }
  for (uint32_t i = 0; i < v.n_nodes; ++i) {
    const Node& n = v.nodes[i];
    if (n.plus_child != NONE && ((n.plus_child & REF_X) != 0) != ((v.nodes[n.plus_child & REF_MASK].flags & NF_HAS_EXACT) != 0))
      fail("plus REF_X");
    for (uint32_t x : {n.end_filter, n.hash_filter})
      if (x != NONE && x >= cur.size()) fail("stale node filter id");
  }
  // no filter id outside the set (deleted ones cleared, the rest renumbered)
  for (int t = 0; t < HOT_TABLES; ++t)
    for (uint64_t s = 0; s < v.hot_cap[t]; ++s) {
      const HotSlot& h = v.hot[v.hot_off[t] + s];
      if (h.key == EDGE_EMPTY) continue;
      for (uint32_t x : {h.end_filter, h.p_end})
        if (x != NONE && (x & ID_MASK) >= cur.size()) fail("stale hot end id");
      for (uint32_t x : {h.hf, h.p_hf})
        if ((x & HF_MASK) != HF_NONE && (x & HF_MASK) >= cur.size()) fail("stale hot hf id");
      if ((h.p_hf & HOT_CHAIN) || ((h.hf & HOT_CHAIN) && (h.p_hf != HF_NONE || (h.hf & HOT_PLUS))))
        fail("chain fields");
    }
  return bad;
}

std::string rand_filter(std::mt19937_64& rng, int max_depth) {
  static const char* W[] = {"a", "b", "c", "", "$x", "long-word-over-8-bytes", "w1", "w22", "+"};
  const int n = 1 + int(rng() % max_depth);
  std::string f;
  for (int i = 0; i < n; ++i) f += (i ? "/" : "") + std::string(W[rng() % 9]);
  if (rng() % 3 == 0) f += "/#";
  if (rng() % 40 == 0) f = "#";
  return f;
}

emqx_gm_index* host_build(const std::set<std::string>& fs) {
  std::vector<uint8_t> b;
  std::vector<uint64_t> o{0};
  for (auto& f : fs) {
    b.insert(b.end(), f.begin(), f.end());
    o.push_back(b.size());
  }
  b.resize(b.size() + 64, 0);
  emqx_gm_index* idx = nullptr;
  if (gm::build_index(nullptr, b.data(), o.data(), fs.size(), nullptr, nullptr, nullptr, &idx)) return nullptr;
  return idx;
}

emqx_gm_index* host_update(emqx_gm_index* prev, const std::vector<std::pair<std::string, bool>>& ops) {
  std::vector<uint8_t> b, k;
  std::vector<uint64_t> o{0};
  for (auto& op : ops) {
    b.insert(b.end(), op.first.begin(), op.first.end());
    o.push_back(b.size());
    k.push_back(op.second ? 1 : 0);
  }
  b.resize(b.size() + 64, 0);
  k.push_back(0);
  emqx_gm_index* out = nullptr;
  if (gm::update_index(nullptr, prev, b.data(), o.data(), k.data(), ops.size(), &out)) return nullptr;
  return out;
}

// gm_filters.h FilterTable: random delete / insert batches against a std::set,
// with a small compaction threshold so shared-base tables, deltas over deltas
// and compactions all occur; every id, every rank_of and the in-order walk checked.
int filter_table_check() {
  int bad = 0;
  std::mt19937_64 rng(11);
  std::set<std::string> ref;
  for (int i = 0; i < 300; ++i) ref.insert(rand_filter(rng, 4));
  auto sf = std::make_shared<SortedFilters>();
  for (auto& f : ref) sf->push(reinterpret_cast<const uint8_t*>(f.data()), f.size());
  FilterTable ft;
  ft.set_base(sf);
  for (int round = 0; round < 200; ++round) {
    std::vector<uint64_t> dels;
    std::set<std::string> adds, gone;
    const int nd = int(rng() % 6), na = int(rng() % 6);
    for (int i = 0; i < nd && !ref.empty(); ++i) {
      auto it = ref.begin();
      std::advance(it, rng() % ref.size());
      gone.insert(*it);
    }
    for (auto& g : gone) dels.push_back(uint64_t(std::distance(ref.begin(), ref.find(g))));
    std::sort(dels.begin(), dels.end());
    for (int i = 0; i < na; ++i) {
      std::string f = rand_filter(rng, 4);
      if (!ref.count(f) || gone.count(f)) adds.insert(f);  // a deleted filter may come back
    }
    for (auto& g : gone) ref.erase(g);
    for (auto& a : adds) ref.insert(a);
    ft = ft.apply(dels, adds, 8);
    if (ft.size() != ref.size()) {
      if (bad++ < 5) std::fprintf(stderr, "filter table: size %llu vs %zu\n", (unsigned long long)ft.size(), ref.size());
      continue;
    }
    uint64_t r = 0;
    for (auto& f : ref) {
      uint64_t l;
      const uint8_t* p = ft.at(r, &l);
      bool found;
      const uint64_t rk = ft.rank_of(reinterpret_cast<const uint8_t*>(f.data()), f.size(), &found);
      if (std::string(reinterpret_cast<const char*>(p), l) != f || rk != r || !found)
        if (bad++ < 5) std::fprintf(stderr, "filter table: id %llu\n", (unsigned long long)r);
      ++r;
    }
    std::string absent = rand_filter(rng, 4) + "/zz";
    bool found;
    const uint64_t rk = ft.rank_of(reinterpret_cast<const uint8_t*>(absent.data()), absent.size(), &found);
    if (found || rk != uint64_t(std::distance(ref.begin(), ref.lower_bound(absent))))
      if (bad++ < 5) std::fprintf(stderr, "filter table: absent rank\n");
    uint64_t walked = 0;
    auto it = ref.begin();
    ft.for_each([&](uint64_t id, const uint8_t* p, uint64_t l) {
      if (id != walked || it == ref.end() || std::string(reinterpret_cast<const char*>(p), l) != *it)
        if (bad++ < 5) std::fprintf(stderr, "filter table: walk at %llu\n", (unsigned long long)id);
      ++walked;
      if (it != ref.end()) ++it;
    });
    if (walked != ref.size() && bad++ < 5) std::fprintf(stderr, "filter table: walk length\n");
  }
  return bad;
}

int patch_sequences() {
  int bad = 0;
  std::mt19937_64 rng(7);
  for (int run = 0; run < 3; ++run) {
    std::set<std::string> cur;
    const int depth = run == 2 ? 22 : 6;  // run 2: the shared last tables
    for (int i = 0; i < 400; ++i) cur.insert(rand_filter(rng, depth));
    emqx_gm_index* idx = host_build(cur);
    if (!idx) return 1;
    bad += verify(idx, cur, "build");
    for (int round = 0; round < 40; ++round) {
      std::vector<std::pair<std::string, bool>> ops;
      const int n = round % 13 == 12 ? 3000 : 1 + int(rng() % 80);  // now and then past the headroom
      for (int i = 0; i < n; ++i) {
        if (!cur.empty() && rng() % 5 < 2) {
          auto it = cur.begin();
          std::advance(it, rng() % cur.size());
          const std::string f = *it;
          const bool ins = rng() % 4 == 0;  // mostly deletes
          ops.emplace_back(f, ins);
          if (!ins) cur.erase(f);
        } else {
          const std::string f = rand_filter(rng, depth);
          const bool ins = rng() % 5 != 0;  // some deletes of absent filters
          ops.emplace_back(f, ins);
          if (ins) cur.insert(f);
          else cur.erase(f);
        }
      }
      emqx_gm_index* nx = host_update(idx, ops);
      if (!nx) {
        std::fprintf(stderr, "host update failed (run %d round %d)\n", run, round);
        return bad + 1;
      }
      if (nx != idx) gm::free_index(idx);  // host-only: the old view shares the moved mirror
      else nx->refs.fetch_sub(1);
      idx = nx;
      bad += verify(idx, cur, "update");
    }
    gm::free_index(idx);
  }
  return bad;
}


// gm_filters.h SubTable: random batches of (id, new count) and (id, mark)
// against plain vectors, with deltas over deltas and compactions (n = 5,000:
// compaction past 4,096 touched ids); every offset, count and mark checked,
// and the running changes the device shift kernel consumes.
int sub_table_check() {
  int bad = 0;
  std::mt19937_64 rng(13);
  const uint64_t n = 5000;
  std::vector<uint64_t> cnt(n), off(n + 1, 0);
  std::vector<uint8_t> mark(n);
  for (uint64_t f = 0; f < n; ++f) cnt[f] = rng() % 4;
  for (uint64_t f = 0; f < n; ++f) off[f + 1] = off[f] + cnt[f];
  for (uint64_t f = 0; f < n; ++f) mark[f] = cnt[f] == 0;  // a built index: no subscribers = route-only
  gm::SubTable t(off, {});
  for (int round = 0; round < 300; ++round) {
    std::set<uint32_t> ids;
    const int k = 1 + int(rng() % 40);
    for (int i = 0; i < k; ++i) ids.insert(uint32_t(rng() % n));
    std::vector<std::pair<uint32_t, uint64_t>> c;
    std::vector<std::pair<uint32_t, uint8_t>> m;
    for (uint32_t id : ids) {
      cnt[id] = rng() % 6;
      mark[id] = uint8_t(rng() % 2);
      c.emplace_back(id, cnt[id]);
      m.emplace_back(id, mark[id]);
    }
    const gm::SubTable prev = t;
    t = t.apply(c, m);
    for (uint64_t f = 0; f < n; ++f) off[f + 1] = off[f] + cnt[f];
    for (uint64_t f = 0; f <= n; ++f)
      if (t.off(f) != off[f] && bad++ < 5) std::fprintf(stderr, "sub table: off %llu\n", (unsigned long long)f);
    for (uint64_t f = 0; f < n; ++f) {
      if (t.count(f) != cnt[f] && bad++ < 5) std::fprintf(stderr, "sub table: count %llu\n", (unsigned long long)f);
      if (t.pinned(f) != (mark[f] != 0) && bad++ < 5) std::fprintf(stderr, "sub table: mark %llu\n", (unsigned long long)f);
    }
    if (t.total() != off[n] && bad++ < 5) std::fprintf(stderr, "sub table: total\n");
    // what shift_subs_device derives from prev: new off = prev off + the batch's changes below
    int64_t run = 0;
    auto it = ids.begin();
    for (uint64_t f = 0; f <= n; ++f) {
      while (it != ids.end() && *it < f) {
        run += int64_t(cnt[*it]) - int64_t(prev.count(*it));
        ++it;
      }
      if (uint64_t(int64_t(prev.off(f)) + run) != off[f] && bad++ < 5)
        std::fprintf(stderr, "sub table: shifted off %llu\n", (unsigned long long)f);
    }
  }
  if (t.offsets() != off && bad++ < 5) std::fprintf(stderr, "sub table: materialized offsets\n");
  return bad;
}

// ---- index images (gm_image.cpp): validate_image / import_host_part fed a
// valid image cut at every section boundary, with byte flips anywhere in its
// header and host sections, and with counts and offsets rewritten (the
// checksum resealed, as a crafted image would carry): every cut and flip is
// refused with EMQX_GM_EINVAL, every rewritten oversized count too, and
// nothing reads out of bounds (ASan) -- what index_import checks before it
// touches a device.
int image_fuzz() {
  int bad = 0;
  std::mt19937_64 rng(5);
  std::set<std::string> fs;
  for (int i = 0; i < 500; ++i) fs.insert(rand_filter(rng, 6));
  emqx_gm_index* idx = host_build(fs);
  if (!idx) return 1;
  uint64_t size = 0;
  if (gm::index_export(nullptr, idx, 0, nullptr, &size)) return 1;
  std::vector<uint8_t> img(size);
  if (gm::index_export(nullptr, idx, 0, img.data(), &size)) return 1;
  auto attempt = [&](const std::vector<uint8_t>& b, uint64_t sz, bool have_blob) {
    emqx_gm_index t;
    std::string why;
    const int rc = gm::import_host_part(b.data(), sz, have_blob, &t, &why);
    if (rc == 0 && t.ft.size() != t.info.n_filters) ++bad;
    delete t.mirror;
    t.mirror = nullptr;
    return rc;
  };
  if (attempt(img, size, false) != 0) {
    std::fprintf(stderr, "image: the intact image is refused\n");
    ++bad;
  }
  // cuts: every section boundary (and one byte either side), then random sizes
  std::vector<uint64_t> cuts = {0, 1, 8, 100, sizeof(uint64_t) * 3};
  for (int k = 0; k < 6; ++k) {
    const uint64_t o = *gm::image_field(img.data(), "sec_off" + std::to_string(k));
    cuts.insert(cuts.end(), {o - 1, o, o + 1});
  }
  for (int i = 0; i < 200; ++i) cuts.push_back(rng() % size);
  for (uint64_t c : cuts) {
    if (c >= size) continue;
    std::vector<uint8_t> b(img.begin(), img.begin() + c);
    b.resize(std::max<uint64_t>(c, 1));
    if (attempt(b, c, false) != EMQX_GM_EINVAL) {
      std::fprintf(stderr, "image: a cut at %llu is not refused\n", (unsigned long long)c);
      ++bad;
    }
  }
  // byte flips: the header and the host sections (the checksum covers both)
  const uint64_t host_end = *gm::image_field(img.data(), "sec_off5");
  for (int i = 0; i < 3000; ++i) {
    std::vector<uint8_t> b(img);
    const uint64_t at = i < 1500 ? rng() % 2048 : rng() % host_end;
    b[at] ^= uint8_t(1 + rng() % 255);
    if (attempt(b, size, false) != EMQX_GM_EINVAL) {
      std::fprintf(stderr, "image: a flip at %llu is not refused\n", (unsigned long long)at);
      ++bad;
    }
  }
  // rewritten counts and offsets, resealed: oversized ones are refused; any
  // other value may be accepted or refused but is never read out of bounds
  const char* names[] = {"dev_bytes", "flen_off", "n_filters", "ft_bytes", "gmap_n", "soff_n", "pinned_n",
                         "blob_in_image", "total_bytes", "info.n_filters", "info.n_subs", "view.dict_mask",
                         "view.hot_cap1", "view.hot_off2", "view.etab_mask0", "mirror.blob_size", "mirror.nodes_cap",
                         "mirror.arena_cap", "mirror.flen_cap", "mirror.o_hot", "mirror.hot_used1",
                         "mirror.edge_used0", "sec_off0", "sec_off1", "sec_off2", "sec_off3", "sec_off4", "sec_off5",
                         "ptr_off0", "ptr_off1", "ptr_off2", "ptr_off3", "ptr_off4", "ptr_off8", "ptr_off9",
                         "ptr_off10"};
  for (const char* nm : names) {
    const uint64_t orig = *gm::image_field(img.data(), nm);
    const uint64_t vals[] = {orig + size, orig * 2 + 1, ~0ull, ~0ull / 2, 1ull << 40, orig + 1, orig ? orig - 1 : 7, 0};
    for (int vi = 0; vi < 8; ++vi) {
      std::vector<uint8_t> b(img);
      *gm::image_field(b.data(), nm) = vals[vi];
      gm::image_reseal(b.data(), size);
      const int rc = attempt(b, size, false);
      // (the oversized values: past the image / the blob / 2^40; a host-only
      // index has no subscriber tables, so its info.n_subs is a bare count)
      const bool oversized = vi == 0 || (vi >= 2 && vi <= 4);
      // (~0 in a ptr_off field is the encoding of an absent table)
      const bool null_ptr = std::string(nm).compare(0, 7, "ptr_off") == 0 && vals[vi] == ~0ull;
      if (oversized && !null_ptr && vals[vi] != orig && rc != EMQX_GM_EINVAL && std::string(nm) != "info.n_subs") {
        std::fprintf(stderr, "image: %s = %llu is not refused\n", nm, (unsigned long long)vals[vi]);
        ++bad;
      }
    }
  }
  // the view's u32 counts (nodes, edge filter and MPH bucket extents) oversized
  for (int which = 0; which < 3; ++which)
    for (int t = 0; t < 16; ++t) {
      std::vector<uint8_t> b(img);
      gm::image_view_set_u32(b.data(), which, t, 0x7FFFFFFFu);
      gm::image_reseal(b.data(), size);
      if (attempt(b, size, false) != EMQX_GM_EINVAL && !(which == 2 && !gm::image_view_u32(img.data(), which, t))) {
        std::fprintf(stderr, "image: view count %d/%d oversized is not refused\n", which, t);
        ++bad;
      }
      if (which == 0) break;
    }
  gm::free_index(idx);
  return bad;
}
// ---- the parallel trie build (gm_index.cpp: runs of filters with one first
// word, built apart and merged in filter order) and the hot tables' one-sweep
// Robin Hood placement: the image of a host-only index -- every table -- is
// the same byte for byte whether the trie was built as one run
// (GM_TRIE_RUNS=1, the serial walk) or as 2, 3, 7 or 64 runs, and whether the
// hot tables were swept or filled by RH insertion key by key
// (GM_HOT_RH_INSERT: the same sizes; its ties among keys of one home differ),
// on random sets over separators, wildcards, NULs and empty words (small
// tables: keys wrap past the end); with GM_INDEX_VERIFY (set by the test)
// every Robin Hood table is checked in order as it is built.
int trie_runs_check() {
  int bad = 0;
  std::mt19937_64 rng(11);
  const char alpha[] = {'a', 'b', '/', '+', '#', '\0', 'z', 'c'};
  auto image = [&](const std::set<std::string>& fs, const char* runs, std::vector<uint8_t>& img) {
    const bool insert = std::strcmp(runs, "insert") == 0;  // the hot tables by RH insertion, key by key
    setenv("GM_TRIE_RUNS", insert ? "1" : runs, 1);
    if (insert) setenv("GM_HOT_RH_INSERT", "1", 1);
    emqx_gm_index* idx = host_build(fs);
    unsetenv("GM_TRIE_RUNS");
    unsetenv("GM_HOT_RH_INSERT");
    if (!idx) return false;
    uint64_t size = 0;
    bool ok = gm::index_export(nullptr, idx, 0, nullptr, &size) == 0;
    img.assign(size, 0);
    ok = ok && gm::index_export(nullptr, idx, 0, img.data(), &size) == 0;
    gm::free_index(idx);
    return ok;
  };
  for (int round = 0; round < 24; ++round) {
    std::set<std::string> fs;
    const int n = 50 + int(rng() % 3000);
    for (int i = 0; i < n; ++i) {
      if (round % 2) {
        fs.insert(rand_filter(rng, 6));
      } else {
        std::string f;
        const int len = int(rng() % 24);
        for (int k = 0; k < len; ++k) f.push_back(alpha[rng() % sizeof(alpha)]);
        fs.insert(f);
      }
    }
    std::vector<uint8_t> one, many;
    if (!image(fs, "1", one)) {
      ++bad;
      continue;
    }
    // (the header holds the build's own host pointers in its view: compared
    // from the end of the header -- host sections and every table)
    uint32_t hb = 0;
    std::memcpy(&hb, one.data() + 12, 4);
    // (RH insertion orders keys of one home by history: the same sizes and a
    // valid Robin Hood layout -- GM_INDEX_VERIFY, set by the test -- not the same bytes)
    for (const char* runs : {"2", "3", "7", "64", "insert"}) {
      const bool bytes = std::strcmp(runs, "insert") != 0;
      if (!image(fs, runs, many) || many.size() != one.size() || hb > one.size() ||
          (bytes && !std::equal(one.begin() + hb, one.end(), many.begin() + hb))) {
        size_t d0 = hb;
        while (d0 < one.size() && d0 < many.size() && one[d0] == many[d0]) ++d0;
        std::fprintf(stderr, "trie runs %s: image differs (round %d, %zu filters; sizes %zu/%zu, first diff %zu)\n",
                     runs, round, fs.size(), one.size(), many.size(), d0);
        ++bad;
      }
    }
  }
  return bad;
}
}  // namespace

int main() {
  std::mt19937_64 rng(42);
  const char alpha[] = {'a', 'b', '/', '+', '#', '\0', '\xff', '$', 'z'};
  int bad = 0;
  auto check = [&](const char* what, const std::vector<std::string>& fs) {
    const int rc = compile(fs);
    if (rc) {
      std::fprintf(stderr, "%s: rc %d\n", what, rc);
      ++bad;
    }
  };
  check("empty set", {});
  check("one empty filter", {""});
  check("separators only", {"/", "//", "///", "+", "#", "+/#", "/+/", "#/#"});
  for (int round = 0; round < 200; ++round) {
    std::vector<std::string> fs;
    const int n = int(rng() % 300);
    for (int i = 0; i < n; ++i) {
      std::string f;
      const int len = int(rng() % 40);
      for (int k = 0; k < len; ++k) f.push_back(alpha[rng() % sizeof(alpha)]);
      fs.push_back(f);
      if (rng() % 5 == 0) fs.push_back(f);  // duplicates
    }
    check("random", fs);
  }
  check("65535-byte filters", {std::string(65535, 'w'), std::string(65534, 'w') + "#",
                               std::string(32767, 'a') + "/" + std::string(32767, 'b')});
  std::string deep;
  for (int i = 0; i < 5000; ++i) deep += (i ? "/" : "") + std::string(1, char('a' + i % 26));
  check("5000 levels", {deep, deep + "/#", "+/" + deep});
  std::string nul_laden("a\0b/\0/+\0", 8);
  check("NUL-laden", {nul_laden, std::string("\0", 1), std::string("\0/#", 3)});

  // overlay id mapping over a host-only base (gm_overlay.cpp overlay_filter)
  {
    emqx_gm_index base;
    std::vector<std::string> fs = {"a", "a/+", "b/#", "c", "d/e/f", "x"};
    {
      auto sf = std::make_shared<gm::SortedFilters>();
      for (auto& f : fs) sf->push(reinterpret_cast<const uint8_t*>(f.data()), f.size());
      base.ft.set_base(sf);
    }
    base.info.n_filters = fs.size();
    emqx_gm_index ov;
    ov.ov = new gm::OverlayState;
    ov.ov->base = &base;
    ov.ov->tomb = {1, 4};          // "a/+" and "d/e/f" deleted
    ov.ov->ins = {3, 6};           // "bb" sorts before "c" (3 base filters before it), "y" after all
    ov.ov->dgid = {2, 5};          // final ids: a b/# bb c x y
    const std::string d = "bby";
    ov.ov->dbytes.assign(d.begin(), d.end());
    ov.ov->doff = {0, 2, 3};
    ov.info.n_filters = 6;
    const char* want[] = {"a", "b/#", "bb", "c", "x", "y"};
    for (uint32_t id = 0; id < 6; ++id) {
      const uint8_t* p = nullptr;
      uint64_t len = 0;
      if (gm::overlay_filter(&ov, id, &p, &len) || std::string(reinterpret_cast<const char*>(p), len) != want[id]) {
        std::fprintf(stderr, "overlay id %u\n", id);
        ++bad;
      }
    }
    const uint8_t* p = nullptr;
    uint64_t len = 0;
    if (gm::overlay_filter(&ov, 6, &p, &len) != EMQX_GM_EINVAL) ++bad;  // out of range
    ov.ov->base = nullptr;
    delete ov.ov;
    ov.ov = nullptr;
  }
  bad += filter_table_check();
  bad += patch_sequences();
  bad += image_fuzz();
  bad += sub_table_check();
  bad += trie_runs_check();
  std::printf(bad ? "ASAN_HOST_CHECK_FAILED %d\n" : "ASAN_HOST_CHECK_OK\n", bad);
  return bad ? 1 : 0;
}
