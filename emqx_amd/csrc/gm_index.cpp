// gm_index.cpp — host compiler: filter set -> flat level trie in HBM.
//
// Input is the set of route filters (emqx_route topics; wildcard ones are the
// emqx_trie entries, apps/emqx/src/emqx_router.erl:112-125) plus, optionally,
// each filter's subscriber list (the emqx_subscriber bag with the shard
// indirection of emqx_broker.erl:147-165 / 445-454 already flattened).
//
// Filter ids are the lexicographic rank of the filter bytes (Erlang binary
// order), so a row sorted by id equals lists:sort/1 of the reference result.
//
// Layout (gm_common.h): nodes are numbered breadth-first so the hot upper
// levels of the trie are contiguous in HBM and stay resident in L2/MALL.
#include <algorithm>
#include <array>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <numeric>
#include <string_view>
#include <thread>
#include <unordered_map>

#include "gm_internal.h"

namespace gm {
namespace {

struct ViewHash {
  size_t operator()(std::string_view s) const {
    return size_t(hash_word_host(reinterpret_cast<const uint8_t*>(s.data()), s.size()));
  }
};

uint64_t next_pow2(uint64_t x) {
  uint64_t p = 64;
  while (p < x) p <<= 1;
  return p;
}

// Open-addressing (u64 key -> u32) map with the same slot function as the
// device edge table, so the host table IS the device table.
struct EdgeMap {
  std::vector<EdgeSlot> slots;
  uint64_t mask = 0, used = 0;
  explicit EdgeMap(uint64_t expect) {
    uint64_t cap = next_pow2(expect * 2 + 2);
    slots.assign(cap, EdgeSlot{EDGE_EMPTY, NONE, 0});
    mask = cap - 1;
  }
  void grow() {
    std::vector<EdgeSlot> old;
    old.swap(slots);
    uint64_t cap = old.size() * 2;
    slots.assign(cap, EdgeSlot{EDGE_EMPTY, NONE, 0});
    mask = cap - 1;
    used = 0;
    for (auto& s : old)
      if (s.key != EDGE_EMPTY) put(s.key, s.child);
  }
  uint32_t get(uint64_t key) const {
    for (uint64_t s = edge_slot(key, mask);; s = (s + 1) & mask) {
      if (slots[s].key == key) return slots[s].child;
      if (slots[s].key == EDGE_EMPTY) return NONE;
    }
  }
  void put(uint64_t key, uint32_t child) {
    if ((used + 1) * 2 > slots.size()) grow();
    for (uint64_t s = edge_slot(key, mask);; s = (s + 1) & mask) {
      if (slots[s].key == EDGE_EMPTY) {
        slots[s] = EdgeSlot{key, child, 0};
        ++used;
        return;
      }
      if (slots[s].key == key) {
        slots[s].child = child;
        return;
      }
    }
  }
};

// (a plain aggregate, so that a vector of 10^8 of them can be left unwritten
// until the merge fills it: kNewNode is a node's starting value)
struct HNode {
  uint32_t plus_child, hash_child, end_filter, flags;
  uint32_t depth;
  uint32_t parent, word;  // incoming edge
  uint32_t sig;           // exact-child word signature (HotSlot::sig)
  uint8_t kind;           // incoming edge: 0 exact, 1 '+', 2 '#'
};
constexpr HNode kNewNode{NONE, NONE, NONE, 0u, 0u, NONE, NONE, 0u, 0u};

bool less_bytes(const uint8_t* a, uint64_t la, const uint8_t* b, uint64_t lb) {
  int c = std::memcmp(a, b, std::min(la, lb));
  if (c) return c < 0;
  return la < lb;
}

// f(begin, end) over [0, n) in one contiguous range per thread (small n: one call).
template <class F> void parallel_for(uint64_t n, F f) {
  const unsigned T = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  if (n < (1u << 16) || T == 1) {
    f(uint64_t(0), n);
    return;
  }
  std::vector<std::thread> th;
  for (unsigned k = 1; k < T; ++k) th.emplace_back([&, k] { f(n * k / T, n * (k + 1) / T); });
  f(uint64_t(0), n / T);
  for (auto& t : th) t.join();
}

// A parallel merge sort: T chunks sorted with std::sort on T threads, then
// rounds of pairwise merges, each merge cut into pieces along its merge path
// (co-ranks by binary search) so every round keeps all T threads busy.
template <class V, class Cmp> void par_sort(V& v, Cmp cmp) {
  using K = typename V::value_type;
  const size_t n = v.size();
  const unsigned T = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  if (n < 200000 || T == 1) {
    std::sort(v.begin(), v.end(), cmp);
    return;
  }
  std::vector<size_t> b(T + 1);
  for (unsigned k = 0; k <= T; ++k) b[k] = n * k / T;
  {
    std::vector<std::thread> th;
    for (unsigned k = 0; k < T; ++k) th.emplace_back([&, k] { std::sort(v.begin() + b[k], v.begin() + b[k + 1], cmp); });
    for (auto& t : th) t.join();
  }
  std::vector<K, DefaultInit<K>> tmp(n);
  K* src = v.data();
  K* dst = tmp.data();
  // how many of a's first elements the first d outputs of merge(a, b) take (a first on ties)
  auto corank = [&](const K* a, size_t na, const K* bb, size_t nb, size_t d) {
    size_t lo = d > nb ? d - nb : 0, hi = std::min(d, na);
    while (lo < hi) {
      const size_t i = (lo + hi) / 2, j = d - i;
      if (j > 0 && i < na && !cmp(bb[j - 1], a[i])) lo = i + 1;
      else hi = i;
    }
    return lo;
  };
  for (size_t width = 1; width < T; width *= 2) {
    std::vector<std::function<void()>> jobs;
    for (size_t k = 0; k < T; k += 2 * width) {
      const size_t lo = b[k], mid = b[std::min<size_t>(k + width, T)], hi = b[std::min<size_t>(k + 2 * width, T)];
      const unsigned P = unsigned(std::min<size_t>(T, 2 * width));  // threads per merge
      for (unsigned p = 0; p < P; ++p)
        jobs.emplace_back([&, lo, mid, hi, P, p] {
          const K* a = src + lo;
          const K* bb = src + mid;
          const size_t na = mid - lo, nb = hi - mid, tot = na + nb;
          const size_t d0 = tot * p / P, d1 = tot * (p + 1) / P;
          const size_t i0 = corank(a, na, bb, nb, d0), i1 = corank(a, na, bb, nb, d1);
          std::merge(a + i0, a + i1, bb + (d0 - i0), bb + (d1 - i1), dst + lo + d0, cmp);
        });
    }
    std::vector<std::thread> th;
    for (size_t j = 1; j < jobs.size(); ++j) th.emplace_back(jobs[j]);
    jobs[0]();
    for (auto& t : th) t.join();
    std::swap(src, dst);
  }
  if (src != v.data()) std::copy(src, src + n, v.data());
}

// Parallel sort of filter indices by bytes: (big-endian first 8 bytes, index)
// pairs, so most comparisons are one integer compare on contiguous memory and
// only equal prefixes compare the filters' bytes.
void sort_filters_impl(std::vector<uint32_t>& ord, const uint8_t* fb, const uint64_t* fo) {
  const size_t n = ord.size();
  struct K {
    uint64_t key;
    uint32_t i;
  };
  std::vector<K, DefaultInit<K>> ks(n);
  parallel_for(n, [&](uint64_t a, uint64_t z) {
    for (size_t k = a; k < z; ++k) {
      const uint32_t x = ord[k];
      const uint64_t len = fo[x + 1] - fo[x];
      uint64_t key = 0;
      for (uint64_t q = 0; q < 8; ++q) key = (key << 8) | (q < len ? fb[fo[x] + q] : 0u);
      ks[k] = K{key, x};
    }
  });
  par_sort(ks, [&](const K& a, const K& b) {
    if (a.key != b.key) return a.key < b.key;
    return less_bytes(fb + fo[a.i], fo[a.i + 1] - fo[a.i], fb + fo[b.i], fo[b.i + 1] - fo[b.i]);
  });
  parallel_for(n, [&](uint64_t a, uint64_t z) {
    for (size_t k = a; k < z; ++k) ord[k] = ks[k].i;
  });
}

// Parallel sort of u64 values.
void sort_u64(std::vector<uint64_t>& v) { par_sort(v, std::less<uint64_t>()); }

// Host tables to a device blob without assembling it on the host: the blob
// zeroed on the device, each region (offset, source, bytes) copied into
// page-locked staging by all threads and sent by DMA, two buffers in turn.
hipError_t upload_regions(emqx_gm_ctx* ctx, uint8_t* dev, size_t total,
                          const std::pair<size_t, std::pair<const void*, size_t>>* regions, size_t n_regions,
                          size_t o_small, const void* small, size_t small_bytes) {
  const size_t CH = std::min<size_t>(size_t(128) << 20, (total + 4095) & ~size_t(4095));
  hipStream_t st = ctx->stream;
  hipError_t e = hipMemsetAsync(dev, 0, total, st);
  void* buf[2] = {nullptr, nullptr};
  hipEvent_t done[2] = {nullptr, nullptr};
  bool staged = e == hipSuccess;
  for (int k = 0; k < 2 && staged; ++k)
    staged = hipHostMalloc(&buf[k], CH, hipHostMallocDefault) == hipSuccess &&
             hipEventCreateWithFlags(&done[k], hipEventDisableTiming) == hipSuccess;
  if (e == hipSuccess && !staged) {  // no page-locked memory to spare: each region from where it lies
    (void)hipGetLastError();
    for (size_t r = 0; r < n_regions && e == hipSuccess; ++r)
      if (regions[r].second.second)
        e = hipMemcpyAsync(dev + regions[r].first, regions[r].second.first, regions[r].second.second,
                           hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipMemcpyAsync(dev + o_small, small, small_bytes, hipMemcpyHostToDevice, st);
    const hipError_t es = hipStreamSynchronize(st);
    for (int q = 0; q < 2; ++q) {
      if (done[q]) (void)hipEventDestroy(done[q]);
      if (buf[q]) (void)hipHostFree(buf[q]);
    }
    return e == hipSuccess ? es : e;
  }
  int k = 0;
  bool used[2] = {false, false};
  auto send = [&](size_t off, const uint8_t* src, size_t bytes) {
    for (size_t c = 0; c < bytes && e == hipSuccess; c += CH) {
      const size_t n = std::min(CH, bytes - c);
      if (used[k]) e = hipEventSynchronize(done[k]);  // (the buffer's previous chunk has crossed)
      if (e != hipSuccess) break;
      uint8_t* b = static_cast<uint8_t*>(buf[k]);
      parallel_for(n, [&](uint64_t a, uint64_t z) { std::memcpy(b + a, src + c + a, z - a); });
      e = hipMemcpyAsync(dev + off + c, b, n, hipMemcpyHostToDevice, st);
      if (e == hipSuccess) e = hipEventRecord(done[k], st);
      used[k] = true;
      k ^= 1;
    }
  };
  for (size_t r = 0; r < n_regions; ++r)
    if (regions[r].second.second)
      send(regions[r].first, static_cast<const uint8_t*>(regions[r].second.first), regions[r].second.second);
  send(o_small, static_cast<const uint8_t*>(small), small_bytes);
  const hipError_t es = hipStreamSynchronize(st);
  if (e == hipSuccess) e = es;
  for (int q = 0; q < 2; ++q) {
    if (done[q]) (void)hipEventDestroy(done[q]);
    if (buf[q]) (void)hipHostFree(buf[q]);
  }
  return e;
}

// An empty EdgeMap filled with distinct keys in one sweep instead of key-by-key
// probes (random lines): the keys sorted by home slot, each at max(its home,
// the next free slot); the few that run past the end take the first free
// slots from 0 (where their probe continues).  A valid linear-probing table.
void sweep_fill(EdgeMap& m, const std::vector<std::pair<uint64_t, uint32_t>>& kv) {
  const uint64_t cap = m.slots.size();
  std::vector<uint64_t> hk(kv.size());
  for (size_t j = 0; j < kv.size(); ++j) hk[j] = (edge_slot(kv[j].first, m.mask) << 32) | j;
  sort_u64(hk);
  std::vector<uint32_t> wrap;
  uint64_t pos = 0;
  for (const uint64_t x : hk) {
    const uint64_t home = x >> 32;
    const uint32_t j = uint32_t(x);
    if (pos < home) pos = home;
    if (pos >= cap) {
      wrap.push_back(j);
      continue;
    }
    m.slots[pos++] = EdgeSlot{kv[j].first, kv[j].second, 0};
  }
  uint64_t sl = 0;
  for (const uint32_t j : wrap) {
    while (m.slots[sl].key != EDGE_EMPTY) ++sl;
    m.slots[sl] = EdgeSlot{kv[j].first, kv[j].second, 0};
  }
  m.used = kv.size();
}

}  // namespace

void sort_filters(std::vector<uint32_t>& ord, const uint8_t* fb, const uint64_t* fo) { sort_filters_impl(ord, fb, fo); }

int build_index(emqx_gm_ctx* ctx, const uint8_t* fb, const uint64_t* fo, uint64_t n, const uint64_t* sub_off,
                const uint32_t* sub_ids, uint32_t* perm_out, emqx_gm_index** out, emqx_gm_index_info_t* host_only,
                const uint32_t* gids) {
  if (!out && !host_only) return set_err(ctx, EMQX_GM_EINVAL, "index_build: out is NULL");
  if (n && (!fb || !fo)) return set_err(ctx, EMQX_GM_EINVAL, "index_build: NULL filter buffers");
  if (n >= 0x7FFFFFFFull) return set_err(ctx, EMQX_GM_EINVAL, "index_build: too many filters");
  if (sub_off && !sub_ids && n && sub_off[n] > 0)
    return set_err(ctx, EMQX_GM_EINVAL, "index_build: sub_ids is NULL");
  for (uint64_t i = 0; i < n; ++i)
    if (fo[i + 1] < fo[i]) return set_err(ctx, EMQX_GM_EINVAL, "index_build: filter offsets not monotone");

  auto* idx = new emqx_gm_index;
  idx->device = ctx ? ctx->device : -1;
  // GM_INDEX_STATS: phase times on stderr (diagnostics)
  const bool stats = knob("GM_INDEX_STATS") != nullptr;
  auto t_last = std::chrono::steady_clock::now();
  auto phase = [&](const char* what) {
    if (!stats) return;
    const auto t = std::chrono::steady_clock::now();
    fprintf(stderr, "[gm_index] %-12s %9.1f ms\n", what, std::chrono::duration<double, std::milli>(t - t_last).count());
    t_last = t;
  };

  // ---- 1. ids = lexicographic rank of unique filters
  std::vector<uint32_t> ord(n);
  std::iota(ord.begin(), ord.end(), 0u);
  sort_filters_impl(ord, fb, fo);
  std::vector<uint32_t> id_of(n);
  uint32_t nf = 0;
  auto sorted = std::make_shared<SortedFilters>();  // becomes idx->ft's base
  std::vector<uint8_t>& FBV = sorted->bytes;
  std::vector<uint64_t>& FOV = sorted->off;
  {
    // duplicates collapse; the unique filters packed in order.  On all threads:
    // per range of the sorted order, its uniques and their bytes are counted,
    // then each range writes its part at its prefix offsets
    const unsigned T = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    const unsigned R = n < (1u << 16) ? 1u : T;
    auto same_as_prev = [&](uint64_t k) {
      if (!k) return false;
      const uint32_t p = ord[k - 1], i = ord[k];
      const uint64_t lp = fo[p + 1] - fo[p], li = fo[i + 1] - fo[i];
      return lp == li && std::memcmp(fb + fo[p], fb + fo[i], li) == 0;
    };
    std::vector<uint64_t> r_uni(R + 1, 0), r_bytes(R + 1, 0);
    std::vector<uint8_t> dup(n);
    auto run_ranges = [&](auto body) {
      std::vector<std::thread> th;
      for (unsigned r = 1; r < R; ++r) th.emplace_back([&, r] { body(r, n * r / R, n * (r + 1) / R); });
      body(0u, uint64_t(0), n / R);
      for (auto& t : th) t.join();
    };
    run_ranges([&](unsigned r, uint64_t a, uint64_t b) {
      uint64_t u = 0, by = 0;
      for (uint64_t k = a; k < b; ++k) {
        dup[k] = same_as_prev(k);
        if (!dup[k]) {
          ++u;
          by += fo[ord[k] + 1] - fo[ord[k]];
        }
      }
      r_uni[r + 1] = u;
      r_bytes[r + 1] = by;
    });
    for (unsigned r = 0; r < R; ++r) {
      r_uni[r + 1] += r_uni[r];
      r_bytes[r + 1] += r_bytes[r];
    }
    nf = uint32_t(std::min<uint64_t>(r_uni[R], 0xFFFFFFFFull));
    FBV.resize(r_bytes[R]);
    FOV.assign(r_uni[R] + 1, 0);
    run_ranges([&](unsigned r, uint64_t a, uint64_t b) {
      uint64_t u = r_uni[r], by = r_bytes[r];
      for (uint64_t k = a; k < b; ++k) {
        const uint32_t i = ord[k];
        if (!dup[k]) {
          const uint64_t l = fo[i + 1] - fo[i];
          if (l) std::memcpy(FBV.data() + by, fb + fo[i], l);
          by += l;
          FOV[++u] = by;
        }
        id_of[i] = uint32_t(u - 1);
      }
    });
  }
  idx->ft.set_base(sorted);  // (the same vectors: FBV / FOV stay valid)
  if (perm_out)
    for (uint64_t i = 0; i < n; ++i) perm_out[i] = id_of[i];
  // shard index: rows carry the filters' global ids, which
  // must follow the byte order (a shard's local order is then the global one)
  if (gids) {
    idx->gmap.assign(nf, NONE);
    for (uint64_t i = 0; i < n; ++i) {
      uint32_t& g = idx->gmap[id_of[i]];
      if (g != NONE && g != gids[i]) {
        delete idx;
        return set_err(ctx, EMQX_GM_EINVAL, "index_build_shard: equal filters with different global ids");
      }
      g = gids[i];
    }
    for (uint32_t f = 0; f < nf; ++f)
      if (idx->gmap[f] >= 0x7FFFFFFFu || (f && idx->gmap[f] <= idx->gmap[f - 1])) {
        delete idx;
        return set_err(ctx, EMQX_GM_EINVAL, "index_build_shard: global ids must ascend with the filter bytes");
      }
  }

  if (nf >= HF_NONE) {  // filter ids share HotSlot::hf with two flag bits
    delete idx;
    return set_err(ctx, EMQX_GM_EINVAL, "index_build: more than 2^30 - 2 distinct filters");
  }
  phase("sort+ids");
  // ---- 2. intern words, build the level trie
  std::unordered_map<std::string_view, uint32_t, ViewHash> wid;  // word -> arena offset
  std::vector<uint8_t> arena;
  std::vector<uint32_t> word_hash;  // per distinct word (parallel to insertion order)
  std::vector<uint32_t> word_ids;
  std::vector<uint32_t> word_len;
  std::vector<uint64_t> word_head;
  uint64_t total_words = 0;
  for (uint32_t f = 0; f < nf; ++f) {
    uint64_t a = FOV[f], b = FOV[f + 1];
    total_words += 1 + std::count(FBV.begin() + a, FBV.begin() + b, uint8_t('/'));
  }
  wid.reserve(std::min<uint64_t>(total_words, 1u << 26));
  std::vector<HNode, DefaultInit<HNode>> nodes(1, kNewNode);
  uint64_t n_wild = 0;
  uint32_t max_depth = 0;
  const uint8_t* FB = FBV.data();

  auto intern = [&](const uint8_t* p, uint64_t len) -> uint32_t {
    std::string_view v(reinterpret_cast<const char*>(p), len);
    auto it = wid.find(v);
    if (it != wid.end()) return it->second;
    uint32_t off = uint32_t(arena.size());
    arena.insert(arena.end(), p, p + len);
    if (len == 0) arena.push_back(0);  // every word owns >= 1 byte: ids stay unique
    wid.emplace(v, off);  // view into FBV (stable for the build)
    word_hash.push_back(dict_hash_host(p, len));
    word_ids.push_back(off);
    word_len.push_back(uint32_t(len));
    word_head.push_back(word_head_host(p, len));
    if (arena.size() >= 0xFFFFFFF0ull) throw std::length_error("word arena exceeds 4 GiB");
    return off;
  };

  // The trie is built in parallel over runs of filters, cut at filters
  // where the walk may start from a path of nodes the earlier runs made (the
  // k words the cut's two neighbours share: the run's seed) and every deeper
  // node of the run is new (safe_cut).  Each run builds a local trie (local
  // node and word numbers, its own edge map) with the root and its seed as
  // stand-ins; the runs are then merged IN FILTER ORDER -- new nodes
  // concatenated, words interned in each run's first-occurrence order, each
  // stand-in's changes folded into the node it stands for -- which is exactly
  // the serial build's creation order and word order (the BFS renumbering,
  // the arena and every table below come out the same).
  struct TrieRun {
    uint32_t f0 = 0, f1 = 0;              // filters [f0, f1)
    uint32_t k = 0;                       // seed depth: nodes[1..k] stand for the path of f0's first k words
    std::vector<uint64_t> seed_end;       // end byte of each seed word (in f0 and f0 - 1 alike)
    std::vector<HNode> nodes;             // [0]: the root's stand-in, [1..k]: the seed's
    std::vector<std::string_view> words;  // distinct words, first occurrence first
    std::vector<uint32_t> last_path;      // local nodes of the last filter's words
    uint64_t n_wild = 0;
    uint32_t max_depth = 0;
  };
  auto filt = [&](uint32_t f) {
    return std::string_view(reinterpret_cast<const char*>(FB + FOV[f]), FOV[f + 1] - FOV[f]);
  };
  auto lower_filter = [&](std::string_view key) {  // the first filter >= key (byte order)
    uint32_t lo = 0, hi = nf;
    while (lo < hi) {
      const uint32_t mid = lo + (hi - lo) / 2;
      const std::string_view m = filt(mid);
      if (less_bytes(reinterpret_cast<const uint8_t*>(m.data()), m.size(),
                     reinterpret_cast<const uint8_t*>(key.data()), key.size()))
        lo = mid + 1;
      else
        hi = mid;
    }
    return lo;
  };
  auto exists = [&](std::string_view key) {
    const uint32_t x = lower_filter(key);
    return x < nf && filt(x) == key;
  };
  // the end bytes of the words filter b shares with filter a (the walk's own rule below)
  auto shared_ends = [&](uint32_t a, uint32_t b) {
    const std::string_view pa = filt(a), pb = filt(b);
    const uint64_t m = std::min(pa.size(), pb.size());
    uint64_t cp = 0;
    while (cp < m && pa[cp] == pb[cp]) ++cp;
    std::vector<uint64_t> ends;
    for (uint64_t i = 0; i <= pb.size(); ++i) {
      if (i < pb.size() && pb[i] != '/') continue;
      const bool sh = i < cp || (i == cp && (cp == pb.size() || (cp == pa.size() && cp < pb.size() && pb[cp] == '/')));
      if (!sh) break;
      ends.push_back(i);
    }
    return ends;
  };
  // A cut before filter e is safe when every node the filters from e on make
  // -- beyond the k words e shares with e - 1, the seed -- is new.  The
  // filters whose words start with a path P are "P" itself and the contiguous
  // block "P/...", and between the two only filters "P" + c... (c < '/') can
  // lie.  So P's node is made on both sides of the cut only when the filter
  // "P" lies before it and P's block at or after it; then every filter in
  // between starts with P's bytes, e - 1 included.  Safe: no byte prefix P of
  // e - 1 is a filter whose block reaches past the cut, unless P is one of the
  // seed's paths (a word prefix of e of at most k words).  Returns k, or -1.
  auto safe_cut = [&](uint32_t e, std::vector<uint64_t>& seed) -> int {
    seed = shared_ends(e - 1, e);
    const std::string_view pa = filt(e - 1);
    std::string key;
    for (uint64_t L = 0; L <= pa.size(); ++L) {
      const std::string_view P = pa.substr(0, L);
      if (!exists(P)) continue;
      if (std::find(seed.begin(), seed.end(), L) != seed.end()) continue;  // a seed node: shared, not made twice
      key.assign(P.data(), P.size());
      key.push_back('/');
      const uint32_t b = lower_filter(key);
      if (b >= e && b < nf && filt(b).substr(0, key.size()) == key) return -1;
    }
    return int(seed.size());
  };
  const unsigned T = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  std::vector<TrieRun> runs;
  {
    // GM_TRIE_RUNS: the number of runs asked for (1: the serial build; tests)
    const char* rk = knob("GM_TRIE_RUNS");
    const uint32_t want = rk ? std::max(1u, uint32_t(strtoul(rk, nullptr, 10)))
                             : (nf < 200000 || T == 1) ? 1u : 4u * T;
    uint32_t f0 = 0;
    std::vector<uint64_t> seed, next_seed;
    int k0 = 0;
    for (uint32_t q = 1; q <= want && f0 < nf; ++q) {
      uint32_t e = q == want ? nf : uint32_t(uint64_t(nf) * q / want);
      if (e <= f0) continue;
      int k = -1;
      while (e < nf && (k = safe_cut(e, next_seed)) < 0) ++e;
      TrieRun r;
      r.f0 = f0;
      r.f1 = e;
      r.k = uint32_t(k0);
      r.seed_end = seed;
      runs.push_back(std::move(r));
      f0 = e;
      k0 = k < 0 ? 0 : k;
      seed.swap(next_seed);
    }
  }
  // one run: the serial walk below, on local numbers
  auto build_run = [&](TrieRun& R) {
    uint64_t tw = 0;
    for (uint32_t f = R.f0; f < R.f1; ++f) tw += 1 + std::count(FB + FOV[f], FB + FOV[f + 1], uint8_t('/'));
    std::unordered_map<std::string_view, uint32_t, ViewHash> lw;  // word -> local word number
    lw.reserve(std::min<uint64_t>(tw, 1u << 26));
    EdgeMap edges(std::min<uint64_t>(tw + 1, 1ull << 30));
    std::vector<HNode>& nd = R.nodes;
    nd.assign(1 + R.k, kNewNode);
    nd.reserve(std::min<uint64_t>(tw + 1 + R.k, 1ull << 30));
    auto lintern = [&](const uint8_t* p, uint64_t len) -> uint32_t {
      std::string_view v(reinterpret_cast<const char*>(p), len);
      auto it = lw.find(v);
      if (it != lw.end()) return it->second;
      const uint32_t id = uint32_t(R.words.size());
      R.words.push_back(v);
      lw.emplace(v, id);
      return id;
    };
    // Filters are in byte order, so a filter usually shares its leading words
    // with the previous one: those words' nodes are taken from the previous
    // filter's path (no interning, no edge lookup).  Word j of the previous
    // filter (ending at byte e) is shared when the two agree on every byte up
    // to e and the word ends at e in both.  A run starts from its seed: the
    // previous filter (the last of the run before) and the stand-ins of the
    // words the two share.
    std::vector<uint32_t> pnode;  // node after word j of the previous filter
    std::vector<uint64_t> pend;   // end byte of word j
    std::vector<uint8_t> pwild;   // a wildcard word among words 0..j
    const uint8_t* ps = nullptr;
    uint64_t plen = 0;
    if (R.k) {
      ps = FB + FOV[R.f0 - 1];
      plen = FOV[R.f0] - FOV[R.f0 - 1];
      bool wild = false;
      for (uint32_t d = 0; d < R.k; ++d) {
        const uint64_t ws = d ? R.seed_end[d - 1] + 1 : 0, wl = R.seed_end[d] - ws;
        const bool plus = wl == 1 && ps[ws] == '+', hash = wl == 1 && ps[ws] == '#';
        wild |= plus || hash;
        nd[d + 1].depth = d + 1;
        nd[d + 1].parent = d;
        nd[d + 1].kind = plus ? 1 : hash ? 2 : 0;
        pnode.push_back(d + 1);
        pend.push_back(R.seed_end[d]);
        pwild.push_back(wild);
      }
    }
    for (uint32_t f = R.f0; f < R.f1; ++f) {
      const uint8_t* s = FB + FOV[f];
      uint64_t len = FOV[f + 1] - FOV[f];
      uint64_t cp = 0;
      if (ps) {
        const uint64_t m = std::min(len, plen);
        while (cp < m && s[cp] == ps[cp]) ++cp;
      }
      size_t j = 0;
      while (j < pend.size()) {
        const uint64_t e = pend[j];
        const bool shared = e < cp || (e == cp && (cp == len || (cp == plen && cp < len && s[cp] == '/')));
        if (!shared) break;
        ++j;
      }
      pnode.resize(j);
      pend.resize(j);
      pwild.resize(j);
      uint32_t node = j ? pnode[j - 1] : 0, depth = uint32_t(j);
      bool wild = j ? pwild[j - 1] != 0 : false;
      const uint64_t ws0 = j ? pend[j - 1] + 1 : 0;
      uint64_t ws = ws0;
      ps = s;
      plen = len;
      for (uint64_t i = ws0; i <= len; ++i) {
        if (i < len && s[i] != '/') continue;
        const uint8_t* w = s + ws;
        uint64_t wl = i - ws;
        bool plus = wl == 1 && w[0] == '+', hash = wl == 1 && w[0] == '#';
        wild |= plus || hash;
        uint32_t id = lintern(w, wl);
        uint64_t key = edge_key(node, id);
        uint32_t child = edges.get(key);
        if (child == NONE) {
          if (nd.size() >= REF_X) throw std::length_error("too many trie nodes (>= 2^31)");
          child = uint32_t(nd.size());
          nd.push_back(kNewNode);
          nd.back().depth = depth + 1;
          nd.back().parent = node;
          nd.back().word = id;
          nd.back().kind = plus ? 1 : hash ? 2 : 0;
          edges.put(key, child);
          if (plus) { nd[node].plus_child = child; nd[node].flags |= NF_HAS_PLUS; }
          else if (hash) nd[node].hash_child = child;
          else nd[node].flags |= NF_HAS_EXACT;  // (sig: from the final word ids, after the merge)
        }
        node = child;
        ++depth;
        ws = i + 1;
        pnode.push_back(node);
        pend.push_back(i);
        pwild.push_back(wild);
      }
      nd[node].end_filter = f;
      if (wild) { nd[node].flags |= NF_END_WILD; ++R.n_wild; }
      R.max_depth = std::max(R.max_depth, depth);
    }
    R.last_path = pnode;
  };
  {
    std::atomic<size_t> next{0};
    std::vector<std::exception_ptr> errs(runs.size());
    auto worker = [&] {
      for (size_t r; (r = next.fetch_add(1)) < runs.size();) {
        try {
          build_run(runs[r]);
        } catch (...) {
          errs[r] = std::current_exception();
        }
      }
    };
    const unsigned nt = unsigned(std::min<size_t>(T, runs.size()));
    std::vector<std::thread> th;
    for (unsigned k = 1; k < nt; ++k) th.emplace_back(worker);
    worker();
    for (auto& t : th) t.join();
    for (auto& e : errs)
      if (e) std::rethrow_exception(e);
  }
  // merge in filter order: words first (the serial first-occurrence order), then
  // the runs' new nodes; a run's seed stand-ins are the nodes of the previous
  // run's last filter's first k words
  const size_t NR = runs.size();
  std::vector<uint32_t> base(NR);
  std::vector<std::vector<uint32_t>> seedg(NR), lastg(NR);
  uint64_t n_all = 1;
  for (size_t r = 0; r < NR; ++r) {
    TrieRun& R = runs[r];
    base[r] = uint32_t(std::min<uint64_t>(n_all, NONE));
    n_all += R.nodes.size() - 1 - R.k;
    if (n_all > REF_X) throw std::length_error("too many trie nodes (>= 2^31)");
    if (R.k && (!r || lastg[r - 1].size() < R.k)) throw std::logic_error("trie run: seed outside the previous run");
    seedg[r].assign(R.k ? lastg[r - 1].begin() : lastg[0].begin(), R.k ? lastg[r - 1].begin() + R.k : lastg[0].begin());
    lastg[r].reserve(R.last_path.size());
    for (const uint32_t l : R.last_path)
      lastg[r].push_back(l == 0 ? 0u : l <= R.k ? seedg[r][l - 1] : base[r] + (l - 1 - R.k));
  }
  std::vector<std::vector<uint32_t>> gword(NR);
  for (size_t r = 0; r < NR; ++r) {
    gword[r].reserve(runs[r].words.size());
    for (std::string_view v : runs[r].words) gword[r].push_back(intern(reinterpret_cast<const uint8_t*>(v.data()), v.size()));
    std::vector<std::string_view>().swap(runs[r].words);
  }
  nodes.resize(n_all);
  auto gmap = [&](size_t r, uint32_t l) {
    const TrieRun& R = runs[r];
    return l == NONE ? NONE : l == 0 ? 0u : l <= R.k ? seedg[r][l - 1] : base[r] + (l - 1 - R.k);
  };
  {
    auto merge_run = [&](size_t r) {
      TrieRun& R = runs[r];
      const uint32_t b = base[r], K = R.k;
      for (size_t l = K + 1; l < R.nodes.size(); ++l) {
        HNode h = R.nodes[l];
        const uint32_t lp = h.parent;
        h.parent = gmap(r, lp);
        h.word = gword[r][h.word];
        h.plus_child = gmap(r, h.plus_child);
        h.hash_child = gmap(r, h.hash_child);
        nodes[b + (l - 1 - K)] = h;
        // exact-child signatures over the final word ids (a new parent is older:
        // already written; a stand-in's, which other runs share, gathered apart)
        if (h.kind == 0) {
          if (lp > K) nodes[h.parent].sig |= sig_bit(h.word);
          else R.nodes[lp].sig |= sig_bit(h.word);
        }
      }
      R.nodes.resize(K + 1);  // (only the stand-ins are still needed)
      R.nodes.shrink_to_fit();
    };
    std::atomic<size_t> next{0};
    auto worker = [&] {
      for (size_t r; (r = next.fetch_add(1)) < NR;) merge_run(r);
    };
    const unsigned nt = unsigned(std::min<size_t>(T, NR));
    std::vector<std::thread> th;
    for (unsigned k = 1; k < nt; ++k) th.emplace_back(worker);
    worker();
    for (auto& t : th) t.join();
  }
  for (size_t r = 0; r < NR; ++r) {  // the root and the seeds: the union of the runs' changes
    const TrieRun& R = runs[r];
    for (uint32_t l = 0; l <= R.k; ++l) {
      const HNode& h = R.nodes[l];
      HNode& g = nodes[gmap(r, l)];
      g.flags |= h.flags;
      g.sig |= h.sig;
      if (h.plus_child != NONE) g.plus_child = gmap(r, h.plus_child);
      if (h.hash_child != NONE) g.hash_child = gmap(r, h.hash_child);
      if (h.end_filter != NONE) g.end_filter = h.end_filter;
    }
    n_wild += R.n_wild;
    max_depth = std::max(max_depth, R.max_depth);
  }
  std::vector<TrieRun>().swap(runs);

  phase("trie");
  // ---- 3. breadth-first renumbering (stable by creation order within a level)
  uint64_t NN = nodes.size();
  std::vector<uint64_t> per_depth(max_depth + 2, 0);
  for (auto& nd : nodes) per_depth[nd.depth + 1]++;
  idx->level_nodes = *std::max_element(per_depth.begin(), per_depth.end());
  for (size_t d = 1; d < per_depth.size(); ++d) per_depth[d] += per_depth[d - 1];
  std::vector<uint32_t> newid(NN);
  for (uint64_t i = 0; i < NN; ++i) newid[i] = uint32_t(per_depth[nodes[i].depth]++);

  phase("v1: renumber");
  auto ref = [&](uint32_t old) -> uint32_t {  // child reference with the child's HAS_EXACT bit
    if (old == NONE) return NONE;
    return newid[old] | ((nodes[old].flags & NF_HAS_EXACT) ? REF_X : 0u);
  };
  std::vector<Node> dnodes(NN);
  parallel_for(NN, [&](uint64_t a, uint64_t b) {  // (newid is a permutation: distinct writes)
    for (uint64_t i = a; i < b; ++i) {
      const HNode& h = nodes[i];
      Node& d = dnodes[newid[i]];
      d.plus_child = ref(h.plus_child);
      d.hash_filter = h.hash_child == NONE ? NONE : nodes[h.hash_child].end_filter;
      d.end_filter = h.end_filter;
      d.flags = h.flags;
    }
  });
  // edge tables partitioned by the parent's depth
  // (each depth's table built on its own thread from its bucket of edges)
  std::vector<std::vector<std::pair<uint64_t, uint32_t>>> by_tab(EDGE_DEPTHS);
  {  // (every non-root node is the child of exactly one edge: (parent, word)); the
     // buckets filled in node order by all threads: per-range counts, then offsets
    const unsigned T = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    const unsigned R = NN < (1u << 16) ? 1u : T;
    std::vector<std::array<uint64_t, EDGE_DEPTHS>> cnt(R);
    auto range = [&](unsigned r, auto f) {
      for (uint64_t i = std::max<uint64_t>(1, NN * r / R), e = NN * (r + 1) / R; i < e; ++i) f(i);
    };
    auto run_ranges = [&](auto body) {
      std::vector<std::thread> th;
      for (unsigned r = 1; r < R; ++r) th.emplace_back([&, r] { body(r); });
      body(0u);
      for (auto& t : th) t.join();
    };
    run_ranges([&](unsigned r) {
      cnt[r].fill(0);
      range(r, [&](uint64_t i) { cnt[r][edge_depth(nodes[i].depth - 1)]++; });
    });
    for (int d = 0; d < EDGE_DEPTHS; ++d) {
      uint64_t o = 0;
      for (unsigned r = 0; r < R; ++r) {
        const uint64_t c = cnt[r][d];
        cnt[r][d] = o;
        o += c;
      }
      by_tab[d].resize(o);
    }
    run_ranges([&](unsigned r) {
      range(r, [&](uint64_t i) {
        const int d = edge_depth(nodes[i].depth - 1);
        by_tab[d][cnt[r][d]++] = {edge_key(newid[nodes[i].parent], nodes[i].word), ref(uint32_t(i))};
      });
    });
  }
  phase("v1: buckets");
  const bool verify_tables = knob("GM_INDEX_VERIFY") != nullptr;
  std::vector<EdgeMap> tabs;
  tabs.reserve(EDGE_DEPTHS);
  for (int d = 0; d < EDGE_DEPTHS; ++d) tabs.emplace_back(by_tab[d].empty() ? 1 : 0);  // (sized on its thread)
  {
    std::vector<std::thread> th;
    std::atomic<bool> lost{false};
    for (int d = 0; d < EDGE_DEPTHS; ++d)
      if (!by_tab[d].empty())
        th.emplace_back([&, d] {
          tabs[d] = EdgeMap(by_tab[d].size() + 1);
          sweep_fill(tabs[d], by_tab[d]);  // (each edge once: distinct keys)
          if (verify_tables)  // GM_INDEX_VERIFY: every edge found by the probe the kernels make
            for (const auto& kv : by_tab[d])
              if (tabs[d].get(kv.first) != kv.second) lost = true;
          std::vector<std::pair<uint64_t, uint32_t>>().swap(by_tab[d]);
        });
    for (auto& t : th) t.join();
    if (lost) throw std::logic_error("edge table: an edge not found");
  }
  phase("v1: edge maps");
  uint64_t etab_off[EDGE_DEPTHS], etab_mask[EDGE_DEPTHS], n_edges = 0, n_eslots = 0;
  for (int d = 0; d < EDGE_DEPTHS; ++d) {
    etab_off[d] = n_eslots;
    etab_mask[d] = tabs[d].mask;
    n_edges += tabs[d].used;
    n_eslots += tabs[d].slots.size();
  }
  std::vector<EdgeSlot, DefaultInit<EdgeSlot>> dedges(n_eslots);  // (each table copied in by a thread of its own)
  {
    std::vector<std::thread> th;
    for (int d = 0; d < EDGE_DEPTHS; ++d)
      th.emplace_back([&, d] {
        std::copy(tabs[d].slots.begin(), tabs[d].slots.end(), dedges.begin() + etab_off[d]);
        std::vector<EdgeSlot>().swap(tabs[d].slots);
      });
    for (auto& t : th) t.join();
  }

  phase("v1 tables");
  // ---- 3b. hot tables: one 32-B slot per node reached through an exact edge
  // (or a '+' edge from the root or from an inline node), slot index = the
  // node's hot id; the '+' child of a slot-owning node is inline in its
  // parent's slot (gm_common.h).  Built depth by depth because a key holds the
  // parent's hot id.
  std::vector<uint32_t> by_depth_off(max_depth + 2, 0);  // old nodes bucketed by depth
  for (uint64_t i = 1; i < NN; ++i) by_depth_off[nodes[i].depth + 1]++;
  for (size_t d = 1; d < by_depth_off.size(); ++d) by_depth_off[d] += by_depth_off[d - 1];
  std::vector<uint32_t> by_depth(by_depth_off.back());
  {
    std::vector<uint32_t> cur(by_depth_off.begin(), by_depth_off.end() - 1);
    for (uint64_t i = 1; i < NN; ++i) by_depth[cur[nodes[i].depth]++] = uint32_t(i);
  }
  // a parent is always created before its child, so one pass in index order
  std::vector<uint8_t> inl(NN, 0);
  for (uint64_t i = 1; i < NN; ++i) {
    const HNode& h = nodes[i];
    inl[i] = h.kind == 1 && nodes[h.parent].kind != 2 && plus_inline(nodes[h.parent].depth, h.parent != 0 && !inl[h.parent]);
  }
  uint64_t hot_n[HOT_TABLES] = {0};
  for (uint64_t i = 1; i < NN; ++i)
    if (nodes[i].kind != 2 && !inl[i]) hot_n[hot_table(nodes[i].depth)]++;
  uint64_t hot_off[HOT_TABLES], hot_cap[HOT_TABLES], hot_total = 0;
  // Minimal-perfect-hash tables (gm_common.h, mph_*), placed by hash-and-displace
  // at load ~0.97:
  //  * a per-depth table of [GM_MPH_MIN_KEYS, GM_MPH_MAX_KEYS] keys (C2/C3: the
  //    depth-2 table, 66.5k keys, 8.5 MB at 0.25 load -> 2.2 MB, which one XCD's
  //    4 MB L2 keeps); smaller tables stay in L2 anyway;
  //  * a table whose parents average >= 4 exact children -- the ones that get an
  //    exact-edge filter, a dependent L2 read in front of every exact probe --
  //    when its bucket words (2 B per key) fit 2 MB: the bucket word is that
  //    read, filters better (12 Bloom bits per key) and the table shrinks 4x
  //    (C2's depth-3 table, 600k keys: 77 -> 20 MB, kernel 8.76 -> 8.56 ms;
  //    placing the depth-4/5 tables too, which have no filter read to replace,
  //    was slower: profiles/r03_ab/mph_tables.txt).
  // GM_NO_MPH / the two bounds / GM_MPH_TABLES (a table bit mask): A/B knobs.
  uint32_t mph_cap[HOT_TABLES] = {0}, mph_nb[HOT_TABLES] = {0};
  uint64_t mph_off[HOT_TABLES] = {0}, mph_total = 0;
  uint64_t x_keys[HOT_TABLES] = {0}, x_parents[HOT_TABLES] = {0};  // exact edges into table t, their parents
  for (uint64_t i = 1; i < NN; ++i)
    if (nodes[i].kind == 0) x_keys[hot_table(nodes[i].depth)]++;
  for (uint64_t i = 0; i < NN; ++i)
    if ((nodes[i].flags & NF_HAS_EXACT) && nodes[i].kind != 2) x_parents[hot_table(nodes[i].depth + 1)]++;
  {
    uint64_t lo = 4096, hi = 131072;
    if (const char* e = knob("GM_MPH_MIN_KEYS")) lo = strtoull(e, nullptr, 10);
    if (const char* e = knob("GM_MPH_MAX_KEYS")) hi = strtoull(e, nullptr, 10);
    // GM_MPH_TABLES: A/B knob, a bit mask of the tables to place this way (overrides the bounds)
    const char* mt = knob("GM_MPH_TABLES");
    const uint32_t mask = mt ? uint32_t(strtoul(mt, nullptr, 0)) : 0u;
    for (int t = 1; t < HOT_TABLES - 1; ++t) {  // (the shared last table mixes depths: open addressing)
      if (knob("GM_NO_MPH") || !hot_n[t]) continue;
      const bool small = hot_n[t] >= lo && hot_n[t] <= hi;
      const bool filtered = x_keys[t] >= 4 * x_parents[t] && hot_n[t] <= (1u << 20) && !knob("GM_MPH_NO_FILTERED");
      if (mt ? !((mask >> t) & 1u) : !(small || filtered)) continue;
      uint64_t slack = 16;  // GM_MPH_SLACK (A/B knob): spare slots = keys / slack (6 keys per bucket need 1/16 to place without overflow)
      if (const char* e = knob("GM_MPH_SLACK")) slack = std::max<uint64_t>(4, strtoull(e, nullptr, 10));
      mph_cap[t] = uint32_t(hot_n[t] + hot_n[t] / slack + 16);
      // GM_MPH_LAMBDA (A/B knob): keys per bucket -- fewer bucket words (an L2-resident
      // table) against a fuller 48-bit Bloom filter and harder displacement searches
      uint32_t lam = MPH_LAMBDA;
      if (const char* e = knob("GM_MPH_LAMBDA")) lam = std::max<uint32_t>(1, std::min<uint32_t>(16, uint32_t(atoi(e))));
      mph_nb[t] = uint32_t((hot_n[t] + lam - 1) / lam);
      mph_off[t] = mph_total;
      mph_total += mph_nb[t];
    }
  }
  uint32_t mph_ovf = 0;
  uint64_t mph_ovf_n[HOT_TABLES] = {0};
  std::vector<uint64_t> mph_word(mph_total + 1, 0);
  uint64_t hot_sparse = 0;
  if (const char* e = knob("GM_HOT_SPARSE")) hot_sparse = std::min<uint64_t>(1u << 22, strtoull(e, nullptr, 10));
  // load factor (%) of the hash-placed hot tables; GM_HOT_LOAD_PCT: A/B knob (10..90).
  // 0.15 (round 6): the walk's found probes end at their home slot more often
  // and its failed ones stop sooner -- the kernel against 0.25, same box: C2
  // -0.5 %, C3 -1.0 % (profiles/r05_r, r05_q), C5 -3.0 % (17.24 -> 16.72 ms,
  // profiles/r06_a/ab.txt) for 1.38x the table bytes (C5: 38.4 -> 53.0 GB of 288)
  uint64_t hot_load_pct = 15;
  if (const char* e = knob("GM_HOT_LOAD_PCT")) hot_load_pct = std::min<uint64_t>(90, std::max<uint64_t>(10, strtoull(e, nullptr, 10)));
  for (int t = 0; t < HOT_TABLES; ++t) {
    // a low load: shorter probe chains beat a smaller footprint (C2, round 2's
    // fused kernel, 4-8 bit/key edge filter: load 0.40 / 0.35 / 0.30 / 0.25 /
    // 0.20 / 0.15 / 0.10 -> 9.73 / 9.51 / 9.39 / 9.20 / 9.22 / 9.24 / 9.35 ms;
    // round 6 above); at least 8 slots so the probe loop always finds an empty one
    uint64_t pct = hot_load_pct;
    if (const char* e = knob("GM_HOT_LOAD_PCT_UPPER"))  // A/B knob: load of the depth 1-2 tables
      if (t <= 2) pct = std::min<uint64_t>(90, std::max<uint64_t>(10, strtoull(e, nullptr, 10)));
    hot_cap[t] = hot_n[t] ? std::max<uint64_t>(8, hot_n[t] * 100 / pct + 1) : 0;
    // GM_HOT_SPARSE=65536 (A/B knob, off by default until measured): a small
    // table (<= 1,024 keys: the depth-1 table of every config) is spread over
    // 65,536 slots (2 MB, of which only its ~n lines are ever read), so
    // almost every key sits at its home slot and a lookup decides in one read:
    // at load 0.25 one key in eight is off home, and any lane that probes one
    // makes its whole wave wait a dependent round (as with the dictionary).
    if (hot_n[t] && hot_n[t] * 64 <= hot_sparse) hot_cap[t] = std::max<uint64_t>(hot_cap[t], hot_sparse);
    // an MPH table: its perfect-hash region plus an overflow region for in-place
    // inserts (load <= 0.5 there, Patcher::hot_add)
    if (mph_cap[t]) hot_cap[t] = mph_cap[t] + std::max<uint64_t>(64, hot_n[t] / 16);
    if (hot_cap[t] > SLOT_MASK) throw std::length_error("hot table exceeds 2^30 slots");
    hot_off[t] = hot_total;
    hot_total += hot_cap[t];
  }
  phase("hot: counts");
  // (uninitialised, then filled by all threads: the first touch of GBs of pages is the cost)
  std::vector<HotSlot, DefaultInit<HotSlot>> hot(hot_total);
  parallel_for(hot_total, [&](uint64_t a, uint64_t b) {
    std::fill(hot.begin() + a, hot.begin() + b, HotSlot{EDGE_EMPTY, 0, HF_NONE, NONE, 0, HF_NONE, NONE});
  });
  phase("hot: alloc");
  std::vector<uint32_t> hid(NN, NONE);
  hid[0] = 0;  // the root (depth 0) is not stored; its record goes to IndexView
  auto end_of = [&](const HNode& h) -> uint32_t {
    if (h.end_filter == NONE) return NONE;
    return h.end_filter | ((h.flags & NF_END_WILD) ? END_WILD : 0u);
  };
  auto hf_of = [&](const HNode& h) -> uint32_t {
    // (a '#' node holding no filter -- "a/#/b" without "a/#" -- is no 'match_#')
    const uint32_t hf = h.hash_child == NONE ? NONE : nodes[h.hash_child].end_filter;
    return (hf == NONE ? HF_NONE : hf) | (h.plus_child != NONE ? HOT_PLUS : 0u);
  };
  // Tables of one depth (t < HOT_TABLES-1) are Robin Hood ordered: a key is
  // placed so that no key between its home slot and its slot is closer to its
  // own home, which lets a lookup of an absent key stop at the first slot
  // whose key sits nearer its home than the probe (hot_resolve).  Slots move
  // while a depth is placed, so its hot ids are assigned once the whole depth
  // is in (the next depth's keys hold them).  The shared last table keeps
  // plain linear probing (its earlier depths' ids are already referenced).
  std::vector<uint32_t> occ;  // old node index per slot of the table being placed
  const bool rh_insert = knob("GM_HOT_RH_INSERT") != nullptr;  // A/B: RH insertion key by key
  const bool verify = knob("GM_INDEX_VERIFY") != nullptr;
  auto fill_slot = [&](HotSlot& o, const HNode& h) {
    o.sig = h.sig;
    o.hf = hf_of(h);
    o.end_filter = end_of(h);
  };
  for (uint32_t d = 1; d <= max_depth; ++d) {
    const int t = hot_table(d);
    HotSlot* tab = hot.data() + hot_off[t];
    const uint64_t cap = hot_cap[t];
    if (mph_cap[t]) {  // hash-and-displace (the depth is one table: t < HOT_TABLES-1)
      std::vector<std::pair<uint64_t, uint32_t>> ks;  // (key, node) of the depth's slot owners
      for (uint32_t k = by_depth_off[d]; k < by_depth_off[d + 1]; ++k) {
        const uint32_t i = by_depth[k];
        const HNode& h = nodes[i];
        if (h.kind == 2 || hid[h.parent] == NONE) continue;
        if (inl[i]) {
          HotSlot& p = hot[hot_off[hot_table(d - 1)] + hid[h.parent]];
          p.p_sig = h.sig;
          p.p_hf = hf_of(h);
          p.p_end = end_of(h);
          hid[i] = hid[h.parent] | HOT_INLINE;
          continue;
        }
        ks.emplace_back(hot_key(hid[h.parent], h.word, d - 1), i);
      }
      const uint32_t mc = mph_cap[t], nb = mph_nb[t];
      std::vector<uint32_t> boff(nb + 1, 0), bk(ks.size());
      for (const auto& kv : ks) boff[mph_bucket(kv.first, nb) + 1]++;
      for (uint32_t b = 0; b < nb; ++b) boff[b + 1] += boff[b];
      {
        std::vector<uint32_t> cur(boff.begin(), boff.end() - 1);
        for (uint32_t j = 0; j < ks.size(); ++j) bk[cur[mph_bucket(ks[j].first, nb)]++] = j;
      }
      std::vector<uint32_t> order(nb);
      for (uint32_t b = 0; b < nb; ++b) order[b] = b;
      std::stable_sort(order.begin(), order.end(),
                       [&](uint32_t a, uint32_t b) { return boff[a + 1] - boff[a] > boff[b + 1] - boff[b]; });
      std::vector<uint8_t> used(mc, 0);
      uint32_t sl[64];
      auto put = [&](uint32_t s, uint32_t j) {
        tab[s].key = ks[j].first;
        fill_slot(tab[s], nodes[ks[j].second]);
        hid[ks[j].second] = s;
      };
      for (uint32_t b : order) {
        const uint32_t sz = boff[b + 1] - boff[b];
        if (!sz) break;  // (sorted by size)
        bool ok = false;
        if (sz <= 64) {
          for (uint32_t dd = 0; dd < 65536 && !ok; ++dd) {
            ok = true;
            for (uint32_t q = 0; q < sz && ok; ++q) {
              const uint32_t s2 = mph_slot(ks[bk[boff[b] + q]].first, dd, mc);
              ok = !used[s2];
              for (uint32_t r = 0; r < q && ok; ++r) ok = sl[r] != s2;
              sl[q] = s2;
            }
            if (ok) {
              mph_word[mph_off[t] + b] = dd;
              for (uint32_t q = 0; q < sz; ++q) {
                used[sl[q]] = 1;
                put(sl[q], bk[boff[b] + q]);
              }
            }
          }
        }
        for (uint32_t q = 0; q < sz; ++q) mph_word[mph_off[t] + b] |= mph_bloom(ks[bk[boff[b] + q]].first);
        if (!ok) {  // (not expected at this load) the bucket's keys go to the overflow region
          mph_ovf |= 1u << t;
          for (uint32_t q = 0; q < sz; ++q) {
            const uint32_t j = bk[boff[b] + q];
            uint64_t s2 = mph_ovf_home(ks[j].first, mc, uint32_t(cap));
            while (tab[s2].key != EDGE_EMPTY) s2 = s2 + 1 == cap ? mc : s2 + 1;
            put(uint32_t(s2), j);
            ++mph_ovf_n[t];
          }
        }
      }
      continue;
    }
    const bool rh = t < HOT_TABLES - 1;
    if (rh) occ.assign(cap, NONE);
    if (rh && !rh_insert) {
      // Robin Hood placement in one sweep (no random probes): the depth's keys
      // sorted by home slot (ties in node order), each at max(its home, the
      // next free slot); keys that run past the end continue at slot 0 ahead of
      // the keys homed there.  A Robin Hood layout like inserting them one by
      // one (GM_HOT_RH_INSERT=1, the A/B twin), up to the order of keys with
      // the same home (insertion's depends on which resident got displaced).
      // the depth's keys in node order, on all threads (per range: count, then
      // fill at the range's offset); an inline '+' node goes into its parent's
      // slot instead (one per parent: distinct writes)
      const uint64_t k0 = by_depth_off[d], nk = by_depth_off[d + 1] - k0;
      const unsigned T = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
      const unsigned R = nk < (1u << 16) ? 1u : T;
      std::vector<uint64_t> r_off(R + 1, 0);
      auto owns_slot = [&](uint32_t i) {
        const HNode& h = nodes[i];
        return h.kind != 2 && hid[h.parent] != NONE && !inl[i];
      };
      auto ranges = [&](auto body) {
        std::vector<std::thread> th;
        for (unsigned r = 1; r < R; ++r) th.emplace_back([&, r] { body(r, k0 + nk * r / R, k0 + nk * (r + 1) / R); });
        body(0u, k0, k0 + nk / R);
        for (auto& t : th) t.join();
      };
      ranges([&](unsigned r, uint64_t a, uint64_t b) {
        uint64_t c = 0;
        for (uint64_t k = a; k < b; ++k) c += owns_slot(by_depth[k]);
        r_off[r + 1] = c;
      });
      for (unsigned r = 0; r < R; ++r) r_off[r + 1] += r_off[r];
      std::vector<uint64_t> hk(r_off[R]);  // (home << 32) | position in keys
      std::vector<uint64_t> keys(r_off[R]);
      std::vector<uint32_t> owner(r_off[R]);
      ranges([&](unsigned r, uint64_t a, uint64_t b) {
        uint64_t q = r_off[r];
        for (uint64_t k = a; k < b; ++k) {
          const uint32_t i = by_depth[k];
          const HNode& h = nodes[i];
          if (h.kind == 2 || hid[h.parent] == NONE) continue;
          if (inl[i]) {
            HotSlot& p = hot[hot_off[hot_table(d - 1)] + hid[h.parent]];
            p.p_sig = h.sig;
            p.p_hf = hf_of(h);
            p.p_end = end_of(h);
            hid[i] = hid[h.parent] | HOT_INLINE;
            continue;
          }
          const uint64_t key = hot_key(hid[h.parent], h.word, d - 1);
          hk[q] = (hot_slot(key, cap) << 32) | q;
          keys[q] = key;
          owner[q] = i;
          ++q;
        }
      });
      sort_u64(hk);
      uint64_t pos = 0;
      std::vector<uint32_t> wrap;  // positions in keys that ran past the end
      for (const uint64_t e : hk) {
        const uint64_t home = e >> 32;
        const uint32_t j = uint32_t(e);
        if (pos < home) pos = home;
        if (pos >= cap) {
          wrap.push_back(j);
          continue;
        }
        occ[pos] = j;
        tab[pos].key = keys[j];
        ++pos;
      }
      // the wrapped keys take slots 0.. and push the residents there along
      // (a FIFO: the wrapped keys, then each resident met, one per slot)
      for (size_t head = 0, sl = 0; head < wrap.size(); ++sl) {
        if (sl >= cap) throw std::length_error("hot table full");
        if (occ[sl] != NONE) wrap.push_back(occ[sl]);
        occ[sl] = wrap[head++];
        tab[sl].key = keys[occ[sl]];
      }
      for (uint64_t sl = 0; sl < cap; ++sl)  // owners: from positions to nodes
        if (occ[sl] != NONE) occ[sl] = owner[occ[sl]];
    }
    auto home_dist = [&](uint64_t key, uint64_t pos) {
      const uint64_t h = hot_slot(key, cap);
      return pos >= h ? pos - h : pos + cap - h;
    };
    for (uint32_t k = rh && !rh_insert ? by_depth_off[d + 1] : by_depth_off[d]; k < by_depth_off[d + 1]; ++k) {
      const uint32_t i = by_depth[k];
      const HNode& h = nodes[i];
      if (h.kind == 2 || hid[h.parent] == NONE) continue;  // '#' nodes and their (unmatchable) subtrees
      if (inl[i]) {  // into the parent's slot (table of depth d-1, already final)
        HotSlot& p = hot[hot_off[hot_table(d - 1)] + hid[h.parent]];
        p.p_sig = h.sig;
        p.p_hf = hf_of(h);
        p.p_end = end_of(h);
        hid[i] = hid[h.parent] | HOT_INLINE;
        continue;
      }
      uint64_t key = hot_key(hid[h.parent], h.word, d - 1);
      uint64_t s = hot_slot(key, cap);
      if (!rh) {
        while (tab[s].key != EDGE_EMPTY) s = s + 1 == cap ? 0 : s + 1;
        HotSlot& o = tab[s];
        o.key = key;
        o.sig = h.sig;
        o.hf = hf_of(h);
        o.end_filter = end_of(h);
        hid[i] = uint32_t(s);
        continue;
      }
      uint32_t node = i;
      uint64_t dist = 0;
      for (;;) {
        if (tab[s].key == EDGE_EMPTY) {
          tab[s].key = key;
          occ[s] = node;
          break;
        }
        const uint64_t d2 = home_dist(tab[s].key, s);
        if (d2 < dist) {  // the resident is nearer its home: it moves on
          std::swap(tab[s].key, key);
          std::swap(occ[s], node);
          dist = d2;
        }
        s = s + 1 == cap ? 0 : s + 1;
        ++dist;
      }
    }
    if (rh && verify) {  // GM_INDEX_VERIFY: the table is Robin Hood ordered (what hot_resolve's early exit needs)
      auto dist_at = [&](uint64_t sl) {
        const uint64_t h = hot_slot(tab[sl].key, cap);
        return sl >= h ? sl - h : sl + cap - h;
      };
      for (uint64_t sl = 0; sl < cap; ++sl) {
        if (tab[sl].key == EDGE_EMPTY) continue;
        const uint64_t pv = sl ? sl - 1 : cap - 1;
        const uint64_t dd = dist_at(sl);
        if (tab[pv].key == EDGE_EMPTY ? dd != 0 : dd > dist_at(pv) + 1)
          throw std::logic_error("hot table not in Robin Hood order");
      }
    }
    if (rh)  // (slot ranges on all threads: each slot's owner is its own node)
      parallel_for(cap, [&](uint64_t a, uint64_t b) {
        for (uint64_t s = a; s < b; ++s)
          if (occ[s] != NONE) {
            const HNode& h = nodes[occ[s]];
            HotSlot& o = tab[s];
            o.sig = h.sig;
            o.hf = hf_of(h);
            o.end_filter = end_of(h);
            hid[occ[s]] = uint32_t(s);
          }
      });
  }

  phase("hot: place");
  // ---- 3b'. chain nodes (gm_common.h): path compression of single-filter
  // tails.  tcl[i] = the length of the chain that starts at exact node i (1: i
  // is a leaf holding a filter; 2: i holds nothing but one exact child that is
  // such a leaf), 0 if none.  A parent is created before its children, so one
  // pass in reverse index order sees every child first.
  // A chain trades one L2-hit read of the chain node's second half for the
  // probes of c1 and c2; those are Infinity-Cache hits while the hot tables fit
  // it (256 MiB), and there the trade does not pay (C2, 240 MB of tables: +0.9 %
  // kernel time; C3, 2.4 GB: -3 %, profiles/r03_ab/chain_ab.txt).  So chains are
  // built for larger tables only; GM_CHAIN=0/1 forces (A/B knob).
  uint64_t n_chain = 0;
  bool chains = hot_total * sizeof(HotSlot) > (256ull << 20);
  if (const char* e = knob("GM_CHAIN")) chains = atoi(e) != 0;
  if (knob("GM_NO_CHAIN")) chains = false;
  if (chains) {
    std::vector<uint32_t> nex(NN, 0), exch(NN, NONE);
    for (uint64_t i = 1; i < NN; ++i)
      if (nodes[i].kind == 0) {
        nex[nodes[i].parent]++;
        exch[nodes[i].parent] = uint32_t(i);
      }
    std::vector<uint8_t> tcl(NN, 0);
    for (uint64_t i = NN; i-- > 1;) {
      const HNode& h = nodes[i];
      if (h.kind != 0 || h.plus_child != NONE || h.hash_child != NONE) continue;
      if (nex[i] == 0) tcl[i] = h.end_filter != NONE ? 1 : 0;
      else if (nex[i] == 1 && h.end_filter == NONE && tcl[exch[i]] == 1) tcl[i] = 2;
    }
    for (uint64_t i = 1; i < NN; ++i) {
      const HNode& h = nodes[i];
      if (h.kind == 2 || h.plus_child != NONE || nex[i] != 1 || hid[i] == NONE || (hid[i] & HOT_INLINE)) continue;
      const uint32_t c1 = exch[i];
      if (!tcl[c1]) continue;
      HotSlot& o = hot[hot_off[hot_table(h.depth)] + hid[i]];
      const HNode& leaf = tcl[c1] == 1 ? nodes[c1] : nodes[exch[c1]];
      o.sig = nodes[c1].word;
      o.hf |= HOT_CHAIN;
      o.p_sig = tcl[c1] == 1 ? NONE : nodes[exch[c1]].word;
      o.p_hf = HF_NONE;
      o.p_end = end_of(leaf);
      ++n_chain;
    }
  }
  if (knob("GM_INDEX_STATS")) {  // diagnostics: the hot tables' sizes (stderr)
    fprintf(stderr, "[gm_index] chain nodes %llu\n", (unsigned long long)n_chain);
    uint64_t inl_n = 0;
    for (uint64_t i = 1; i < NN; ++i) inl_n += inl[i];
    fprintf(stderr, "[gm_index] nodes %llu, inline '+' nodes %llu\n", (unsigned long long)NN,
            (unsigned long long)inl_n);
    for (int t = 0; t < HOT_TABLES; ++t)
      if (hot_n[t])
        fprintf(stderr, "[gm_index] hot table %d: %llu slots used of %llu (%.1f MB)%s\n", t,
                (unsigned long long)hot_n[t], (unsigned long long)hot_cap[t], hot_cap[t] * 32.0 / 1e6,
                mph_cap[t] ? ((mph_ovf >> t) & 1u ? " mph+overflow" : " mph") : "");
  }
  phase("hot tables");
  // ---- 3c. exact-edge filters (gm_common.h), for tables whose parents have
  // on average >= 4 exact children and whose filter fits the L2 budget
  std::vector<uint64_t> ex_edges(HOT_TABLES, 0), ex_parents(HOT_TABLES, 0);
  for (uint64_t i = 1; i < NN; ++i) {
    const HNode& h = nodes[i];
    if (h.kind != 0 || hid[i] == NONE) continue;
    ex_edges[hot_table(h.depth)]++;
  }
  for (uint64_t i = 0; i < NN; ++i)
    if ((nodes[i].flags & NF_HAS_EXACT) && hid[i] != NONE) ex_parents[hot_table(nodes[i].depth + 1)]++;
  uint64_t efilt_off[HOT_TABLES] = {0}, efilt_total = 0;
  uint32_t efilt_mask[HOT_TABLES] = {0};
  for (int t = 0; t < HOT_TABLES; ++t) {
    if (knob("GM_NO_EDGE_FILTER")) break;  // A/B knob
    if (!ex_edges[t] || (ex_edges[t] < 4 * ex_parents[t] && !knob("GM_EFILT_ALL"))) continue;  // A/B knob
    if (mph_cap[t]) continue;  // an MPH table's bucket words carry its filter
    // 4-8 bits per key: the filter is a dependent read in front of every exact
    // probe and pays only while it stays in L2 (C2 A/B, bits per key -> kernel ms:
    // 16-32 10.04, 8-16 9.54, 4-8 9.37, 2-4 9.40, 1-2 9.60, no filter 9.50)
    uint64_t div = 8;  // GM_EFILT_DIV: A/B knob (words = keys / div)
    if (const char* e = knob("GM_EFILT_DIV")) div = std::min<uint64_t>(64, std::max<uint64_t>(1, strtoull(e, nullptr, 10)));
    const uint64_t words = std::max<uint64_t>(32, next_pow2(ex_edges[t] / div + 1));
    // an L2 budget (a filter that does not stay in L2 costs more than it saves:
    // C3's 4 MB one took its kernel from 14.1 to 14.9 ms); GM_EFILT_MAX_KB: A/B knob
    uint64_t max_kb = 1024;
    if (const char* e = knob("GM_EFILT_MAX_KB")) max_kb = strtoull(e, nullptr, 10);
    if (words * 4 > max_kb * 1024) continue;
    efilt_off[t] = efilt_total;
    efilt_mask[t] = uint32_t(words - 1);
    efilt_total += words;
  }
  std::vector<uint32_t> efilt(efilt_total, 0u);
  for (uint64_t i = 1; i < NN; ++i) {
    const HNode& h = nodes[i];
    if (h.kind != 0 || hid[i] == NONE) continue;
    const int t = hot_table(h.depth);
    if (!efilt_mask[t]) continue;
    const uint32_t fh = edge_filter_hash(hot_key(hid[h.parent], h.word, h.depth - 1));
    efilt[efilt_off[t] + edge_filter_word(fh, efilt_mask[t])] |= edge_filter_bits(fh);
  }

  phase("edge filter");
  // ---- 4. word dictionary (open addressing by hash, verified by bytes)
  uint64_t nw = word_ids.size();
  // Load <= 0.25, and a small vocabulary spread over up to 2 MB (32 slots per
  // word): a word off its home slot costs its wave a dependent L2 round trip
  // whenever any of the 64 lanes holds it, and the few words of the upper
  // levels are in nearly every wave (C2's 2,192 words: 4 -> 32 slots per word
  // took k_match_fused 8.72 -> 8.48 ms, profiles/r03_ab/dict_load.txt).  Only
  // the slots holding words are ever read, so the sparse table's cache
  // footprint stays ~one line per word.  GM_DICT_MUL (A/B knob): slots per word.
  uint64_t dslots = std::max<uint64_t>(nw * 4 + 4, std::min<uint64_t>(nw * 32, 1ull << 17));
  if (const char* e = knob("GM_DICT_MUL"))
    dslots = nw * std::min<uint64_t>(64, std::max<uint64_t>(1, strtoull(e, nullptr, 10))) + 4;
  uint64_t dcap = next_pow2(dslots);
  std::vector<DictSlot> dict(dcap, DictSlot{0, DICT_EMPTY_LEN, 0});
  for (uint64_t k = 0; k < nw; ++k) {
    uint64_t s = dict_slot(word_hash[k], dcap - 1);
    while (dict[s].len != DICT_EMPTY_LEN) s = (s + 1) & (dcap - 1);
    dict[s] = DictSlot{word_head[k], word_len[k], word_ids[k]};
  }
  uint32_t plus_word = NONE, hash_word = NONE;
  {
    auto it = wid.find(std::string_view("+", 1));
    if (it != wid.end()) plus_word = it->second;
    it = wid.find(std::string_view("#", 1));
    if (it != wid.end()) hash_word = it->second;
  }

  phase("dictionary");
  // ---- 5. subscriber CSR per unique filter id (duplicates concatenated)
  std::vector<uint64_t> soff(nf + 1, 0);
  std::vector<uint32_t> sids;
  if (sub_off) {
    for (uint64_t i = 0; i < n; ++i) soff[id_of[i] + 1] += sub_off[i + 1] - sub_off[i];
    for (uint32_t f = 0; f < nf; ++f) soff[f + 1] += soff[f];
    sids.resize(soff[nf]);
    std::vector<uint64_t> cur(soff.begin(), soff.end() - 1);
    for (uint64_t i = 0; i < n; ++i) {
      uint64_t c = sub_off[i + 1] - sub_off[i];
      if (c) std::memcpy(&sids[cur[id_of[i]]], sub_ids + sub_off[i], c * 4);
      cur[id_of[i]] += c;
    }
  }
  std::vector<uint16_t> flen(nf);
  for (uint32_t f = 0; f < nf; ++f) flen[f] = uint16_t(std::min<uint64_t>(FOV[f + 1] - FOV[f], 65535));

  phase("subscribers");
  // ---- 6. upload: one allocation, 256-B aligned sections, the subscriber
  // CSR last.  An index without shard ids keeps a host mirror of the blob up
  // to the subscriber CSR for in-place updates, with headroom for appended
  // nodes, words and filters (an update of the subscriber lists writes a new
  // CSR of its own, gm_subs.cpp).
  // (no context but an `out`: a host-only index whose view points into its
  // mirror -- the CPU test of the in-place update, tests/asan/)
  const bool host_mirror = !ctx && out && !host_only;
  if (host_mirror && (gids || sub_off)) {
    delete idx;
    return set_err(ctx, EMQX_GM_EINVAL, "index_build: host-only index without subscribers or shard ids only");
  }
  // keep_mirror: the layout reserves update headroom and the index carries a
  // Mirror; its host copy of the blob is kept from here (eager) or downloaded
  // on the line's first update (load_mirror_blob), see EMQX_GM_OPEN_MIRROR_*
  const bool keep_mirror = host_mirror || (ctx && !gids && !knob("GM_NO_MIRROR"));
  const uint64_t nodes_cap = keep_mirror ? NN + NN / 4 + 1024 : NN;
  const uint64_t arena_cap = keep_mirror ? arena.size() + arena.size() / 4 + 65536 : arena.size();
  const uint64_t flen_cap = keep_mirror ? uint64_t(nf) + nf / 4 + 1024 : nf;
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  size_t o_nodes = 0;
  size_t o_dict = o_nodes + al(nodes_cap * sizeof(Node));
  size_t o_edges = o_dict + al(dcap * sizeof(DictSlot));
  size_t o_hot = o_edges + al(dedges.size() * sizeof(EdgeSlot));
  size_t o_arena = o_hot + al(hot.size() * sizeof(HotSlot));
  size_t o_flen = o_arena + al(arena_cap + 64);
  size_t o_gmap = o_flen + al(flen_cap * 2 + 2);
  size_t o_efilt = o_gmap + al(idx->gmap.size() * 4 + 4);
  size_t o_mph = o_efilt + al(efilt.size() * 4 + 4);
  size_t o_d0 = o_mph + al(mph_word.size() * 8);
  size_t o_soff = o_d0 + al(16);
  // (a plain index's offsets stay zero past nf: appended filters have no subscribers)
  size_t o_sids = o_soff + al((keep_mirror && !sub_off ? flen_cap + 1 : soff.size()) * 8);
  size_t total = o_sids + al(sids.size() * 4 + 4);

  if (host_only) {  // compile-only self check (no device): report the table sizes
    emqx_gm_index_info_t& in = *host_only;
    in = emqx_gm_index_info_t{};
    in.n_filters = nf;
    in.n_wildcard = n_wild;
    in.n_nodes = NN;
    in.n_edges = n_edges;
    in.n_words = nw;
    in.n_subs = sids.size();
    in.device_bytes = total;
    in.max_depth = max_depth;
    in.trie_empty = n_wild == 0;
    delete idx;
    return EMQX_GM_OK;
  }
  hipError_t e = hipSuccess;
  if (!host_mirror) {
    e = hipSetDevice(ctx->device);
    if (e == hipSuccess) e = hipMalloc(&idx->dev_base, total);
    if (e != hipSuccess) {
      delete idx;
      return set_err(ctx, EMQX_GM_ENOMEM, std::string("index_build: hipMalloc: ") + hipGetErrorString(e));
    }
  }
  idx->dev_bytes = total;
  bool eager = host_mirror || o_soff <= kEagerMirrorBytes;  // (keep_mirror: the mirror's policy)
  if (keep_mirror && !host_mirror) {
    if (const char* pol = knob("GM_MIRROR")) eager = !strcmp(pol, "eager");  // A/B and test knob
    if (ctx->open_flags & EMQX_GM_OPEN_MIRROR_EAGER) eager = true;
    if (ctx->open_flags & EMQX_GM_OPEN_MIRROR_LAZY) eager = false;
  }
  // the tables, region by region (offset in the blob, source, bytes)
  const std::pair<size_t, std::pair<const void*, size_t>> regions[] = {
      {o_nodes, {dnodes.data(), NN * sizeof(Node)}},
      {o_dict, {dict.data(), dcap * sizeof(DictSlot)}},
      {o_edges, {dedges.data(), dedges.size() * sizeof(EdgeSlot)}},
      {o_hot, {hot.data(), hot.size() * sizeof(HotSlot)}},
      {o_arena, {arena.data(), arena.size()}},
      {o_soff, {soff.data(), soff.size() * 8}},
      {o_sids, {sids.data(), sids.size() * 4}},
      {o_flen, {flen.data(), flen.size() * 2}},
      {o_gmap, {idx->gmap.data(), idx->gmap.size() * 4}},
      {o_efilt, {efilt.data(), efilt.size() * 4}},
      {o_mph, {mph_word.data(), mph_word.size() * 8}}};
  const uint32_t d0_none[4] = {NONE, 0, HF_NONE, NONE};
  HostBytes hb;
  if (host_mirror || (keep_mirror && eager) || total < (size_t(1) << 20)) {
    // the blob assembled on the host (it stays as the mirror) and sent in one copy
    hb.assign(total, 0);
    for (const auto& r : regions)
      if (r.second.second) std::memcpy(hb.data() + r.first, r.second.first, r.second.second);
    std::memcpy(hb.data() + o_d0, d0_none, sizeof d0_none);
    if (!host_mirror) e = hipMemcpy(idx->dev_base, hb.data(), total, hipMemcpyHostToDevice);
  } else {
    // no host copy of the blob is kept: the device blob zeroed, then each table
    // streamed through two page-locked buffers (all threads fill one while the
    // other crosses PCIe) -- no 38-GB host assembly, no pageable copy (C5: 11.3 s
    // for the assembly and the copy before)
    e = upload_regions(ctx, static_cast<uint8_t*>(idx->dev_base), total, regions, sizeof regions / sizeof regions[0],
                       o_d0, d0_none, sizeof d0_none);
  }
  if (e != hipSuccess) {
    (void)hipFree(idx->dev_base);
    delete idx;
    return set_err(ctx, EMQX_GM_EDEVICE, std::string("index_build: upload: ") + hipGetErrorString(e));
  }
  if (keep_mirror) {
    auto* m = new Mirror;
    m->blob_size = o_soff;  // the mirror stops at the subscriber CSR
    if (eager) {
      hb.resize(o_soff);
      hb.shrink_to_fit();
      m->blob = std::move(hb);
    }
    m->o_nodes = o_nodes;
    m->o_dict = o_dict;
    m->o_edges = o_edges;
    m->o_hot = o_hot;
    m->o_arena = o_arena;
    m->o_flen = o_flen;
    m->o_efilt = o_efilt;
    m->o_mph = o_mph;
    m->nodes_n = NN;
    m->nodes_cap = nodes_cap;
    m->arena_n = arena.size();
    m->arena_cap = arena_cap;
    m->flen_cap = flen_cap;
    m->dict_used = nw;
    for (int d = 0; d < EDGE_DEPTHS; ++d) m->edge_used[d] = tabs[d].used;
    for (int t = 0; t < HOT_TABLES; ++t) m->hot_used[t] = hot_n[t];
    for (int t = 0; t < HOT_TABLES; ++t) m->mph_ovf_used[t] = mph_ovf_n[t];
    idx->mirror = m;
  }
  // the view's base: the device blob, or (host-only index) the mirror
  uint8_t* B = host_mirror ? idx->mirror->blob.data() : static_cast<uint8_t*>(idx->dev_base);
  HostBytes().swap(hb);  // (a lazy mirror: no host copy of the tables stays)

  phase("upload");
  IndexView& v = idx->view;
  v.nodes = reinterpret_cast<const Node*>(B + o_nodes);
  v.dict = reinterpret_cast<const DictSlot*>(B + o_dict);
  v.d0_root = reinterpret_cast<const uint32_t*>(B + o_d0);
  v.edges = reinterpret_cast<const EdgeSlot*>(B + o_edges);
  v.hot = reinterpret_cast<const HotSlot*>(B + o_hot);
  v.arena = B + o_arena;
  v.sub_off = host_mirror ? nullptr : reinterpret_cast<const uint64_t*>(B + o_soff);
  v.sub_ids = host_mirror ? nullptr : reinterpret_cast<const uint32_t*>(B + o_sids);
  v.gmap = idx->gmap.empty() ? nullptr : reinterpret_cast<const uint32_t*>(B + o_gmap);
  v.dict_mask = dcap - 1;
  for (int d = 0; d < EDGE_DEPTHS; ++d) {
    v.etab_off[d] = etab_off[d];
    v.etab_mask[d] = etab_mask[d];
  }
  for (int t = 0; t < HOT_TABLES; ++t) {
    v.hot_off[t] = hot_off[t];
    v.hot_cap[t] = hot_cap[t];
    v.efilt_off[t] = efilt_off[t];
    v.efilt_mask[t] = efilt_mask[t];
  }
  v.efilt = reinterpret_cast<const uint32_t*>(B + o_efilt);
  v.mph_word = reinterpret_cast<const uint64_t*>(B + o_mph);
  v.mph_ovf = mph_ovf;
  v.l1_bypass = 0;
  v.hot_policy = 1;  // (sc1, for the tables GM_L1_BYPASS selects; both A/B knobs, read per call too)
  if (const char* e = knob("GM_L1_BYPASS")) v.l1_bypass = uint32_t(strtoul(e, nullptr, 0));
  for (int t = 0; t < HOT_TABLES; ++t) {
    v.mph_off[t] = mph_off[t];
    v.mph_nb[t] = mph_nb[t];
    v.mph_cap[t] = mph_cap[t];
  }
  v.root_sig = nodes[0].sig;
  v.root_hash = nodes[0].hash_child == NONE ? NONE : nodes[nodes[0].hash_child].end_filter;
  v.root_flags = nodes[0].plus_child != NONE ? HOT_PLUS : 0u;
  v.flags = 0;
  for (int t = 0; t < HOT_TABLES; ++t)
    if (hot_cap[t] * sizeof(HotSlot) >= (1ull << 31)) v.flags |= IX_HOT_FLAT;
  if (knob("GM_HOT_FLAT")) v.flags |= IX_HOT_FLAT;  // test knob: exercise the flat-load path
  // every per-depth table is Robin Hood ordered; the shared last one is not (GM_NO_RH_EXIT: A/B knob)
  v.rh_mask = knob("GM_NO_RH_EXIT") ? 0u : (1u << (HOT_TABLES - 1)) - 1u;
  v.n_nodes = uint32_t(NN);
  v.n_filters = nf;
  v.plus_word = plus_word;
  v.hash_word = hash_word;
  idx->dev_flen = reinterpret_cast<uint16_t*>(B + o_flen);
  // the root's '+' record, from the depth-1 hot table on the device
  // (gm_match.hip); IX_D0 once it is written
  if (!host_mirror) {
    const int rc = refresh_d0(ctx, v, static_cast<uint8_t*>(idx->dev_base) + o_d0);
    if (rc < 0) {
      free_index(idx);
      return rc;
    }
    if (rc == 0) v.flags |= IX_D0;
  }

  if (sub_off) idx->subs = SubTable(std::move(soff), {});
  emqx_gm_index_info_t& in = idx->info;
  in.n_filters = nf;
  in.n_wildcard = n_wild;
  in.n_nodes = NN;
  in.n_edges = n_edges;
  in.n_words = nw;
  in.n_subs = sids.size();
  in.device_bytes = total;
  in.max_depth = max_depth;
  in.trie_empty = n_wild == 0;
  *out = idx;
  return EMQX_GM_OK;
}

// (the device build defines it in gm_match.hip; the host-only ASAN build of
// this file links this stand-in, which reports "not written")
__attribute__((weak)) int refresh_d0(emqx_gm_ctx*, const IndexView&, void*) { return 1; }

namespace {
struct SpareBlob {
  void* p = nullptr;
  size_t bytes = 0;
};
constexpr int kSpareDevices = 64;
std::mutex g_spare_mu;
// per device, oldest first: at most one per context open there (a
// multi-device context listing a device twice opens two: each replica line
// frees and reuses its own size)
std::vector<SpareBlob> g_spare[kSpareDevices];
int g_ctx_open[kSpareDevices] = {};  // (under g_spare_mu)
// blobs below this size allocate quickly anyway (GM_SPARE_BLOB_MIN, bytes; 0: off)
size_t spare_min() {
  const char* e = knob("GM_SPARE_BLOB_MIN");
  return e ? size_t(strtoull(e, nullptr, 10)) : size_t(256) << 20;
}
}  // namespace

void* take_spare_blob(int device, size_t bytes) {
  const size_t lo = spare_min();
  if (device < 0 || device >= kSpareDevices || !lo || bytes < lo) return nullptr;
  std::lock_guard<std::mutex> lk(g_spare_mu);
  auto& v = g_spare[device];
  size_t best = v.size();
  for (size_t i = 0; i < v.size(); ++i)
    if (v[i].bytes >= bytes && v[i].bytes - bytes <= bytes / 4 && (best == v.size() || v[i].bytes < v[best].bytes))
      best = i;
  if (best == v.size()) return nullptr;
  void* p = v[best].p;
  v.erase(v.begin() + best);
  return p;
}

void give_spare_blob(int device, void* p, size_t bytes) {
  if (!p) return;
  const size_t lo = spare_min();
  std::vector<void*> drop{p};
  bool keep = device >= 0 && device < kSpareDevices && lo && bytes >= lo;
  if (keep) {
    std::lock_guard<std::mutex> lk(g_spare_mu);
    keep = g_ctx_open[device] > 0;  // (no context left on the device: nothing would reuse or trim it)
  }
  if (keep) {
    // hipFree waits for the device's work; so does keeping the blob for reuse
    (void)hipDeviceSynchronize();
    std::lock_guard<std::mutex> lk(g_spare_mu);
    auto& v = g_spare[device];
    drop.clear();
    v.push_back(SpareBlob{p, bytes});  // the newest stays (a line of updates frees its own size)
    while (v.size() > size_t(std::max(1, g_ctx_open[device]))) {
      drop.push_back(v.front().p);
      v.erase(v.begin());
    }
  }
  for (void* q : drop) (void)hipFree(q);
}

void note_ctx_open(int device) {
  if (device < 0 || device >= kSpareDevices) return;
  std::lock_guard<std::mutex> lk(g_spare_mu);
  ++g_ctx_open[device];
}

void note_ctx_close(int device) {
  if (device < 0 || device >= kSpareDevices) return;
  std::lock_guard<std::mutex> lk(g_spare_mu);
  if (g_ctx_open[device] > 0) --g_ctx_open[device];
}

void trim_spare_blob(int device) {
  if (device < 0 || device >= kSpareDevices) return;
  std::vector<SpareBlob> v;
  {
    std::lock_guard<std::mutex> lk(g_spare_mu);
    v.swap(g_spare[device]);
  }
  if (!v.empty()) (void)hipSetDevice(device);
  for (const SpareBlob& b : v) (void)hipFree(b.p);
}

void free_index(emqx_gm_index* idx) {
  if (!idx) return;
  for (emqx_gm_index* r : idx->reps)
    if (r && r->refs.fetch_sub(1) == 1) free_index(r);
  idx->reps.clear();
  for (emqx_gm_index* s : idx->shards)
    if (s && s->refs.fetch_sub(1) == 1) free_index(s);
  idx->shards.clear();
  if (idx->route) free_route(idx->route);
  if (idx->ov) free_overlay(idx);
  delete idx->mirror;
  if (idx->dev_base || idx->dev_subs) {
    (void)hipSetDevice(idx->device);
    if (idx->dev_base && !idx->blob_owner) give_spare_blob(idx->device, idx->dev_base, idx->dev_bytes);
    if (idx->dev_subs) (void)hipFree(idx->dev_subs);
  }
  if (idx->blob_owner && idx->blob_owner->refs.fetch_sub(1) == 1) free_index(idx->blob_owner);
  delete idx;
}

}  // namespace gm
