// gm_match.hip — CDNA4 (gfx950) kernels for batch topic matching and fan-out.
//
// Hot path (replaces emqx_trie:match/1 + emqx_router:match_routes/1,
// apps/emqx/src/emqx_trie.erl:147-333, apps/emqx/src/emqx_router.erl:128-145):
//
//   k_match_fused  main pass (default): a block stages its 256 topics' text in
//                  LDS; each lane splits its topic into words, hashes them and
//                  resolves them in the word dictionary (verified
//                  byte-for-byte) into registers; then each wave walks its
//                  64-topic tile with the frontier of all 64 topics as ONE
//                  compacted LDS work list (ballot + mbcnt), one entry per
//                  lane per round: an exact probe and a '+' probe per entry,
//                  each one 16-B raw buffer load of a 32-B hot slot (edge probe
//                  and node record in one line).  Matches are staged per tile
//                  as [slot][lane].
//   k_tokenize + k_walk_coop / k_walk
//                  the same work as two kernels through HBM word ids (A/B
//                  forms, GM_MATCH_MAIN; k_walk keeps a lane-private frontier
//                  in registers).
//   k_match_lds    the same walk with the frontier in LDS (capacity FC).  As
//                  the LISTED pass it re-walks the topics whose frontier or
//                  row outgrew the main pass (count read on the device, so no
//                  host round trip between the passes).
//   (k_walk tile sums) / scan / k_assemble
//                  count -> scan -> write: builds the CSR (row_off u64, ids u32).
//   k_slow_walk / k_slow_emit / k_copy_slow
//                  device slow path: one workgroup per topic the listed pass
//                  could not hold, frontier in HBM (bounded by the node
//                  count), matches as a bitmap over filter ids, emitted in
//                  ascending id order.  No truncation, no CPU fallback.
//
// Fan-out (replaces emqx_broker:dispatch/2 + do_dispatch, emqx_broker.erl:
// 296-322, 506-530): k_fanout_seglen -> scan -> k_fanout_copy, a load-balanced
// CSR gather in which every workgroup owns a fixed range of OUTPUT elements,
// so a 1M-subscriber row is split across many workgroups.
//
// Everything here is integer/byte work bound by HBM/L2 latency and bandwidth;
// there is no MFMA.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "gm_gather.h"
#include "gm_internal.h"

namespace gm {

// ---------------------------------------------------------------------------
// device helpers
// ---------------------------------------------------------------------------

// Stream accesses (topic text, word ids, headers, staging, counts, the CSR)
// touch each byte once; NT = non-temporal, so they do not evict the index
// tables from L2 / the Infinity Cache (GM_NT knob, A/B).
template <bool NT, class T>
__device__ __forceinline__ T ld_s(const T* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT, class T>
__device__ __forceinline__ void st_s(T* p, T v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// Byte reader over a lane's topic with an 8-byte cache (aligned 8-B loads;
// topic buffers are padded, emqx_gpu_match.h).
struct ByteReader {
  const uint8_t* base;
  uint64_t cached_addr;
  uint64_t cached;
  __device__ __forceinline__ uint32_t get(uint64_t p) {
    const uint64_t a = p & ~7ull;
    if (a != cached_addr) {
      cached_addr = a;
      cached = *reinterpret_cast<const uint64_t*>(base + a);
    }
    return uint32_t(cached >> ((p & 7) * 8)) & 0xFFu;
  }
};

// One tokenized level word: hash, first 8 bytes, length, first byte.
struct WordTok {
  uint32_t h;  // dict_hash
  uint64_t head;
  uint64_t start;
  uint32_t len;
  uint32_t b0;
};

// Tokenize the word starting at `pos`; leaves `pos` on the '/' (or end).
template <class RD>
__device__ __forceinline__ WordTok next_word(RD& rd, uint64_t& pos, uint64_t end) {
  WordTok w;
  w.start = pos;
  w.head = 0;
  uint32_t h = DICT_HASH_SEED;
  uint64_t chunk = 0;
  uint32_t k = 0;
  while (pos < end) {
    const uint32_t b = rd.get(pos);
    if (b == '/') break;
    chunk |= uint64_t(b) << ((k & 7) * 8);
    ++k;
    ++pos;
    if ((k & 7) == 0) {
      if (k == 8) w.head = chunk;
      h = dict_hash_step(h, chunk);
      chunk = 0;
    }
  }
  if (k & 7) {
    if (k < 8) w.head = chunk;
    h = dict_hash_step(h, chunk);
  }
  w.h = dict_hash_final(h, k);
  w.len = k;
  w.b0 = uint32_t(w.head & 0xFF);
  return w;
}

__device__ __noinline__ bool tail_equal(const uint8_t* a, const uint8_t* b, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i)
    if (a[i] != b[i]) return false;
  return true;
}

__device__ __forceinline__ DictSlot dict_at(const IndexView& ix, uint64_t s) { return ix.dict[s]; }
// a depth-1 node's record as the level-0 round takes it: {hot id, sig, hf, end_filter}
constexpr uint4 D1_NONE = {NONE, 0u, HF_NONE, NONE};

// Resolve a word in the dictionary starting from the (prefetched) first slot.
// A hit is exact: length + first 8 bytes compared inline, the rest against
// the arena (only for words longer than 8 bytes).
__device__ __forceinline__ uint32_t dict_resolve(const IndexView& ix, const WordTok& w, DictSlot d,
                                                 const uint8_t* tb) {
  // the common outcomes decided from the prefetched slot with selects
  const bool empty0 = d.len == DICT_EMPTY_LEN;
  const bool hit0 = d.len == w.len && d.head == w.head && w.len <= 8;
  if (empty0 || hit0) return hit0 ? d.word : NONE;
  for (uint64_t s = dict_slot(w.h, ix.dict_mask);;) {
    if (d.len == DICT_EMPTY_LEN) return NONE;
    if (d.len == w.len && d.head == w.head &&
        (w.len <= 8 || tail_equal(ix.arena + d.word + 8, tb + w.start + 8, w.len - 8)))
      return d.word;
    s = (s + 1) & ix.dict_mask;
    d = dict_at(ix, s);
  }
}

__device__ __forceinline__ DictSlot dict_first(const IndexView& ix, const WordTok& w) {
  return dict_at(ix, dict_slot(w.h, ix.dict_mask));
}


__device__ __forceinline__ uint32_t edge_lookup(const IndexView& ix, uint32_t depth, uint32_t parent,
                                                uint32_t word) {
  const int d = edge_depth(depth);
  const EdgeSlot* tab = ix.edges + ix.etab_off[d];
  const uint64_t mask = ix.etab_mask[d];
  const uint64_t key = edge_key(parent, word);
  for (uint64_t s = edge_slot(key, mask);; s = (s + 1) & mask) {
    const EdgeSlot e = tab[s];
    if (e.key == key) return e.child;
    if (e.key == EDGE_EMPTY) return NONE;
  }
}

// Literal lookup of a wildcard topic as a filter string: emqx_router:
// lookup_routes(Topic) for a topic containing '+' / '#' words
// (emqx_router.erl:128-134 with match_trie = []).
__device__ uint32_t literal_lookup(const IndexView& ix, const uint8_t* tb, uint64_t pos, uint64_t end) {
  ByteReader rd{tb, ~0ull, 0};
  uint32_t node = 0;
  for (uint32_t depth = 0;; ++depth) {
    const WordTok w = next_word(rd, pos, end);
    const uint32_t wid = dict_resolve(ix, w, dict_first(ix, w), tb);
    if (wid == NONE) return NONE;
    const uint32_t c = edge_lookup(ix, depth, node, wid);
    if (c == NONE) return NONE;
    node = c & REF_MASK;
    if (pos >= end) break;
    ++pos;
  }
  return ix.nodes[node].end_filter;
}

__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t& total) {
  const int lane = threadIdx.x & 63;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  total = __shfl(x, 63, 64);
  return x - v;
}

// ---------------------------------------------------------------------------
// match kernels
// ---------------------------------------------------------------------------
// Staging layout per 64-topic tile: [slot k][lane], FAST_MC slots, so the k-th
// match of every lane is one coalesced 256-B row.
__device__ __forceinline__ uint64_t stage_index(uint64_t tile, uint32_t k, int lane) {
  return tile * (64ull * FAST_MC) + uint64_t(k) * 64u + uint32_t(lane);
}

// A hot slot as the kernel reads it: {key, sig, hf} in one dwordx4; the end
// filter (a second dword of the same line) only on the topic's last level.
struct HotRec {
  uint4 a;      // key lo, key hi, sig, hf (| HOT_PLUS)
  uint32_t ef;  // end_filter (NONE unless loaded)
};
// Hot-table loads go through a buffer resource (raw buffer loads, 32-bit byte
// offset from the table base): at C2 they took 4 % less time and ~10 % fewer
// L2 requests per topic than the same loads as flat global_load (A/B in
// scripts/mem_experiment.sh).  An index with a table of 2 GiB or more
// (IX_HOT_FLAT) uses flat loads.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t hot_rsrc(const HotSlot* tab) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<HotSlot*>(tab), (short)0, 0x7FFFFFFF, 0x00020000);
}
// pol (wave-uniform; 0 = default): the cache policy of a probe of a table
// selected by IndexView::l1_bypass (A/B knobs GM_L1_BYPASS, GM_HOT_POLICY):
// 1 sc1 (no L1 fill), 2 sc0 sc1 (system scope), 3 nt, 4 sc1 nt
__device__ __forceinline__ HotRec hot_load(const HotSlot* tab, uint32_t s, bool with_end, bool flat, uint32_t pol = 0) {
  HotRec r;
  if (!flat) {
    const __amdgpu_buffer_rsrc_t rs = hot_rsrc(tab);
    const auto v = pol == 0 ? __builtin_amdgcn_raw_buffer_load_b128(rs, s * 32u, 0, 0)
                   : pol == 1 ? __builtin_amdgcn_raw_buffer_load_b128(rs, s * 32u, 0, 16)
                   : pol == 2 ? __builtin_amdgcn_raw_buffer_load_b128(rs, s * 32u, 0, 17)
                   : pol == 3 ? __builtin_amdgcn_raw_buffer_load_b128(rs, s * 32u, 0, 2)
                              : __builtin_amdgcn_raw_buffer_load_b128(rs, s * 32u, 0, 18);
    r.a = make_uint4(v[0], v[1], v[2], v[3]);
    r.ef = with_end ? __builtin_amdgcn_raw_buffer_load_b32(rs, s * 32u + 16u, 0, 0) : NONE;
  } else {
    const uint32_t* p = reinterpret_cast<const uint32_t*>(tab + s);
    r.a = *reinterpret_cast<const uint4*>(p);
    r.ef = with_end ? p[4] : NONE;
  }
  return r;
}
__device__ __forceinline__ bool hot_is(const HotRec& r, uint64_t key) {
  return r.a.x == uint32_t(key) && r.a.y == uint32_t(key >> 32);
}
__device__ __forceinline__ bool hot_empty(const HotRec& r) { return r.a.x == 0xFFFFFFFFu && r.a.y == 0xFFFFFFFFu; }
// Linear probing from the home slot s of `key` (whose record r is already
// loaded); returns the slot index of `key` or NONE.  rh: the table is Robin
// Hood ordered (gm_index.cpp), so an absent key is known at the first slot
// whose key lies nearer its own home than this probe is from `key`'s.
__device__ __forceinline__ uint32_t hot_resolve(const HotSlot* tab, uint32_t cap, uint64_t key, uint32_t s,
                                                HotRec& r, bool with_end, bool flat, bool rh) {
  uint32_t dist = 0;
  while (!hot_is(r, key)) {
    if (hot_empty(r)) return NONE;
    if (rh) {
      const uint32_t h = uint32_t(hot_slot((uint64_t(r.a.y) << 32) | r.a.x, cap));
      if ((s >= h ? s - h : s + cap - h) < dist) return NONE;
    }
    s = s + 1 == cap ? 0 : s + 1;
    ++dist;
    r = hot_load(tab, s, with_end, flat);
  }
  return s;
}

// The home slot of `key` in hot table ht (wave-uniform): an MPH table first
// reads the key's bucket displacement (a small array that stays in L2), then
// its one perfect slot; an open-addressing table hashes straight to the home.
__device__ __forceinline__ uint32_t hot_home(const IndexView& ix, int ht, uint64_t key, uint64_t cap) {
  if (const uint32_t mc = ix.mph_cap[ht]) {
    const uint64_t w = ix.mph_word[ix.mph_off[ht] + mph_bucket(key, ix.mph_nb[ht])];
    return mph_slot(key, uint32_t(w) & 0xFFFFu, mc);
  }
  return uint32_t(hot_slot(key, cap));
}
// An MPH table's bucket word for `key` (one L2 read): whether the table may
// hold the key (its Bloom bits) and, if so, the key's perfect slot.
__device__ __forceinline__ bool mph_gate(const IndexView& ix, int ht, uint64_t key, uint32_t mc, uint32_t& s) {
  const uint64_t w = ix.mph_word[ix.mph_off[ht] + mph_bucket(key, ix.mph_nb[ht])];
  s = mph_slot(key, uint32_t(w) & 0xFFFFu, mc);
  return mph_may_hold(w, key);
}
// hot_resolve for either kind of table: an MPH table's key is at its perfect
// slot, or (once an in-place update put keys there) in the overflow region.
__device__ __forceinline__ uint32_t hot_resolve_x(const IndexView& ix, int ht, const HotSlot* tab, uint32_t cap,
                                                  uint64_t key, uint32_t s, HotRec& r, bool with_end, bool flat,
                                                  bool rh) {
  if (const uint32_t mc = ix.mph_cap[ht]) {
    if (hot_is(r, key)) return s;
    if (!((ix.mph_ovf >> ht) & 1u)) return NONE;
    for (s = mph_ovf_home(key, mc, cap);; s = s + 1 == cap ? mc : s + 1) {
      r = hot_load(tab, s, with_end, flat);
      if (hot_is(r, key)) return s;
      if (hot_empty(r)) return NONE;
    }
  }
  return hot_resolve(tab, cap, key, s, r, with_end, flat, rh);
}

// A compact staging list entry (IX_STAGE_SC1, A/B knob GM_STAGE_SC1: an sc1
// store, which leaves the line out of the XCD's L2 instead of keeping it there
// until eviction; the list is read by the next kernel anyway)
template <bool NT>
__device__ __forceinline__ void stage_st(uint32_t* base, uint32_t k, uint32_t v, bool sc1) {
  if (sc1) {
    __builtin_amdgcn_raw_buffer_store_b32(v, __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7FFFFFFF, 0x00020000),
                                          int(k * 4u), 0, 16);
  } else {
    st_s<NT>(base + k, v);
  }
}

// Per-lane match staging: emit one filter id into the topic's row (slot m_n
// of the topic's lane column in its tile; srow = &stage[stage_index(tile, 0,
// lane)]).
#define GM_EMIT(f)                                \
  do {                                            \
    if (m_n < MC) srow[m_n * sstr] = (f);         \
    ++m_n;                                        \
  } while (0)

// Visit a node reached at this level (its record r, hot id hs): emit
// 'match_#' for it; on the topic's last word also its own filter
// (lookup_topic/3: only wildcard filters in trie mode; the '$X' quirk of
// emqx_trie.erl:275-276 for single-word '$' topics); otherwise push it onto
// the next frontier (GM_PUSH is defined per kernel).
#define GM_VISIT(hs, r)                                                                 \
  do {                                                                                  \
    if (((r).a.w & HF_MASK) != HF_NONE) GM_EMIT((r).a.w & HF_MASK);                     \
    if (last) {                                                                         \
      if ((r).ef != NONE && (EXACT || ((r).ef & END_WILD) || (dollar && level == 0)))   \
        GM_EMIT((r).ef & ID_MASK);                                                      \
      ++nfinal;                                                                         \
    } else {                                                                            \
      GM_PUSH((hs) | ((r).a.w & FR_PLUS), hot_sig((r).a.w, (r).a.z));                   \
    }                                                                                   \
  } while (0)

// A wildcard publish topic: [] from the trie (emqx_trie.erl:149-158); with
// match_routes semantics the literal route lookup_routes(Topic)
// (emqx_router.erl:128-134).
#define GM_WILD_ROW()                                        \
  do {                                                       \
    m_n = 0;                                                 \
    ovf = false;                                             \
    if (EXACT) {                                             \
      const uint32_t f = literal_lookup(ix, tb, start, end); \
      if (f != NONE) {                                       \
        srow[0] = f;                                         \
        m_n = 1;                                             \
      }                                                      \
    }                                                        \
  } while (0)

// ---- probes shared by the walk kernels -------------------------------------
// Frontier (k_walk): at most RFC entries {hot id | FR_PLUS, exact-child
// signature} in registers (pushes are select chains over static indices, so
// nothing spills to scratch).  A lane whose frontier outgrows RFC, or whose row
// outgrows FAST_MC, is queued for the listed LDS pass and contributes nothing
// in the main pass.
constexpr int RFC = 4;

// The record of the '+' child held inline by slot `id` of its parent's table
// (gm_common.h): the slot's second 16 bytes, a line this walk read one level
// earlier when it visited the parent.
__device__ __forceinline__ HotRec plus_inline_load(const HotSlot* ptab, uint32_t id, bool flat) {
  uint4 q;
  if (!flat) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(hot_rsrc(ptab), (id & SLOT_MASK) * 32u + 16u, 0, 0);
    q = make_uint4(v[0], v[1], v[2], v[3]);
  } else {
    q = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint32_t*>(ptab + (id & SLOT_MASK)) + 4);
  }
  HotRec r;
  r.a = make_uint4(0u, 0u, q.y, q.z);
  r.ef = q.w;
  return r;
}
// The second 16 bytes of slot s: {end_filter, p_sig, p_hf, p_end} (a chain
// node's tail: {end_filter, s2, HF_NONE, F}).
__device__ __forceinline__ uint4 hot_tail_load(const HotSlot* tab, uint32_t s, bool flat) {
  if (!flat) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(hot_rsrc(tab), s * 32u + 16u, 0, 0);
    return make_uint4(v[0], v[1], v[2], v[3]);
  }
  return *reinterpret_cast<const uint4*>(reinterpret_cast<const uint32_t*>(tab + s) + 4);
}
// Whether the '+' child of frontier entry `id` (a node at depth lvl) is inline.
__device__ __forceinline__ bool plus_is_inline(uint32_t lvl, uint32_t id) { return plus_inline(lvl, !(id & HOT_INLINE)); }

// Issue (load the home slot of) / take (resolve and visit) one probe of a
// frontier entry: the exact edge (word wid) or the '+' edge.  An inline '+'
// child is "issued" as the re-read of its parent's slot (sx = NONE).
#define GM_PROBE_ISSUE(c, e_id, plus, sx, rx)                                           \
  do {                                                                                  \
    if (c) {                                                                            \
      if ((plus) && plus_is_inline(lvl, (e_id))) {                                      \
        sx = NONE;                                                                      \
        rx = plus_inline_load(ptab, (e_id), hflat);                                        \
      } else {                                                                          \
        sx = hot_home(ix, ht, hot_key((e_id), (plus) ? ix.plus_word : wid, lvl), cap);    \
        rx = hot_load(tab, sx, last, hflat);                                            \
      }                                                                                 \
    }                                                                                   \
  } while (0)

#define GM_PROBE_TAKE(c, e_id, plus, sx, rx)                                                              \
  do {                                                                                                    \
    if (c) {                                                                                              \
      if ((plus) && sx == NONE) {                                                                         \
        GM_VISIT((e_id) | HOT_INLINE, rx);                                                                \
      } else {                                                                                            \
        const uint32_t hs_ = hot_resolve_x(ix, ht, tab, capu, hot_key((e_id), (plus) ? ix.plus_word : wid, lvl), sx, rx, last, hflat, hrh); \
        if (hs_ != NONE) GM_VISIT(hs_, rx);                                                               \
      }                                                                                                   \
    }                                                                                                     \
  } while (0)

// ---- k_match_lds ----------------------------------------------------------
// Frontier entries double buffered in LDS, FC per lane.  LISTED: grid-stride
// over the topics list_in[0 .. *list_n) (the main pass's overflow queue; the
// count is read on the device); otherwise one topic per thread.  Overflow
// here (frontier > FC or row > FAST_MC) is queued for k_slow_walk.
#define GM_PUSH(idv, sigv)                                                 \
  do {                                                                     \
    if (nn < FC) s_fr[nb][nn][threadIdx.x] = make_uint2((idv), (sigv));    \
    ++nn;                                                                  \
  } while (0)

// CMP (the main pass staged compactly): the listed rows go to their own
// buffer, row `item` of lstage (FAST_MC ids, stride 1), their length to
// lcnt[item] and cnt[t] = LIST_BIT | item; items past lcap go to the slow path.
template <bool EXACT, int FC, bool LISTED, bool CMP = false>
__global__ __launch_bounds__(256) void k_match_lds(const uint8_t* __restrict__ tb,
                                                   const uint64_t* __restrict__ toff, uint64_t n, IndexView ix,
                                                   uint32_t* __restrict__ cnt, uint32_t* __restrict__ stage,
                                                   const uint32_t* __restrict__ list_in,
                                                   const uint32_t* __restrict__ list_n,
                                                   uint32_t* __restrict__ ovf_list, uint32_t* __restrict__ ovf_n,
                                                   unsigned long long* __restrict__ probe_ctr,
                                                   unsigned long long* __restrict__ wild_ctr,
                                                   uint64_t* __restrict__ tsum, uint32_t* __restrict__ lstage = nullptr,
                                                   uint32_t* __restrict__ lcnt = nullptr, uint64_t lcap = 0) {
  constexpr int MC = FAST_MC;
  constexpr uint32_t sstr = CMP ? 1u : 64u;
  // frontier entry: {hot id | FR_PLUS, exact-child signature}, double buffered
  __shared__ uint2 s_fr[2][FC][256];
  const int tid = threadIdx.x, lane = tid & 63;
  const uint64_t n_items = LISTED ? uint64_t(*list_n) : n;
  uint32_t probes = 0, wilds = 0;

  for (uint64_t item = uint64_t(blockIdx.x) * 256u + tid; item < n_items;
       item += uint64_t(gridDim.x) * 256u) {
    const uint64_t t = LISTED ? uint64_t(list_in[item]) : item;
    const uint64_t tile = t >> 6;
    if (CMP && item >= lcap) {  // no listed row left: the slow path
      cnt[t] = OVF_BIT;
      ovf_list[atomicAdd(ovf_n, 1u)] = uint32_t(t);
      continue;
    }
    uint32_t* const srow = CMP ? lstage + item * uint64_t(MC) : stage + stage_index(tile, 0, int(t & 63));
    uint32_t m_n = 0, tprobes = 0;
    bool ovf = false, wild = false;
    uint64_t pos = toff[t];
    const uint64_t end = toff[t + 1];
    const uint64_t start = pos;
    ByteReader rd{tb, ~0ull, 0};
    WordTok w = next_word(rd, pos, end);
    DictSlot d0 = dict_first(ix, w);
    const bool dollar = w.len > 0 && w.b0 == '$';  // emqx_trie.erl:271-278
    if (!dollar && ix.root_hash != NONE) GM_EMIT(ix.root_hash);
    int cur = 0;
    uint32_t cur_n = 1, nfinal = 0;
    s_fr[0][0][tid] = make_uint2((!dollar && (ix.root_flags & HOT_PLUS)) ? FR_PLUS : 0u, ix.root_sig);
    uint32_t level = 0;
    for (;;) {
      const bool last = pos >= end;
      if (w.len == 1 && (w.b0 == '+' || w.b0 == '#')) {
        wild = true;
        break;
      }
      const uint32_t wid = cur_n ? dict_resolve(ix, w, d0, tb) : NONE;
      const uint32_t wbit = sig_bit(wid);
      WordTok wn;
      DictSlot dn;
      if (!last) {
        ++pos;
        wn = next_word(rd, pos, end);
        dn = dict_first(ix, wn);
      }
      if (cur_n) {
        tprobes += 3 * cur_n;
        const int nb = cur ^ 1;
        uint32_t nn = 0;
        const uint32_t lvl = __builtin_amdgcn_readfirstlane(level);  // wave-uniform
        const int ht = hot_table(lvl + 1);
        const HotSlot* tab = ix.hot + ix.hot_off[ht];
        const HotSlot* ptab = ix.hot + ix.hot_off[hot_table(lvl)];  // the frontier nodes' own table
        const bool hflat = (ix.flags & IX_HOT_FLAT) != 0;
        const bool hrh = ((ix.rh_mask >> ht) & 1u) != 0;  // Robin Hood ordered table
        const uint64_t cap = ix.hot_cap[ht];
        const uint32_t capu = uint32_t(cap);
        for (uint32_t i = 0; i < cur_n; ++i) {
          const uint2 e = s_fr[cur][i][tid];
          const uint32_t id = e.x & ID_MASK;
          const bool dx = wid != NONE && (e.y & wbit);
          const bool dp = (e.x & FR_PLUS) != 0;
          uint32_t sx = 0, sp = 0;
          HotRec rx{}, rp{};
          GM_PROBE_ISSUE(dx, id, false, sx, rx);
          GM_PROBE_ISSUE(dp, id, true, sp, rp);
          GM_PROBE_TAKE(dx, id, false, sx, rx);
          GM_PROBE_TAKE(dp, id, true, sp, rp);
        }
        if (nn > FC) {
          ovf = true;
          break;
        }
        cur = nb;
        cur_n = nn;
      }
      if (last) break;
      w = wn;
      d0 = dn;
      ++level;
    }
    if (wild) {
      GM_WILD_ROW();
    } else if (!ovf) {
      tprobes += 2 * nfinal + 1;
      if (m_n > MC) ovf = true;
    }
    if (CMP) {
      cnt[t] = ovf ? OVF_BIT : (LIST_BIT | uint32_t(item));
      if (!ovf) lcnt[item] = m_n;
    } else {
      cnt[t] = ovf ? OVF_BIT : m_n;
    }
    if (ovf) ovf_list[atomicAdd(ovf_n, 1u)] = uint32_t(t);
    else if (LISTED) atomicAdd(reinterpret_cast<unsigned long long*>(tsum + tile), (unsigned long long)m_n);
    probes += tprobes;
    wilds += wild ? 1u : 0u;
    if (!LISTED) break;
  }
  // per-wave counters (one atomic per wave)
  uint32_t ptot, wtot;
  wave_excl_scan(probes, ptot);
  wave_excl_scan(wilds, wtot);
  if (lane == 0) {
    if (LISTED) {
      if (ptot) atomicAdd(probe_ctr, (unsigned long long)ptot);  // (an idle listed grid adds nothing: 2,048
    }                                                             //  same-address atomics cost ~20 us)
    else if (((uint64_t(blockIdx.x) * 256u + tid) >> 6) * 64 < n)
      probe_ctr[(uint64_t(blockIdx.x) * 256u + tid) >> 6] = ptot;  // per-tile slot, see k_match_reg
    if (wtot) atomicAdd(wild_ctr, (unsigned long long)wtot);
  }
}
#undef GM_PUSH

// ---- split form: k_tokenize + k_walk --------------------------------------
// The per-topic front end (byte scan, word hash, dictionary lookup) and the
// trie walk have different shapes: the first is streaming ALU work over the
// topic bytes, the second a chain of dependent gathers.  Split, each kernel
// keeps only its own state live, so the walk runs at full occupancy.
//
// k_tokenize writes, per topic, hdr = levels | TOK_DOLLAR | TOK_WILD | TOK_DEEP
// and the word id of each level (NONE for a word no filter uses) into
// wids[level][topic] (level < TOK_LMAX), a layout the walk reads coalesced.
constexpr int TOK_LMAX = 8;
constexpr uint32_t TOK_DOLLAR = 1u << 8, TOK_WILD = 1u << 9, TOK_DEEP = 1u << 10;

// Reader over topic text staged in LDS (8-byte words; `lo` = the absolute
// batch offset of lds[0]), with the same one-word cache as ByteReader.
struct LdsReader {
  const uint64_t* lds;
  uint64_t lo;
  uint64_t cached_addr;
  uint64_t cached;
  __device__ __forceinline__ uint32_t get(uint64_t p) {
    const uint64_t a = p & ~7ull;
    if (a != cached_addr) {
      cached_addr = a;
      cached = lds[(a - lo) >> 3];
    }
    return uint32_t(cached >> ((p & 7) * 8)) & 0xFFu;
  }
};

// Word scan over LDS-staged text, 8 bytes per step (SWAR): the next '/' is the
// lowest zero byte of (word ^ 0x2F..2F) at or after the start (an exact
// per-byte test: the usual (y - 0x01..) & ~y trick borrows across bytes and
// can flag a byte just above an earlier '/'); a word's 8-byte
// chunks (from its own first byte, the last one zero padded -- the same
// chunking as the byte reader, so the same hash) are funnel shifts of two
// aligned LDS words.  Needs one staged word of slack past the text.
__device__ __forceinline__ uint64_t funnel8(const uint64_t* lds, uint64_t wi, uint32_t sh) {
  const uint64_t a = lds[wi];
  return sh ? (a >> sh) | (lds[wi + 1] << (64 - sh)) : a;
}

__device__ __forceinline__ WordTok next_word(LdsReader& rd, uint64_t& pos, uint64_t end) {
  constexpr uint64_t SL = 0x2F2F2F2F2F2F2F2Full, M7 = 0x7F7F7F7F7F7F7F7Full;
  // exact per-byte zero test (no borrow between bytes): bit 7 of a byte of
  // zbytes(y) is set iff that byte of y is 0
  auto zbytes = [](uint64_t y) { return ~(((y & M7) + M7) | y | M7); };
  WordTok w;
  w.start = pos;
  const uint64_t rel = pos - rd.lo;
  const uint64_t w0 = rel >> 3;
  const uint32_t sh = uint32_t(rel & 7) * 8;
  // find the end of the word
  uint64_t wi = w0, e = end;
  uint64_t z = zbytes(rd.lds[wi] ^ SL) & (~0ull << sh);  // bytes before pos do not count
  for (;;) {
    if (z) {
      const uint64_t at = rd.lo + wi * 8 + (__builtin_ctzll(z) >> 3);
      e = at < end ? at : end;
      break;
    }
    if (rd.lo + (wi + 1) * 8 >= end) break;
    ++wi;
    z = zbytes(rd.lds[wi] ^ SL);
  }
  const uint32_t len = uint32_t(e - pos);
  uint32_t h = DICT_HASH_SEED;
  uint64_t head = 0;
  for (uint32_t k = 0; k < len; k += 8) {
    uint64_t c = funnel8(rd.lds, w0 + (k >> 3), sh);
    if (len - k < 8) c &= (1ull << ((len - k) * 8)) - 1;
    if (k == 0) head = c;
    h = dict_hash_step(h, c);
  }
  w.h = dict_hash_final(h, len);
  w.head = head;
  w.len = len;
  w.b0 = uint32_t(head & 0xFF);
  pos = e;
  return w;
}

// The same scan in 32-bit offsets relative to the block's staged text (at
// most TOK_STAGE bytes): no 64-bit position arithmetic in the byte scan.
// `w.start` is relative too, so the word's tail is read from `tb + lo`.
__device__ __forceinline__ WordTok next_word_s(const uint64_t* lds, uint32_t& pos, uint32_t end) {
  constexpr uint64_t SL = 0x2F2F2F2F2F2F2F2Full, M7 = 0x7F7F7F7F7F7F7F7Full;
  auto zbytes = [](uint64_t y) { return ~(((y & M7) + M7) | y | M7); };
  WordTok w;
  w.start = pos;
  const uint32_t w0 = pos >> 3;
  const uint32_t sh = (pos & 7u) * 8u;
  // The two staged words that hold any word of up to 8 bytes, loaded
  // unconditionally: the common word is cut and hashed with selects, no
  // divergent loop (the kernels were issue bound on the exec-mask SALU work
  // of those loops as much as on VALU).  Index w0 + 1 stays inside s_txt
  // (staged text <= TOK_STAGE - 8 bytes, one word of slack).
  const uint64_t a0 = lds[w0], a1 = lds[w0 + 1];
  const uint64_t z0 = zbytes(a0 ^ SL) & (~0ull << sh);  // bytes before pos do not count
  const uint64_t z1 = zbytes(a1 ^ SL);
  uint32_t at = z0 ? w0 * 8u + (uint32_t(__builtin_ctzll(z0)) >> 3)
                   : (z1 ? w0 * 8u + 8u + (uint32_t(__builtin_ctzll(z1)) >> 3) : w0 * 8u + 16u);
  if (!z0 && !z1 && (w0 + 2u) * 8u < end) {  // a word reaching past the second staged word
    uint32_t wi = w0 + 2u;
    at = end;
    for (;;) {
      const uint64_t z = zbytes(lds[wi] ^ SL);
      if (z) {
        at = wi * 8u + (uint32_t(__builtin_ctzll(z)) >> 3);
        break;
      }
      if ((wi + 1u) * 8u >= end) break;
      ++wi;
    }
  }
  const uint32_t e = at < end ? at : end;
  const uint32_t len = e - pos;
  uint64_t c = sh ? (a0 >> sh) | (a1 << (64 - sh)) : a0;
  c &= len >= 8 ? ~0ull : (1ull << ((len & 7u) * 8u)) - 1;
  uint32_t h = len ? dict_hash_step(DICT_HASH_SEED, c) : DICT_HASH_SEED;
  for (uint32_t k = 8; k < len; k += 8) {  // words longer than 8 bytes
    uint64_t ck = funnel8(lds, w0 + (k >> 3), sh);
    if (len - k < 8) ck &= (1ull << ((len - k) * 8)) - 1;
    h = dict_hash_step(h, ck);
  }
  w.h = dict_hash_final(h, len);
  w.head = c;
  w.len = len;
  w.b0 = uint32_t(c & 0xFF);
  pos = e;
  return w;
}

// Staged-text form of tokenize_topic: relative 32-bit positions, and the
// level's wids[] slot advanced by n (no lev * n product per level).
__device__ __forceinline__ uint32_t tokenize_staged(const uint64_t* lds, uint32_t pos, uint32_t end,
                                                    const IndexView& ix, const uint8_t* tb_lo, uint64_t n,
                                                    uint32_t* __restrict__ wp) {
  uint32_t lev = 0, fl = 0;
  WordTok w = next_word_s(lds, pos, end);
  DictSlot d = dict_first(ix, w);
  if (w.len > 0 && w.b0 == '$') fl |= TOK_DOLLAR;  // emqx_trie.erl:271-278
  for (;;) {
    if (w.len == 1 && (w.b0 == '+' || w.b0 == '#')) {  // emqx_topic:wildcard/1
      fl |= TOK_WILD;
      break;
    }
    const bool more = pos < end;
    WordTok wn;
    DictSlot dn;
    if (more) {
      ++pos;
      wn = next_word_s(lds, pos, end);
      dn = dict_first(ix, wn);
    }
    if (lev < TOK_LMAX) {
      *wp = dict_resolve(ix, w, d, tb_lo);
      wp += n;
    }
    ++lev;
    if (!more) break;
    w = wn;
    d = dn;
  }
  if (lev > TOK_LMAX) fl |= TOK_DEEP;
  return (lev < 255u ? lev : 255u) | fl;
}

// Grouped form: the words of G levels are scanned first and their first
// dictionary slots loaded together, then resolved -- G L2 round trips in
// flight per lane instead of the one-ahead prefetch above (the tokenizer
// waits on the dictionary most of its time).  A word is kept as 4 VGPRs
// (head, hash, start | len << 16; staged text is < 64 KiB) until it resolves.
// Same hdr/wids as tokenize_topic: levels past TOK_LMAX are only counted
// and checked for wildcards.
// Where the word ids of one topic go: level-major HBM for k_walk / k_walk_coop,
// registers for the fused kernel.  Called for levels 0, 1, 2, ... in order.
template <bool NT>
struct WidsToHbm {
  uint32_t* wp;  // wids + t
  uint64_t n;
  __device__ __forceinline__ void operator()(uint32_t, uint32_t v) {
    st_s<NT>(wp, v);
    wp += n;
  }
};
struct WidsToRegs {
  uint32_t (&w)[TOK_LMAX];
  __device__ __forceinline__ void operator()(uint32_t lev, uint32_t v) {
#pragma unroll
    for (int q = 0; q < TOK_LMAX; ++q)
      if (lev == uint32_t(q)) w[q] = v;
  }
};

template <int G, class SINK>
__device__ __forceinline__ uint32_t tokenize_grouped(const uint64_t* lds, uint32_t pos, uint32_t end,
                                                     const IndexView& ix, const uint8_t* tb_lo, SINK&& sink) {
  uint32_t lev = 0, fl = 0;
  bool more = true, wild = false;
  while (more && lev < uint32_t(TOK_LMAX)) {
    uint64_t hd[G];
    uint32_t hh[G], sl[G];
    DictSlot d[G];
    bool have[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      have[g] = more && lev + g < uint32_t(TOK_LMAX);
      if (have[g]) {
        const WordTok w = next_word_s(lds, pos, end);
        if (g == 0 && lev == 0 && w.len > 0 && w.b0 == '$') fl |= TOK_DOLLAR;  // emqx_trie.erl:271-278
        if (w.len == 1 && (w.b0 == '+' || w.b0 == '#')) {  // emqx_topic:wildcard/1
          wild = true;
          have[g] = more = false;
        } else {
          hd[g] = w.head;
          hh[g] = w.h;
          sl[g] = uint32_t(w.start) | (w.len << 16);
          d[g] = dict_first(ix, w);
          more = pos < end;
          pos += more ? 1u : 0u;
        }
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (have[g]) {
        WordTok w;
        w.h = hh[g];
        w.head = hd[g];
        w.start = sl[g] & 0xFFFFu;
        w.len = sl[g] >> 16;
        w.b0 = uint32_t(hd[g] & 0xFF);
        sink(lev, dict_resolve(ix, w, d[g], tb_lo));
        ++lev;
      }
    }
  }
  while (more) {  // deep topic: count the remaining levels
    const WordTok w = next_word_s(lds, pos, end);
    if (w.len == 1 && (w.b0 == '+' || w.b0 == '#')) {
      wild = true;
      break;
    }
    ++lev;
    more = pos < end;
    pos += more ? 1u : 0u;
  }
  if (wild) fl |= TOK_WILD;
  if (lev > uint32_t(TOK_LMAX)) fl |= TOK_DEEP;
  return (lev < 255u ? lev : 255u) | fl;
}

// One topic: words -> dictionary ids, the next word's first dictionary slot
// loaded while this word resolves.
template <class RD, class SINK>
__device__ __forceinline__ uint32_t tokenize_topic(RD& rd, uint64_t pos, uint64_t end, const IndexView& ix,
                                                   const uint8_t* tb, SINK&& sink) {
  uint32_t lev = 0, fl = 0;
  WordTok w = next_word(rd, pos, end);
  DictSlot d = dict_first(ix, w);
  if (w.len > 0 && w.b0 == '$') fl |= TOK_DOLLAR;  // emqx_trie.erl:271-278
  for (;;) {
    if (w.len == 1 && (w.b0 == '+' || w.b0 == '#')) {  // emqx_topic:wildcard/1
      fl |= TOK_WILD;
      break;
    }
    const bool more = pos < end;
    WordTok wn;
    DictSlot dn;
    if (more) {
      ++pos;
      wn = next_word(rd, pos, end);
      dn = dict_first(ix, wn);
    }
    if (lev < TOK_LMAX) sink(lev, dict_resolve(ix, w, d, tb));
    ++lev;
    if (!more) break;
    w = wn;
    d = dn;
  }
  if (lev > TOK_LMAX) fl |= TOK_DEEP;
  return (lev < 255u ? lev : 255u) | fl;
}

// The block's topic text [toff[t0], toff[t0+256]) is staged in LDS with
// coalesced 8-byte loads when it fits TOK_STAGE bytes (a wave's lanes then
// scan their own topics from LDS instead of issuing dependent global loads
// at every 8-byte boundary); a longer block reads global memory directly.
constexpr int TOK_STAGE = 16384;

template <int G, bool NT>
__global__ __launch_bounds__(256) void k_tokenize(const uint8_t* __restrict__ tb, const uint64_t* __restrict__ toff,
                                                  uint64_t n, IndexView ix, uint32_t* __restrict__ hdr,
                                                  uint32_t* __restrict__ wids, uint64_t t_base) {
  __shared__ uint64_t s_txt[TOK_STAGE / 8 + 1];  // + one word of slack for the funnel shifts
  const uint64_t t0 = t_base + uint64_t(blockIdx.x) * 256u;
  const uint64_t t = t0 + threadIdx.x;
  const uint64_t tl = t0 + 256 < n ? t0 + 256 : n;
  const uint64_t lo = toff[t0] & ~7ull, hi = toff[tl];
  const bool staged = hi - lo <= uint64_t(TOK_STAGE) - 8;  // block-uniform
  if (staged) {
    const uint64_t nw = ((hi - lo + 7) >> 3) + 1;  // topic buffers are padded by 64 bytes
    for (uint64_t i = threadIdx.x; i < nw; i += 256) s_txt[i] = ld_s<NT>(reinterpret_cast<const uint64_t*>(tb + lo + 8 * i));
  }
  __syncthreads();
  if (t >= n) return;
  const uint64_t pos = toff[t], end = toff[t + 1];
  uint32_t h;
  if (staged) {
    if constexpr (G == 1)
      h = tokenize_staged(s_txt, uint32_t(pos - lo), uint32_t(end - lo), ix, tb + lo, n, wids + t);
    else
      h = tokenize_grouped<G>(s_txt, uint32_t(pos - lo), uint32_t(end - lo), ix, tb + lo, WidsToHbm<NT>{wids + t, n});
  } else {
    ByteReader rd{tb, ~0ull, 0};
    h = tokenize_topic(rd, pos, end, ix, tb, WidsToHbm<NT>{wids + t, n});
  }
  st_s<NT>(hdr + t, h);
}

// k_walk: the NFA walk over pre-resolved word ids, frontier in registers as
// in k_match_reg.  Deep topics (more than TOK_LMAX levels) are queued for the
// listed pass, which tokenizes for itself.
#define GM_PUSH(idv, sigv)                                \
  do {                                                    \
    const uint32_t pid_ = (idv), psig_ = (sigv);          \
    _Pragma("unroll") for (int q_ = 0; q_ < RFC; ++q_) {  \
      if (nn == uint32_t(q_)) {                           \
        nid[q_] = pid_;                                   \
        nsig[q_] = psig_;                                 \
      }                                                   \
    }                                                     \
    ++nn;                                                 \
  } while (0)

template <bool EXACT, int MINW, bool PAIR>
__global__ __launch_bounds__(256, MINW) void k_walk(const uint8_t* __restrict__ tb, const uint64_t* __restrict__ toff,
                                                    uint64_t n, IndexView ix, const uint32_t* __restrict__ hdr,
                                                    const uint32_t* __restrict__ wids, uint32_t* __restrict__ cnt,
                                                    uint32_t* __restrict__ stage, uint32_t* __restrict__ ovf_list,
                                                    uint32_t* __restrict__ ovf_n,
                                                    unsigned long long* __restrict__ probe_tile,
                                                    unsigned long long* __restrict__ wild_ctr,
                                                    uint64_t* __restrict__ tsum, uint64_t t_base) {
  constexpr int MC = FAST_MC;
  const int lane = threadIdx.x & 63;
  const uint64_t t = t_base + uint64_t(blockIdx.x) * 256u + threadIdx.x;
  const uint64_t tile = t >> 6;
  const bool valid = t < n;
  uint32_t* const srow = stage + stage_index(tile, 0, lane);
  constexpr uint32_t sstr = 64u;
  uint32_t m_n = 0, probes = 0;
  bool ovf = false, wild = false;

  if (valid) {
    const uint32_t h = hdr[t];
    const uint32_t nlev = h & 0xFFu;
    const bool dollar = (h & TOK_DOLLAR) != 0;
    wild = (h & TOK_WILD) != 0;
    if (h & TOK_DEEP) {
      ovf = true;
    } else if (wild) {
      const uint64_t start = toff[t], end = toff[t + 1];
      GM_WILD_ROW();
    } else {
      if (!dollar && ix.root_hash != NONE) GM_EMIT(ix.root_hash);  // '#' at the virtual root
      uint32_t fid[RFC], fsig[RFC];
#pragma unroll
      for (int q = 0; q < RFC; ++q) fid[q] = fsig[q] = 0;
      fid[0] = (!dollar && (ix.root_flags & HOT_PLUS)) ? FR_PLUS : 0u;
      fsig[0] = ix.root_sig;
      uint32_t cur_n = 1, nfinal = 0;
      uint32_t wid_next = wids[t];
      for (uint32_t level = 0; level < nlev && cur_n; ++level) {
        const bool last = level + 1 == nlev;
        const uint32_t wid = wid_next;
        if (!last) wid_next = wids[uint64_t(level + 1) * n + t];  // prefetch
        const uint32_t wbit = sig_bit(wid);
        probes += 3 * cur_n;
        uint32_t nid[RFC], nsig[RFC], nn = 0;
#pragma unroll
        for (int q = 0; q < RFC; ++q) nid[q] = nsig[q] = 0;
        const uint32_t lvl = __builtin_amdgcn_readfirstlane(level);  // wave-uniform
        const int ht = hot_table(lvl + 1);
        const HotSlot* tab = ix.hot + ix.hot_off[ht];
        const HotSlot* ptab = ix.hot + ix.hot_off[hot_table(lvl)];  // the frontier nodes' own table
        const bool hflat = (ix.flags & IX_HOT_FLAT) != 0;
        const bool hrh = ((ix.rh_mask >> ht) & 1u) != 0;  // Robin Hood ordered table
        const uint64_t cap = ix.hot_cap[ht];
        const uint32_t capu = uint32_t(cap);
        const bool wok = wid != NONE;
        // bit q: the exact probe of entry q can hit (signature, then the
        // table's exact-edge filter when it has one: an L2 hit that saves a
        // random line for most of the probes the signature lets through)
        uint32_t xmask = 0;
#pragma unroll
        for (int q = 0; q < RFC; ++q)
          if (uint32_t(q) < cur_n && wok && (fsig[q] & wbit)) xmask |= 1u << q;
        const uint32_t fmask = ix.efilt_mask[ht];  // wave-uniform
        if (fmask && xmask) {
          const uint32_t* ft = ix.efilt + ix.efilt_off[ht];
          uint32_t fw[RFC], fb[RFC];
#pragma unroll
          for (int q = 0; q < RFC; ++q) {
            fw[q] = fb[q] = 0;
            if (xmask & (1u << q)) {
              const uint32_t fh = edge_filter_hash(hot_key(fid[q] & ID_MASK, wid, lvl));
              fb[q] = edge_filter_bits(fh);
              fw[q] = ft[edge_filter_word(fh, fmask)];
            }
          }
#pragma unroll
          for (int q = 0; q < RFC; ++q)
            if ((fw[q] & fb[q]) != fb[q]) xmask &= ~(1u << q);
        }
        if (PAIR) {
#pragma unroll
          for (int i = 0; i < RFC; i += 2) {
            if (uint32_t(i) < cur_n) {
              const bool hb = uint32_t(i + 1) < cur_n;
              const uint32_t ia = fid[i] & ID_MASK, ib = fid[i + 1] & ID_MASK;
              const bool ax = (xmask >> i) & 1u, ap = (fid[i] & FR_PLUS) != 0;
              const bool bx = (xmask >> (i + 1)) & 1u, bp = hb && (fid[i + 1] & FR_PLUS) != 0;
              uint32_t sax = 0, sap = 0, sbx = 0, sbp = 0;
              HotRec rax{}, rap{}, rbx{}, rbp{};
              GM_PROBE_ISSUE(ax, ia, false, sax, rax);
              GM_PROBE_ISSUE(ap, ia, true, sap, rap);
              GM_PROBE_ISSUE(bx, ib, false, sbx, rbx);
              GM_PROBE_ISSUE(bp, ib, true, sbp, rbp);
              GM_PROBE_TAKE(ax, ia, false, sax, rax);
              GM_PROBE_TAKE(ap, ia, true, sap, rap);
              GM_PROBE_TAKE(bx, ib, false, sbx, rbx);
              GM_PROBE_TAKE(bp, ib, true, sbp, rbp);
            }
          }
        } else {
#pragma unroll
          for (int i = 0; i < RFC; ++i) {
            if (uint32_t(i) < cur_n) {
              const uint32_t ia = fid[i] & ID_MASK;
              const bool ax = (xmask >> i) & 1u, ap = (fid[i] & FR_PLUS) != 0;
              uint32_t sax = 0, sap = 0;
              HotRec rax{}, rap{};
              GM_PROBE_ISSUE(ax, ia, false, sax, rax);
              GM_PROBE_ISSUE(ap, ia, true, sap, rap);
              GM_PROBE_TAKE(ax, ia, false, sax, rax);
              GM_PROBE_TAKE(ap, ia, true, sap, rap);
            }
          }
        }
        if (nn > RFC) {
          ovf = true;
          break;
        }
#pragma unroll
        for (int q = 0; q < RFC; ++q) {
          fid[q] = nid[q];
          fsig[q] = nsig[q];
        }
        cur_n = nn;
      }
      if (!ovf) {
        probes += 2 * nfinal + 1;
        if (m_n > MC) ovf = true;
      }
    }
    if (ovf) probes = 0;  // the listed pass walks this topic again and counts it
  }

  if (valid) {
    cnt[t] = ovf ? OVF_BIT : m_n;
    if (ovf) ovf_list[atomicAdd(ovf_n, 1u)] = uint32_t(t);
  }
  // per-tile probe count and match count (the CSR scan's input; rows the
  // listed / slow passes finish add theirs there): plain stores into the
  // tile's slots, not atomics on one address
  uint32_t ptot, mtot;
  wave_excl_scan(probes, ptot);
  wave_excl_scan(valid && !ovf ? m_n : 0u, mtot);
  const unsigned long long wb = __ballot(valid && wild);
  if (lane == 0) {
    if (tile * 64 < n) {  // waves wholly past n have no slot
      probe_tile[tile] = ptot;
      tsum[tile] = mtot;
    }
    if (wb) atomicAdd(wild_ctr, (unsigned long long)__popcll(wb));
  }
}
#undef GM_PUSH
#undef GM_PROBE_ISSUE
#undef GM_PROBE_TAKE
#undef GM_VISIT
#undef GM_WILD_ROW
#undef GM_EMIT

// ---- k_walk_coop: the wave's frontier as one compacted work list ---------
// k_walk gives every lane its own topic's frontier, so at each level a wave
// runs as many probe rounds as its LONGEST frontier (C2: ~1.6 entries per
// topic on average, but the longest of 64 lanes is 3-4) and pays the exec-mask
// bookkeeping of those divergent rounds.  Here the frontier entries of all 64
// topics of the tile form one list in LDS, {node | FR_PLUS, signature, topic
// lane}; every round each lane takes the next entry of the list, so a level
// costs ceil(entries / 64) rounds with every lane busy.  Children are
// appended to the next level's list with ballot + mbcnt compaction; matches go
// to the topic's staging column through an LDS counter per topic (one
// ds_add_rtn per match).  A topic whose entries do not fit the list, or whose
// row outgrows FAST_MC, is marked (CW_OVF) and queued for the listed pass
// like k_walk's overflow.  Same hdr / wids input, same stage / cnt / tile-sum
// output as k_walk, so the listed pass, the scan and k_assemble are shared.
// Frontier entries per wave and level: 9 B each, two lists, so a 4-wave
// block's LDS is 72 * CW_CAP + 3 KB; 236 keeps it under 20 KB, i.e. 8 blocks
// (32 waves) per CU in 160 KB.  (192 -> 236 cut C3's list overflow rows; the
// overflowed topics are re-walked by the listed pass.)
#ifndef GM_CW_CAP
#define GM_CW_CAP 236
#endif
constexpr int CW_CAP = GM_CW_CAP;
constexpr uint32_t CW_OVF = 0x40000000u;   // in a topic's LDS match counter: queued for the listed pass
// compact staging entry: filter id (< 2^22) | lane << 22 | the match's rank in its row << 28
constexpr uint32_t CMP_SHIFT = 22, CMP_RANK = 28;

#ifdef GM_PROBE_STATS
// Diagnostic build only (-DGM_PROBE_STATS): a census of the coop walk's
// probes per level [level][k]: 0 entries, 1 exact candidates (a word), 2 past
// the signature, 3 past the exact-edge filter (= exact probes issued), 4 exact
// children found, 5 '+' slot probes issued, 6 '+' children found (slot), 7
// '+' children taken inline.  Printed by run_match after each call.
__device__ unsigned long long g_pstats[8][8];
#endif
#ifdef GM_PHASE_STATS
// Diagnostic build only (-DGM_PHASE_STATS): per wave of k_match_fused, one
// record of 16 words in g_phase_rec[tile], accumulated in registers and
// written once at the wave's end (no atomics, no read-modify-write in the
// walk): [0] staging, [1] tokenizer, [2+l] walk level l (l < 8) in s_memtime
// ticks, [10] epilogue, [11] rounds of levels 0-3 (8 bits each), [12] rounds of
// levels 4-7, [13] rounds with a chain tail load, [14..15] the wave's start
// tick.  run_match reduces them after each call.
__device__ uint32_t* g_phase_rec;
struct PhaseRec {
  uint32_t v[32];  // [16 + l] ticks of level l's rounds up to the probes' data, [24 + l] the rest of them
};
#define GM_PHASE_ADD(k, x) (PH.v[k] += uint32_t(x))
// level-indexed adds with constant indices (a dynamic index would put the
// record in scratch memory)
__device__ __forceinline__ void phase_level(PhaseRec& PH, uint32_t level, uint32_t ticks, uint32_t rounds, uint32_t t_data,
                                            uint32_t t_rest) {
  switch (level) {
#define GM_PH_CASE(L)                                          \
  case L:                                                      \
    PH.v[2 + L] += ticks;                                      \
    PH.v[L < 4 ? 11 : 12] += rounds << (8 * (L & 3));          \
    PH.v[16 + L] += t_data;                                    \
    PH.v[24 + L] += t_rest;                                    \
    break;
    GM_PH_CASE(0) GM_PH_CASE(1) GM_PH_CASE(2) GM_PH_CASE(3) GM_PH_CASE(4) GM_PH_CASE(5) GM_PH_CASE(6)
    default:
      PH.v[9] += ticks;
      PH.v[12] += rounds << 24;
      PH.v[23] += t_data;
      PH.v[31] += t_rest;
      break;
#undef GM_PH_CASE
  }
}
#else
struct PhaseRec {};
#define GM_PHASE_ADD(k, x) \
  do {                     \
  } while (0)
#endif

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ uint32_t lane_prefix(unsigned long long mask) {
  return __builtin_amdgcn_mbcnt_hi(uint32_t(mask >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(mask), 0u));
}

// One wave's walk over its 64-topic tile (k_walk_coop and k_match_fused).
// h = the topic's tokenizer header; WORDS yields the topic's word id of
// level 0 (first()) and of the next level (next(level)); the LDS arrays are
// the wave's own.
struct CoopLds {
  uint2 e[2][CW_CAP];      // {hot id | FR_PLUS, exact-child signature}
  uint8_t ln[2][CW_CAP];   // the entry's topic (lane of the tile)
  uint2 lw[64];            // per topic: {this level's word id, levels | TOK_DOLLAR}
  uint32_t mc[64];         // per topic: matches emitted | CW_OVF
};

// CMP (compact staging, k_match_fused): the tile's matches go to ONE list in
// emission order, each entry (filter id | lane | rank in the row), written by
// ballot + mbcnt; tlen[tile] = the list's length.  k_assemble_c sorts them
// into rows.  A tile whose list would pass 64 x FAST_MC entries sends every
// topic to the listed pass.  Otherwise ([slot][lane]): one column per topic.
// IX_D0: a topic's level-0 exact probe, issued by k_match_fused right after
// its tokenizer (the home slot of (root, level-0 word) in the depth-1 table;
// s = NONE: no probe) and resolved in the walk's level-0 round.
struct D0Probe {
  uint4 a;     // the home slot's head {key lo, key hi, sig, hf}
  uint32_t s;  // its slot index, or NONE
};
__device__ __forceinline__ D0Probe d0_issue(const IndexView& ix, uint32_t w0, uint32_t h, bool valid) {
  D0Probe p{make_uint4(0u, 0u, 0u, 0u), NONE};
  const bool walk = valid && !(h & (TOK_WILD | TOK_DEEP));
  if (!walk || w0 == NONE || !(ix.root_sig & sig_bit(w0))) return p;
  const int ht = hot_table(1);
  const uint64_t key = hot_key(0u, w0, 0u);
  uint32_t s;
  if (const uint32_t mc = ix.mph_cap[ht]) {
    if (!mph_gate(ix, ht, key, mc, s)) return p;
  } else {
    s = uint32_t(hot_slot(key, ix.hot_cap[ht]));
  }
  p.a = hot_load(ix.hot + ix.hot_off[ht], s, false, (ix.flags & IX_HOT_FLAT) != 0).a;
  p.s = s;
  return p;
}

// D0 (k_match_fused with IX_D0): level 0 issues no probe of its own.  Each
// walking lane takes its own topic's root entry, resolves the exact probe its
// tokenizer issued (d1; parked in the level-0 list's LDS, which a level-0
// round from registers does not use) and takes the root's '+' child from
// ix.d0_root (one uniform load); the rest of the round -- visits, chains,
// pushes, probe counts -- is the general round's.
template <bool EXACT, bool NT, class WORDS, bool CMP = false, bool D0 = false>
__device__ __forceinline__ void coop_walk_tile(CoopLds& L, uint32_t h, WORDS& words, bool valid, uint64_t t,
                                               int lane, const uint8_t* __restrict__ tb,
                                               const uint64_t* __restrict__ toff, const IndexView& ix,
                                               uint32_t* __restrict__ cnt, uint32_t* __restrict__ stage,
                                               uint32_t* __restrict__ ovf_list, uint32_t* __restrict__ ovf_n,
                                               unsigned long long* __restrict__ probe_tile,
                                               unsigned long long* __restrict__ wild_ctr,
                                               uint64_t* __restrict__ tsum, uint32_t* __restrict__ tlen = nullptr,
                                               uint8_t* __restrict__ cnt8 = nullptr, PhaseRec* php = nullptr,
                                               D0Probe d1 = D0Probe{}) {
  PhaseRec ph_dummy{};
  PhaseRec& PH = php ? *php : ph_dummy;
  (void)PH;
  constexpr uint32_t MC = FAST_MC;
  constexpr uint32_t TCAP = 64u * FAST_MC;  // a tile's staging entries
  constexpr bool KC = WORDS::kChain;        // the topic's future words are in its lane's registers
  // d0: the lanes' issued level-0 probes wait in the level-0 list's LDS (a
  // level-0 round from registers reads no list), not in VGPRs: stored first
  // thing, before the wildcard topics' literal lookup needs its registers
  uint4* const D1L = reinterpret_cast<uint4*>(L.e[0]);
  uint32_t* const D1S = reinterpret_cast<uint32_t*>(D1L + 64);
  static_assert(sizeof(L.e[0]) >= 64 * (sizeof(uint4) + 4), "the level-0 list holds 64 probes");
  if (D0 && (ix.flags & IX_D0)) {
    D1L[lane] = d1.a;
    D1S[lane] = d1.s;
  }
  const uint64_t tile = t >> 6;
  uint32_t* const MCNT = L.mc;
  uint2* const LW = L.lw;
  uint32_t* const stile = stage + tile * (64ull * MC);
  const uint32_t nlev = h & 0xFFu;
  const bool dollar = (h & TOK_DOLLAR) != 0, wild = valid && (h & TOK_WILD), deep = valid && (h & TOK_DEEP);
  const bool walk = valid && !wild && !deep;
  uint32_t m0 = deep ? CW_OVF : 0u;  // deep topics: the listed pass tokenizes them itself
  uint32_t f0 = NONE;
  if (wild && EXACT) {  // a wildcard publish topic: the literal route only (emqx_router.erl:128-134)
    f0 = literal_lookup(ix, tb, toff[t], toff[t + 1]);
  }
  if (walk && !dollar && ix.root_hash != NONE) f0 = ix.root_hash;  // '#' at the virtual root ('$' rule: emqx_trie.erl:271-278)
  uint32_t wbase = 0;  // CMP: entries in the tile's list (wave-uniform)
  if (f0 != NONE) m0 = 1;
  if constexpr (CMP) {  // (rank 0 of the lane's row)
    const unsigned long long b0 = __ballot(f0 != NONE);
    if (f0 != NONE) stage_st<NT>(stile, lane_prefix(b0), f0 | (uint32_t(lane) << CMP_SHIFT), ix.flags & IX_STAGE_SC1);
    wbase = uint32_t(__popcll(b0));
  } else {
    if (f0 != NONE) stile[lane] = f0;
  }
  MCNT[lane] = m0;
  uint32_t probes = walk ? 1u : 0u;  // + the exact-route probe
  // level 0: one root entry per walking topic
  const unsigned long long bw = __ballot(walk);
  uint32_t wnext = walk ? words.first() : NONE;
  if (walk && !(D0 && (ix.flags & IX_D0))) {
    const uint32_t p = lane_prefix(bw);
    L.e[0][p] = make_uint2((!dollar && (ix.root_flags & HOT_PLUS)) ? FR_PLUS : 0u, ix.root_sig);
    L.ln[0][p] = uint8_t(lane);
  }
  uint32_t cur_total = uint32_t(__popcll(bw));
  const bool hflat = (ix.flags & IX_HOT_FLAT) != 0;
  const bool d0 = D0 && (ix.flags & IX_D0);  // (wave-uniform)
  uint4 rq = D1_NONE;                       // the root's '+' child {hot id, sig, hf, end}
  if (d0) rq = *reinterpret_cast<const uint4*>(ix.d0_root);
  int cur = 0;
#ifdef GM_PHASE_STATS
  uint64_t tph = __builtin_amdgcn_s_memtime();
#endif
  // One level of the walk (a lambda, so that level 0 under D0 -- the round
  // from registers -- is its own instance and its extra live values do not
  // raise the general loop's register pressure)
  auto walk_level = [&](uint32_t level, auto d0r_tag) {
    constexpr bool D0R = decltype(d0r_tag)::value;
#ifdef GM_PHASE_STATS
    const uint32_t ph_rounds = (cur_total + 63) / 64;
    uint32_t ph_data = 0, ph_rest = 0;
#endif
    LW[lane] = make_uint2(wnext, nlev | (dollar ? TOK_DOLLAR : 0u));
    if (walk && level + 1 < nlev) wnext = words.next(level);  // next level's word, in flight
    uint32_t wnext2 = NONE;  // KC: the word after it (chain nodes of two words)
    if constexpr (KC) wnext2 = words.peek1();
    wave_lds_sync();
    const uint32_t lvl = __builtin_amdgcn_readfirstlane(level);
    const int ht = hot_table(lvl + 1);
    const HotSlot* tab = ix.hot + ix.hot_off[ht];
    const HotSlot* ptab = ix.hot + ix.hot_off[hot_table(lvl)];  // the frontier nodes' own table
    const bool hrh = ((ix.rh_mask >> ht) & 1u) != 0;
    const uint64_t cap = ix.hot_cap[ht];
    const uint32_t capu = uint32_t(cap);
    const uint32_t fmask = ix.efilt_mask[ht];
    const uint32_t* ft = ix.efilt + ix.efilt_off[ht];
    const uint2* E = L.e[cur];
    const uint8_t* LNc = L.ln[cur];
    uint2* EN = L.e[cur ^ 1];
    uint8_t* LNn = L.ln[cur ^ 1];
    uint32_t nxt_total = 0;
    for (uint32_t base = 0; base < (D0R ? 1u : cur_total); base += 64) {
#ifdef GM_PHASE_STATS
      const uint64_t tr0 = __builtin_amdgcn_s_memtime();
#endif
      // (d0r: level 0 from registers; every walking lane takes its own root entry)
      constexpr bool d0r = D0R;
      const uint32_t e = base + uint32_t(lane);
      const bool act = d0r ? walk : e < cur_total;
      const uint2 en = d0r ? make_uint2((!dollar && (ix.root_flags & HOT_PLUS)) ? FR_PLUS : 0u, ix.root_sig)
                           : act ? E[e] : make_uint2(0u, 0u);
      const uint32_t tl = d0r ? uint32_t(lane) : act ? LNc[e] : 0u;
      const uint2 lw = LW[tl];
      const uint32_t wid = lw.x, id = en.x & ID_MASK;
      const bool last = act && level + 1 == (lw.y & 0xFFu);
      const bool ldollar = (lw.y & TOK_DOLLAR) != 0;
      bool dx = act && wid != NONE && (en.y & sig_bit(wid));
#ifdef GM_PROBE_STATS
      const bool st_cand = act && wid != NONE, st_sig = dx;
#endif
      bool dp = act && (en.x & FR_PLUS);
      probes += act ? 3u : 0u;
      const bool pin = dp && plus_is_inline(lvl, id);
      const uint64_t kx = hot_key(id, wid, lvl), kp = hot_key(id, ix.plus_word, lvl);
      uint32_t sx = 0, sp = 0;
      HotRec rx{}, rp{};
      uint32_t hx = NONE, hp = NONE;
      if (d0r) {
        const uint32_t s1 = D1S[lane];
        dx = dx && s1 != NONE;  // (NONE: the tokenizer's gates -- root sig, MPH Bloom bits -- ruled it out)
        if (dx) {  // resolve the issued probe; the end filter (a one-level topic) from the found slot
          rx.a = D1L[lane];
          rx.ef = NONE;
          hx = hot_resolve_x(ix, ht, tab, capu, kx, s1, rx, false, hflat, hrh);
          if (last && hx != NONE) rx.ef = hot_load(tab, hx, true, hflat).ef;
        }
        if (dp) {
          hp = rq.x;
          rp.a = make_uint4(0u, 0u, rq.y, rq.z);
          rp.ef = last ? rq.w : NONE;
        }
      } else {
      if (const uint32_t mc = ix.mph_cap[ht]) {
        // an MPH table (wave-uniform): one L2 read of the key's bucket word
        // filters the probe and gives its slot, in place of the exact-edge filter
        if (dx) dx = mph_gate(ix, ht, kx, mc, sx);
        if (dp && !pin) dp = mph_gate(ix, ht, kp, mc, sp);
      } else {
        if (fmask && dx) {  // the table's exact-edge filter (an L2 hit) before a random line
          const uint32_t fh = edge_filter_hash(kx);
          const uint32_t fb = edge_filter_bits(fh);
          dx = (ft[edge_filter_word(fh, fmask)] & fb) == fb;
        }
        if (dx) sx = uint32_t(hot_slot(kx, cap));
        if (dp && !pin) sp = uint32_t(hot_slot(kp, cap));
      }
      // issue both probes, then resolve
      const uint32_t nol1 = ((ix.l1_bypass >> ht) & 1u) ? ix.hot_policy : 0u;
      if (dx) rx = hot_load(tab, sx, last, hflat, nol1);
      if (pin) {
        rp = plus_inline_load(ptab, id, hflat);
      } else if (dp) {
        rp = hot_load(tab, sp, last, hflat, nol1);
      }
      hx = dx ? hot_resolve_x(ix, ht, tab, capu, kx, sx, rx, last, hflat, hrh) : NONE;
      hp = pin ? (id | HOT_INLINE) : dp ? hot_resolve_x(ix, ht, tab, capu, kp, sp, rp, last, hflat, hrh) : NONE;
      }
#ifdef GM_PHASE_STATS
      __builtin_amdgcn_s_waitcnt(0);  // (diagnostic build: the probes' data is in)
      const uint64_t tr1 = __builtin_amdgcn_s_memtime();
      ph_data += uint32_t(tr1 - tr0);
#endif
      // The topic's next word (its own lane holds it: wnext), for the push
      // filter and the chain nodes below; the kernel forms without future words
      // in registers (KC false) push every node with children.
      uint32_t w1 = NONE;
      if constexpr (KC) w1 = uint32_t(__builtin_amdgcn_ds_bpermute(int(tl) << 2, int(wnext)));
#ifdef GM_PROBE_STATS
      {
        const unsigned long long c[8] = {__ballot(act), __ballot(st_cand), __ballot(st_sig), __ballot(dx),
                                         __ballot(hx != NONE), __ballot(dp && !pin), __ballot(dp && !pin && hp != NONE),
                                         __ballot(pin)};
        if (lane == 0)
          for (int k = 0; k < 8; ++k)
            if (c[k]) atomicAdd(&g_pstats[lvl < 7 ? lvl : 7][k], (unsigned long long)__popcll(c[k]));
      }
#endif
      const bool ex = hx != NONE, ep = hp != NONE;
      // Chain nodes (gm_common.h): the topic must continue with s1 (the head's
      // sig field) and end after the chain's Lc words; the tail {end, s2, -, F}
      // is read (an L2 hit: the head's line was just fetched) only when s1 agrees.
      const bool chx = KC && ex && !last && (rx.a.w & HOT_CHAIN);
      const bool chp = KC && ep && !last && (rp.a.w & HOT_CHAIN);
      const bool tx = chx && w1 == rx.a.z, tp = chp && w1 == rp.a.z;
      const uint32_t rem = (lw.y & 0xFFu) - (level + 1);  // the topic's words after this level (>= 1 when !last)
      uint32_t fx = NONE, fp = NONE, vx = 0, vp = 0;  // the chain's filter on a match; virtual probes
      if constexpr (KC) {
        if (__ballot(tx || tp)) {
          GM_PHASE_ADD(13, 1);
          const uint32_t w2 = uint32_t(__builtin_amdgcn_ds_bpermute(int(tl) << 2, int(wnext2)));
          uint4 qx{}, qp{};
          if (tx) qx = hot_tail_load(tab, hx, hflat);
          if (tp) qp = hot_tail_load(tab, hp, hflat);
          // the probes the reference NFA makes along the chain (SURVEY §8d's P):
          // c1 found at level+1 (+2 there if it is the topic's last level,
          // else +3 for c1's own frontier entry), c2 found at level+2 alike
          auto chain = [&](const uint4& q, uint32_t& f, uint32_t& vpr) {
            const uint32_t lc = q.y == NONE ? 1u : 2u;
            const bool two = lc == 2u && w2 == q.y;
            if (rem == lc && (lc == 1u || two)) f = q.w;
            vpr = rem == 1u ? 2u : 3u + (two ? (rem == 2u ? 2u : 3u) : 0u);
          };
          if (tx) chain(qx, fx, vx);
          if (tp) chain(qp, fp, vp);
        }
      }
      const bool e5 = fx != NONE && (EXACT || (fx & END_WILD));
      const bool e6 = fp != NONE && (EXACT || (fp & END_WILD));
      // a node goes on to the next level only if one of its probes there can
      // find something: a '+' child, or an exact child the next word's
      // signature bit admits (KC; otherwise any exact child).  A node that
      // stays behind (and a chain node) is counted with the probes the
      // reference NFA would make for it there.
      const uint32_t b1 = KC ? (w1 != NONE ? sig_bit(w1) : 0u) : 0xFFFFFFFFu;
      const uint32_t yx = ex ? hot_sig(rx.a.w, rx.a.z) : 0u, yp = ep ? hot_sig(rp.a.w, rp.a.z) : 0u;
      const bool cx = ex && !last && !chx && ((rx.a.w & FR_PLUS) || (yx & b1));
      const bool cp = ep && !last && !chp && ((rp.a.w & FR_PLUS) || (yp & b1));
      probes += (ex && !last && !cx ? 3u + vx : 0u) + (ep && !last && !cp ? 3u + vp : 0u);
      // visits: 'match_#', the end filter on the last level, else the next frontier
      if constexpr (CMP) {
        const bool e1 = ex && (rx.a.w & HF_MASK) != HF_NONE;
        const bool e2 = ex && last && rx.ef != NONE && (EXACT || (rx.ef & END_WILD) || (ldollar && level == 0));
        const bool e3 = ep && (rp.a.w & HF_MASK) != HF_NONE;
        const bool e4 = ep && last && rp.ef != NONE && (EXACT || (rp.ef & END_WILD) || (ldollar && level == 0));
        probes += last ? 2u * (uint32_t(ex) + uint32_t(ep)) : 0u;
        // the row's counter hands this lane's matches their ranks in the row
        const uint32_t ne = uint32_t(e1) + uint32_t(e2) + uint32_t(e3) + uint32_t(e4) + uint32_t(e5) + uint32_t(e6);
        uint32_t rk = ne ? atomicAdd(&MCNT[tl], ne) : 0u;
        const uint32_t tag = uint32_t(tl) << CMP_SHIFT;
        const bool sc1st = (ix.flags & IX_STAGE_SC1) != 0;
#define GM_CW_PUT(c, f)                                                                         \
  do {                                                                                          \
    const unsigned long long b_ = __ballot(c);                                                  \
    if (c) {                                                                                    \
      const uint32_t k_ = wbase + lane_prefix(b_);                                              \
      if (k_ < TCAP) stage_st<NT>(stile, k_, (f) | tag | ((rk < MC ? rk : MC - 1) << CMP_RANK), sc1st); \
      ++rk;                                                                                     \
    }                                                                                           \
    wbase += uint32_t(__popcll(b_));                                                            \
  } while (0)
        GM_CW_PUT(e1, rx.a.w & HF_MASK);
        GM_CW_PUT(e2, rx.ef & ID_MASK);
        GM_CW_PUT(e3, rp.a.w & HF_MASK);
        GM_CW_PUT(e4, rp.ef & ID_MASK);
        if (__ballot(e5 || e6)) {
          GM_CW_PUT(e5, fx & ID_MASK);
          GM_CW_PUT(e6, fp & ID_MASK);
        }
#undef GM_CW_PUT
      } else {
#define GM_CW_EMIT(f)                                   \
  do {                                                  \
    const uint32_t k_ = atomicAdd(&MCNT[tl], 1u);       \
    if (k_ < MC) st_s<NT>(stile + k_ * 64u + tl, (f));  \
  } while (0)
#define GM_CW_VISIT(r)                                                                          \
  do {                                                                                          \
    if (((r).a.w & HF_MASK) != HF_NONE) GM_CW_EMIT((r).a.w & HF_MASK);                          \
    if (last) {                                                                                 \
      if ((r).ef != NONE && (EXACT || ((r).ef & END_WILD) || (ldollar && level == 0)))          \
        GM_CW_EMIT((r).ef & ID_MASK);                                                           \
      probes += 2u;                                                                             \
    }                                                                                           \
  } while (0)
        if (ex) GM_CW_VISIT(rx);
        if (ep) GM_CW_VISIT(rp);
        if (e5) GM_CW_EMIT(fx & ID_MASK);
        if (e6) GM_CW_EMIT(fp & ID_MASK);
#undef GM_CW_VISIT
#undef GM_CW_EMIT
      }
      const unsigned long long bx = __ballot(cx), bp = __ballot(cp);
      const uint32_t nx = uint32_t(__popcll(bx));
      if (cx) {
        const uint32_t q = nxt_total + lane_prefix(bx);
        if (q < uint32_t(CW_CAP)) {
          EN[q] = make_uint2(hx | (rx.a.w & FR_PLUS), yx);
          LNn[q] = uint8_t(tl);
        } else {
          atomicOr(&MCNT[tl], CW_OVF);
        }
      }
      if (cp) {
        const uint32_t q = nxt_total + nx + lane_prefix(bp);
        if (q < uint32_t(CW_CAP)) {
          EN[q] = make_uint2(hp | (rp.a.w & FR_PLUS), yp);
          LNn[q] = uint8_t(tl);
        } else {
          atomicOr(&MCNT[tl], CW_OVF);
        }
      }
      nxt_total += nx + uint32_t(__popcll(bp));
#ifdef GM_PHASE_STATS
      ph_rest += uint32_t(__builtin_amdgcn_s_memtime() - tr1);
#endif
    }
    cur ^= 1;
    cur_total = nxt_total < uint32_t(CW_CAP) ? nxt_total : uint32_t(CW_CAP);
    wave_lds_sync();
#ifdef GM_PHASE_STATS
    {
      const uint64_t tn = __builtin_amdgcn_s_memtime();
      phase_level(PH, level, uint32_t(tn - tph), ph_rounds, ph_data, ph_rest);
      tph = tn;
    }
#endif
  };
  uint32_t level0 = 0;
  if (d0 && cur_total) {
    walk_level(0u, std::true_type{});
    level0 = 1;
  }
  uint32_t level = level0;
  while (cur_total != 0) walk_level(level++, std::false_type{});  // (each level updates cur_total)
  wave_lds_sync();
  const uint32_t m_n = MCNT[lane];
  // CW_OVF or a row past the staging capacity; CMP: the tile's list past its capacity
  const bool ovf = valid && (m_n > MC || (CMP && wbase > TCAP));
  if (valid) {
    // CMP: one byte per row (0xFF: the listed and slow passes write the row's cnt word)
    if constexpr (CMP) {
      st_s<NT>(cnt8 + t, uint8_t(ovf ? 0xFFu : m_n));
      // (the listed pass writes its rows' cnt words; until it has run -- it is
      // deferred to the host's read-back, MatchCall::finish -- the row reads
      // as a slow row with no ids, so an assembly before it stays in bounds)
      if (ovf) cnt[t] = OVF_BIT;
    } else {
      st_s<NT>(cnt + t, ovf ? OVF_BIT : m_n);
    }
    if (ovf) ovf_list[atomicAdd(ovf_n, 1u)] = uint32_t(t);
  }
  if (CMP && lane == 0) st_s<NT>(tlen + tile, wbase < TCAP ? wbase : TCAP);
  uint32_t ptot, mtot;
  wave_excl_scan(probes, ptot);
  wave_excl_scan(valid && !ovf ? m_n : 0u, mtot);
  const unsigned long long wb = __ballot(wild);
  if (lane == 0) {
    probe_tile[tile] = ptot;
    tsum[tile] = mtot;
    if (wb) atomicAdd(wild_ctr, (unsigned long long)__popcll(wb));
  }
#ifdef GM_PHASE_STATS
  GM_PHASE_ADD(10, __builtin_amdgcn_s_memtime() - tph);
  if (lane == 0 && g_phase_rec)
    for (int k = 0; k < 32; ++k) g_phase_rec[tile * 32 + k] = PH.v[k];
#endif
}


struct WordsFromHbm {  // k_walk_coop: the tokenizer's level-major word ids
  static constexpr bool kChain = false;
  __device__ __forceinline__ uint32_t peek1() { return NONE; }
  const uint32_t* wp;  // wids + t
  uint64_t n;
  bool nt;
  __device__ __forceinline__ uint32_t first() { return nt ? __builtin_nontemporal_load(wp) : *wp; }
  __device__ __forceinline__ uint32_t next(uint32_t level) {
    const uint32_t* p = wp + uint64_t(level + 1) * n;
    return nt ? __builtin_nontemporal_load(p) : *p;
  }
};

template <bool EXACT, bool NT>
__global__ __launch_bounds__(256, 8) void k_walk_coop(const uint8_t* __restrict__ tb,
                                                      const uint64_t* __restrict__ toff, uint64_t n, IndexView ix,
                                                      const uint32_t* __restrict__ hdr,
                                                      const uint32_t* __restrict__ wids, uint32_t* __restrict__ cnt,
                                                      uint32_t* __restrict__ stage, uint32_t* __restrict__ ovf_list,
                                                      uint32_t* __restrict__ ovf_n,
                                                      unsigned long long* __restrict__ probe_tile,
                                                      unsigned long long* __restrict__ wild_ctr,
                                                      uint64_t* __restrict__ tsum, uint64_t t_base) {
  __shared__ CoopLds s_w[4];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t t = t_base + uint64_t(blockIdx.x) * 256u + threadIdx.x;
  if ((t >> 6) * 64 >= n) return;  // wave-uniform: no workgroup barrier below
  const bool valid = t < n;
  const uint32_t h = valid ? ld_s<NT>(hdr + t) : 0u;
  WordsFromHbm words{wids + (valid ? t : 0), n, NT};
  coop_walk_tile<EXACT, NT>(s_w[wv], h, words, valid, t, lane, tb, toff, ix, cnt, stage, ovf_list, ovf_n, probe_tile,
                            wild_ctr, tsum);
}

// ---- k_match_fused: tokenize + coop walk in one kernel --------------------
// The block stages its topics' text in LDS and each lane tokenizes its topic
// into REGISTERS (word ids of up to TOK_LMAX levels, the header); then each
// wave walks its tile as k_walk_coop does, in the same LDS.  The word ids
// and headers never go through HBM (k_tokenize + k_walk_coop write and read
// back ~48 B per C2 topic of them), and the tokenizer's ALU work of one wave
// overlaps the walk's gathers of the others.
struct WordsFromRegs {
  static constexpr bool kChain = true;
  uint32_t (&w)[TOK_LMAX];
  __device__ __forceinline__ uint32_t peek1() { return w[1]; }  // after next(level): the word of level + 2
  __device__ __forceinline__ uint32_t first() { return w[0]; }
  __device__ __forceinline__ uint32_t next(uint32_t) {  // shift the levels down: w[0] = the next level's word
#pragma unroll
    for (int q = 0; q + 1 < TOK_LMAX; ++q) w[q] = w[q + 1];
    return w[0];
  }
};

constexpr size_t FUSED_LDS = sizeof(CoopLds) * 4 > (TOK_STAGE + 8) ? sizeof(CoopLds) * 4 : (TOK_STAGE + 8);

template <int G, bool EXACT, bool NT, bool TOKPRIO, bool CMP, bool D0 = true>
__global__ __launch_bounds__(256, 8) void k_match_fused(const uint8_t* __restrict__ tb,
                                                        const uint64_t* __restrict__ toff, uint64_t n, IndexView ix,
                                                        uint32_t* __restrict__ cnt, uint32_t* __restrict__ stage,
                                                        uint32_t* __restrict__ ovf_list, uint32_t* __restrict__ ovf_n,
                                                        unsigned long long* __restrict__ probe_tile,
                                                        unsigned long long* __restrict__ wild_ctr,
                                                        uint64_t* __restrict__ tsum, uint32_t* __restrict__ tlen,
                                                        uint8_t* __restrict__ cnt8) {
  __shared__ __align__(16) uint8_t s_raw[FUSED_LDS];  // the staged text, then the walk's lists
  uint64_t* const s_txt = reinterpret_cast<uint64_t*>(s_raw);
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // TOKPRIO: staging and tokenizing at wave priority 1, the walk at 0.  A block
  // holds its 20 KB of LDS (one of the CU's 8 block slots) through both phases
  // but only the walk keeps lines in flight, so the SIMD's issue arbiter favours
  // the waves that are still getting their block to the walk (C2 9.20 -> 9.10
  // ms, C3 13.68 -> 13.54; raising late walk levels instead was slower:
  // profiles/r02_ab/prio*_c*.txt)
  if constexpr (TOKPRIO) __builtin_amdgcn_s_setprio(1);
#ifdef GM_PHASE_STATS
  const uint64_t tp0 = __builtin_amdgcn_s_memtime();
#endif
  const uint64_t t0 = uint64_t(blockIdx.x) * 256u;
  const uint64_t t = t0 + threadIdx.x;
  const uint64_t tl = t0 + 256 < n ? t0 + 256 : n;
  const uint64_t lo = toff[t0] & ~7ull, hi = toff[tl];
  const bool staged = hi - lo <= uint64_t(TOK_STAGE) - 8;  // block-uniform
  if (staged) {
    const uint64_t nw = ((hi - lo + 7) >> 3) + 1;  // topic buffers are padded by 64 bytes
    for (uint64_t i = threadIdx.x; i < nw; i += 256) s_txt[i] = ld_s<NT>(reinterpret_cast<const uint64_t*>(tb + lo + 8 * i));
  }
  __syncthreads();
  PhaseRec PH{};
#ifdef GM_PHASE_STATS
  const uint64_t tp1 = __builtin_amdgcn_s_memtime();
  PH.v[0] = uint32_t(tp1 - tp0);
#endif
  const bool valid = t < n;
  uint32_t w[TOK_LMAX];
#pragma unroll
  for (int q = 0; q < TOK_LMAX; ++q) w[q] = NONE;
  uint32_t h = 0;
  if (valid) {
    const uint64_t pos = toff[t], end = toff[t + 1];
    if (staged) {
      h = tokenize_grouped<G>(s_txt, uint32_t(pos - lo), uint32_t(end - lo), ix, tb + lo, WidsToRegs{w});
    } else {
      ByteReader rd{tb, ~0ull, 0};
      h = tokenize_topic(rd, pos, end, ix, tb, WidsToRegs{w});
    }
  }
  __syncthreads();  // every lane is done with the staged text: the walk reuses the LDS
#ifdef GM_PHASE_STATS
  PH.v[1] = uint32_t(__builtin_amdgcn_s_memtime() - tp1);
#endif
  if constexpr (TOKPRIO) __builtin_amdgcn_s_setprio(0);
  if ((t >> 6) * 64 >= n) return;  // wave-uniform, after the last workgroup barrier
  // IX_D0: the level-0 exact probe -- the depth-1 node (root, level-0 word) --
  // issued before the walk's setup and resolved in its level-0 round (held
  // across the block barrier it spilled)
  D0Probe d1{make_uint4(0u, 0u, 0u, 0u), NONE};
  if (D0 && (ix.flags & IX_D0)) d1 = d0_issue(ix, w[0], h, valid);
  WordsFromRegs words{w};
  coop_walk_tile<EXACT, NT, WordsFromRegs, CMP, D0>(reinterpret_cast<CoopLds*>(s_raw)[wv], h, words, valid, t, lane,
                                                    tb, toff, ix, cnt, stage, ovf_list, ovf_n, probe_tile, wild_ctr,
                                                    tsum, tlen, cnt8, &PH, d1);
}

// ---------------------------------------------------------------------------
// scan (u64, exclusive, n+1 outputs: out[n] = total)
// ---------------------------------------------------------------------------
constexpr int SCAN_T = 256, SCAN_V = 4, SCAN_B = SCAN_T * SCAN_V;
// one-launch form for short inputs (up to 4,096 values: a match call of up to
// 262,144 topics): one workgroup of SCAN1_T threads, SCAN1_V per thread.  (16
// per thread, 16,384 values, took 25.6 us against 14 us for the three-launch
// form at C1's 15,625 tiles: one CU's address unit serializes the lanes'
// separate lines.)
constexpr int SCAN1_T = 1024, SCAN1_V = 4, SCAN1_B = SCAN1_T * SCAN1_V;

// A second array summed alongside the scan (the main pass's per-tile probe
// counts -> the probe counter), one atomic add per workgroup: saves the
// separate reduction launch of a match call.
struct SideSum {
  const unsigned long long* a = nullptr;
  uint64_t n = 0;
  unsigned long long* acc = nullptr;
};

// Scan of one workgroup's T*V inputs (exclusive, from `pre`); returns the
// workgroup's total to every thread.  s_w: T/64 + 1 words of LDS.
template <int T, int V, class LOAD>
__device__ __forceinline__ uint64_t block_scan(LOAD load, uint64_t base, uint64_t n_in, uint64_t n_out, uint64_t pre,
                                               uint64_t* __restrict__ out, uint64_t* s_w, const SideSum& side) {
  uint64_t v[V];
  uint64_t run = 0, ssum = 0;
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const uint64_t i = base + k;
    const uint64_t x = i < n_in ? load(i) : 0;
    v[k] = run;
    run += x;
    if (side.a && i < side.n) ssum += side.a[i];
  }
  // wave inclusive scan of per-thread totals
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint64_t x = run;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (side.a) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) ssum += __shfl_down(ssum, d, 64);
  }
  if (lane == 63) s_w[wv] = x;
  if (side.a && lane == 0) s_w[T / 64 + wv] = ssum;
  __syncthreads();
  uint64_t wpre = 0, tot = 0;
  for (int k = 0; k < T / 64; ++k) {
    wpre += k < wv ? s_w[k] : 0;
    tot += s_w[k];
  }
  const uint64_t tpre = pre + wpre + x - run;
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const uint64_t i = base + k;
    if (i < n_out) out[i] = tpre + v[k];
  }
  if (side.a && threadIdx.x == 0) {
    uint64_t st = 0;
    for (int k = 0; k < T / 64; ++k) st += s_w[T / 64 + k];
    if (st) atomicAdd(side.acc, (unsigned long long)st);
  }
  return tot;
}

__global__ void k_zero16(uint32_t* __restrict__ p) {  // 16 words (64 B)
  if (threadIdx.x < 16) p[threadIdx.x] = 0u;
}

template <class LOAD>
__global__ __launch_bounds__(SCAN_T) void k_scan_local(LOAD load, uint64_t n_in, uint64_t n_out,
                                                        uint64_t* __restrict__ out,
                                                        uint64_t* __restrict__ block_sums, SideSum side) {
  __shared__ uint64_t s_w[2 * (SCAN_T / 64)];
  const uint64_t base = uint64_t(blockIdx.x) * SCAN_B + threadIdx.x * SCAN_V;
  const uint64_t tot = block_scan<SCAN_T, SCAN_V>(load, base, n_in, n_out, 0, out, s_w, side);
  if (threadIdx.x == 0) block_sums[blockIdx.x] = tot;
}

template <class LOAD>
__global__ __launch_bounds__(SCAN1_T) void k_scan_one(LOAD load, uint64_t n_in, uint64_t n_out,
                                                       uint64_t* __restrict__ out, SideSum side,
                                                       uint64_t* __restrict__ mirror) {
  __shared__ uint64_t s_w[2 * (SCAN1_T / 64)];
  const uint64_t tot = block_scan<SCAN1_T, SCAN1_V>(load, uint64_t(threadIdx.x) * SCAN1_V, n_in, n_out, 0, out, s_w,
                                                    side);
  if (mirror && threadIdx.x == 0) *mirror = tot;  // the grand total, also at the caller's out[n]
}

// A small call's scan of up to 8 x SCAN1_B values in ONE launch: the workgroup
// walks the chunks with a running carry (a publish window's fan-out: ~5-15k
// matches, where the three-launch form idled the queue ~20 us between launches)
template <class LOAD>
__global__ __launch_bounds__(SCAN1_T) void k_scan_loop(LOAD load, uint64_t n_in, uint64_t n_out,
                                                        uint64_t* __restrict__ out) {
  __shared__ uint64_t s_w[2 * (SCAN1_T / 64)];
  uint64_t pre = 0;
  for (uint64_t b0 = 0; b0 < n_out; b0 += SCAN1_B) {
    pre += block_scan<SCAN1_T, SCAN1_V>(load, b0 + uint64_t(threadIdx.x) * SCAN1_V, n_in, n_out, pre, out, s_w,
                                        SideSum{});
    __syncthreads();  // (s_w is rewritten by the next chunk)
  }
}
constexpr uint64_t SCAN_LOOP_MAX = 8ull * SCAN1_B;

__global__ __launch_bounds__(SCAN_T) void k_scan_add(uint64_t* __restrict__ out, uint64_t n_out,
                                                      const uint64_t* __restrict__ block_off) {
  const uint64_t base = uint64_t(blockIdx.x) * SCAN_B;
  const uint64_t add = block_off[blockIdx.x];
  for (int k = threadIdx.x; k < SCAN_B; k += SCAN_T) {
    const uint64_t i = base + k;
    if (i < n_out) out[i] += add;
  }
}

struct LoadU64 {
  const uint64_t* p;
  __device__ uint64_t operator()(uint64_t i) const { return p[i]; }
};
struct LoadCnt {  // masked match counts
  const uint32_t* p;
  __device__ uint64_t operator()(uint64_t i) const { return p[i] & CNT_MASK; }
};
struct LoadSegLen {  // subscriber count of the filter of match entry i
  const uint32_t* ids;
  const uint64_t* sub_off;
  __device__ uint64_t operator()(uint64_t i) const {
    const uint32_t f = ids[i];
    return sub_off[f + 1] - sub_off[f];
  }
};

// LoadSegLen over a small call's SPECULATIVE rows (emqx_gm_match_fanout): the
// fan-out is queued before the host knows the match count, so entries past the
// device's own count (*nnz, the rows' row_off[n]) and ids out of range (an
// overflowed speculative buffer holds stale words) count 0 -- such a fan-out
// is discarded, but it reads nothing out of bounds
struct LoadSegLenSpec {
  const uint32_t* ids;
  const uint64_t* sub_off;
  const uint64_t* nnz;
  uint32_t nf;
  __device__ uint64_t operator()(uint64_t i) const {
    if (i >= *nnz) return 0;
    const uint32_t f = ids[i];
    return f < nf ? sub_off[f + 1] - sub_off[f] : 0;
  }
};

// Exclusive scan of n_in loaded values into out[0..n_in] (out[n_in] = total).
// split (optional): for a two-level scan, leave out[0..n_in) block-local and
// hand back the blocks' offsets in *split (out[i] + (*split)[i / SCAN_B] is the
// scan; out[n_in] is the grand total) -- the consumer adds them, one launch
// (k_scan_add) fewer.  split->p stays null when the scan was not split.
// st: the stream (default: the context's).  On another stream the scan's
// workspace goes back to the pool behind an event on that stream (the pool's
// immediate reuse assumes the context stream's order).
// split_sums (optional, with split): a scan of at most 64 blocks may hand
// back the blocks' SUMS instead (*split_sums = their count): no second launch;
// the consumer (k_assemble_c) sums the prefixes and writes out[n_in] itself.
template <class LOAD>
int scan_excl(emqx_gm_ctx* ctx, LOAD load, uint64_t n_in, uint64_t* out, SideSum side = SideSum{},
              PoolBuf* split = nullptr, hipStream_t st = nullptr, uint32_t* split_sums = nullptr) {
  if (split_sums) *split_sums = 0;
  if (!st) st = ctx->stream;
  const uint64_t n_out = n_in + 1;
  if (n_out <= uint64_t(SCAN1_B)) {  // one launch
    hipLaunchKernelGGL(k_scan_one<LOAD>, dim3(1), dim3(SCAN1_T), 0, st, load, n_in, n_out, out, side,
                       static_cast<uint64_t*>(nullptr));
    GM_HIP(ctx, hipGetLastError());
    return 0;
  }
  const uint64_t nb = (n_out + SCAN_B - 1) / SCAN_B;
  PoolBuf sums(ctx->pool, nb * 8 + 8), offs(ctx->pool, (nb + 1) * 8 + 8);
  if (!sums.p || !offs.p) return set_err(ctx, EMQX_GM_ENOMEM, "scan: workspace");
  struct Later {  // (another stream: release the workspace behind that stream's work)
    emqx_gm_ctx* c;
    hipStream_t s;
    PoolBuf* b[2];
    ~Later() {
      if (s == c->stream) return;
      for (PoolBuf* x : b)
        if (x->p) c->pool->release_after(x->release_ownership(), s);
    }
  } later{ctx, st, {&sums, &offs}};
  hipLaunchKernelGGL(k_scan_local<LOAD>, dim3(nb), dim3(SCAN_T), 0, st, load, n_in, n_out, out,
                     sums.as<uint64_t>(), side);
  if (split && split_sums && nb <= 64) {
    GM_HIP(ctx, hipGetLastError());
    *split = std::move(sums);
    *split_sums = uint32_t(nb);
    return 0;
  }
  if (split && nb + 1 <= uint64_t(SCAN1_B)) {  // the blocks' offsets, and the total into out[n_in]
    hipLaunchKernelGGL(k_scan_one<LoadU64>, dim3(1), dim3(SCAN1_T), 0, st, LoadU64{sums.as<uint64_t>()}, nb,
                       nb + 1, offs.as<uint64_t>(), SideSum{}, out + n_in);
    GM_HIP(ctx, hipGetLastError());
    *split = std::move(offs);
    return 0;
  }
  if (nb > 1) {
    int rc = scan_excl(ctx, LoadU64{sums.as<uint64_t>()}, nb, offs.as<uint64_t>(), SideSum{}, nullptr, st);
    if (rc) return rc;
    hipLaunchKernelGGL(k_scan_add, dim3(nb), dim3(SCAN_T), 0, st, out, n_out, offs.as<uint64_t>());
  }
  GM_HIP(ctx, hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------------------
// assembly
// ---------------------------------------------------------------------------
// Sort a row held in FAST_MC registers (unused slots = 0xFFFFFFFF) with a
// bitonic network over its first N slots; every index is static after
// unrolling.  Valid when every slot at or past N holds the sentinel.
template <int N>
__device__ __forceinline__ void sort_row(uint32_t (&m)[FAST_MC]) {
  static_assert(N <= FAST_MC && (N & (N - 1)) == 0, "bitonic width");
#pragma unroll
  for (int k = 2; k <= N; k <<= 1)
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1)
#pragma unroll
      for (int i = 0; i < N; ++i) {
        const int l = i ^ j;
        if (l > i) {
          const uint32_t a = m[i], b = m[l];
          const bool up = (i & k) == 0;
          const uint32_t lo = a < b ? a : b, hi = a < b ? b : a;
          m[i] = up ? lo : hi;
          m[l] = up ? hi : lo;
        }
      }
}

// One tile's rows once the wave's longest row is known to fit W slots (W is
// wave-uniform): W stage loads, the W-wide bitonic network and W stores per
// lane instead of FAST_MC.  At C2 (2.9 matches per topic) most waves take
// W = 8 (24 compare-exchanges instead of 80); k_assemble was bound by that
// VALU work (C2: 1.07 ms -> 0.91 ms with the network sized alone, 0.80 ms
// with loads and stores sized too).
template <int W>
__device__ __forceinline__ void assemble_tile(const uint32_t* __restrict__ stage, uint64_t tile, int lane,
                                              uint32_t cf, bool any_slow, uint64_t base, uint32_t pa,
                                              uint32_t tall, uint32_t* out, uint32_t* __restrict__ ids,
                                              uint64_t tile_base, const uint32_t* __restrict__ gmap) {
  uint32_t m[FAST_MC];
#pragma unroll
  for (int k = 0; k < FAST_MC; ++k)
    m[k] = (k < W && uint32_t(k) < cf) ? stage[stage_index(tile, k, lane)] : 0xFFFFFFFFu;
  if (W > 1) sort_row<W>(m);
  if (any_slow) {
#pragma unroll
    for (int k = 0; k < W; ++k)
      if (uint32_t(k) < cf) ids[base + k] = gmap ? gmap[m[k]] : m[k];  // shard index: global ids (ascending)
    return;
  }
#pragma unroll
  for (int k = 0; k < W; ++k)
    if (uint32_t(k) < cf) out[pa + k] = gmap ? gmap[m[k]] : m[k];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  uint32_t* const dst = ids + tile_base;
  for (uint32_t i = lane; i < tall; i += 64) dst[i] = out[i];
}

// One wave per 64-topic tile: row offsets from the wave's scan, each lane's
// row sorted in registers, then the tile's ids (one contiguous range of the
// output) written through LDS as coalesced 256-B rows.  A tile holding a
// slow-path row (its ids land later, k_copy_slow) stores lane by lane so
// that row's range is left alone.
// cap: the ids buffer's capacity; a tile whose rows would pass it writes no
// ids (the host, seeing a total past cap, assembles again into a larger buffer).
__global__ __launch_bounds__(256) void k_assemble(const uint32_t* __restrict__ cnt, uint64_t n,
                                                  const uint64_t* __restrict__ tile_off,
                                                  const uint32_t* __restrict__ stage,
                                                  uint64_t* __restrict__ row_off, uint32_t* __restrict__ ids,
                                                  const uint32_t* __restrict__ gmap, uint64_t cap) {
  __shared__ uint32_t s_out[4][64 * FAST_MC];
  const int lane = threadIdx.x & 63;
  uint32_t* const out = s_out[threadIdx.x >> 6];
  const uint64_t t = uint64_t(blockIdx.x) * 256u + threadIdx.x;
  const uint64_t tile = t >> 6;
  if (tile * 64 >= n) return;  // wave-uniform; no block barrier below
  const uint32_t c = t < n ? cnt[t] : 0;
  const bool slow = (c & OVF_BIT) != 0;
  const uint32_t call = c & CNT_MASK, cf = slow ? 0 : call;
  uint32_t tall;
  const uint32_t pa = wave_excl_scan(call, tall);
  const uint64_t base = tile_off[tile] + pa;
  if (t < n) row_off[t] = base;
  if (t == n - 1) row_off[n] = base + call;
  const bool any_slow = __ballot(slow) != 0;
  const uint64_t tb0 = tile_off[tile];
  if (tb0 + tall > cap) return;  // wave-uniform
#define GM_ASM(W) assemble_tile<W>(stage, tile, lane, cf, any_slow, base, pa, tall, out, ids, tb0, gmap)
  if (__ballot(cf > 8))
    GM_ASM(FAST_MC);
  else if (__ballot(cf > 4))
    GM_ASM(8);
  else if (__ballot(cf > 2))
    GM_ASM(4);
  else if (__ballot(cf > 1))
    GM_ASM(2);
  else
    GM_ASM(1);
#undef GM_ASM
}

// One lane's row of k_assemble_c once the wave's longest row fits W slots:
// W gathers (LDS, or the listed row), the W-wide network, W writes back (or,
// beside a slow row, straight to the output).
template <int W>
__device__ __forceinline__ void assemble_rows_c(uint32_t* out, const uint32_t* __restrict__ lrow, bool listed,
                                                uint32_t lpa, uint32_t cf, bool any_slow, uint32_t* __restrict__ ids,
                                                uint64_t base, const uint32_t* __restrict__ gmap) {
  uint32_t m[FAST_MC];
#pragma unroll
  for (int k = 0; k < FAST_MC; ++k)
    m[k] = (k < W && uint32_t(k) < cf) ? (listed ? lrow[k] : out[lpa + k]) : 0xFFFFFFFFu;
  if (W > 1) sort_row<W>(m);
  if (any_slow) {  // leave the slow rows' ranges alone: lane by lane
#pragma unroll
    for (int k = 0; k < W; ++k)
      if (uint32_t(k) < cf) ids[base + k] = gmap ? gmap[m[k]] : m[k];
    return;
  }
  wave_lds_sync();
#pragma unroll
  for (int k = 0; k < W; ++k)
    if (uint32_t(k) < cf) out[lpa + k] = gmap ? gmap[m[k]] : m[k];  // (no slow row: lpa == pa)
}

// Compact staging (k_match_fused<CMP>): the tile's list holds its matches in
// emission order as (filter id | lane | rank in its row), tlen[tile] of them, the
// partial rows of topics that went on to the listed pass included.  Each
// wave places its main-pass rows' entries in LDS at the row's offset (one
// LDS counter per row), sorts each row in registers, and writes the tile's
// ids as one coalesced range; a listed row comes from its own lstage row.
// The list is ~11.5 B per C2 topic against the ~20 B of [slot][lane] rows
// k_assemble reads.
struct AsmCLoads {  // one tile's loads of k_assemble_c, issued before any is used
  static constexpr int PRE = 4;
  uint32_t pre[PRE];  // the list's first 256 entries (a C2 tile holds ~184)
  uint32_t len, c;
  uint64_t tb0;
};
// blk_sums: blk holds the split scan's block SUMS (a scan of at most 64
// blocks: the prefix is summed here by the wave, one scan launch fewer), not
// their offsets.
__device__ __forceinline__ uint64_t blk_prefix(const uint64_t* __restrict__ sums, uint32_t j, int lane) {
  uint64_t v = uint32_t(lane) < j ? sums[lane] : 0ull;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}
__device__ __forceinline__ void asm_c_load(AsmCLoads& L, uint64_t tile, uint64_t n, int lane,
                                           const uint8_t* __restrict__ cnt8, const uint64_t* __restrict__ tile_off,
                                           const uint32_t* __restrict__ stage, const uint32_t* __restrict__ tlen,
                                           const uint64_t* __restrict__ blk, bool blk_sums = false) {
  const uint32_t* const lst = stage + tile * (64ull * FAST_MC);
#pragma unroll
  for (int q = 0; q < AsmCLoads::PRE; ++q) L.pre[q] = ld_s<true>(lst + q * 64 + lane);
  L.len = tlen[tile];
  const uint64_t t = tile * 64 + lane;
  L.c = t < n ? ld_s<true>(cnt8 + t) : 0u;  // 0xFF: the row's cnt word (asm_c_tile)
  L.tb0 = tile_off[tile] + (!blk ? 0ull : blk_sums ? blk_prefix(blk, uint32_t(tile / SCAN_B), lane)
                                                   : blk[tile / SCAN_B]);  // blk: a split scan's block offsets
}

// One tile of k_assemble_c from its loads (out, s_pa: the wave's LDS).
__device__ __forceinline__ void asm_c_tile(const AsmCLoads& L, uint64_t tile, uint64_t n, int lane, uint32_t* out,
                                           uint32_t* s_pa, const uint32_t* __restrict__ cnt,
                                           const uint32_t* __restrict__ stage,
                                           const uint32_t* __restrict__ lstage, const uint32_t* __restrict__ lcnt,
                                           uint64_t* __restrict__ row_off, uint32_t* __restrict__ ids,
                                           const uint32_t* __restrict__ gmap, uint64_t cap) {
  const uint64_t t = tile * 64 + lane;
  const uint32_t c = L.c == 0xFFu ? cnt[t] : L.c;  // a listed or slow row: its cnt word
  const bool slow = (c & OVF_BIT) != 0, listed = !slow && (c & LIST_BIT);
  const uint32_t call = slow ? (c & CNT_MASK) : listed ? lcnt[c & ~LIST_BIT] : c;
  const uint32_t cf = slow ? 0 : call;  // rows placed here (a slow row's ids land later, k_copy_slow)
  uint32_t tall, lall;
  const uint32_t pa = wave_excl_scan(call, tall);
  const uint32_t lpa = wave_excl_scan(cf, lall);  // the row's place in LDS (slow rows take none)
  const uint64_t base = L.tb0 + pa;
  if (t < n) row_off[t] = base;
  if (t == n - 1) row_off[n] = base + call;
  if (L.tb0 + tall > cap) return;  // wave-uniform
  const bool any_slow = __ballot(slow) != 0;
  // main-pass rows: scatter the list into LDS at each row's offset + the entry's rank
  s_pa[lane] = (slow || listed || t >= n) ? NONE : lpa;
  wave_lds_sync();
#define GM_PLACE(e)                                                               \
  do {                                                                            \
    const uint32_t rp = s_pa[((e) >> CMP_SHIFT) & 63u];                           \
    if (rp != NONE) out[rp + ((e) >> CMP_RANK)] = (e) & ((1u << CMP_SHIFT) - 1u); \
  } while (0)
#pragma unroll
  for (int q = 0; q < AsmCLoads::PRE; ++q)
    if (uint32_t(q * 64 + lane) < L.len) GM_PLACE(L.pre[q]);
  const uint32_t* const lst = stage + tile * (64ull * FAST_MC);
  for (uint32_t i = AsmCLoads::PRE * 64 + lane; i < L.len; i += 64) {
    const uint32_t e = ld_s<true>(lst + i);
    GM_PLACE(e);
  }
#undef GM_PLACE
  wave_lds_sync();
  // each row sorted in registers (W = the wave's longest row, a power of two)
  const uint32_t* const lrow = listed ? lstage + uint64_t(c & ~LIST_BIT) * FAST_MC : nullptr;
#define GM_ASMC(W) assemble_rows_c<W>(out, lrow, listed, lpa, cf, any_slow, ids, base, gmap)
  if (__ballot(cf > 8)) GM_ASMC(FAST_MC);
  else if (__ballot(cf > 4)) GM_ASMC(8);
  else if (__ballot(cf > 2)) GM_ASMC(4);
  else if (__ballot(cf > 1)) GM_ASMC(2);
  else GM_ASMC(1);
#undef GM_ASMC
  if (any_slow) return;
  wave_lds_sync();
  uint32_t* const dst = ids + L.tb0;
  for (uint32_t i = lane; i < tall; i += 64) st_s<true>(dst + i, out[i]);
}

// ASM_TPW tiles per wave, every tile's loads issued together (one round trip
// for all).  2 was slower at C2: 0.83-0.84 ms against 0.79-0.80 for 1, at 6
// waves/SIMD (74 VGPRs) or at 8 with spills.
constexpr int ASM_TPW = 1;
__global__ __launch_bounds__(256) void k_assemble_c(const uint8_t* __restrict__ cnt8, const uint32_t* __restrict__ cnt,
                                                    uint64_t n,
                                                    const uint64_t* __restrict__ tile_off,
                                                    const uint32_t* __restrict__ stage,
                                                    const uint32_t* __restrict__ tlen,
                                                    const uint32_t* __restrict__ lstage,
                                                    const uint32_t* __restrict__ lcnt,
                                                    uint64_t* __restrict__ row_off, uint32_t* __restrict__ ids,
                                                    const uint32_t* __restrict__ gmap, uint64_t cap,
                                                    const uint64_t* __restrict__ blk,
                                                    const uint32_t* __restrict__ rb_total,
                                                    const uint32_t* __restrict__ rb_ctr, uint32_t* __restrict__ rb_dst,
                                                    uint32_t* __restrict__ zero16, uint32_t blk_sums,
                                                    uint64_t* __restrict__ total_out) {
  __shared__ uint32_t s_out[4][64 * FAST_MC];
  __shared__ uint32_t s_pa[4][64];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // rb_dst (the call's pinned host words): the 40-B read-back -- the match
  // total and the pass counters, final before this kernel -- written by the
  // first wave's lanes (vector stores), so the call needs no copy packet; the
  // host reads it once this launch's stop event has completed
  // blk_sums (= the number of scan blocks): no launch wrote the grand total;
  // the first wave sums the blocks and writes it behind the tile offsets
  uint64_t gtot = 0;
  if (blk_sums && blockIdx.x == 0 && wv == 0) {
    gtot = blk_prefix(blk, blk_sums, lane);
    if (lane == 0) *total_out = gtot;
  }
  if (rb_dst && blockIdx.x == 0 && wv == 0) {
    if (lane < 10)
      rb_dst[lane] = lane < 2 ? (blk_sums ? uint32_t(gtot >> (32 * lane)) : rb_total[lane]) : rb_ctr[lane - 2];
    __threadfence_system();  // (out to host memory before the kernel's end is signalled)
  }
  // zero16: the next call's pass-counter block (the context's ring), zeroed
  // for it here so that call needs no zeroing launch
  if (zero16 && blockIdx.x == 0 && wv == 1 && lane < 16) zero16[lane] = 0u;
  const uint64_t n_tiles = (n + 63) / 64;
  const uint64_t tile0 = (uint64_t(blockIdx.x) * 4 + wv) * ASM_TPW;
  if (tile0 >= n_tiles) return;  // wave-uniform; no block barrier below
  AsmCLoads L[ASM_TPW];
#pragma unroll
  for (int k = 0; k < ASM_TPW; ++k)
    if (tile0 + k < n_tiles) asm_c_load(L[k], tile0 + k, n, lane, cnt8, tile_off, stage, tlen, blk, blk_sums != 0);
#pragma unroll
  for (int k = 0; k < ASM_TPW; ++k) {
    if (tile0 + k >= n_tiles) break;
    if (k) wave_lds_sync();  // the previous tile is done with the wave's LDS
    asm_c_tile(L[k], tile0 + k, n, lane, s_out[wv], s_pa[wv], cnt, stage, lstage, lcnt, row_off, ids, gmap, cap);
  }
}

// ---------------------------------------------------------------------------
// slow path
// ---------------------------------------------------------------------------
template <bool EXACT>
__global__ __launch_bounds__(256) void k_slow_walk(const uint8_t* __restrict__ tb,
                                                   const uint64_t* __restrict__ toff, IndexView ix,
                                                   const uint32_t* __restrict__ list, uint64_t k0, uint64_t kn,
                                                   uint32_t* __restrict__ fr_all, uint64_t fr_cap,
                                                   uint32_t* __restrict__ bm_all, uint64_t bm_words,
                                                   uint32_t* __restrict__ cnt, uint64_t* __restrict__ slow_cnt,
                                                   uint64_t* __restrict__ tsum) {
  const uint64_t k = k0 + blockIdx.x;
  if (k >= kn) return;
  const uint32_t t = list[k];
  uint32_t* fr0 = fr_all + uint64_t(blockIdx.x) * 2 * fr_cap;
  uint32_t* fr1 = fr0 + fr_cap;
  uint32_t* bm = bm_all + uint64_t(blockIdx.x) * bm_words;
  __shared__ uint32_t s_cur_n, s_nxt_n, s_wid, s_flags;  // flags: 1 last, 2 wild, 4 dollar
  __shared__ uint64_t s_pos;
  __shared__ uint32_t s_level;
  __shared__ uint32_t s_red[256];
  const int tid = threadIdx.x;
  for (uint64_t i = tid; i < bm_words; i += 256) bm[i] = 0;
  const uint64_t end = toff[t + 1];
  if (tid == 0) {
    s_pos = toff[t];
    s_cur_n = 1;
    s_nxt_n = 0;
    s_level = 0;
    s_flags = 0;
    fr0[0] = 0;
  }
  __syncthreads();
  uint32_t* cur = fr0;
  uint32_t* nxt = fr1;
  for (;;) {
    if (tid == 0) {
      ByteReader rd{tb, ~0ull, 0};
      uint64_t pos = s_pos;
      const WordTok w = next_word(rd, pos, end);
      uint32_t fl = s_flags & 4u;
      if (pos >= end) fl |= 1u;
      if (w.len == 1 && (w.b0 == '+' || w.b0 == '#')) fl |= 2u;
      if (s_level == 0 && w.len > 0 && w.b0 == '$') fl |= 4u;
      s_flags = fl;
      s_wid = (fl & 2u) ? NONE : dict_resolve(ix, w, dict_first(ix, w), tb);
      s_pos = pos + 1;
    }
    __syncthreads();
    const uint32_t fl = s_flags;
    if (fl & 2u) break;
    const uint32_t wid = s_wid, cn = s_cur_n, lvl = s_level;
    const bool rootskip = (fl & 4u) && lvl == 0;
    for (uint32_t i = tid; i < cn; i += 256) {
      const uint32_t nd = cur[i] & REF_MASK;
      const Node node = ix.nodes[nd];
      if (!rootskip) {
        if (node.hash_filter != NONE) atomicOr(&bm[node.hash_filter >> 5], 1u << (node.hash_filter & 31));
        if (node.plus_child != NONE) nxt[atomicAdd(&s_nxt_n, 1u)] = node.plus_child;
      }
      if (wid != NONE && (node.flags & NF_HAS_EXACT)) {
        const uint32_t c = edge_lookup(ix, lvl, nd, wid);
        if (c != NONE) nxt[atomicAdd(&s_nxt_n, 1u)] = c;
      }
    }
    __syncthreads();
    if (tid == 0) {
      s_cur_n = s_nxt_n;
      s_nxt_n = 0;
      if (!(fl & 1u)) s_level = s_level + 1;
    }
    uint32_t* tmp = cur;
    cur = nxt;
    nxt = tmp;
    __syncthreads();
    if (fl & 1u) break;
  }
  const uint32_t fl = s_flags;
  if (fl & 2u) {  // wildcard topic: [] (trie) or the literal filter (routes)
    __syncthreads();
    for (uint64_t i = tid; i < bm_words; i += 256) atomicAnd(&bm[i], 0u);
    __syncthreads();
    if (EXACT && tid == 0) {
      const uint32_t f = literal_lookup(ix, tb, toff[t], end);
      if (f != NONE) atomicOr(&bm[f >> 5], 1u << (f & 31));
    }
  } else {
    const uint32_t cn = s_cur_n;
    const bool single = s_level == 0 && (fl & 4u);
    for (uint32_t i = tid; i < cn; i += 256) {
      const Node node = ix.nodes[cur[i] & REF_MASK];
      if (node.hash_filter != NONE) atomicOr(&bm[node.hash_filter >> 5], 1u << (node.hash_filter & 31));
      if (node.end_filter != NONE && (EXACT || (node.flags & NF_END_WILD) || single))
        atomicOr(&bm[node.end_filter >> 5], 1u << (node.end_filter & 31));
    }
  }
  __syncthreads();
  uint32_t c = 0;
  for (uint64_t i = tid; i < bm_words; i += 256)
    c += __popc(__hip_atomic_load(&bm[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  s_red[tid] = c;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) s_red[tid] += s_red[tid + s];
    __syncthreads();
  }
  if (tid == 0) {
    slow_cnt[k] = s_red[0];
    cnt[t] = OVF_BIT | s_red[0];
    atomicAdd(reinterpret_cast<unsigned long long*>(tsum + (t >> 6)), (unsigned long long)s_red[0]);
  }
}

__global__ __launch_bounds__(256) void k_slow_emit(uint64_t k0, uint64_t kn, const uint32_t* __restrict__ bm_all,
                                                   uint64_t bm_words, const uint64_t* __restrict__ slow_off,
                                                   uint32_t* __restrict__ slow_ids) {
  const uint64_t k = k0 + blockIdx.x;
  if (k >= kn) return;
  const uint32_t* bm = bm_all + uint64_t(blockIdx.x) * bm_words;
  __shared__ uint32_t s_w[4];
  uint64_t out = slow_off[k];
  for (uint64_t b = 0; b < bm_words; b += 256) {
    const uint64_t i = b + threadIdx.x;
    uint32_t w = i < bm_words ? bm[i] : 0;
    uint32_t tot;
    const uint32_t pre = wave_excl_scan(__popc(w), tot);
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) s_w[wv] = tot;
    __syncthreads();
    uint32_t wpre = 0, all = 0;
    for (int q = 0; q < 4; ++q) {
      if (q < wv) wpre += s_w[q];
      all += s_w[q];
    }
    uint64_t o = out + wpre + pre;
    while (w) {
      const int bit = __ffs(w) - 1;
      slow_ids[o++] = uint32_t(i * 32 + bit);
      w &= w - 1;
    }
    out += all;
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void k_copy_slow(const uint32_t* __restrict__ list, uint64_t kn,
                                                   const uint64_t* __restrict__ row_off,
                                                   const uint64_t* __restrict__ slow_off,
                                                   const uint32_t* __restrict__ slow_ids, uint32_t* __restrict__ ids,
                                                   const uint32_t* __restrict__ gmap) {
  const uint64_t k = blockIdx.x;
  if (k >= kn) return;
  const uint32_t t = list[k];
  const uint64_t dst = row_off[t], src = slow_off[k], len = slow_off[k + 1] - src;
  for (uint64_t i = threadIdx.x; i < len; i += 256) {
    const uint32_t f = slow_ids[src + i];
    ids[dst + i] = gmap ? gmap[f] : f;
  }
}

// ---------------------------------------------------------------------------
// fan-out
// ---------------------------------------------------------------------------
// (nseg: the segments seg_dst holds -- a speculative call's row offsets may point past them)
__global__ __launch_bounds__(256) void k_fanout_rowoff(const uint64_t* __restrict__ m_off, uint64_t n,
                                                       const uint64_t* __restrict__ seg_dst,
                                                       uint64_t* __restrict__ out_off, uint64_t nseg) {
  const uint64_t i = uint64_t(blockIdx.x) * 256u + threadIdx.x;
  if (i <= n) out_off[i] = seg_dst[min(m_off[i], nseg)];
}

// Output elements per workgroup: from 1,024 (a publish window's ~100k
// deliveries in ~100 workgroups, not 30: 63 -> ~20 us) up to 65,536 for large
// fan-outs (C4: 0.94 -> 0.81 ms against 4,096, fewer per-block segment
// searches), a multiple of 1,024 (4 per thread step).
inline uint64_t fan_per_block(uint64_t total) {
  uint64_t per = total / 2048;  // ~8 workgroups per CU
  per = per < 1024 ? 1024 : per > 65536 ? 65536 : per;
  return (per + 1023) & ~uint64_t(1023);
}

// Segment of output element p: the last segment whose start <= p, searched in
// [a, b] (the block's first and last segments).
__device__ __forceinline__ uint64_t fan_seg(const uint64_t* __restrict__ seg_dst, uint64_t a, uint64_t b, uint64_t p) {
  if (a == b) return a;
  ++b;
  while (b - a > 1) {
    const uint64_t m = (a + b) >> 1;
    if (seg_dst[m] <= p) a = m;
    else b = m;
  }
  return a;
}

// Every workgroup owns per_block consecutive output elements; a thread
// moves 4 consecutive elements at a time, as one 16-B non-temporal store (the
// output is streamed out once) when they lie in one segment -- the usual case,
// a hot row being one long segment -- and element by element across a
// segment boundary.
__global__ __launch_bounds__(256) void k_fanout_copy(const uint64_t* __restrict__ seg_dst, uint64_t nseg,
                                                     const uint32_t* __restrict__ m_ids,
                                                     const uint64_t* __restrict__ sub_off,
                                                     const uint32_t* __restrict__ sub_ids, uint64_t glo,
                                                     uint64_t total, uint64_t per_block, uint32_t* __restrict__ out0,
                                                     bool clamp) {
  // this launch produces the global delivery range [glo, total); out0[0] is delivery glo
  // (clamp: never past the device's own total -- a small host fan-out sizes
  // the launch by a speculative capacity, gm_host.cpp run_fanout_small)
  if (clamp) total = min(total, seg_dst[nseg]);
  const uint64_t lo = glo + uint64_t(blockIdx.x) * per_block;
  if (lo >= total) return;
  const uint64_t hi = min(total, lo + per_block);
  uint32_t* const out = out0 - glo;  // indexed by global delivery number
  __shared__ uint64_t s_seg[2];
  if (threadIdx.x < 2) {
    // last segment whose start <= x (segments may be empty)
    const uint64_t x = threadIdx.x == 0 ? lo : hi - 1;
    uint64_t a = 0, b = nseg;  // seg_dst[a] <= x < seg_dst[b]
    while (b - a > 1) {
      const uint64_t m = (a + b) >> 1;
      if (seg_dst[m] <= x) a = m;
      else b = m;
    }
    s_seg[threadIdx.x] = a;
  }
  __syncthreads();
  const uint64_t s0 = s_seg[0], s1 = s_seg[1];
  if (s0 == s1) {
    // the whole range lies in one segment (a hot row): the source offset is
    // loop invariant, so each step is an independent load + store with no
    // dependent segment lookups in between
    const uint64_t off = sub_off[m_ids[s0]] - seg_dst[s0];  // element q comes from sub_ids[off + q] (mod 2^64)
    uint64_t q = lo + uint64_t(threadIdx.x) * 4;
    for (; q + 4 <= hi; q += 256 * 4) {
      const uint32_t* src = sub_ids + (off + q);
      const uint4 v = make_uint4(src[0], src[1], src[2], src[3]);
      __builtin_nontemporal_store(v.x, out + q);
      __builtin_nontemporal_store(v.y, out + q + 1);
      __builtin_nontemporal_store(v.z, out + q + 2);
      __builtin_nontemporal_store(v.w, out + q + 3);
    }
    for (uint64_t p = q; p < hi; ++p) out[p] = sub_ids[off + p];  // q + 4 > hi here: at most 3 left
    return;
  }
  for (uint64_t q = lo + uint64_t(threadIdx.x) * 4; q < hi; q += 256 * 4) {
    const uint64_t s = fan_seg(seg_dst, s0, s1, q);
    const uint64_t sd = seg_dst[s];
    if (q + 4 <= hi && q + 4 <= seg_dst[s + 1]) {
      const uint32_t* src = sub_ids + sub_off[m_ids[s]] + (q - sd);
      const uint4 v = make_uint4(src[0], src[1], src[2], src[3]);
      __builtin_nontemporal_store(v.x, out + q);
      __builtin_nontemporal_store(v.y, out + q + 1);
      __builtin_nontemporal_store(v.z, out + q + 2);
      __builtin_nontemporal_store(v.w, out + q + 3);
    } else {
      for (uint64_t p = q; p < q + 4 && p < hi; ++p) {
        const uint64_t sp = fan_seg(seg_dst, s0, s1, p);
        out[p] = sub_ids[sub_off[m_ids[sp]] + (p - seg_dst[sp])];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// stats helper: sum of matched filter lengths (for algorithmic bytes)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lower_bound_u32(const uint32_t* a, uint32_t n, uint32_t x) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t m = (lo + hi) >> 1;
    if (a[m] < x) lo = m + 1;
    else hi = m;
  }
  return lo;
}

__global__ __launch_bounds__(256) void k_sum_flen(const uint32_t* __restrict__ ids, uint64_t nnz,
                                                  const uint16_t* __restrict__ flen,
                                                  const uint32_t* __restrict__ gmap, uint32_t nf,
                                                  unsigned long long* __restrict__ acc) {
  uint64_t s = 0;
  for (uint64_t i = uint64_t(blockIdx.x) * 256u + threadIdx.x; i < nnz; i += uint64_t(gridDim.x) * 256u)
    s += flen[gmap ? lower_bound_u32(gmap, nf, ids[i]) : ids[i]];
  for (int d = 32; d > 0; d >>= 1) s += __shfl_down(s, d, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(acc, (unsigned long long)s);
}

// ---------------------------------------------------------------------------
// row merge (sharded index)
// ---------------------------------------------------------------------------
// Pieces p = 0..P-1 each hold, for the same n rows, a sorted list of filter
// ids; the lists of one row are disjoint (filters are partitioned over the
// shards).  lens is [P][stride] (rows >= n have length 0), ids the pieces'
// rows concatenated piece-major, row-minor (the all-to-all's output), so an
// exclusive scan of lens gives every (piece, row) list's offset in ids.  Each
// element's rank in its merged row = its index in its own list + its
// lower_bound in every other list of the row.
struct LoadU32 {
  const uint32_t* p;
  __device__ uint64_t operator()(uint64_t i) const { return p[i]; }
};
struct LoadRowSum {  // merged row length
  const uint32_t* lens;
  uint64_t stride;
  uint32_t pieces;
  __device__ uint64_t operator()(uint64_t t) const {
    uint64_t s = 0;
    for (uint32_t p = 0; p < pieces; ++p) s += lens[p * stride + t];
    return s;
  }
};

__global__ __launch_bounds__(256) void k_merge_rows(const uint32_t* __restrict__ lens, const uint64_t* __restrict__ pos,
                                                    const uint32_t* __restrict__ ids, uint64_t n, uint64_t stride,
                                                    uint32_t pieces, const uint64_t* __restrict__ row_off,
                                                    uint32_t* __restrict__ out) {
  const uint64_t t = uint64_t(blockIdx.x) * 256u + threadIdx.x;
  if (t >= n) return;
  const uint64_t o = row_off[t];
  for (uint32_t p = 0; p < pieces; ++p) {
    const uint64_t src = pos[p * stride + t];
    const uint32_t len = lens[p * stride + t];
    for (uint32_t j = 0; j < len; ++j) {
      const uint32_t x = ids[src + j];
      uint64_t r = j;
      for (uint32_t q = 0; q < pieces; ++q)
        if (q != p) r += lower_bound_u32(ids + pos[q * stride + t], lens[q * stride + t], x);
      out[o + r] = x;
    }
  }
}

__global__ __launch_bounds__(256) void k_row_lengths(const uint64_t* __restrict__ row_off, uint64_t n,
                                                     uint32_t* __restrict__ out) {
  const uint64_t t = uint64_t(blockIdx.x) * 256u + threadIdx.x;
  if (t < n) out[t] = uint32_t(row_off[t + 1] - row_off[t]);
}

// ---------------------------------------------------------------------------
// overlay snapshot merge (incremental updates, gm_overlay.cpp)
// ---------------------------------------------------------------------------
struct OvView {
  const uint32_t* tbm;   // tombstone bitmap over base ids
  const uint32_t* tpre;  // tombstones in the words before each bitmap word
  const uint32_t* ins;   // insertion point of each delta filter, ascending
  uint32_t n_ins;
};
__device__ __forceinline__ bool ov_dead(const OvView& o, uint32_t b) { return (o.tbm[b >> 5] >> (b & 31)) & 1u; }
// final id of a surviving base id: + delta filters sorting before it - tombstones below it
__device__ __forceinline__ uint32_t ov_remap(const OvView& o, uint32_t b) {
  uint32_t lo = 0, hi = o.n_ins;
  while (lo < hi) {
    const uint32_t m = (lo + hi) >> 1;
    if (o.ins[m] <= b) lo = m + 1;
    else hi = m;
  }
  const uint32_t w = b >> 5;
  return b + lo - (o.tpre[w] + __popc(o.tbm[w] & ((1u << (b & 31)) - 1u)));
}
struct LoadOvLen {  // merged row length: surviving base ids + delta ids
  const uint64_t* bo;
  const uint32_t* bi;
  const uint64_t* dof;
  OvView o;
  __device__ uint64_t operator()(uint64_t t) const {
    uint64_t c = dof ? dof[t + 1] - dof[t] : 0;
    for (uint64_t k = bo[t]; k < bo[t + 1]; ++k) c += ov_dead(o, bi[k]) ? 0 : 1;
    return c;
  }
};
__global__ __launch_bounds__(256) void k_ov_merge(const uint64_t* __restrict__ bo, const uint32_t* __restrict__ bi,
                                                  const uint64_t* __restrict__ dof, const uint32_t* __restrict__ di,
                                                  OvView o, uint64_t n, const uint64_t* __restrict__ row_off,
                                                  uint32_t* __restrict__ out) {
  const uint64_t t = uint64_t(blockIdx.x) * 256u + threadIdx.x;
  if (t >= n) return;
  uint64_t i = bo[t], w = row_off[t];
  const uint64_t ie = bo[t + 1];
  uint64_t j = dof ? dof[t] : 0;
  const uint64_t je = dof ? dof[t + 1] : 0;
  auto next_base = [&]() -> uint32_t {
    while (i < ie && ov_dead(o, bi[i])) ++i;
    return i < ie ? ov_remap(o, bi[i]) : 0xFFFFFFFFu;
  };
  uint32_t b = next_base(), d = j < je ? di[j] : 0xFFFFFFFFu;
  while (b != 0xFFFFFFFFu || d != 0xFFFFFFFFu) {
    if (b < d) {
      out[w++] = b;
      ++i;
      b = next_base();
    } else {
      out[w++] = d;
      ++j;
      d = j < je ? di[j] : 0xFFFFFFFFu;
    }
  }
}

// Offsets of the host-buffer path: topics cross PCIe with u32 chunk-relative
// offsets (4 B per topic instead of 8) and rows come back the same way.
__global__ __launch_bounds__(256) void k_off32_to_64(const uint32_t* __restrict__ in, uint64_t n1,
                                                     uint64_t* __restrict__ out) {
  for (uint64_t i = uint64_t(blockIdx.x) * 256u + threadIdx.x; i < n1; i += uint64_t(gridDim.x) * 256u) out[i] = in[i];
}
__global__ __launch_bounds__(256) void k_off64_to_32(const uint64_t* __restrict__ in, uint64_t n1,
                                                     uint32_t* __restrict__ out) {
  for (uint64_t i = uint64_t(blockIdx.x) * 256u + threadIdx.x; i < n1; i += uint64_t(gridDim.x) * 256u)
    out[i] = uint32_t(in[i]);
}
int launch_off32_to_64(hipStream_t st, const uint32_t* in, uint64_t n1, uint64_t* out) {
  const uint64_t g = std::min<uint64_t>(2048, (n1 + 255) / 256);
  hipLaunchKernelGGL(k_off32_to_64, dim3(g ? g : 1), dim3(256), 0, st, in, n1, out);
  return hipGetLastError() == hipSuccess ? 0 : EMQX_GM_EDEVICE;
}
int launch_off64_to_32(hipStream_t st, const uint64_t* in, uint64_t n1, uint32_t* out) {
  const uint64_t g = std::min<uint64_t>(2048, (n1 + 255) / 256);
  hipLaunchKernelGGL(k_off64_to_32, dim3(g ? g : 1), dim3(256), 0, st, in, n1, out);
  return hipGetLastError() == hipSuccess ? 0 : EMQX_GM_EDEVICE;
}
// Small host-buffer calls (gm_host.cpp run_host_small): inputs in and rows out
// through page-locked host memory the device addresses directly -- two copies
// in one launch on the call's own queue, so no copy engine has to hand over to
// the compute queue between the call's kernels (~10 us a hand-over).  n1_max
// (optional): the second copy stops at the count the device wrote there (a
// result's row_off[n]: the rows' true length inside a speculative capacity)
__global__ __launch_bounds__(256) void k_copy_u32x2(const uint32_t* __restrict__ s0, uint32_t* __restrict__ d0,
                                                    uint64_t n0, const uint32_t* __restrict__ s1,
                                                    uint32_t* __restrict__ d1, uint64_t n1,
                                                    const uint64_t* __restrict__ n1_max) {
  if (n1_max) n1 = min(n1, *n1_max);
  const uint64_t t = uint64_t(blockIdx.x) * 256u + threadIdx.x, stride = uint64_t(gridDim.x) * 256u;
  const uint64_t q0 = n0 / 4, q1 = n1 / 4;  // (16-B units; every buffer here is 16-B aligned)
  for (uint64_t i = t; i < q0; i += stride)
    reinterpret_cast<uint4*>(d0)[i] = reinterpret_cast<const uint4*>(s0)[i];
  for (uint64_t i = t; i < q1; i += stride)
    reinterpret_cast<uint4*>(d1)[i] = reinterpret_cast<const uint4*>(s1)[i];
  if (t < (n0 & 3)) d0[q0 * 4 + t] = s0[q0 * 4 + t];
  if (t < (n1 & 3)) d1[q1 * 4 + t] = s1[q1 * 4 + t];
  __threadfence_system();  // (host-bound stores visible before the call's end event)
}
int launch_copy_u32x2(hipStream_t st, const uint32_t* s0, uint32_t* d0, uint64_t n0, const uint32_t* s1, uint32_t* d1,
                      uint64_t n1, const uint64_t* n1_max) {
  const uint64_t q = (std::max(n0, n1) + 3) / 4;
  const uint64_t g = std::min<uint64_t>(1024, (q + 255) / 256);
  hipLaunchKernelGGL(k_copy_u32x2, dim3(g ? g : 1), dim3(256), 0, st, s0, d0, n0, s1, d1, n1, n1_max);
  return hipGetLastError() == hipSuccess ? 0 : EMQX_GM_EDEVICE;
}
// p[0..n1) += add, in place (a chunk's row offsets rebased to the whole call's rows)
__global__ __launch_bounds__(256) void k_add_u64(uint64_t* __restrict__ p, uint64_t n1, uint64_t add) {
  for (uint64_t i = uint64_t(blockIdx.x) * 256u + threadIdx.x; i < n1; i += uint64_t(gridDim.x) * 256u) p[i] += add;
}
int launch_add_u64(hipStream_t st, uint64_t* p, uint64_t n1, uint64_t add) {
  if (!n1) return 0;
  const uint64_t g = std::min<uint64_t>(2048, (n1 + 255) / 256);
  hipLaunchKernelGGL(k_add_u64, dim3(g), dim3(256), 0, st, p, n1, add);
  return hipGetLastError() == hipSuccess ? 0 : EMQX_GM_EDEVICE;
}

// ---- in-place update (gm_overlay.cpp, patch_update) -----------------------
// The host-patched byte ranges, cut into pieces of <= PATCH_PIECE bytes, one
// workgroup per piece: desc[3b..3b+2] = (offset in the blob, offset in the
// payload, bytes).
constexpr uint32_t PATCH_PIECE = 4096;
__global__ __launch_bounds__(256) void k_patch_scatter(uint8_t* __restrict__ dst, const uint64_t* __restrict__ desc,
                                                       const uint8_t* __restrict__ pay) {
  const uint64_t d = desc[3 * blockIdx.x], p = desc[3 * blockIdx.x + 1], n = desc[3 * blockIdx.x + 2];
  for (uint64_t i = threadIdx.x; i < n; i += 256) dst[d + i] = pay[p + i];
}
// The id table of an in-place update (IdShift::map, gm_internal.h), built on
// the device from the O(delta) lists: dels (prev ids deleted, ascending) and
// addpos (per new filter, byte order: prev filters sorting before it).
__device__ __forceinline__ uint32_t count_below(const uint32_t* a, uint32_t n, uint32_t x) {  // a[i] < x
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t m = (lo + hi) >> 1;
    if (a[m] < x) lo = m + 1;
    else hi = m;
  }
  return lo;
}
__global__ __launch_bounds__(256) void k_shift_table(uint32_t* __restrict__ rmap, uint64_t nb,
                                                     const uint32_t* __restrict__ dels, uint32_t nd,
                                                     const uint32_t* __restrict__ addpos, uint32_t na) {
  const uint64_t id = uint64_t(blockIdx.x) * 256u + threadIdx.x;
  if (id >= nb + na) return;
  if (id >= nb) {
    const uint32_t k = uint32_t(id - nb), p = addpos[k];
    rmap[id] = p - count_below(dels, nd, p) + k;
    return;
  }
  const uint32_t x = uint32_t(id), below = count_below(dels, nd, x);
  if (below < nd && dels[below] == x) {
    rmap[id] = NONE;
    return;
  }
  rmap[id] = x - below + count_below(addpos, na, x + 1);  // inserts at or before it
}
// Flag bits set on words whose other bits are filter ids (HOT_PLUS on hf /
// p_hf): the host mirror's ids are stale (not renumbered), so these go as ORs.
__global__ __launch_bounds__(256) void k_patch_or(uint32_t* __restrict__ dst, const uint64_t* __restrict__ ops,
                                                  uint64_t n) {
  const uint64_t i = uint64_t(blockIdx.x) * 256u + threadIdx.x;
  if (i >= n) return;
  const uint64_t off = ops[2 * i];
  if (off & PATCH_AND) atomicAnd(dst + ((off & ~PATCH_AND) >> 2), ~uint32_t(ops[2 * i + 1]));
  else atomicOr(dst + (off >> 2), uint32_t(ops[2 * i + 1]));
}
// Every filter-id field renumbered (renum_field, the device twin of
// gm_overlay.cpp's renumber_host): hot slots [0, n_hot), nodes [0, n_nodes).
__global__ __launch_bounds__(256) void k_renumber(HotSlot* __restrict__ hot, uint64_t n_hot, Node* __restrict__ nodes,
                                                  uint64_t n_nodes, const uint32_t* __restrict__ rmap) {
  const uint64_t stride = uint64_t(gridDim.x) * 256u;
  for (uint64_t s = uint64_t(blockIdx.x) * 256u + threadIdx.x; s < n_hot; s += stride) {
    HotSlot h = hot[s];
    if (h.key == EDGE_EMPTY) continue;
    h.hf = renum_field(h.hf, HF_NONE, HF_FLAGS, rmap);
    h.end_filter = renum_field(h.end_filter, NONE, END_WILD, rmap);
    h.p_hf = renum_field(h.p_hf, HF_NONE, HF_FLAGS, rmap);
    h.p_end = renum_field(h.p_end, NONE, END_WILD, rmap);
    hot[s] = h;
  }
  for (uint64_t i = uint64_t(blockIdx.x) * 256u + threadIdx.x; i < n_nodes; i += stride) {
    Node nd = nodes[i];
    nd.hash_filter = renum_field(nd.hash_filter, NONE, 0, rmap);
    nd.end_filter = renum_field(nd.end_filter, NONE, 0, rmap);
    nodes[i] = nd;
  }
}

// k_renumber fused with the blob copy: dst's hot slots and nodes = src's,
// renumbered (every slot written, empty ones as they are), so an update reads
// and writes the id-bearing tables once instead of copying them and then
// renumbering them in place (C5: ~26 of the 38 GB blob)
__global__ __launch_bounds__(256) void k_renumber_copy(const HotSlot* __restrict__ shot, HotSlot* __restrict__ hot,
                                                       uint64_t n_hot, const Node* __restrict__ snodes,
                                                       Node* __restrict__ nodes, uint64_t n_nodes,
                                                       const uint32_t* __restrict__ rmap) {
  const uint64_t stride = uint64_t(gridDim.x) * 256u;
  for (uint64_t s = uint64_t(blockIdx.x) * 256u + threadIdx.x; s < n_hot; s += stride) {
    HotSlot h = shot[s];
    if (h.key != EDGE_EMPTY) {
      h.hf = renum_field(h.hf, HF_NONE, HF_FLAGS, rmap);
      h.end_filter = renum_field(h.end_filter, NONE, END_WILD, rmap);
      h.p_hf = renum_field(h.p_hf, HF_NONE, HF_FLAGS, rmap);
      h.p_end = renum_field(h.p_end, NONE, END_WILD, rmap);
    }
    hot[s] = h;
  }
  for (uint64_t i = uint64_t(blockIdx.x) * 256u + threadIdx.x; i < n_nodes; i += stride) {
    Node nd = snodes[i];
    nd.hash_filter = renum_field(nd.hash_filter, NONE, 0, rmap);
    nd.end_filter = renum_field(nd.end_filter, NONE, 0, rmap);
    nodes[i] = nd;
  }
}

namespace {
// The filter-id fields of the records k_renumber rewrites: (offset, empty value, flag bits)
struct IdField {
  uint32_t off, none, flag;
};
constexpr IdField kHotIds[] = {{offsetof(HotSlot, hf), HF_NONE, HF_FLAGS},
                               {offsetof(HotSlot, end_filter), NONE, END_WILD},
                               {offsetof(HotSlot, p_hf), HF_NONE, HF_FLAGS},
                               {offsetof(HotSlot, p_end), NONE, END_WILD}};
constexpr IdField kNodeIds[] = {{offsetof(Node, hash_filter), NONE, 0u}, {offsetof(Node, end_filter), NONE, 0u}};
// The id fields of the table [o, o + n * rec) lying inside the patched range
// [a, b) (buf = its bytes), renumbered in place by the shift (IdShift::map:
// O(log delta) per field).  false: a field holds an id outside the shift.
template <size_t K>
bool renum_payload(uint8_t* buf, uint64_t a, uint64_t b, uint64_t o, uint64_t n, uint64_t rec,
                   const IdField (&fs)[K], const IdShift& sh, uint64_t n_map) {
  const uint64_t lo = std::max(a, o), hi = std::min(b, o + n * rec);
  for (uint64_t r = lo < hi ? (lo - o) / rec : 0, re = lo < hi ? (hi - o + rec - 1) / rec : 0; r < re; ++r)
    for (const IdField& f : fs) {
      const uint64_t at = o + r * rec + f.off;
      if (at < a || at + 4 > b) continue;  // (the patcher writes id fields whole)
      uint32_t x;
      std::memcpy(&x, buf + (at - a), 4);
      const uint32_t id = x & ~f.flag;
      if (x != f.none && id != (f.none & ~f.flag) && id >= n_map) return false;
      x = renum_field(x, f.none, f.flag, sh);
      std::memcpy(buf + (at - a), &x, 4);
    }
  return true;
}
}  // namespace

int apply_patch_device(emqx_gm_ctx* ctx, void* dst, const void* src, size_t bytes,
                       const std::vector<std::pair<uint64_t, uint32_t>>& ranges, const uint8_t* host,
                       const IndexView& v, uint64_t o_hot, uint64_t o_nodes, uint64_t n_nodes,
                       const IdShift& shift, const std::vector<std::pair<uint64_t, uint32_t>>& orops) {
  uint64_t n_hot = 0;
  for (int t = 0; t < HOT_TABLES; ++t) n_hot = std::max<uint64_t>(n_hot, v.hot_off[t] + v.hot_cap[t]);
  const uint64_t hot_end = o_hot + n_hot * sizeof(HotSlot), nodes_end = o_nodes + n_nodes * sizeof(Node);
  if (hot_end > bytes || nodes_end > bytes) return set_err(ctx, EMQX_GM_EINVAL, "index_update: tables outside the blob");
  const bool unfused = knob("GM_UPDATE_UNFUSED") != nullptr;
  // fused (one pass): the two id-bearing tables must not overlap
  const bool fused = !unfused && (hot_end <= o_nodes || nodes_end <= o_hot);
  // coalesce overlapping / adjacent ranges only (the bytes between two written
  // fields may differ: the host mirror's untouched filter ids are stale), then
  // cut into pieces
  std::vector<std::pair<uint64_t, uint64_t>> seg;  // [begin, end)
  {
    std::vector<std::pair<uint64_t, uint32_t>> r(ranges);
    std::sort(r.begin(), r.end());
    for (const auto& x : r) {
      if (!x.second) continue;
      if (x.first + x.second > bytes) return set_err(ctx, EMQX_GM_EINVAL, "index_update: patch outside the blob");
      if (!seg.empty() && x.first <= seg.back().second) seg.back().second = std::max(seg.back().second, x.first + x.second);
      else seg.emplace_back(x.first, x.first + x.second);
    }
  }
  for (const auto& o : orops)
    if ((o.first & 3) || (o.first & ~PATCH_AND) + 4 > bytes)
      return set_err(ctx, EMQX_GM_EINVAL, "index_update: OR/AND op outside the blob");
  std::vector<uint64_t> desc;
  uint64_t pay_n = 0;
  for (const auto& g : seg) {
    for (uint64_t b = g.first; b < g.second; b += PATCH_PIECE) {
      const uint64_t n = std::min<uint64_t>(PATCH_PIECE, g.second - b);
      desc.insert(desc.end(), {b, pay_n + (b - g.first), n});
    }
    pay_n += g.second - g.first;
  }
  const uint64_t n_pieces = desc.size() / 3;
  if (n_pieces > 0x7FFFFFFFull) return set_err(ctx, EMQX_GM_EINVAL, "index_update: patch too large");
  // staging: desc | payload | dels | addpos | OR ops (one upload); the id table after them (device-built)
  const uint64_t nd = shift.dels.size(), na = shift.addpos.size(), n_map = shift.nb + na;
  const size_t o_pay = (desc.size() * 8 + 255) & ~size_t(255);
  const size_t o_dels = (o_pay + pay_n + 255) & ~size_t(255);
  const size_t o_adds = (o_dels + nd * 4 + 4 + 255) & ~size_t(255);
  const size_t o_ors = (o_adds + na * 4 + 4 + 255) & ~size_t(255);
  const size_t up = o_ors + orops.size() * 16 + 16;
  const size_t o_rmap = (up + 255) & ~size_t(255);
  const size_t total = o_rmap + n_map * 4 + 4;
  std::vector<uint8_t> st(up, 0);
  if (!desc.empty()) std::memcpy(st.data(), desc.data(), desc.size() * 8);
  {
    uint64_t q = o_pay;
    for (const auto& g : seg) {
      uint8_t* const pb = st.data() + q;
      std::memcpy(pb, host + g.first, g.second - g.first);
      // fused: the range's filter ids (this update's temporary numbering) go up final
      if (fused && !(renum_payload(pb, g.first, g.second, o_hot, n_hot, sizeof(HotSlot), kHotIds, shift, n_map) &&
                     renum_payload(pb, g.first, g.second, o_nodes, n_nodes, sizeof(Node), kNodeIds, shift, n_map)))
        return set_err(ctx, EMQX_GM_EINVAL, "index_update: a patched filter id outside the update's ids");
      q += g.second - g.first;
    }
  }
  for (uint64_t k = 0; k < nd; ++k) reinterpret_cast<uint32_t*>(st.data() + o_dels)[k] = uint32_t(shift.dels[k]);
  for (uint64_t k = 0; k < na; ++k) reinterpret_cast<uint32_t*>(st.data() + o_adds)[k] = uint32_t(shift.addpos[k]);
  for (size_t k = 0; k < orops.size(); ++k) {
    const uint64_t w[2] = {orops[k].first, orops[k].second};
    std::memcpy(st.data() + o_ors + 16 * k, w, 16);
  }
  PoolBuf dbuf(ctx->pool, total);
  if (!dbuf.p) return set_err(ctx, EMQX_GM_ENOMEM, "index_update: staging buffer");
  hipStream_t s = ctx->stream;
  uint8_t* D = static_cast<uint8_t*>(dst);
  const uint8_t* S = dbuf.as<uint8_t>();
  uint32_t* const RM = reinterpret_cast<uint32_t*>(dbuf.as<uint8_t>() + o_rmap);
  auto shift_table = [&]() -> int {
    if (n_map) {
      hipLaunchKernelGGL(k_shift_table, dim3(uint32_t((n_map + 255) / 256)), dim3(256), 0, s, RM, shift.nb,
                         reinterpret_cast<const uint32_t*>(S + o_dels), uint32_t(nd),
                         reinterpret_cast<const uint32_t*>(S + o_adds), uint32_t(na));
      GM_HIP(ctx, hipGetLastError());
    }
    return 0;
  };
  const uint64_t g = std::min<uint64_t>(8192, (std::max(n_hot, n_nodes) + 255) / 256);
  if (fused) {
    GM_HIP(ctx, hipMemcpyAsync(dbuf.p, st.data(), up, hipMemcpyHostToDevice, s));
    if (const int rc = shift_table()) return rc;
    // the bytes around the two tables as they are, the tables renumbered on the way
    const uint64_t a0 = std::min(o_hot, o_nodes), a1 = std::min(hot_end, nodes_end);
    const uint64_t b0 = std::max(o_hot, o_nodes), b1 = std::max(hot_end, nodes_end);
    const uint64_t gaps[3][2] = {{0, a0}, {a1, b0}, {b1, bytes}};
    for (const auto& gp : gaps)
      if (gp[1] > gp[0])
        GM_HIP(ctx, hipMemcpyAsync(D + gp[0], static_cast<const uint8_t*>(src) + gp[0], gp[1] - gp[0],
                                   hipMemcpyDeviceToDevice, s));
    const uint8_t* SRC = static_cast<const uint8_t*>(src);
    hipLaunchKernelGGL(k_renumber_copy, dim3(uint32_t(g ? g : 1)), dim3(256), 0, s,
                       reinterpret_cast<const HotSlot*>(SRC + o_hot), reinterpret_cast<HotSlot*>(D + o_hot), n_hot,
                       reinterpret_cast<const Node*>(SRC + o_nodes), reinterpret_cast<Node*>(D + o_nodes), n_nodes, RM);
    GM_HIP(ctx, hipGetLastError());
  } else {
    GM_HIP(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s));
    GM_HIP(ctx, hipMemcpyAsync(dbuf.p, st.data(), up, hipMemcpyHostToDevice, s));
  }
  if (n_pieces) {
    hipLaunchKernelGGL(k_patch_scatter, dim3(uint32_t(n_pieces)), dim3(256), 0, s, D,
                       reinterpret_cast<const uint64_t*>(S), S + o_pay);
    GM_HIP(ctx, hipGetLastError());
  }
  if (!orops.empty()) {
    hipLaunchKernelGGL(k_patch_or, dim3(uint32_t((orops.size() + 255) / 256)), dim3(256), 0, s,
                       reinterpret_cast<uint32_t*>(D), reinterpret_cast<const uint64_t*>(S + o_ors),
                       uint64_t(orops.size()));
    GM_HIP(ctx, hipGetLastError());
  }
  if (!fused) {
    if (const int rc = shift_table()) return rc;
    hipLaunchKernelGGL(k_renumber, dim3(uint32_t(g ? g : 1)), dim3(256), 0, s, reinterpret_cast<HotSlot*>(D + o_hot),
                       n_hot, reinterpret_cast<Node*>(D + o_nodes), n_nodes, RM);
    GM_HIP(ctx, hipGetLastError());
  }
  GM_HIP(ctx, hipStreamSynchronize(s));  // the staging buffers go back to the pool / the host
  return EMQX_GM_OK;
}

// ---- the new subscriber CSR of emqx_gm_index_update_subs (gm_subs.cpp) ----
// Output element p of the new CSR belongs to filter f (the last segment whose
// start <= p); its source is f's edited list from the host (f in aff_ids) or
// element p - nsoff[f] of the previous list of f's old id inv[f].  Every
// workgroup owns per_block consecutive outputs, as k_fanout_copy does.
__device__ __forceinline__ uint64_t seg_of(const uint64_t* __restrict__ s, uint64_t a, uint64_t b, uint64_t p) {
  // s[a] <= p < s[b]: the last segment of [a, b) starting at or before p
  while (b - a > 1) {
    const uint64_t m = (a + b) >> 1;
    if (s[m] <= p) a = m;
    else b = m;
  }
  return a;
}
__global__ __launch_bounds__(256) void k_subs_copy(const uint64_t* __restrict__ nsoff, uint64_t nf,
                                                   const uint32_t* __restrict__ inv, const uint64_t* __restrict__ osoff,
                                                   const uint32_t* __restrict__ oids, const uint32_t* __restrict__ aff_ids,
                                                   uint64_t n_aff, const uint64_t* __restrict__ aff_off,
                                                   const uint32_t* __restrict__ aff_buf, uint64_t total,
                                                   uint64_t per_block, uint32_t* __restrict__ out) {
  const uint64_t lo = uint64_t(blockIdx.x) * per_block;
  if (lo >= total) return;
  const uint64_t hi = min(total, lo + per_block);
  __shared__ uint64_t s_seg[2];
  if (threadIdx.x < 2) s_seg[threadIdx.x] = seg_of(nsoff, 0, nf, threadIdx.x == 0 ? lo : hi - 1);
  __syncthreads();
  const uint64_t s0 = s_seg[0], s1 = s_seg[1] + 1;
  for (uint64_t p = lo + threadIdx.x; p < hi; p += 256) {
    const uint64_t f = seg_of(nsoff, s0, s1, p);
    const uint64_t q = p - nsoff[f];
    uint64_t a = 0, b = n_aff;  // is f a touched filter?
    while (a < b) {
      const uint64_t m = (a + b) >> 1;
      if (aff_ids[m] < f) a = m + 1;
      else b = m;
    }
    out[p] = (a < n_aff && aff_ids[a] == f) ? aff_buf[aff_off[a] + q] : oids[osoff[inv ? inv[f] : f] + q];
  }
}

// A subscriber-only batch (ids unchanged): new sub_off[i] = old sub_off[i] +
// the count changes of the touched filters below i (tid ascending, tcum their
// running sum) -- the host uploads only the touched ids
__global__ __launch_bounds__(256) void k_soff_shift(const uint64_t* __restrict__ osoff, uint64_t n1,
                                                    const uint32_t* __restrict__ tid, const int64_t* __restrict__ tcum,
                                                    uint64_t nt, uint64_t* __restrict__ nsoff) {
  for (uint64_t i = uint64_t(blockIdx.x) * 256u + threadIdx.x; i < n1; i += uint64_t(gridDim.x) * 256u) {
    uint64_t a = 0, b = nt;  // touched ids below i
    while (a < b) {
      const uint64_t m = (a + b) >> 1;
      if (tid[m] < i) a = m + 1;
      else b = m;
    }
    nsoff[i] = uint64_t(int64_t(osoff[i]) + (a ? tcum[a - 1] : 0));
  }
}

__global__ __launch_bounds__(256) void k_gather_segments(const uint32_t* __restrict__ src,
                                                         const uint64_t* __restrict__ src_off,
                                                         const uint64_t* __restrict__ dst_off, uint64_t m,
                                                         uint64_t total, uint64_t per_block,
                                                         uint32_t* __restrict__ out) {
  const uint64_t lo = uint64_t(blockIdx.x) * per_block;
  if (lo >= total) return;
  const uint64_t hi = min(total, lo + per_block);
  __shared__ uint64_t s_seg[2];
  if (threadIdx.x < 2) s_seg[threadIdx.x] = seg_of(dst_off, 0, m, threadIdx.x == 0 ? lo : hi - 1);
  __syncthreads();
  const uint64_t s0 = s_seg[0], s1 = s_seg[1] + 1;
  for (uint64_t p = lo + threadIdx.x; p < hi; p += 256) {
    const uint64_t j = seg_of(dst_off, s0, s1, p);
    out[p] = src[src_off[j] + (p - dst_off[j])];
  }
}

int gather_segments(emqx_gm_ctx* ctx, const uint32_t* src, const std::vector<uint64_t>& src_off,
                    const std::vector<uint64_t>& dst_off, uint32_t* out) {
  const uint64_t m = src_off.size(), total = dst_off.back();
  if (!total) return EMQX_GM_OK;
  hipStream_t st = ctx->stream;
  PoolBuf so(ctx->pool, m * 8 + 8), dof(ctx->pool, (m + 1) * 8), buf(ctx->pool, total * 4 + 16);
  if (!so.p || !dof.p || !buf.p) return set_err(ctx, EMQX_GM_ENOMEM, "gather_segments: workspace");
  GM_HIP(ctx, hipMemcpyAsync(so.p, src_off.data(), m * 8, hipMemcpyHostToDevice, st));
  GM_HIP(ctx, hipMemcpyAsync(dof.p, dst_off.data(), (m + 1) * 8, hipMemcpyHostToDevice, st));
  const uint64_t per = fan_per_block(total);
  hipLaunchKernelGGL(k_gather_segments, dim3((total + per - 1) / per), dim3(256), 0, st, src, so.as<uint64_t>(),
                     dof.as<uint64_t>(), m, total, per, buf.as<uint32_t>());
  GM_HIP(ctx, hipGetLastError());
  GM_HIP(ctx, hipMemcpyAsync(out, buf.p, total * 4, hipMemcpyDeviceToHost, st));
  GM_HIP(ctx, hipStreamSynchronize(st));
  return EMQX_GM_OK;
}

// The new subscriber CSR of a subscriber-only emqx_gm_index_update_subs batch
// (gm_subs.cpp; filter ids unchanged): O(delta) host work -- the touched
// filters' ids, count changes and lists go up -- and the device derives the
// offsets (k_soff_shift) and copies every other filter's segment from prev's
// CSR (k_subs_copy with the identity id map).
int shift_subs_device(emqx_gm_ctx* ctx, const emqx_gm_index* prev, emqx_gm_index* idx,
                      const std::vector<uint32_t>& aff_ids, const std::vector<uint64_t>& aff_off,
                      const std::vector<uint32_t>& aff_buf) {
  const uint64_t nf = prev->info.n_filters, na = aff_ids.size();
  std::vector<int64_t> tcum(na + 1, 0);
  int64_t cum = 0;
  for (uint64_t k = 0; k < na; ++k) {
    if (aff_ids[k] >= nf || (k && aff_ids[k] <= aff_ids[k - 1]))
      return set_err(ctx, EMQX_GM_EINVAL, "index_update_subs: touched ids");
    cum += int64_t(aff_off[k + 1] - aff_off[k]) - int64_t(prev->subs.count(aff_ids[k]));
    tcum[k] = cum;
  }
  const uint64_t total = uint64_t(int64_t(prev->subs.total()) + cum);
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  const size_t o_ids = al((nf + 1) * 8);
  GM_HIP(ctx, hipMalloc(&idx->dev_subs, o_ids + total * 4 + 16));
  idx->subs_bytes = o_ids + total * 4 + 16;
  uint8_t* D = static_cast<uint8_t*>(idx->dev_subs);
  hipStream_t st = ctx->stream;
  // staging: tid | tcum | aff_off | aff_buf
  const size_t o_cum = al(na * 4 + 4), o_aoff = o_cum + al((na + 1) * 8), o_abuf = o_aoff + al(aff_off.size() * 8),
               n_st = o_abuf + aff_buf.size() * 4 + 4;
  std::vector<uint8_t> h(n_st, 0);
  if (na) std::memcpy(h.data(), aff_ids.data(), na * 4);
  std::memcpy(h.data() + o_cum, tcum.data(), (na + 1) * 8);
  std::memcpy(h.data() + o_aoff, aff_off.data(), aff_off.size() * 8);
  if (!aff_buf.empty()) std::memcpy(h.data() + o_abuf, aff_buf.data(), aff_buf.size() * 4);
  PoolBuf sbuf(ctx->pool, n_st);
  if (!sbuf.p) return set_err(ctx, EMQX_GM_ENOMEM, "index_update_subs: staging");
  GM_HIP(ctx, hipMemcpyAsync(sbuf.p, h.data(), n_st, hipMemcpyHostToDevice, st));
  const uint8_t* S = sbuf.as<uint8_t>();
  const uint64_t g = std::min<uint64_t>(4096, (nf + 1 + 255) / 256);
  hipLaunchKernelGGL(k_soff_shift, dim3(g), dim3(256), 0, st, prev->view.sub_off, nf + 1,
                     reinterpret_cast<const uint32_t*>(S), reinterpret_cast<const int64_t*>(S + o_cum), na,
                     reinterpret_cast<uint64_t*>(D));
  GM_HIP(ctx, hipGetLastError());
  if (total) {
    const uint64_t per = fan_per_block(total);
    hipLaunchKernelGGL(k_subs_copy, dim3((total + per - 1) / per), dim3(256), 0, st,
                       reinterpret_cast<const uint64_t*>(D), nf, static_cast<const uint32_t*>(nullptr),
                       prev->view.sub_off, prev->view.sub_ids, reinterpret_cast<const uint32_t*>(S), na,
                       reinterpret_cast<const uint64_t*>(S + o_aoff), reinterpret_cast<const uint32_t*>(S + o_abuf),
                       total, per, reinterpret_cast<uint32_t*>(D + o_ids));
    GM_HIP(ctx, hipGetLastError());
  }
  GM_HIP(ctx, hipStreamSynchronize(st));  // the staging goes back to the pool / the host
  idx->view.sub_off = reinterpret_cast<const uint64_t*>(D);
  idx->view.sub_ids = reinterpret_cast<const uint32_t*>(D + o_ids);
  idx->info.device_bytes += o_ids + total * 4 + 16;
  return EMQX_GM_OK;
}

int rebuild_subs_device(emqx_gm_ctx* ctx, const emqx_gm_index* prev, emqx_gm_index* idx,
                        const std::vector<uint64_t>& new_soff, const std::vector<uint32_t>& inv,
                        const std::vector<uint32_t>& aff_ids, const std::vector<uint64_t>& aff_off,
                        const std::vector<uint32_t>& aff_buf) {
  const uint64_t nf = new_soff.size() - 1, total = new_soff.back();
  for (uint64_t f = 0; f < nf; ++f)  // host-side check of what the kernel will index
    if (inv[f] == NONE && !std::binary_search(aff_ids.begin(), aff_ids.end(), uint32_t(f)) &&
        new_soff[f + 1] != new_soff[f])
      return set_err(ctx, EMQX_GM_EINVAL, "index_update_subs: a new filter without its list");
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  const size_t o_ids = al((nf + 1) * 8);
  GM_HIP(ctx, hipMalloc(&idx->dev_subs, o_ids + total * 4 + 16));
  idx->subs_bytes = o_ids + total * 4 + 16;
  uint8_t* D = static_cast<uint8_t*>(idx->dev_subs);
  hipStream_t st = ctx->stream;
  GM_HIP(ctx, hipMemcpyAsync(D, new_soff.data(), (nf + 1) * 8, hipMemcpyHostToDevice, st));
  // staging: inv | aff_ids | aff_off | aff_buf
  const size_t o_aid = al(nf * 4 + 4), o_aoff = o_aid + al(aff_ids.size() * 4 + 4),
               o_abuf = o_aoff + al(aff_off.size() * 8), n_st = o_abuf + aff_buf.size() * 4 + 4;
  std::vector<uint8_t> h(n_st, 0);
  std::memcpy(h.data(), inv.data(), nf * 4);
  if (!aff_ids.empty()) std::memcpy(h.data() + o_aid, aff_ids.data(), aff_ids.size() * 4);
  std::memcpy(h.data() + o_aoff, aff_off.data(), aff_off.size() * 8);
  if (!aff_buf.empty()) std::memcpy(h.data() + o_abuf, aff_buf.data(), aff_buf.size() * 4);
  PoolBuf sbuf(ctx->pool, n_st);
  if (!sbuf.p) return set_err(ctx, EMQX_GM_ENOMEM, "index_update_subs: staging");
  GM_HIP(ctx, hipMemcpyAsync(sbuf.p, h.data(), n_st, hipMemcpyHostToDevice, st));
  if (total) {
    const uint8_t* S = sbuf.as<uint8_t>();
    const uint64_t per = fan_per_block(total);
    hipLaunchKernelGGL(k_subs_copy, dim3((total + per - 1) / per), dim3(256), 0, st,
                       reinterpret_cast<const uint64_t*>(D), nf, reinterpret_cast<const uint32_t*>(S),
                       prev->view.sub_off, prev->view.sub_ids, reinterpret_cast<const uint32_t*>(S + o_aid),
                       uint64_t(aff_ids.size()), reinterpret_cast<const uint64_t*>(S + o_aoff),
                       reinterpret_cast<const uint32_t*>(S + o_abuf), total, per,
                       reinterpret_cast<uint32_t*>(D + o_ids));
    GM_HIP(ctx, hipGetLastError());
  }
  GM_HIP(ctx, hipStreamSynchronize(st));  // the staging goes back to the pool / the host
  idx->view.sub_off = reinterpret_cast<const uint64_t*>(D);
  idx->view.sub_ids = reinterpret_cast<const uint32_t*>(D + o_ids);
  idx->info.device_bytes += o_ids + total * 4 + 16;
  return EMQX_GM_OK;
}


// ---------------------------------------------------------------------------
// host orchestration
// ---------------------------------------------------------------------------
namespace {

int finish_csr(emqx_gm_ctx* ctx, uint64_t n, uint64_t nnz, PoolBuf& row_off, PoolBuf& ids, bool device_out,
               emqx_gm_csr* out) {
  out->n_rows = n;
  out->nnz = nnz;
  out->priv = ctx;  // the owning context (emqx_gm_csr_free checks it)
  if (device_out) {
    out->row_off = static_cast<uint64_t*>(row_off.release_ownership());
    out->ids = static_cast<uint32_t*>(ids.release_ownership());
    out->on_device = 1;
    return 0;
  }
  uint64_t* h_off = static_cast<uint64_t*>(ctx->hpool->alloc((n + 1) * 8));
  uint32_t* h_ids = static_cast<uint32_t*>(ctx->hpool->alloc(nnz * 4 + 4));
  if (!h_off || !h_ids) {
    ctx->hpool->release(h_off);
    ctx->hpool->release(h_ids);
    return set_err(ctx, EMQX_GM_ENOMEM, "csr: host allocation");
  }
  GM_HIP(ctx, hipMemcpyAsync(h_off, row_off.p, (n + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
  if (nnz) GM_HIP(ctx, hipMemcpyAsync(h_ids, ids.p, nnz * 4, hipMemcpyDeviceToHost, ctx->stream));
  GM_HIP(ctx, hipStreamSynchronize(ctx->stream));
  out->row_off = h_off;
  out->ids = h_ids;
  out->on_device = 0;
  return 0;
}

float ev_ms(hipEvent_t a, hipEvent_t b) {
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, a, b) != hipSuccess) {
    (void)hipGetLastError();  // (an event not recorded for this call: no timing, and no sticky error)
    return 0.f;
  }
  return ms;
}

// Main-pass kernel selection.  GM_MATCH_MAIN (A/B knob, read per call so tests
// cover every kind): fused (k_match_fused: tokenizer into registers + the
// compacted wave walk in one kernel, default; C2 10.2 ms vs 12.0 for the
// split coop pair), coop (k_tokenize + k_walk_coop, the wave's frontier as
// one compacted list), splitw8 (k_tokenize + k_walk, lane-private register
// frontier, 8-wave register budget), split (budget left to the compiler),
// split2 (k_walk expanding frontier entries in pairs).
enum MainKind { MAIN_SPLIT, MAIN_SPLITW8, MAIN_SPLIT2, MAIN_COOP, MAIN_FUSED };
MainKind main_kind() {
  const char* e = knob("GM_MATCH_MAIN");
  static const struct { const char* name; MainKind kind; } names[] = {
      {"split", MAIN_SPLIT}, {"splitw8", MAIN_SPLITW8}, {"split2", MAIN_SPLIT2}, {"coop", MAIN_COOP},
      {"fused", MAIN_FUSED}};
  if (e)
    for (const auto& nk : names)
      if (!strcmp(e, nk.name)) return nk.kind;
  return MAIN_FUSED;
}

constexpr int LISTED_FC = 16;  // frontier capacity of the listed pass

// Tokenizer group size.  GM_TOK_GROUP (A/B knob, read once): 1 = one-ahead
// dictionary prefetch, 3 (default) / 5 = words scanned and their dictionary
// slots loaded G at a time.  Measured at C2: 3.54 / 3.42 / 3.90 ms (G = 5
// needs 80 VGPRs, 6 waves per SIMD).  Read per call, so tests cover all three.
int tok_group() {
  const char* e = knob("GM_TOK_GROUP");
  const int v = e ? atoi(e) : 3;
  return (v == 1 || v == 5) ? v : 3;
}

// Non-temporal stream accesses.  GM_NT (A/B knob, read per call): the topic
// text, word ids, headers, staging and counts as nt loads / stores (default;
// C2: 12.15 -> 12.03 ms for the split pair, 10.45 -> 10.24 ms fused), 0 = plain.
bool nt_streams() {
  const char* e = knob("GM_NT");
  return !e || atoi(e) != 0;
}

// Compact staging of the fused main pass (k_match_fused<CMP> + k_assemble_c).
// GM_STAGE_COMPACT (A/B knob, read per call so tests cover both; default on):
// used when the index's filter ids fit CMP_SHIFT bits.
// The assembly stream (MatchCall::submit) for device-buffer calls of at least
// this many topics; GM_ASM_STREAM (A/B knob, read per call): 0 = never, N =
// from N topics.
// (Off by default: at C2 the overlapped assembly slowed the walk by what it
// hid, 9.16 vs 9.16 ms per step, profiles/r04_ab/asm_stream_c2.txt.)
// GM_SCAN_SUMS (A/B knob, read per call; default on): a split tile scan of at
// most 64 blocks (calls up to ~4M topics: C1) ends after its first launch and
// k_assemble_c sums the block prefixes itself.
bool sums_mode() {
  const char* e = knob("GM_SCAN_SUMS");
  return !e || atoi(e) != 0;
}

uint64_t asm_stream_min() {
  const char* e = knob("GM_ASM_STREAM");
  return e ? strtoull(e, nullptr, 10) : 0;
}

bool stage_compact() {
  const char* e = knob("GM_STAGE_COMPACT");
  return !e || atoi(e) != 0;
}
struct CmpBufs {
  uint8_t* cnt8;     // per topic: its row length, 0xFF = see cnt (listed / slow rows)
  uint32_t* tlen;    // per tile: entries in its list
  uint32_t* lstage;  // listed rows, FAST_MC ids each
  uint32_t* lcnt;    // listed row lengths
  uint64_t lcap;     // listed rows available
};
void launch_assemble(hipStream_t st, uint64_t nblk, const CmpBufs* cb, const uint32_t* cnt, uint64_t n,
                     const uint64_t* toff, const uint32_t* stage, uint64_t* row_off, uint32_t* ids,
                     const uint32_t* gmap, uint64_t cap, const uint64_t* blk = nullptr, uint32_t* rb_dst = nullptr,
                     const uint32_t* rb_ctr = nullptr, hipEvent_t done = nullptr, uint32_t* zero16 = nullptr,
                     uint32_t blk_sums = 0) {
  // blk (compact staging only): toff is a split scan's block-local part, blk its block offsets
  // (blk_sums != 0: blk holds that many block SUMS, and the kernel writes the grand total at toff[n_tiles])
  // rb_dst (compact staging only): the read-back words (the total behind toff, the
  // counters at rb_ctr) written by the kernel, `done` its stop event
  // zero16 (compact staging only): a 64-B counter block the kernel zeroes
  const uint32_t* rb_total = reinterpret_cast<const uint32_t*>(toff + (n + 63) / 64);
  if (cb)
    hipExtLaunchKernelGGL(k_assemble_c, dim3((nblk + ASM_TPW - 1) / ASM_TPW), dim3(256), 0, st, nullptr, done, 0,
                          cb->cnt8, cnt, n, toff, stage, cb->tlen, cb->lstage, cb->lcnt, row_off, ids, gmap, cap, blk,
                          rb_total, rb_ctr, rb_dst, zero16, blk_sums,
                          const_cast<uint64_t*>(toff) + (n + 63) / 64);
  else
    hipLaunchKernelGGL(k_assemble, dim3(nblk), dim3(256), 0, st, cnt, n, toff, stage, row_off, ids, gmap, cap);
}

void launch_tokenize(hipStream_t st, uint64_t nblk, const uint8_t* tb, const uint64_t* to, uint64_t n,
                     const IndexView& v, uint32_t* hdr, uint32_t* wids, uint64_t t_base) {
  const bool nt = nt_streams();
#define GM_TOK(G)                                                                                          \
  do {                                                                                                     \
    if (nt) hipLaunchKernelGGL((k_tokenize<G, true>), dim3(nblk), dim3(256), 0, st, tb, to, n, v, hdr, wids, t_base); \
    else hipLaunchKernelGGL((k_tokenize<G, false>), dim3(nblk), dim3(256), 0, st, tb, to, n, v, hdr, wids, t_base); \
  } while (0)
  switch (tok_group()) {
    case 1: GM_TOK(1); break;
    case 5: GM_TOK(5); break;
    default: GM_TOK(3);
  }
#undef GM_TOK
}

// Tokenize / walk overlap.  GM_OVERLAP = K (A/B knob, read per call; 1 = off):
// the batch is cut into K block ranges; chunk i is tokenized on a second
// stream while the walk of chunk i-1 runs on the context's stream (the
// tokenizer is VALU bound, the walk waits on the fabric, so the two can share
// the CUs).  Kernels index by t_base + their own grid, so the layouts are
// those of one launch.
int overlap_chunks() {
  const char* e = knob("GM_OVERLAP");
  const int v = e ? atoi(e) : 1;
  return v < 1 ? 1 : (v > 8 ? 8 : v);
}

// Main pass, then the listed pass over its overflow queue (count read on the
// device).  `after_main` is recorded between the two: the roofline times the
// main pass alone, the same kernel rocprofv3 reports.
template <bool EXACT>
void launch_listed(hipStream_t st, const IndexView& v, const uint8_t* tb, const uint64_t* to, uint64_t n, uint32_t* cnt,
                   uint32_t* stage, uint32_t* list1, uint32_t* n1, uint32_t* list2, uint32_t* n2,
                   unsigned long long* probe_ctr, unsigned long long* wild_ctr, uint64_t* tsum, const CmpBufs* cb);
template <bool EXACT>
void launch_match(emqx_gm_ctx* ctx, const IndexView& v, const uint8_t* tb, const uint64_t* to, uint64_t n,
                  uint32_t* cnt, uint32_t* stage, uint32_t* list1, uint32_t* n1, uint32_t* list2, uint32_t* n2,
                  unsigned long long* probe_ctr, unsigned long long* wild_ctr, uint32_t* hdr, uint32_t* wids,
                  unsigned long long* probe_tile, uint64_t* tsum, hipEvent_t before_main, hipEvent_t after_main,
                  const CmpBufs* cb, bool* listed_deferred) {
  hipStream_t st = ctx->stream;
  const uint64_t nblk = (n + 255) / 256;
  *listed_deferred = false;
#define GM_LAUNCH_WALK(W, P, sw, g, base)                                                                        \
  hipLaunchKernelGGL((k_walk<EXACT, W, P>), dim3(g), dim3(256), 0, sw, tb, to, n, v, hdr, wids, cnt, stage, list1, n1, \
                     probe_tile, wild_ctr, tsum, base)
#define GM_WALK(sw, g, base)                                  \
  do {                                                        \
    switch (main_kind()) {                                    \
      case MAIN_SPLIT: GM_LAUNCH_WALK(1, false, sw, g, base); break;  \
      case MAIN_SPLIT2: GM_LAUNCH_WALK(1, true, sw, g, base); break;  \
      case MAIN_COOP:                                         \
        if (nt_streams())                                     \
          hipLaunchKernelGGL((k_walk_coop<EXACT, true>), dim3(g), dim3(256), 0, sw, tb, to, n, v, hdr, wids, cnt, \
                             stage, list1, n1, probe_tile, wild_ctr, tsum, base);                                 \
        else                                                  \
          hipLaunchKernelGGL((k_walk_coop<EXACT, false>), dim3(g), dim3(256), 0, sw, tb, to, n, v, hdr, wids, cnt, \
                             stage, list1, n1, probe_tile, wild_ctr, tsum, base);                                  \
        break;                                                \
      default: GM_LAUNCH_WALK(8, false, sw, g, base);         \
    }                                                         \
  } while (0)
  int K = overlap_chunks();
  if (K > 1 && nblk < uint64_t(K) * 1024) K = 1;  // small batches: one launch each
  if (K > 1 && !ctx->stream2 && hipStreamCreateWithFlags(&ctx->stream2, hipStreamNonBlocking) != hipSuccess) {
    ctx->stream2 = nullptr;
    K = 1;
  }
  for (int i = 0; K > 1 && i <= K; ++i)
    if (!ctx->ov_ev[i] && hipEventCreateWithFlags(&ctx->ov_ev[i], hipEventDisableTiming) != hipSuccess) K = 1;
#ifdef GM_PHASE_STATS
  uint32_t* phase_rec = nullptr;
  if (main_kind() == MAIN_FUSED && n && hipStreamSynchronize(st) == hipSuccess &&
      hipMalloc(&phase_rec, (n + 63) / 64 * 128) == hipSuccess) {
    (void)hipMemset(phase_rec, 0, (n + 63) / 64 * 128);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_phase_rec), &phase_rec, sizeof phase_rec);
  }
#endif
  if (main_kind() == MAIN_FUSED) {
    const char* pe = knob("GM_FUSED_PRIO");  // A/B knob (read per call): 0 = every phase at priority 0
    const bool tp = !pe || atoi(pe) != 0;
    uint32_t* const tl = cb ? cb->tlen : nullptr;
    uint8_t* const c8 = cb ? cb->cnt8 : nullptr;
    // the kernel's own start / stop timestamps (hipExtLaunchKernel) instead of
    // two event records around it: each record is a barrier packet that costs
    // the stream ~5.5 us of idle GPU (C1 per-call trace, profiles/r03_c1_trace.txt)
#define GM_FUSED(NT, P, C)                                                                                          \
  hipExtLaunchKernelGGL((k_match_fused<3, EXACT, NT, P, C>), dim3(nblk), dim3(256), 0, st, kt ? before_main : nullptr,   \
                        kt ? after_main : nullptr, 0,                                                                     \
                        tb, to, n, v, cnt, stage, list1, n1, probe_tile, wild_ctr, tsum, tl, c8)
    const bool kt = before_main != nullptr;  // (an untimed call: EMQX_GM_NO_TIMING)
    if (cb) {
      if (nt_streams() && tp) GM_FUSED(true, true, true);
      else if (nt_streams()) GM_FUSED(true, false, true);
      else if (tp) GM_FUSED(false, true, true);
      else GM_FUSED(false, false, true);
    } else if (nt_streams()) {
      if (tp) GM_FUSED(true, true, false);
      else GM_FUSED(true, false, false);
    } else {
      if (tp) GM_FUSED(false, true, false);
      else GM_FUSED(false, false, false);
    }
#undef GM_FUSED
  } else if (K == 1) {
    hipEventRecord(before_main, st);
    launch_tokenize(st, nblk, tb, to, n, v, hdr, wids, 0);
    GM_WALK(st, nblk, 0ull);
  } else {
    hipEventRecord(before_main, st);
    hipStream_t st2 = ctx->stream2;
    hipEventRecord(ctx->ov_ev[0], st);  // the tokenizer stream starts after the work queued so far
    hipStreamWaitEvent(st2, ctx->ov_ev[0], 0);
    const uint64_t cb = (nblk + K - 1) / K;
    for (int i = 0; i < K; ++i) {
      const uint64_t b0 = uint64_t(i) * cb;
      if (b0 >= nblk) break;
      const uint64_t nb = std::min<uint64_t>(cb, nblk - b0);
      launch_tokenize(st2, nb, tb, to, n, v, hdr, wids, b0 * 256);
      hipEventRecord(ctx->ov_ev[i + 1], st2);
      hipStreamWaitEvent(st, ctx->ov_ev[i + 1], 0);
      GM_WALK(st, nb, b0 * 256);
    }
  }
#undef GM_WALK
#undef GM_LAUNCH_WALK
#ifdef GM_PROBE_STATS
  {
    unsigned long long h[8][8], z[8][8] = {};
    if (hipStreamSynchronize(st) == hipSuccess && hipMemcpyFromSymbol(h, HIP_SYMBOL(g_pstats), sizeof h) == hipSuccess) {
      (void)hipMemcpyToSymbol(HIP_SYMBOL(g_pstats), z, sizeof z);
      for (int l = 0; l < 8; ++l)
        if (h[l][0])
          fprintf(stderr, "[probe_stats] level %d entries %llu cand %llu sig %llu efilt %llu found %llu plus_slot %llu "
                  "plus_found %llu plus_inline %llu\n", l, h[l][0], h[l][1], h[l][2], h[l][3], h[l][4], h[l][5], h[l][6],
                  h[l][7]);
    }
  }
#endif
#ifdef GM_PHASE_STATS
  if (phase_rec) {
    const uint64_t nt = (n + 63) / 64;
    std::vector<uint32_t> h(nt * 32);
    uint32_t* null_rec = nullptr;
    if (hipStreamSynchronize(st) == hipSuccess &&
        hipMemcpy(h.data(), phase_rec, h.size() * 4, hipMemcpyDeviceToHost) == hipSuccess) {
      double sum[32] = {0}, rounds[8] = {0};
      for (uint64_t i = 0; i < nt; ++i) {
        const uint32_t* r = &h[i * 32];
        for (int k = 0; k < 32; ++k) sum[k] += r[k];
        for (int l = 0; l < 8; ++l) rounds[l] += (r[l < 4 ? 11 : 12] >> (8 * (l & 3))) & 0xFFu;
      }
      const double w = double(nt);
      fprintf(stderr, "[phase_stats] waves %llu; ticks/wave: stage %.0f tok %.0f", (unsigned long long)nt, sum[0] / w,
              sum[1] / w);
      for (int l = 0; l < 8; ++l)
        if (rounds[l] > 0)
          fprintf(stderr, " L%d %.0f (%.2f rounds: to data %.0f, rest %.0f)", l, sum[2 + l] / w, rounds[l] / w,
                  sum[16 + l] / w, sum[24 + l] / w);
      fprintf(stderr, " epi %.0f; chain-tail rounds/wave %.2f\n", sum[10] / w, sum[13] / w);
    }
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_phase_rec), &null_rec, sizeof null_rec);
    (void)hipFree(phase_rec);
  }
#endif
  if (main_kind() != MAIN_FUSED) hipEventRecord(after_main, st);
  (void)probe_tile;  // summed into the probe counter by the tile scan (run_match)
  // The fused main pass with compact staging leaves the listed pass to the
  // host's read-back (MatchCall::finish): it launches it only when the main
  // pass queued rows, instead of an (almost always idle) launch per call.
  // GM_LISTED_DEFER=0: launch it here (A/B knob).
  if (cb && main_kind() == MAIN_FUSED) {
    const char* le = knob("GM_LISTED_DEFER");
    if (!le || atoi(le) != 0) {
      *listed_deferred = true;
      return;
    }
  }
  launch_listed<EXACT>(st, v, tb, to, n, cnt, stage, list1, n1, list2, n2, probe_ctr, wild_ctr, tsum, cb);
}

// The listed pass over the main pass's overflow queue (list1, its count n1 on the device)
template <bool EXACT>
void launch_listed(hipStream_t st, const IndexView& v, const uint8_t* tb, const uint64_t* to, uint64_t n, uint32_t* cnt,
                   uint32_t* stage, uint32_t* list1, uint32_t* n1, uint32_t* list2, uint32_t* n2,
                   unsigned long long* probe_ctr, unsigned long long* wild_ctr, uint64_t* tsum, const CmpBufs* cb) {
  const uint64_t nblk = (n + 255) / 256;
  const uint64_t lblk = std::min<uint64_t>(nblk, 512);
  if (cb)
    hipLaunchKernelGGL((k_match_lds<EXACT, LISTED_FC, true, true>), dim3(lblk), dim3(256), 0, st, tb, to, n, v, cnt,
                       stage, list1, n1, list2, n2, probe_ctr, wild_ctr, tsum, cb->lstage, cb->lcnt, cb->lcap);
  else
    hipLaunchKernelGGL((k_match_lds<EXACT, LISTED_FC, true>), dim3(lblk), dim3(256), 0, st, tb, to, n, v, cnt, stage,
                       list1, n1, list2, n2, probe_ctr, wild_ctr, tsum);
}

}  // namespace

// One match call in two phases (emqx_gm_match = submit then finish at once;
// emqx_gm_match_submit / emqx_gm_match_wait split them, so the next batch's
// launches queue behind this one's before the host has read its total):
//   submit(): every kernel of the call, the speculative assembly and the
//     40-B read-back of the match total + pass counters into the call's own
//     pinned words, then an event -- no host wait;
//   finish(): waits on that event (without the context lock when it was
//     submitted alone), then either hands out the speculative rows or runs
//     the slow path / exact-size assembly and waits again.
// A call owns its workspaces (PoolBufs), events and pinned words until
// finish(), so several can be in flight on one context stream.
struct MatchCall {
  emqx_gm_ctx* ctx;
  const emqx_gm_index* idx = nullptr;
  uint64_t n = 0, n_tiles = 0, nblk = 0, cap_spec = 0;
  bool dev_io = false, exact = false, cmp = false, spec = false, split = false, submitted = false;
  uint32_t split_sums = 0;       // the split scan handed back block sums (k_assemble_c sums them)
  bool listed_deferred = false;  // the listed pass is left to finish() (launched only for queued rows)
  bool timed = true;             // the main pass's start / stop events (EMQX_GM_NO_TIMING: none)
  bool asm_overlap = false;      // scan + speculative assembly on ctx->stream_asm (wanted)
  bool on_asm = false;           // ... and queued there
  int ctr_slot = -1;             // the pass-counter block of the context's ring, or -1 (counters behind toff)
  const uint8_t* tb = nullptr;
  const uint64_t* to = nullptr;
  PoolBuf d_tb_own, d_to_own, row_off, cnt, stage, list1, list2, tsum, toff, probe_tile, hdr, wids;
  PoolBuf c_tlen, c_lstage, c_lcnt, c_cnt8, scan_blk, ids;
  CmpBufs cmpb{};
  uint64_t* toff_p = nullptr;
  uint8_t* ctrs_p = nullptr;
  uint64_t* pin = nullptr;  // [0] match total, [1..4] the pass counters
  hipEvent_t ev[3] = {};    // start, after the main pass, done
  emqx_gm_match_stats st_copy{};  // the stats finish() wrote for this call
  explicit MatchCall(emqx_gm_ctx* c) : ctx(c) {}
  MatchCall(const MatchCall&) = delete;
  MatchCall& operator=(const MatchCall&) = delete;
  ~MatchCall() {
    // (caller holds ctx->mu: the pools are not thread safe)
    if (submitted) {  // an abandoned call: its kernels may still use the buffers
      hipStreamSynchronize(ctx->stream);
      if (on_asm) hipStreamSynchronize(ctx->stream_asm);
    }
    for (hipEvent_t& e : ev)
      if (e) ctx->ev_free.push_back(e);
    if (pin) ctx->pin_free.push_back(pin);
    if (ctr_slot >= 0) ctx->ctr_state[ctr_slot] = 2;  // dirty: zeroed before its next use
    if (idx) const_cast<emqx_gm_index*>(idx)->refs.fetch_sub(1) == 1 ? free_index(const_cast<emqx_gm_index*>(idx))
                                                                     : void();
  }
  // the 40-B read-back (match total + pass counters) into the pinned words
  int readback(hipStream_t st) {
    if (ctr_slot < 0) {
      GM_HIP(ctx, hipMemcpyAsync(pin, toff_p + n_tiles, 40, hipMemcpyDeviceToHost, st));
    } else {
      GM_HIP(ctx, hipMemcpyAsync(pin, toff_p + n_tiles, 8, hipMemcpyDeviceToHost, st));
      GM_HIP(ctx, hipMemcpyAsync(pin + 1, ctrs_p, 32, hipMemcpyDeviceToHost, st));
    }
    return 0;
  }
  int take_event(hipEvent_t* e) {
    if (!ctx->ev_free.empty()) {
      *e = ctx->ev_free.back();
      ctx->ev_free.pop_back();
      return 0;
    }
    GM_HIP(ctx, hipEventCreate(e));
    return 0;
  }
  int submit(const emqx_gm_index* index, const uint8_t* tb_in, const uint64_t* to_in, uint64_t n_topics,
             uint32_t flags, MatchTail* tail);
  int finish(emqx_gm_csr* out, MatchTail* tail, bool locked);
};

int MatchCall::submit(const emqx_gm_index* index, const uint8_t* tb_in, const uint64_t* to_in, uint64_t n_topics,
                      uint32_t flags, MatchTail* tail) {
  dev_io = flags & EMQX_GM_DEVICE_IO;
  exact = flags & EMQX_GM_WITH_EXACT;
  timed = !(flags & EMQX_GM_NO_TIMING);
  n = n_topics;
  asm_overlap = dev_io && !tail && asm_stream_min() && n >= asm_stream_min();
  const_cast<emqx_gm_index*>(index)->refs.fetch_add(1);  // the snapshot stays alive until finish (RCU)
  idx = index;
  hipStream_t st = ctx->stream;
  for (hipEvent_t& e : ev)
    if (int rc = take_event(&e)) return rc;
  if (!ctx->pin_free.empty()) {
    pin = static_cast<uint64_t*>(ctx->pin_free.back());
    ctx->pin_free.pop_back();
  } else {
    void* p = nullptr;
    if (hipHostMalloc(&p, 64, hipHostMallocDefault) != hipSuccess)
      return set_err(ctx, EMQX_GM_ENOMEM, "match: pinned read-back words");
    ctx->pin_all.push_back(p);
    pin = static_cast<uint64_t*>(p);
  }

  // ---- inputs on the device
  tb = tb_in;
  to = to_in;
  if (!dev_io) {
    const uint64_t bytes = n ? to_in[n] : 0;
    for (uint64_t i = 0; i < n; ++i)
      if (to_in[i + 1] < to_in[i]) return set_err(ctx, EMQX_GM_EINVAL, "match: topic offsets not monotone");
    d_tb_own = PoolBuf(ctx->pool, bytes + 64);
    d_to_own = PoolBuf(ctx->pool, (n + 1) * 8);
    if (!d_tb_own.p || !d_to_own.p) return set_err(ctx, EMQX_GM_ENOMEM, "match: input workspace");
    submitted = true;
    if (bytes) GM_HIP(ctx, hipMemcpyAsync(d_tb_own.p, tb_in, bytes, hipMemcpyHostToDevice, st));
    GM_HIP(ctx, hipMemsetAsync(static_cast<uint8_t*>(d_tb_own.p) + bytes, 0, 64, st));
    GM_HIP(ctx, hipMemcpyAsync(d_to_own.p, to_in, (n + 1) * 8, hipMemcpyHostToDevice, st));
    tb = d_tb_own.as<uint8_t>();
    to = d_to_own.as<uint64_t>();
  }

  row_off = PoolBuf(ctx->pool, (n + 1) * 8);
  if (!row_off.p) return set_err(ctx, EMQX_GM_ENOMEM, "match: row_off");
  submitted = true;
  if (n == 0) {
    GM_HIP(ctx, hipMemsetAsync(row_off.p, 0, 8, st));
    ids = PoolBuf(ctx->pool, 16);
    GM_HIP(ctx, hipEventRecord(ev[0], st));
    GM_HIP(ctx, hipEventRecord(ev[1], st));
    GM_HIP(ctx, hipEventRecord(ev[2], st));
    pin[0] = pin[1] = pin[2] = pin[3] = pin[4] = 0;
    return 0;
  }

  n_tiles = (n + 63) / 64;
  nblk = (n + 255) / 256;
  cnt = PoolBuf(ctx->pool, n * 4 + 16);
  stage = PoolBuf(ctx->pool, n_tiles * 64ull * FAST_MC * 4);
  list1 = PoolBuf(ctx->pool, n * 4 + 16);
  list2 = PoolBuf(ctx->pool, n * 4 + 16);
  tsum = PoolBuf(ctx->pool, n_tiles * 8 + 8);
  // tile offsets [n_tiles + 1] and, right behind the total, the pass counters:
  // one read-back brings the match total and the counters together
  toff = PoolBuf(ctx->pool, (n_tiles + 1) * 8 + 128);
  if (!cnt.p || !stage.p || !list1.p || !list2.p || !tsum.p || !toff.p)
    return set_err(ctx, EMQX_GM_ENOMEM, "match: workspace");
  // the counters start 64-B aligned, so zeroing them is one fill launch (an
  // unaligned 64-B memset is split into three)
  const uintptr_t ctrs_a = (reinterpret_cast<uintptr_t>(toff.p) + (n_tiles + 1) * 8 + 63) & ~uintptr_t(63);
  ctrs_p = reinterpret_cast<uint8_t*>(ctrs_a);
  toff_p = reinterpret_cast<uint64_t*>(ctrs_p) - (n_tiles + 1);
  // the pass counters: the next block of the context's ring when it is free
  // (zeroed by the previous call's assembly, or here if it is dirty), else the
  // 64-B block behind toff, zeroed here
  bool zero_ctrs = true;
  if (!ctx->ctr_ring) {
    void* r = nullptr;
    if (hipMalloc(&r, emqx_gm_ctx::CTR_RING * 64) == hipSuccess) {
      if (hipMemset(r, 0, emqx_gm_ctx::CTR_RING * 64) == hipSuccess) ctx->ctr_ring = r;
      else hipFree(r);
    }
  }
  if (ctx->ctr_ring && ctx->ctr_state[ctx->ctr_next] != 1) {
    ctr_slot = ctx->ctr_next;
    ctx->ctr_next = (ctx->ctr_next + 1) % emqx_gm_ctx::CTR_RING;
    zero_ctrs = ctx->ctr_state[ctr_slot] == 2;
    ctx->ctr_state[ctr_slot] = 1;
    ctrs_p = static_cast<uint8_t*>(ctx->ctr_ring) + 64 * ctr_slot;
  }
  probe_tile = PoolBuf(ctx->pool, n_tiles * 8 + 8);
  if (!probe_tile.p) return set_err(ctx, EMQX_GM_ENOMEM, "match: probe workspace");
  // split forms: per-topic header and word ids [level][topic] (the fused kernel keeps them in registers)
  if (main_kind() != MAIN_FUSED) {
    hdr = PoolBuf(ctx->pool, n * 4 + 16);
    wids = PoolBuf(ctx->pool, uint64_t(TOK_LMAX) * n * 4 + 16);
    if (!hdr.p || !wids.p) return set_err(ctx, EMQX_GM_ENOMEM, "match: word-id workspace");
  }
  // counters: u32 n1 @0 (main-pass overflow), u32 n2 @4 (listed-pass
  // overflow), u64 probes @16, u64 wildcard topics @24
  uint32_t* n1 = reinterpret_cast<uint32_t*>(ctrs_p);
  uint32_t* n2 = n1 + 1;
  unsigned long long* probe_ctr = reinterpret_cast<unsigned long long*>(ctrs_p + 16);
  unsigned long long* wild_ctr = reinterpret_cast<unsigned long long*>(ctrs_p + 24);
  // (a one-wave kernel: a 64-B hipMemsetAsync costs 11-26 us of host time
  // before the main pass can be queued, a launch ~6)
  if (zero_ctrs) hipLaunchKernelGGL(k_zero16, dim3(1), dim3(64), 0, st, reinterpret_cast<uint32_t*>(ctrs_p));

  cmp = main_kind() == MAIN_FUSED && stage_compact() && uint64_t(idx->view.n_filters) < (1ull << CMP_SHIFT);
  if (cmp) {
    const char* le = knob("GM_LISTED_CAP");  // (tests: listed rows past it go to the slow path)
    cmpb.lcap = std::min<uint64_t>(n, le ? strtoull(le, nullptr, 10) : (1u << 20));
    c_tlen = PoolBuf(ctx->pool, n_tiles * 4 + 16);
    c_cnt8 = PoolBuf(ctx->pool, n + 64);
    c_lstage = PoolBuf(ctx->pool, cmpb.lcap * FAST_MC * 4 + 16);
    c_lcnt = PoolBuf(ctx->pool, cmpb.lcap * 4 + 16);
    if (!c_tlen.p || !c_lstage.p || !c_lcnt.p || !c_cnt8.p) return set_err(ctx, EMQX_GM_ENOMEM, "match: compact staging");
    cmpb.cnt8 = c_cnt8.as<uint8_t>();
    cmpb.tlen = c_tlen.as<uint32_t>();
    cmpb.lstage = c_lstage.as<uint32_t>();
    cmpb.lcnt = c_lcnt.as<uint32_t>();
  }
  // ev[0] / ev[1]: the main pass's start and end (also the call's start: total_device_ms);
  // an untimed call of the fused pass launches it without them
  if (main_kind() != MAIN_FUSED) timed = true;  // (the other forms record their events around the launches)
  hipEvent_t main_ev0 = ev[0], main_ev1 = ev[1];
  if (!timed) main_ev0 = main_ev1 = nullptr;
  // GM_D0=0 (A/B knob, read per call): level 0 probed like any other level
  IndexView vcall = idx->view;
  if (const char* de = knob("GM_D0"))
    if (!atoi(de)) vcall.flags &= ~IX_D0;
  if (const char* se = knob("GM_STAGE_SC1"))  // A/B knobs (read per call)
    if (atoi(se)) vcall.flags |= IX_STAGE_SC1;
  if (const char* be = knob("GM_L1_BYPASS")) vcall.l1_bypass = uint32_t(strtoul(be, nullptr, 0));
  if (const char* pe = knob("GM_HOT_POLICY")) vcall.hot_policy = uint32_t(strtoul(pe, nullptr, 0));
  if (exact)
    launch_match<true>(ctx, vcall, tb, to, n, cnt.as<uint32_t>(), stage.as<uint32_t>(), list1.as<uint32_t>(), n1,
                       list2.as<uint32_t>(), n2, probe_ctr, wild_ctr, hdr.as<uint32_t>(), wids.as<uint32_t>(),
                       probe_tile.as<unsigned long long>(), tsum.as<uint64_t>(), main_ev0, main_ev1,
                       cmp ? &cmpb : nullptr, &listed_deferred);
  else
    launch_match<false>(ctx, vcall, tb, to, n, cnt.as<uint32_t>(), stage.as<uint32_t>(), list1.as<uint32_t>(),
                        n1, list2.as<uint32_t>(), n2, probe_ctr, wild_ctr, hdr.as<uint32_t>(), wids.as<uint32_t>(),
                        probe_tile.as<unsigned long long>(), tsum.as<uint64_t>(), main_ev0, main_ev1,
                        cmp ? &cmpb : nullptr, &listed_deferred);
  GM_HIP(ctx, hipGetLastError());

  // Assembly stream: a large device-buffer call's scan and speculative
  // assembly go to ctx->stream_asm behind its main pass (an event), so the
  // NEXT call's main pass, queued on the context stream, starts as soon as
  // this one's ends and overlaps this call's latency-bound assembly and the
  // walk's tail.  (Its pass counters were zeroed on the context stream; the
  // assembly then zeroes no ring block for a later call.)
  hipStream_t sa = st;
  if (asm_overlap && main_kind() == MAIN_FUSED) {
    if (!ctx->stream_asm && hipStreamCreateWithFlags(&ctx->stream_asm, hipStreamNonBlocking) != hipSuccess)
      ctx->stream_asm = nullptr;
    if (ctx->stream_asm) {
      if (!timed) GM_HIP(ctx, hipEventRecord(ev[1], st));  // (a timed call's main pass records it itself)
      GM_HIP(ctx, hipStreamWaitEvent(ctx->stream_asm, ev[1], 0));
      sa = ctx->stream_asm;
    }
  }
  on_asm = sa != st;

  // count -> scan, then ONE host round trip reads the pass counters and the
  // match total together (the slow path below is rare; it re-scans)
  // (tsum: per-tile match counts, written by the main pass and topped up by the listed and slow passes)
  // (compact staging: a two-level scan is left split, k_assemble_c adds the
  // block offsets -- one launch fewer; GM_SCAN_SPLIT=0 turns it off)
  const char* se = knob("GM_SCAN_SPLIT");
  split = cmp && (!se || atoi(se) != 0);
  // Speculative assembly: the rows are written before the host has read the
  // match total, into an ids buffer sized from this context's recent matches
  // per topic (x1.25), so a call makes ONE host round trip.  The total, the
  // pass counters and the assembly come back together; a batch with a listed-
  // pass overflow (slow-path rows) or more matches than the buffer holds is
  // assembled again in finish(), once the host knows the total.
  // (at most FAST_MC per topic: a longer row is a slow-path row, assembled again anyway)
  cap_spec = 1024 + uint64_t(double(n) * std::min(ctx->ids_per_topic, double(FAST_MC)));
  // (no room for the speculative buffer: skip speculation, the rows are
  // assembled at their exact size once the total is known)
  if (!knob("GM_NO_SPEC_IDS")) ids = PoolBuf(ctx->pool, cap_spec * 4 + 16);  // (test knob: as if it failed)
  spec = ids.p != nullptr;
  // The scan may hand back block SUMS (split_sums) only when the speculative
  // assembly runs: that kernel sums them and writes the grand total to
  // toff[n_tiles], which the read-back below copies.  Without it the total
  // would still be k_scan_local's block-local prefix, so the scan
  // then writes its block offsets and total itself.
  int rc = scan_excl(ctx, LoadU64{tsum.as<uint64_t>()}, n_tiles, toff_p,
                     SideSum{probe_tile.as<unsigned long long>(), n_tiles, probe_ctr}, split ? &scan_blk : nullptr, sa,
                     split && spec && sums_mode() ? &split_sums : nullptr);
  if (rc) return rc;
  // (compact staging with no host copy-out queued behind: the assembly kernel
  // writes the read-back words itself and its stop event is the call's end --
  // a copy and an event record fewer, ~10 us of idle stream per call at C1)
  // (a host copy-out queued behind -- the small host-buffer call's tail -- goes
  // between the assembly and the call's end event, recorded after it)
  uint32_t* pin_dev = nullptr;  // the pinned words as the device addresses them
  const bool tail_q = tail && tail->enqueue;
  const bool rb_kernel =
      spec && cmp && hipHostGetDevicePointer(reinterpret_cast<void**>(&pin_dev), pin, 0) == hipSuccess && pin_dev;
  // (compact staging: the assembly also zeroes the ring's next block for the next call, if it is dirty)
  uint32_t* zero_next = nullptr;
  if (spec && cmp && ctr_slot >= 0 && !on_asm) {
    const int z = (ctr_slot + 1) % emqx_gm_ctx::CTR_RING;
    if (ctx->ctr_state[z] == 2) {
      zero_next = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(ctx->ctr_ring) + 64 * z);
      ctx->ctr_state[z] = 0;  // (a kernel queued before any later call zeroes it)
    }
  }
  if (spec) {
    launch_assemble(sa, nblk, cmp ? &cmpb : nullptr, cnt.as<uint32_t>(), n, toff_p, stage.as<uint32_t>(),
                    row_off.as<uint64_t>(), ids.as<uint32_t>(), idx->view.gmap, cap_spec, scan_blk.as<uint64_t>(),
                    rb_kernel ? pin_dev : nullptr, reinterpret_cast<const uint32_t*>(ctrs_p),
                    rb_kernel && !tail_q ? ev[2] : nullptr, zero_next, split_sums);
    GM_HIP(ctx, hipGetLastError());
    if (tail_q) {
      rc = tail->enqueue(row_off.as<uint64_t>(), ids.as<uint32_t>(), cap_spec);
      if (rc) return rc;
      if (rb_kernel) GM_HIP(ctx, hipEventRecord(ev[2], sa));
    }
  }
  if (!rb_kernel) {
    if (int rc2 = readback(sa)) return rc2;
    GM_HIP(ctx, hipEventRecord(ev[2], sa));
  }
  return 0;
}

int MatchCall::finish(emqx_gm_csr* out, MatchTail* tail, bool locked) {
  // wait for the read-back; a call submitted alone waits without the context
  // lock, so other threads can queue their calls meanwhile
  if (locked) {
    GM_HIP(ctx, hipEventSynchronize(ev[2]));
  } else {
    const hipError_t e = hipEventSynchronize(ev[2]);
    if (e != hipSuccess) return set_err(ctx, EMQX_GM_EDEVICE, std::string("match_wait: ") + hipGetErrorString(e));
  }
  std::unique_lock<std::recursive_mutex> lk(ctx->mu, std::defer_lock);
  if (!locked) lk.lock();
  struct StatsCopy {  // this call's stats, kept with it (destroyed before lk: still under the lock)
    MatchCall* c;
    ~StatsCopy() { c->st_copy = c->ctx->stats; }
  } stats_copy{this};
  hipStream_t st = ctx->stream;
  emqx_gm_match_stats& S = ctx->stats;
  S = emqx_gm_match_stats{};
  S.n_topics = n;
  if (n == 0) {
    submitted = false;
    return finish_csr(ctx, 0, 0, row_off, ids, dev_io, out);
  }
  uint64_t nnz = pin[0];
  uint64_t h_ctr[4] = {pin[1], pin[2], pin[3], pin[4]};
  // (an untimed call's events hold an older call's stamps: no figures)
  const float main_ms = timed ? ev_ms(ev[0], ev[1]) : 0.f, call_ms = timed ? ev_ms(ev[0], ev[2]) : 0.f;
  if (listed_deferred && uint32_t(h_ctr[0])) {
    // the main pass queued rows: the listed pass now, a full scan of the
    // topped-up tile sums, the read-back again; the rows are assembled below
    uint32_t* n1 = reinterpret_cast<uint32_t*>(ctrs_p);
    unsigned long long* probe_ctr = reinterpret_cast<unsigned long long*>(ctrs_p + 16);
    unsigned long long* wild_ctr = reinterpret_cast<unsigned long long*>(ctrs_p + 24);
    if (exact)
      launch_listed<true>(st, idx->view, tb, to, n, cnt.as<uint32_t>(), stage.as<uint32_t>(), list1.as<uint32_t>(), n1,
                          list2.as<uint32_t>(), n1 + 1, probe_ctr, wild_ctr, tsum.as<uint64_t>(), &cmpb);
    else
      launch_listed<false>(st, idx->view, tb, to, n, cnt.as<uint32_t>(), stage.as<uint32_t>(), list1.as<uint32_t>(),
                           n1, list2.as<uint32_t>(), n1 + 1, probe_ctr, wild_ctr, tsum.as<uint64_t>(), &cmpb);
    GM_HIP(ctx, hipGetLastError());
    // (the probe counter already holds the main pass's tiles: the side sum is not repeated)
    int rc = scan_excl(ctx, LoadU64{tsum.as<uint64_t>()}, n_tiles, toff_p);
    if (rc) return rc;
    if (int rc2 = readback(st)) return rc2;
    GM_HIP(ctx, hipStreamSynchronize(st));
    nnz = pin[0];
    for (int k = 0; k < 4; ++k) h_ctr[k] = pin[k + 1];
    spec = false;  // the speculative rows lacked the listed rows
    split = false;  // toff is whole now
  }
  S.probes = h_ctr[2];
  S.n_wildcard_topics = h_ctr[3];
  S.n_overflow = uint32_t(h_ctr[0]);
  if (spec && uint32_t(h_ctr[0] >> 32) == 0 && nnz <= cap_spec) {  // no slow-path row, and the rows fit: done
    ctx->ids_per_topic = std::max(1.0, 1.25 * double(nnz) / double(n));
    S.nnz = nnz;
    S.match_kernel_ms = main_ms;
    S.total_device_ms = call_ms;
    if (tail) tail->used = true;
    submitted = false;
    return finish_csr(ctx, n, nnz, row_off, ids, dev_io, out);
  }
  ids.reset();
  if (nnz > cap_spec) ctx->ids_per_topic = std::max(ctx->ids_per_topic, 1.25 * double(nnz) / double(n));
  const uint64_t n_ovf = uint32_t(h_ctr[0] >> 32);

  // ---- slow path for rows the listed pass could not hold
  PoolBuf slow_off, slow_ids;
  uint32_t* ovf_list = list2.as<uint32_t>();
  if (n_ovf) {
    // a frontier holds the nodes of one depth: the widest depth bounds it
    const uint64_t fr_cap = std::min<uint64_t>(uint64_t(idx->view.n_nodes),
                                               idx->level_nodes ? idx->level_nodes : uint64_t(idx->view.n_nodes)) + 1;
    const uint64_t bm_words = (uint64_t(idx->view.n_filters) + 31) / 32 + 1;
    const uint64_t per_blk = (2 * fr_cap + bm_words) * 4;
    // chunks sized by a 1 GiB workspace, up to 16,384 topics (a workgroup each) per launch
    uint64_t chunk = std::max<uint64_t>(1, std::min<uint64_t>(16384, (1ull << 30) / per_blk));
    chunk = std::min(chunk, n_ovf);
    PoolBuf fr(ctx->pool, chunk * 2 * fr_cap * 4);
    PoolBuf bm(ctx->pool, chunk * bm_words * 4);
    PoolBuf scnt(ctx->pool, n_ovf * 8 + 8);
    std::vector<uint64_t> h_off(n_ovf + 1, 0);
    if (!fr.p || !bm.p || !scnt.p) return set_err(ctx, EMQX_GM_ENOMEM, "match: slow-path workspace");
    slow_off = PoolBuf(ctx->pool, (n_ovf + 1) * 8);
    uint64_t cap_ids = std::max<uint64_t>(1024, n_ovf * 64);
    slow_ids = PoolBuf(ctx->pool, cap_ids * 4);
    if (!slow_off.p || !slow_ids.p) return set_err(ctx, EMQX_GM_ENOMEM, "match: slow-path output");
    for (uint64_t k0 = 0; k0 < n_ovf; k0 += chunk) {
      const uint64_t kn = std::min(n_ovf, k0 + chunk);
      if (exact)
        hipLaunchKernelGGL(k_slow_walk<true>, dim3(kn - k0), dim3(256), 0, st, tb, to, idx->view, ovf_list, k0, kn,
                           fr.as<uint32_t>(), fr_cap, bm.as<uint32_t>(), bm_words, cnt.as<uint32_t>(),
                           scnt.as<uint64_t>(), tsum.as<uint64_t>());
      else
        hipLaunchKernelGGL(k_slow_walk<false>, dim3(kn - k0), dim3(256), 0, st, tb, to, idx->view, ovf_list, k0, kn,
                           fr.as<uint32_t>(), fr_cap, bm.as<uint32_t>(), bm_words, cnt.as<uint32_t>(),
                           scnt.as<uint64_t>(), tsum.as<uint64_t>());
      GM_HIP(ctx, hipGetLastError());
      std::vector<uint64_t> c(kn - k0);
      GM_HIP(ctx, hipMemcpyAsync(c.data(), scnt.as<uint64_t>() + k0, (kn - k0) * 8, hipMemcpyDeviceToHost, st));
      GM_HIP(ctx, hipStreamSynchronize(st));
      for (uint64_t k = k0; k < kn; ++k) h_off[k + 1] = h_off[k] + c[k - k0];
      if (h_off[kn] > cap_ids) {  // grow the slow output buffer
        uint64_t ncap = std::max(h_off[kn], cap_ids * 2);
        PoolBuf nb(ctx->pool, ncap * 4);
        if (!nb.p) return set_err(ctx, EMQX_GM_ENOMEM, "match: slow-path output grow");
        if (h_off[k0]) GM_HIP(ctx, hipMemcpyAsync(nb.p, slow_ids.p, h_off[k0] * 4, hipMemcpyDeviceToDevice, st));
        slow_ids = std::move(nb);
        cap_ids = ncap;
      }
      GM_HIP(ctx, hipMemcpyAsync(slow_off.as<uint64_t>() + k0, h_off.data() + k0, (kn - k0 + 1) * 8,
                                 hipMemcpyHostToDevice, st));
      hipLaunchKernelGGL(k_slow_emit, dim3(kn - k0), dim3(256), 0, st, k0, kn, bm.as<uint32_t>(), bm_words,
                         slow_off.as<uint64_t>(), slow_ids.as<uint32_t>());
      GM_HIP(ctx, hipGetLastError());
    }
    // the slow path added its rows' counts to tsum: scan again
    int rc = scan_excl(ctx, LoadU64{tsum.as<uint64_t>()}, n_tiles, toff_p);
    if (rc) return rc;
    GM_HIP(ctx, hipMemcpyAsync(&nnz, toff_p + n_tiles, 8, hipMemcpyDeviceToHost, st));
    GM_HIP(ctx, hipStreamSynchronize(st));
  }

  // ---- write the rows (again: the speculative pass did not fit or missed slow-path rows)
  ids = PoolBuf(ctx->pool, nnz * 4 + 16);
  if (!ids.p) return set_err(ctx, EMQX_GM_ENOMEM, "match: ids");
  // (after a slow-path rescan toff is whole; otherwise it is still the split first scan)
  launch_assemble(st, nblk, cmp ? &cmpb : nullptr, cnt.as<uint32_t>(), n, toff_p, stage.as<uint32_t>(),
                  row_off.as<uint64_t>(), ids.as<uint32_t>(), idx->view.gmap, nnz,
                  (n_ovf || !split) ? nullptr : scan_blk.as<uint64_t>(), nullptr, nullptr, nullptr, nullptr,
                  (n_ovf || !split) ? 0u : split_sums);
  GM_HIP(ctx, hipGetLastError());
  if (n_ovf) {
    hipLaunchKernelGGL(k_copy_slow, dim3(n_ovf), dim3(256), 0, st, ovf_list, n_ovf, row_off.as<uint64_t>(),
                       slow_off.as<uint64_t>(), slow_ids.as<uint32_t>(), ids.as<uint32_t>(), idx->view.gmap);
    GM_HIP(ctx, hipGetLastError());
  }
  GM_HIP(ctx, hipEventRecord(ev[2], st));
  GM_HIP(ctx, hipEventSynchronize(ev[2]));
  S.nnz = nnz;
  S.match_kernel_ms = main_ms;
  S.total_device_ms = timed ? ev_ms(ev[0], ev[2]) : 0.f;
  submitted = false;
  return finish_csr(ctx, n, nnz, row_off, ids, dev_io, out);
}

int run_match(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const uint8_t* tb_in, const uint64_t* to_in, uint64_t n,
              uint32_t flags, emqx_gm_csr* out, MatchTail* tail) {
  MatchCall c(ctx);
  if (int rc = c.submit(idx, tb_in, to_in, n, flags, tail)) return rc;
  return c.finish(out, tail, true);
}

int match_submit(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const uint8_t* tb, const uint64_t* to, uint64_t n,
                 uint32_t flags, void** ticket, MatchTail* tail) {
  auto* c = new MatchCall(ctx);
  if (int rc = c->submit(idx, tb, to, n, flags, tail)) {
    delete c;
    return rc;
  }
  *ticket = c;
  return 0;
}

// (called without ctx->mu; takes it after the wait)
int match_wait(emqx_gm_ctx* ctx, void* ticket, emqx_gm_csr* out, MatchTail* tail, emqx_gm_match_stats* st_out) {
  auto* c = static_cast<MatchCall*>(ticket);
  const int rc = c->finish(out, tail, false);
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  if (st_out) *st_out = c->st_copy;
  delete c;
  return rc;
}

// ---- IX_D0: the root's '+' child's record (IndexView::d0_root), read from
// the depth-1 hot table (the gm_common.h hot_lookup rules: MPH slot + overflow
// region, or linear probing) by one thread, at build and after each in-place
// update (the update renumbers filter ids and may change its sig / hf).
__device__ __forceinline__ uint32_t hot_find(const IndexView& v, int t, uint64_t key) {
  const uint64_t cap = v.hot_cap[t];
  if (!cap) return NONE;
  const HotSlot* tab = v.hot + v.hot_off[t];
  if (const uint32_t mc = v.mph_cap[t]) {
    const uint64_t w = v.mph_word[v.mph_off[t] + mph_bucket(key, v.mph_nb[t])];
    if (!mph_may_hold(w, key)) return NONE;
    const uint32_t s = mph_slot(key, uint32_t(w & 0xFFFFu), mc);
    if (tab[s].key == key) return s;
    if (!((v.mph_ovf >> t) & 1u)) return NONE;
    for (uint64_t o = mph_ovf_home(key, mc, uint32_t(cap));; o = o + 1 == cap ? mc : o + 1) {
      if (tab[o].key == key) return uint32_t(o);
      if (tab[o].key == EDGE_EMPTY) return NONE;
    }
  }
  for (uint64_t s = hot_slot(key, cap);; s = s + 1 == cap ? 0 : s + 1) {
    if (tab[s].key == key) return uint32_t(s);
    if (tab[s].key == EDGE_EMPTY) return NONE;
  }
}
__global__ void k_d0_refresh(IndexView v, uint4* __restrict__ d0) {
  const int t = hot_table(1);
  const uint32_t s = v.plus_word == NONE ? NONE : hot_find(v, t, hot_key(0u, v.plus_word, 0u));
  if (s == NONE) {
    *d0 = D1_NONE;
  } else {
    const HotSlot& h = v.hot[v.hot_off[t] + s];
    *d0 = make_uint4(s, h.sig, h.hf, h.end_filter);
  }
}

int refresh_d0(emqx_gm_ctx* ctx, const IndexView& v, void* d0) {
  if (const char* e = knob("GM_D0"))  // A/B knob: 0 = the walk probes level 0 like any other
    if (!atoi(e)) return 1;
  hipLaunchKernelGGL(k_d0_refresh, dim3(1), dim3(1), 0, ctx->stream, v, static_cast<uint4*>(d0));
  GM_HIP(ctx, hipGetLastError());
  GM_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return 0;
}

int scan_lengths(emqx_gm_ctx* ctx, const uint64_t* len, uint64_t n, uint64_t* out) {
  return scan_excl(ctx, LoadU64{len}, n, out);
}

namespace {
struct LoadU16 {
  const uint16_t* p;
  __device__ uint64_t operator()(uint64_t i) const { return p[i]; }
};
}  // namespace
int scan_len16(emqx_gm_ctx* ctx, hipStream_t st, const uint16_t* len, uint64_t n, uint64_t* out) {
  return scan_excl(ctx, LoadU16{len}, n, out, SideSum{}, nullptr, st);
}

int sum_filter_lengths(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const uint32_t* d_ids, uint64_t nnz,
                       uint64_t* out) {
  if (idx->flen_stale) {  // after an in-place update: the lengths in this snapshot's ids, once
    std::lock_guard<std::mutex> lk(idx->flen_mu);
    if (idx->flen_stale) {
      const uint64_t nf = idx->info.n_filters;
      std::vector<uint16_t> fl(nf + 1, 0);
      idx->ft.for_each([&](uint64_t f, const uint8_t*, uint64_t l) { fl[f] = uint16_t(std::min<uint64_t>(l, 65535)); });
      GM_HIP(ctx, hipMemcpyAsync(idx->dev_flen, fl.data(), nf * 2, hipMemcpyHostToDevice, ctx->stream));
      GM_HIP(ctx, hipStreamSynchronize(ctx->stream));
      idx->flen_stale = false;
    }
  }
  PoolBuf acc(ctx->pool, 16);
  if (!acc.p) return set_err(ctx, EMQX_GM_ENOMEM, "sum_flen");
  GM_HIP(ctx, hipMemsetAsync(acc.p, 0, 8, ctx->stream));
  if (nnz) {
    const uint64_t blocks = std::min<uint64_t>(4096, (nnz + 255) / 256);
    hipLaunchKernelGGL(k_sum_flen, dim3(blocks), dim3(256), 0, ctx->stream, d_ids, nnz, idx->dev_flen,
                       idx->view.gmap, idx->view.n_filters, acc.as<unsigned long long>());
    GM_HIP(ctx, hipGetLastError());
  }
  GM_HIP(ctx, hipMemcpyAsync(out, acc.p, 8, hipMemcpyDeviceToHost, ctx->stream));
  GM_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return 0;
}

int run_fanout(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const emqx_gm_csr* m, uint32_t flags,
               emqx_gm_csr* out, uint32_t part, uint32_t n_parts, uint64_t* first_out) {
  const bool dev_out = flags & EMQX_GM_DEVICE_IO;
  hipStream_t st = ctx->stream;
  const uint64_t n = m->n_rows, nnz = m->nnz;
  ctx->stats = emqx_gm_match_stats{};
  ctx->stats.n_topics = n;
  PoolBuf own_off, own_ids;
  const uint64_t* m_off = m->row_off;
  const uint32_t* m_ids = m->ids;
  if (!m->on_device) {
    for (uint64_t i = 0; i < nnz; ++i)
      if (m->ids[i] >= idx->view.n_filters) return set_err(ctx, EMQX_GM_EINVAL, "fanout: filter id out of range");
    own_off = PoolBuf(ctx->pool, (n + 1) * 8);
    own_ids = PoolBuf(ctx->pool, nnz * 4 + 16);
    if (!own_off.p || !own_ids.p) return set_err(ctx, EMQX_GM_ENOMEM, "fanout: input workspace");
    GM_HIP(ctx, hipMemcpyAsync(own_off.p, m->row_off, (n + 1) * 8, hipMemcpyHostToDevice, st));
    if (nnz) GM_HIP(ctx, hipMemcpyAsync(own_ids.p, m->ids, nnz * 4, hipMemcpyHostToDevice, st));
    m_off = own_off.as<uint64_t>();
    m_ids = own_ids.as<uint32_t>();
  }
  PoolBuf seg_dst(ctx->pool, (nnz + 1) * 8);
  PoolBuf row_off(ctx->pool, (n + 1) * 8);
  if (!seg_dst.p || !row_off.p) return set_err(ctx, EMQX_GM_ENOMEM, "fanout: workspace");
  GM_HIP(ctx, hipEventRecord(ctx->ev[0], st));
  int rc = scan_excl(ctx, LoadSegLen{m_ids, idx->view.sub_off}, nnz, seg_dst.as<uint64_t>());
  if (rc) return rc;
  hipLaunchKernelGGL(k_fanout_rowoff, dim3((n + 1 + 255) / 256), dim3(256), 0, st, m_off, n, seg_dst.as<uint64_t>(),
                     row_off.as<uint64_t>(), nnz);
  GM_HIP(ctx, hipGetLastError());
  uint64_t total = 0;
  GM_HIP(ctx, hipMemcpyAsync(&total, seg_dst.as<uint64_t>() + nnz, 8, hipMemcpyDeviceToHost, st));
  GM_HIP(ctx, hipStreamSynchronize(st));
  // part `part` of n_parts: the contiguous delivery range [glo, ghi) of the
  // whole fan-out (rows and wide rows alike are cut wherever the range ends)
  // (the deliveries per match a small host fan-out sizes its speculative capacity by)
  if (nnz) ctx->subs_per_match = std::max(1.0, double(total) / double(nnz));
  const uint64_t glo = uint64_t((unsigned __int128)total * part / n_parts);
  const uint64_t ghi = uint64_t((unsigned __int128)total * (part + 1) / n_parts);
  const uint64_t cnt = ghi - glo;
  if (first_out) *first_out = glo;
  PoolBuf ids(ctx->pool, cnt * 4 + 16);
  if (!ids.p) return set_err(ctx, EMQX_GM_ENOMEM, "fanout: output");
  GM_HIP(ctx, hipEventRecord(ctx->ev[1], st));
  if (cnt) {
    const uint64_t per = fan_per_block(cnt);
    const uint64_t blocks = (cnt + per - 1) / per;
    hipLaunchKernelGGL(k_fanout_copy, dim3(blocks), dim3(256), 0, st, seg_dst.as<uint64_t>(), nnz, m_ids,
                       idx->view.sub_off, idx->view.sub_ids, glo, ghi, per, ids.as<uint32_t>(), false);
    GM_HIP(ctx, hipGetLastError());
  }
  GM_HIP(ctx, hipEventRecord(ctx->ev[2], st));
  GM_HIP(ctx, hipEventSynchronize(ctx->ev[2]));
  ctx->stats.nnz = cnt;
  ctx->stats.match_kernel_ms = ev_ms(ctx->ev[1], ctx->ev[2]);
  ctx->stats.total_device_ms = ev_ms(ctx->ev[0], ctx->ev[2]);
  return finish_csr(ctx, n, cnt, row_off, ids, dev_out, out);
}

// A small host fan-out's device work (gm_host.cpp run_fanout_small), queued
// without a wait: the deliveries' offsets, the rows' offsets and the delivery
// lists of [0, min(total, the device's count)) -- total: the call's capacity.
int queue_fanout_small(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const uint64_t* d_off, const uint32_t* d_ids,
                       uint64_t n, uint64_t nnz, uint64_t total, uint64_t* seg_dst, uint64_t* row_off, uint32_t* ids) {
  hipStream_t st = ctx->stream;
  if (nnz + 1 <= SCAN_LOOP_MAX) {
    hipLaunchKernelGGL(k_scan_loop<LoadSegLen>, dim3(1), dim3(SCAN1_T), 0, st, LoadSegLen{d_ids, idx->view.sub_off},
                       nnz, nnz + 1, seg_dst);
    GM_HIP(ctx, hipGetLastError());
  } else if (int rc = scan_excl(ctx, LoadSegLen{d_ids, idx->view.sub_off}, nnz, seg_dst)) {
    return rc;
  }
  hipLaunchKernelGGL(k_fanout_rowoff, dim3((n + 1 + 255) / 256), dim3(256), 0, st, d_off, n, seg_dst, row_off, nnz);
  GM_HIP(ctx, hipGetLastError());
  if (total) {
    const uint64_t per = fan_per_block(total);
    hipLaunchKernelGGL(k_fanout_copy, dim3((total + per - 1) / per), dim3(256), 0, st, seg_dst, nnz, d_ids,
                       idx->view.sub_off, idx->view.sub_ids, uint64_t(0), total, per, ids, true);
    GM_HIP(ctx, hipGetLastError());
  }
  return 0;
}

// The fan-out of a small host call's speculative rows, queued right behind its
// assembly (emqx_gm_match_fanout, gm_host.cpp run_host_small): d_ro/d_ids the
// speculative CSR (cap_m ids), the deliveries into cap_f -- both counts checked
// by the host after the call's one wait.
int queue_fanout_spec(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const uint64_t* d_ro, const uint32_t* d_ids,
                      uint64_t n, uint64_t cap_m, uint64_t cap_f, uint64_t* seg_dst, uint64_t* row_off, uint32_t* ids) {
  hipStream_t st = ctx->stream;
  const LoadSegLenSpec ld{d_ids, idx->view.sub_off, d_ro + n, uint32_t(idx->view.n_filters)};
  if (cap_m + 1 <= SCAN_LOOP_MAX) {
    hipLaunchKernelGGL(k_scan_loop<LoadSegLenSpec>, dim3(1), dim3(SCAN1_T), 0, st, ld, cap_m, cap_m + 1, seg_dst);
    GM_HIP(ctx, hipGetLastError());
  } else if (int rc = scan_excl(ctx, ld, cap_m, seg_dst)) {
    return rc;
  }
  hipLaunchKernelGGL(k_fanout_rowoff, dim3((n + 1 + 255) / 256), dim3(256), 0, st, d_ro, n, seg_dst, row_off, cap_m);
  GM_HIP(ctx, hipGetLastError());
  const uint64_t per = fan_per_block(cap_f);
  hipLaunchKernelGGL(k_fanout_copy, dim3((cap_f + per - 1) / per), dim3(256), 0, st, seg_dst, cap_m, d_ids,
                     idx->view.sub_off, idx->view.sub_ids, uint64_t(0), cap_f, per, ids, true);
  GM_HIP(ctx, hipGetLastError());
  return 0;
}

// Rows back in their batch order after a prefix-routed exchange (sharded.py,
// gm_route.hip): out row perm[i] = input row i, the input rows packed in send
// order with u32 lengths lens[i].
__global__ __launch_bounds__(256) void k_unperm_lens(const uint32_t* __restrict__ lens, const uint32_t* __restrict__ perm,
                                                     uint64_t n, uint64_t* __restrict__ lens_out,
                                                     uint64_t* __restrict__ lens_in, uint32_t* __restrict__ inv) {
  const uint64_t i = uint64_t(blockIdx.x) * 256u + threadIdx.x;
  if (i < n) {
    lens_out[perm[i]] = lens[i];
    lens_in[i] = lens[i];
    inv[perm[i]] = uint32_t(i);
  }
}
// output row j = input row inv[j] (k_gather_segs, output-driven: one coalesced write)
struct UnpermSeg {
  const uint64_t* in_off;
  const uint32_t* inv;
  __device__ __forceinline__ SegSpan at(uint64_t j) const {
    const uint64_t a = in_off[inv[j]];
    return {a, in_off[inv[j] + 1] - a};
  }
};
int unpermute_rows(emqx_gm_ctx* ctx, uint64_t n, const uint32_t* d_perm, const uint32_t* d_lens, const uint32_t* d_ids,
                   uint32_t flags, emqx_gm_csr* out) {
  hipStream_t st = ctx->stream;
  PoolBuf row_off(ctx->pool, (n + 1) * 8), in_off(ctx->pool, (n + 1) * 8), l_out(ctx->pool, n * 8 + 8),
      l_in(ctx->pool, n * 8 + 8), inv(ctx->pool, n * 4 + 4);
  if (!row_off.p || !in_off.p || !l_out.p || !l_in.p || !inv.p)
    return set_err(ctx, EMQX_GM_ENOMEM, "unpermute_rows: workspace");
  if (n) {
    hipLaunchKernelGGL(k_unperm_lens, dim3(uint32_t((n + 255) / 256)), dim3(256), 0, st, d_lens, d_perm, n,
                       l_out.as<uint64_t>(), l_in.as<uint64_t>(), inv.as<uint32_t>());
    GM_HIP(ctx, hipGetLastError());
  }
  if (int rc = scan_lengths(ctx, l_out.as<uint64_t>(), n, row_off.as<uint64_t>())) return rc;
  if (int rc = scan_lengths(ctx, l_in.as<uint64_t>(), n, in_off.as<uint64_t>())) return rc;
  uint64_t nnz = 0;
  GM_HIP(ctx, hipMemcpyAsync(&nnz, row_off.as<uint64_t>() + n, 8, hipMemcpyDeviceToHost, st));
  GM_HIP(ctx, hipStreamSynchronize(st));
  PoolBuf ids(ctx->pool, nnz * 4 + 16);
  if (!ids.p) return set_err(ctx, EMQX_GM_ENOMEM, "unpermute_rows: ids");
  if (n) {
    hipLaunchKernelGGL((k_gather_segs<uint32_t, UnpermSeg>), dim3(gather_blocks(n)), dim3(256), 0, st, d_ids,
                       UnpermSeg{in_off.as<uint64_t>(), inv.as<uint32_t>()}, n, row_off.as<uint64_t>(),
                       ids.as<uint32_t>());
    GM_HIP(ctx, hipGetLastError());
  }
  return finish_csr(ctx, n, nnz, row_off, ids, flags & EMQX_GM_DEVICE_IO, out);
}

int run_merge_rows(emqx_gm_ctx* ctx, uint64_t n, uint64_t stride, uint32_t pieces, const uint32_t* d_lens,
                   const uint32_t* d_ids, uint32_t flags, emqx_gm_csr* out) {
  hipStream_t st = ctx->stream;
  ctx->stats = emqx_gm_match_stats{};
  ctx->stats.n_topics = n;
  const uint64_t nl = uint64_t(pieces) * stride;
  PoolBuf pos(ctx->pool, (nl + 1) * 8), row_off(ctx->pool, (n + 1) * 8);
  if (!pos.p || !row_off.p) return set_err(ctx, EMQX_GM_ENOMEM, "merge_rows: workspace");
  GM_HIP(ctx, hipEventRecord(ctx->ev[0], st));
  int rc = scan_excl(ctx, LoadU32{d_lens}, nl, pos.as<uint64_t>());
  if (rc) return rc;
  rc = scan_excl(ctx, LoadRowSum{d_lens, stride, pieces}, n, row_off.as<uint64_t>());
  if (rc) return rc;
  uint64_t nnz = 0;
  GM_HIP(ctx, hipMemcpyAsync(&nnz, row_off.as<uint64_t>() + n, 8, hipMemcpyDeviceToHost, st));
  GM_HIP(ctx, hipStreamSynchronize(st));
  PoolBuf ids(ctx->pool, nnz * 4 + 16);
  if (!ids.p) return set_err(ctx, EMQX_GM_ENOMEM, "merge_rows: output");
  GM_HIP(ctx, hipEventRecord(ctx->ev[1], st));
  if (n) {
    hipLaunchKernelGGL(k_merge_rows, dim3((n + 255) / 256), dim3(256), 0, st, d_lens, pos.as<uint64_t>(), d_ids, n,
                       stride, pieces, row_off.as<uint64_t>(), ids.as<uint32_t>());
    GM_HIP(ctx, hipGetLastError());
  }
  GM_HIP(ctx, hipEventRecord(ctx->ev[2], st));
  GM_HIP(ctx, hipEventSynchronize(ctx->ev[2]));
  ctx->stats.nnz = nnz;
  ctx->stats.match_kernel_ms = ev_ms(ctx->ev[1], ctx->ev[2]);
  ctx->stats.total_device_ms = ev_ms(ctx->ev[0], ctx->ev[2]);
  return finish_csr(ctx, n, nnz, row_off, ids, flags & EMQX_GM_DEVICE_IO, out);
}

int run_row_lengths(emqx_gm_ctx* ctx, const emqx_gm_csr* csr, uint32_t* d_out) {
  if (csr->n_rows) {
    hipLaunchKernelGGL(k_row_lengths, dim3((csr->n_rows + 255) / 256), dim3(256), 0, ctx->stream, csr->row_off,
                       csr->n_rows, d_out);
    GM_HIP(ctx, hipGetLastError());
  }
  GM_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return 0;
}

// Match on an overlay snapshot: the base and the delta snapshots each match
// the batch (inputs copied to the device once), then one pass drops
// tombstoned base ids, remaps the survivors to final ids and merges the delta
// row in (both rows sorted, disjoint).
int run_match_overlay(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const uint8_t* tb_in, const uint64_t* to_in,
                      uint64_t n, uint32_t flags, emqx_gm_csr* out) {
  const OverlayState& ov = *idx->ov;
  const bool dev_io = flags & EMQX_GM_DEVICE_IO;
  hipStream_t st = ctx->stream;
  PoolBuf d_tb_own, d_to_own;
  const uint8_t* tb = tb_in;
  const uint64_t* to = to_in;
  if (!dev_io && n) {
    const uint64_t bytes = to_in[n];
    for (uint64_t i = 0; i < n; ++i)
      if (to_in[i + 1] < to_in[i]) return set_err(ctx, EMQX_GM_EINVAL, "match: topic offsets not monotone");
    d_tb_own = PoolBuf(ctx->pool, bytes + 64);
    d_to_own = PoolBuf(ctx->pool, (n + 1) * 8);
    if (!d_tb_own.p || !d_to_own.p) return set_err(ctx, EMQX_GM_ENOMEM, "match: input workspace");
    if (bytes) GM_HIP(ctx, hipMemcpyAsync(d_tb_own.p, tb_in, bytes, hipMemcpyHostToDevice, st));
    GM_HIP(ctx, hipMemsetAsync(static_cast<uint8_t*>(d_tb_own.p) + bytes, 0, 64, st));
    GM_HIP(ctx, hipMemcpyAsync(d_to_own.p, to_in, (n + 1) * 8, hipMemcpyHostToDevice, st));
    tb = d_tb_own.as<uint8_t>();
    to = d_to_own.as<uint64_t>();
  }
  const uint32_t sub_flags = (flags & EMQX_GM_WITH_EXACT) | EMQX_GM_DEVICE_IO;
  emqx_gm_csr cb{}, cd{};
  int rc = run_match(ctx, ov.base, tb, to, n, sub_flags, &cb);
  if (rc) return rc;
  PoolBuf b_off, b_ids, d_off, d_ids;  // adopt the sub-results' pool buffers
  b_off.pool = b_ids.pool = d_off.pool = d_ids.pool = ctx->pool;
  b_off.p = cb.row_off;
  b_ids.p = cb.ids;
  emqx_gm_match_stats st_b = ctx->stats, st_d{};
  if (ov.delta) {
    rc = run_match(ctx, ov.delta, tb, to, n, sub_flags, &cd);
    if (rc) return rc;
    d_off.p = cd.row_off;
    d_ids.p = cd.ids;
    st_d = ctx->stats;
  }
  PoolBuf row_off(ctx->pool, (n + 1) * 8);
  if (!row_off.p) return set_err(ctx, EMQX_GM_ENOMEM, "match: row_off");
  const OvView o{ov.d_tbm, ov.d_tpre, ov.d_ins, uint32_t(ov.ins.size())};
  rc = scan_excl(ctx, LoadOvLen{cb.row_off, cb.ids, ov.delta ? cd.row_off : nullptr, o}, n, row_off.as<uint64_t>());
  if (rc) return rc;
  uint64_t nnz = 0;
  GM_HIP(ctx, hipMemcpyAsync(&nnz, row_off.as<uint64_t>() + n, 8, hipMemcpyDeviceToHost, st));
  GM_HIP(ctx, hipStreamSynchronize(st));
  PoolBuf ids(ctx->pool, nnz * 4 + 16);
  if (!ids.p) return set_err(ctx, EMQX_GM_ENOMEM, "match: ids");
  if (n) {
    hipLaunchKernelGGL(k_ov_merge, dim3((n + 255) / 256), dim3(256), 0, st, cb.row_off, cb.ids,
                       ov.delta ? cd.row_off : nullptr, ov.delta ? cd.ids : nullptr, o, n, row_off.as<uint64_t>(),
                       ids.as<uint32_t>());
    GM_HIP(ctx, hipGetLastError());
  }
  GM_HIP(ctx, hipStreamSynchronize(st));
  ctx->stats = st_b;
  ctx->stats.nnz = nnz;
  ctx->stats.probes += st_d.probes;
  ctx->stats.n_overflow += st_d.n_overflow;
  ctx->stats.match_kernel_ms += st_d.match_kernel_ms;
  ctx->stats.total_device_ms += st_d.total_device_ms;
  return finish_csr(ctx, n, nnz, row_off, ids, dev_io, out);
}

}  // namespace gm
