// gm_common.h — index layout in HBM and the word hash shared by the host index
// compiler (gm_index.cpp) and the HIP kernels (gm_match.hip).
//
// The flat index replaces the reference's ETS ordered_set of {Key, 0|1} keys
// (apps/emqx/src/emqx_trie.erl:52-58) with a level trie:
//   * nodes[]  : one 16-B record per distinct filter prefix (word list);
//   * dict[]   : open-addressing word dictionary, 16-B slots {hash64, word id, len};
//                a word id IS its byte offset in the word arena, so a hash hit
//                is verified byte-for-byte with one dependent read;
//   * edges[]  : open-addressing (parent node, word id) -> child table, 16-B slots;
//   * arena[]  : distinct word bytes;
//   * subs     : filter -> subscriber CSR (the flattened emqx_subscriber bag).
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define GM_HD __host__ __device__ __forceinline__
#else
#define GM_HD inline
#endif

namespace gm {

constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr uint64_t EDGE_EMPTY = ~0ull;
constexpr uint32_t DICT_EMPTY_LEN = 0xFFFFFFFFu;

// node flags
constexpr uint32_t NF_END_WILD = 1u;   // end_filter is a wildcard filter (held by the trie)
constexpr uint32_t NF_HAS_EXACT = 2u;  // node has children through non-wildcard words
constexpr uint32_t NF_HAS_PLUS = 4u;

// A child reference (Node::plus_child, EdgeSlot::child) carries the child's
// NF_HAS_EXACT flag in bit 31, so a frontier entry knows whether an exact-edge
// probe can hit before its node record has been read.
constexpr uint32_t REF_X = 0x80000000u;
constexpr uint32_t REF_MASK = 0x7FFFFFFFu;

// Edge tables are partitioned by the parent's depth (0..EDGE_DEPTHS-2 each in
// their own table, deeper parents share the last), so the small upper-level
// tables stay resident in each XCD's L2.
constexpr int EDGE_DEPTHS = 16;

struct alignas(16) Node {
  uint32_t plus_child;   // child ref through '+', or NONE
  uint32_t hash_filter;  // filter id of "<this prefix>/#" (or "#" at the root), or NONE
  uint32_t end_filter;   // filter id ending exactly here, or NONE
  uint32_t flags;
};

struct alignas(16) DictSlot {
  uint64_t head;     // first 8 bytes of the word, little endian, zero padded
  uint32_t len;      // word length; DICT_EMPTY_LEN marks an empty slot
  uint32_t word;     // word id == byte offset of the word in the arena
};

struct alignas(16) EdgeSlot {
  uint64_t key;      // (parent << 32) | word id; EDGE_EMPTY marks an empty slot
  uint32_t child;    // child ref (REF_X | node index)
  uint32_t pad;
};

// ---- hot tables (read by the walk kernels) --------------------------------
// One open-addressing table per node depth (1..HOT_TABLES-2 each their own,
// deeper nodes share the last).  A node reached through an exact edge, or
// through a '+' edge from the root or from an inline node, owns exactly one
// 32-B slot, keyed by (parent's hot id, word id); its hot id IS that slot
// index.  The '+' child of a slot-owning node owns no slot: its record sits in
// the second half of its parent's slot (p_sig, p_hf, p_end) and its hot id is
// the parent's slot index | HOT_INLINE.  So a frontier entry's '+' expansion
// re-reads a line the walk fetched one level earlier (an L2 hit) instead of
// probing a new random line.  '#' edges have no node at all: their filter is
// the parent's hf ('match_#').
constexpr int HOT_TABLES = 16;
constexpr uint32_t ID_MASK = 0x7FFFFFFFu;
constexpr uint32_t HOT_INLINE = 0x40000000u;  // in a hot id: the '+' child held inline by slot (id & SLOT_MASK)
constexpr uint32_t SLOT_MASK = 0x3FFFFFFFu;
constexpr uint32_t END_WILD = 0x80000000u;  // in end_filter: the filter is a wildcard one
constexpr uint32_t HOT_PLUS = 0x80000000u;  // in HotSlot::hf: the node has a '+' child
constexpr uint32_t HOT_CHAIN = 0x40000000u; // in HotSlot::hf: a chain node (below)
constexpr uint32_t HF_MASK = 0x3FFFFFFFu;   // the filter id in HotSlot::hf
constexpr uint32_t HF_NONE = 0x3FFFFFFFu;   // HotSlot::hf without a '#' filter (filter ids stay below it)
constexpr uint32_t FR_PLUS = 0x80000000u;   // in a frontier entry: the node has a '+' child
constexpr uint64_t HOT_KEY_MARK = 1ull << 63;  // parent lives in table HOT_TABLES-2, child in the shared last

struct alignas(32) HotSlot {
  uint64_t key;          // hot_key(parent, word); EDGE_EMPTY marks an empty slot
  uint32_t sig;          // bit sig_bit(w) set for each exact child word id w; 0 = no exact child
  uint32_t hf;           // filter id of "<node>/#" (HF_NONE if none) | HOT_PLUS if the node has a '+' child
  uint32_t end_filter;   // filter id ending at the node | END_WILD, or NONE
  uint32_t p_sig;        // the inline '+' child's sig, hf and end_filter (same encodings)
  uint32_t p_hf;
  uint32_t p_end;
};
// The first 16 bytes {key, sig, hf} are all a probe needs below the topic's
// last level (one dwordx4); end_filter is read on the last level, and the
// second 16 bytes {end_filter, p_sig, p_hf, p_end} (one dwordx4) are the
// inline '+' child's record.
//
// Chain nodes (path compression of single-filter tails; HOT_CHAIN in hf): a
// slot-owning node N with no '+' child whose only child c1 is an exact edge
// that ends a chain of Lc = 1 or 2 exact words with no other branch -- c1 (and
// c2) with no '+' or '#' child, only the last one holding a filter F and no
// children at all.  Its slot then holds sig = s1 (c1's word id, not a
// signature: hot_sig() gives the signature back), p_sig = s2 (c2's word id, or
// NONE when Lc = 1), p_hf = HF_NONE and p_end = F | END_WILD flag.  The walk
// of k_match_fused checks the topic's next one or two words against s1/s2 at
// N's visit and emits F there, so c1 and c2 (still in the tables, for the
// listed pass and the in-place update) are never probed by the main pass.
// An in-place update clears HOT_CHAIN on every chain node of a path it writes
// (Patcher::unchain), so chains only need to be right at build time.
GM_HD uint32_t hot_sig(uint32_t hf, uint32_t sig);
// Read-only view of one index resident in HBM (passed by value to kernels).
constexpr uint32_t IX_HOT_FLAT = 1u;  // a hot table reaches 2 GiB: flat loads instead of buffer loads
constexpr uint32_t IX_STAGE_SC1 = 4u;  // A/B: the compact staging list stored sc1 (set per call, GM_STAGE_SC1)
constexpr uint32_t IX_D0 = 2u;        // d0_root is current: k_match_fused's level 0 round without hot-table probes of its own
struct IndexView {
  const Node* nodes;
  const DictSlot* dict;
  const EdgeSlot* edges;
  const HotSlot* hot;
  const uint8_t* arena;
  const uint64_t* sub_off;
  const uint32_t* sub_ids;
  const uint32_t* gmap;     // shard index: local filter id -> global id (ascending); nullptr otherwise
  uint64_t dict_mask;
  uint64_t etab_off[EDGE_DEPTHS];   // slot offset of each depth's table
  uint64_t etab_mask[EDGE_DEPTHS];  // slots - 1
  uint64_t hot_off[HOT_TABLES];     // slot offset of each hot table (index = child depth, capped)
  uint64_t hot_cap[HOT_TABLES];     // slots of each hot table
  const uint32_t* efilt;            // exact-edge filters (see edge_filter_hash), one bit array per hot table
  uint64_t efilt_off[HOT_TABLES];   // u32-word offset of each table's filter
  uint32_t efilt_mask[HOT_TABLES];  // words - 1 of each table's filter; 0 = no filter for that table
  uint32_t n_nodes;
  uint32_t n_filters;
  uint32_t plus_word;   // word id of "+" (NONE if no filter uses it)
  uint32_t hash_word;   // word id of "#"
  uint32_t root_sig;    // the root's exact-child signature
  uint32_t root_hash;   // filter id of "#", or NONE
  uint32_t root_flags;  // HOT_PLUS if "+" starts a filter
  uint32_t flags;       // IX_* below
  uint32_t rh_mask;     // bit t: hot table t is Robin Hood ordered (absent keys may exit early)
  // Minimal-perfect-hash tables (mph_cap[t] != 0): slots [0, mph_cap) are
  // placed by hash-and-displace (mph_slot: one probe, no chain, load ~0.97),
  // slots [mph_cap, hot_cap) are a linear-probing overflow region for keys
  // an in-place update could not put at their perfect slot (mph_ovf bit t set
  // once it holds any).  One 64-bit word per bucket: the displacement (low 16
  // bits) and a 48-bit Bloom filter over the bucket's keys, so ONE L2 read
  // both rules out most absent keys (the exact-edge filter's job) and gives
  // the slot.  See mph_* below.
  const uint64_t* mph_word;          // per bucket: displacement | Bloom bits << 16
  uint64_t mph_off[HOT_TABLES];      // word offset of each table's buckets
  uint32_t mph_nb[HOT_TABLES];       // buckets of each MPH table
  uint32_t mph_cap[HOT_TABLES];      // perfect-hash slots of each table; 0 = not an MPH table
  uint32_t mph_ovf;                  // bit t: table t's overflow region holds keys
  uint32_t l1_bypass;                // bit t: table t's probes use hot_policy (GM_L1_BYPASS A/B knob)
  uint32_t hot_policy;               // their cache policy (gm_match.hip hot_load; 1 = sc1: no L1 fill)
  // IX_D0: the root's '+' child as the walk reads it at level 0 (one uniform
  // 16-B load per wave): {hot id (NONE: no '+' at the root), sig, hf,
  // end_filter}, written from the depth-1 hot table by k_d0_refresh
  const uint32_t* d0_root;
};

GM_HD uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

// Word hash: 8-byte little-endian chunks (last one zero padded), then length.
GM_HD uint64_t hash_step(uint64_t h, uint64_t chunk) {
  h ^= chunk * 0x87c37b91114253d5ull;
  h = (h << 31) | (h >> 33);
  return h * 0x4cf5ad432745937full + 0x52dce729ull;
}
GM_HD uint64_t hash_final(uint64_t h, uint64_t len) { return fmix64(h ^ (len * 0x9E3779B97F4A7C15ull)); }
constexpr uint64_t HASH_SEED = 0x243F6A8885A308D3ull;

inline uint64_t word_head_host(const uint8_t* p, uint64_t len) {
  uint64_t c = 0;
  for (uint64_t k = 0; k < 8 && k < len; ++k) c |= uint64_t(p[k]) << (8 * k);
  return c;
}

inline uint64_t hash_word_host(const uint8_t* p, uint64_t len) {
  uint64_t h = HASH_SEED;
  uint64_t i = 0;
  for (; i + 8 <= len; i += 8) {
    uint64_t c = 0;
    for (int k = 0; k < 8; ++k) c |= uint64_t(p[i + k]) << (8 * k);
    h = hash_step(h, c);
  }
  if (i < len) {
    uint64_t c = 0;
    for (int k = 0; i + k < len; ++k) c |= uint64_t(p[i + k]) << (8 * k);
    h = hash_step(h, c);
  }
  return hash_final(h, len);
}

// Dictionary hash: 32-bit multiply-rotate steps over the same 8-byte chunks
// (two v_mul_lo_u32 per chunk instead of four 64-bit products), then a
// one-multiply xorshift finish (v_mul_lo_u32 is quarter rate and the
// tokenizer is VALU bound; a single-multiply chunk step was tried and lets
// structured words such as "l1w123" collide before the multiply).  A hit is
// verified by bytes, so the hash only spreads slots.
GM_HD uint32_t dict_hash_step(uint32_t h, uint64_t chunk) {
  h ^= uint32_t(chunk);
  h *= 0x9E3779B1u;
  h = ((h << 15) | (h >> 17)) ^ uint32_t(chunk >> 32);
  return h * 0x85EBCA77u;
}
GM_HD uint32_t dict_hash_final(uint32_t h, uint32_t len);
constexpr uint32_t DICT_HASH_SEED = 0x243F6A88u;
GM_HD uint64_t dict_slot(uint32_t h, uint64_t mask) { return uint64_t(h) & mask; }
GM_HD int edge_depth(uint32_t depth) { return depth < uint32_t(EDGE_DEPTHS) ? int(depth) : EDGE_DEPTHS - 1; }
GM_HD uint64_t edge_key(uint32_t parent, uint32_t word) { return (uint64_t(parent) << 32) | word; }
GM_HD uint64_t edge_slot(uint64_t key, uint64_t mask) { return fmix64(key) & mask; }

GM_HD int hot_table(uint32_t depth) { return depth < uint32_t(HOT_TABLES) ? int(depth) : HOT_TABLES - 1; }
// Is the '+' child of a node at `pdepth` held inline in the node's own slot?
// Only under a slot-owning node (not the root, not an inline node), and not
// under a node of depth HOT_TABLES-2: its '+' child's children go to the
// shared last table, whose keys must tell parents apart by slot number, and an
// inline hot id there would name a slot of table HOT_TABLES-2 beside the hot
// ids of the shared table's own inline nodes (same numbers, same INLINE bit).
// Such a '+' child owns a slot of the shared table instead.
GM_HD bool plus_inline(uint32_t pdepth, bool parent_owns_slot) {
  return parent_owns_slot && pdepth != 0 && pdepth != uint32_t(HOT_TABLES - 2);
}
// Key of the child of `parent` (a node at depth `pdepth`) through word `word`.
GM_HD uint64_t hot_key(uint32_t parent, uint32_t word, uint32_t pdepth) {
  return ((uint64_t(parent) << 32) | word) | (pdepth == uint32_t(HOT_TABLES - 2) ? HOT_KEY_MARK : 0ull);
}
GM_HD uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}
GM_HD uint32_t sig_bit(uint32_t word_id);
// a slot's exact-child signature (a chain node holds its one child's word id)
GM_HD uint32_t hot_sig(uint32_t hf, uint32_t sig) { return (hf & HOT_CHAIN) ? sig_bit(sig) : sig; }
GM_HD uint32_t dict_hash_final(uint32_t h, uint32_t len) {
  h ^= len;
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  return h ^ (h >> 13) ^ (h >> 20);
}

inline uint32_t dict_hash_host(const uint8_t* p, uint64_t len) {
  uint32_t h = DICT_HASH_SEED;
  for (uint64_t i = 0; i < len; i += 8) {
    uint64_t c = 0;
    for (uint64_t k = 0; k < 8 && i + k < len; ++k) c |= uint64_t(p[i + k]) << (8 * k);
    h = dict_hash_step(h, c);
  }
  return dict_hash_final(h, uint32_t(len));
}

// Signature bit of a word id (the exact-child filter of HotSlot::sig): a
// function of the id alone, so the walk needs no word hash.
GM_HD uint32_t sig_bit(uint32_t word_id) { return 1u << (fmix32(word_id * 0x9E3779B1u) >> 27); }
// Hot-key hash: two Fibonacci products (parent hot id, word id) xor-ed --
// two v_mul_lo_u32 -- and the home slot is its high bits scaled to the table
// by one v_mul_hi_u32 (any capacity < 2^32, no power-of-two blow-up).  The
// exact-edge filter takes its word and bits from the same hash folded down.
GM_HD uint32_t hot_hash(uint64_t key) { return (uint32_t(key >> 32) * 0x9E3779B1u) ^ (uint32_t(key) * 0x85EBCA77u); }
GM_HD uint64_t hot_slot(uint64_t key, uint64_t cap) {
  const uint32_t h = hot_hash(key);
#if defined(__HIP_DEVICE_COMPILE__)
  return __umulhi(h, uint32_t(cap));
#else
  return (uint64_t(h) * cap) >> 32;
#endif
}

// Hash-and-displace placement of the small upper hot tables (the depth-2
// table, ~66k keys at C2/C3, shared by every topic's first two probes): the
// key's bucket (hot_hash scaled to the bucket count) holds a 16-bit
// displacement d, and the key's slot is mph_hash(key, d) scaled to the
// table's perfect-hash region.  The builder picks each bucket's d so that all
// its keys land on distinct free slots (largest buckets first), which fills
// the region to ~0.97 with ONE probe per lookup: the table is a quarter of its
// open-addressing size (0.25 load) and stays in each XCD's L2.
constexpr uint32_t MPH_LAMBDA = 6;     // keys per bucket (1.33 B of bucket word per key; 4 -> 5: C2 -1 %, 3: +2.7 %, 5 -> 6 with keys/16 spare slots: -0.4 %; profiles/r04_ab/mph_lambda_c2.txt)
GM_HD uint32_t mph_hash(uint64_t key, uint32_t d) {
  uint32_t h = (uint32_t(key >> 32) * 0x7FEB352Du) ^ (uint32_t(key) * 0x846CA68Bu) ^ (d * 0x9E3779B9u);
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  return h;
}
GM_HD uint32_t scale32(uint32_t h, uint32_t n) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umulhi(h, n);
#else
  return uint32_t((uint64_t(h) * n) >> 32);
#endif
}
GM_HD uint32_t mph_bucket(uint64_t key, uint32_t nb) { return scale32(hot_hash(key), nb); }
GM_HD uint32_t mph_slot(uint64_t key, uint32_t d, uint32_t cap) { return scale32(mph_hash(key, d), cap); }
// the key's two Bloom bits in its bucket word (bits 16..63)
GM_HD uint64_t mph_bloom(uint64_t key) {
  const uint32_t h = (uint32_t(key >> 32) * 0x85EBCA6Bu) ^ (uint32_t(key) * 0xC2B2AE35u);
  const uint32_t a = ((h >> 26) * 3u) >> 2, b = (((h >> 20) & 63u) * 3u) >> 2;  // 0..47 each
  return (1ull << (16 + a)) | (1ull << (16 + b));
}
GM_HD bool mph_may_hold(uint64_t word, uint64_t key) {
  const uint64_t m = mph_bloom(key);
  return (word & m) == m;
}
// the overflow region [mph_cap, hot_cap): linear probing from this home
GM_HD uint32_t mph_ovf_home(uint64_t key, uint32_t mcap, uint32_t cap) {
  return mcap + scale32(hot_hash(key) ^ 0x5BD1E995u, cap - mcap);
}

// Host-side lookup of `key` in hot table t of view v, over a host copy of the
// tables: slots from `base`, bucket words from `words` (the in-place update's
// mirror, the host-only test index): the key's slot, or NONE.
inline uint32_t hot_lookup_host(const IndexView& v, const HotSlot* base, const uint64_t* words, int t, uint64_t key) {
  const uint64_t cap = v.hot_cap[t];
  if (!cap) return NONE;
  const HotSlot* tab = base + v.hot_off[t];
  const uint32_t mc = v.mph_cap[t];
  if (mc) {
    const uint64_t w = words[v.mph_off[t] + mph_bucket(key, v.mph_nb[t])];
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

// Exact-edge filter: for a hot table whose parents have many exact children
// (so the 32-bit HotSlot::sig passes most probes that then miss), one bit
// array over the hot keys (parent hot id, word id) of its exact children, two
// bits per key in one 32-bit word (4-8 bits per key: a few times more false
// positives than at 16-32, but a quarter of the L2 footprint, which measured
// faster).  It stays in L2, so a probe it rules out costs an L2 hit instead
// of a random line from HBM / Infinity Cache.
GM_HD uint32_t edge_filter_hash(uint64_t key) {
  const uint32_t h = hot_hash(key);
  return h ^ (h >> 16);
}
GM_HD uint32_t edge_filter_bits(uint32_t h) { return (1u << (h & 31)) | (1u << ((h >> 5) & 31)); }
GM_HD uint32_t edge_filter_word(uint32_t h, uint32_t mask) { return (h >> 10) & mask; }

// In-place update (gm_overlay.cpp, patch_update): a filter-id field under the
// renumbering rmap[old id] -> new id (NONE: deleted).  `none` is the field's
// empty value (NONE or HF_NONE) and `flag` the flag bits it carries (END_WILD,
// HF_FLAGS, or 0 for the level-trie fields).
constexpr uint32_t HF_FLAGS = HOT_PLUS | HOT_CHAIN;
// (rmap: the id table, or anything indexed like it -- the host's IdShift view)
template <class R>
GM_HD uint32_t renum_field(uint32_t f, uint32_t none, uint32_t flag, const R& rmap) {
  if (f == none) return f;
  const uint32_t fl = f & flag, id = f & ~flag;
  if (id == (none & ~flag)) return f;
  const uint32_t r = rmap[id];
  return r == NONE ? (fl ? (fl | (none & ~flag)) : none) : (fl | r);
}

}  // namespace gm
