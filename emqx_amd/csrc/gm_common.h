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

// Read-only view of one index resident in HBM (passed by value to kernels).
struct IndexView {
  const Node* nodes;
  const DictSlot* dict;
  const EdgeSlot* edges;
  const uint8_t* arena;
  const uint64_t* sub_off;
  const uint32_t* sub_ids;
  uint64_t dict_mask;
  uint64_t etab_off[EDGE_DEPTHS];   // slot offset of each depth's table
  uint64_t etab_mask[EDGE_DEPTHS];  // slots - 1
  uint32_t n_nodes;
  uint32_t n_filters;
  uint32_t plus_word;   // word id of "+" (NONE if no filter uses it)
  uint32_t hash_word;   // word id of "#"
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

GM_HD uint64_t dict_slot(uint64_t h, uint64_t mask) { return (h ^ (h >> 29)) & mask; }
GM_HD int edge_depth(uint32_t depth) { return depth < uint32_t(EDGE_DEPTHS) ? int(depth) : EDGE_DEPTHS - 1; }
GM_HD uint64_t edge_key(uint32_t parent, uint32_t word) { return (uint64_t(parent) << 32) | word; }
GM_HD uint64_t edge_slot(uint64_t key, uint64_t mask) { return fmix64(key) & mask; }

}  // namespace gm
