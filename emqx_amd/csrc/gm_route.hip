// gm_route.hip — prefix sharding of a filter set too large to replicate
// (BASELINE.json configs[4]).
//
// Hash sharding (emqx_gm_shard_of) makes every rank walk EVERY topic against
// its shard, so topic throughput cannot grow with the ranks.  Here filters are
// partitioned by their FIRST WORD: a topic can only match filters whose first
// word is its own first word, '+' or '#' (emqx_topic:match/2,
// apps/emqx/src/emqx_topic.erl:65-87), so once the root-wildcard filters are
// on every shard, each topic needs exactly ONE shard -- the one owning its
// first word -- and a rank walks ~1/N of the topics.
//   * first-word partitions are assigned greedily (largest first, to the
//     least loaded shard);
//   * a HOT first word (more than 1/(2N) of the non-root filters) is split by
//     its second word; its filters whose second word is '+' / '#' or absent
//     ('w', 'w/#', 'w/+/...') go to every shard, like the root wildcards;
//   * a topic whose prefix owns no partition can only match replicated
//     filters: any shard does (one picked by hash, for balance).
// The route table (key bytes -> shard) is built on the host and used by the
// host (tests) and by a device kernel (one thread per topic) with the same
// logic; keys are verified byte for byte, so routing never aliases.
#include <algorithm>
#include <cstring>
#include <numeric>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "gm_gather.h"
#include "gm_internal.h"
#include "../../include/emqx_gm_ext.h"

namespace gm {

constexpr uint32_t RT_SPLIT = 0x80000000u;  // in RouteSlot::shard: a hot first word, split by its second word
constexpr uint32_t RT_EMPTY = 0xFFFFFFFFu;

struct RouteSlot {
  uint32_t hash;   // dict_hash of the key bytes
  uint32_t len;    // key length; RT_EMPTY marks an empty slot
  uint32_t off;    // key bytes in the route arena
  uint32_t shard;  // owning shard, or RT_SPLIT
};

}  // namespace gm

struct emqx_gm_route {
  uint32_t n_shards = 1;
  std::vector<gm::RouteSlot> slots;  // open addressing, power-of-two capacity
  std::vector<uint8_t> arena;        // key bytes ('w' or 'w/v')
  // device copy per device (uploaded on first use)
  std::mutex mu;
  std::unordered_map<int, void*> dev;
};

namespace gm {
namespace {

GM_HD uint32_t rt_hash(const uint8_t* p, uint32_t len) {
  uint32_t h = DICT_HASH_SEED;
  for (uint32_t i = 0; i < len; i += 8) {
    uint64_t c = 0;
    for (uint32_t k = 0; k < 8 && i + k < len; ++k) c |= uint64_t(p[i + k]) << (8 * k);
    h = dict_hash_step(h, c);
  }
  return dict_hash_final(h, len);
}

// the shard of a topic (host and device share it): its first word's
// partition, or its two-word prefix's for a split first word, else by hash
GM_HD uint32_t rt_route(const RouteSlot* slots, uint32_t mask, const uint8_t* arena, uint32_t n_shards,
                        const uint8_t* t, uint32_t len) {
  uint32_t e0 = 0;
  while (e0 < len && t[e0] != '/') ++e0;
  auto find = [&](uint32_t klen) -> uint32_t {
    const uint32_t h = rt_hash(t, klen);
    for (uint32_t s = h & mask;; s = (s + 1) & mask) {
      const RouteSlot r = slots[s];
      if (r.len == RT_EMPTY) return RT_EMPTY;
      if (r.hash == h && r.len == klen) {
        bool eq = true;
        for (uint32_t i = 0; i < klen && eq; ++i) eq = arena[r.off + i] == t[i];
        if (eq) return r.shard;
      }
    }
  };
  const uint32_t fallback = fmix32(rt_hash(t, e0) ^ 0x2545F491u) % n_shards;
  uint32_t s = find(e0);
  if (s == RT_EMPTY) return fallback;
  if (!(s & RT_SPLIT)) return s;
  if (e0 == len) return fallback;  // a one-word topic under a split word: only replicated filters match it
  uint32_t e1 = e0 + 1;
  while (e1 < len && t[e1] != '/') ++e1;
  s = find(e1);
  return s == RT_EMPTY || (s & RT_SPLIT) ? fallback : s;
}

// The device form of rt_route, 8 bytes at a time: a topic's bytes come as
// little-endian u64 chunks (two aligned loads and a funnel shift each; the
// batch is padded by 64 readable bytes), the first '/' is found by a SWAR
// compare, the key hash takes whole chunks (bytes past the key zeroed, as
// rt_hash's zero padding), and a hit is verified chunk by chunk against the
// arena (padded by 8).  Same shard as rt_route for every topic
// (test_device_route_equals_host_route); byte-at-a-time global loads had
// made the route 3.1 ms of a 100M-topic step (profiles/r04_l).
__device__ __forceinline__ uint64_t ld8(const uint8_t* base, uint64_t pos) {
  const uint64_t* w = reinterpret_cast<const uint64_t*>(reinterpret_cast<uintptr_t>(base + pos) & ~uintptr_t(7));
  const uint32_t sh = uint32_t(reinterpret_cast<uintptr_t>(base + pos) & 7u) * 8u;
  const uint64_t lo = w[0];
  return sh ? (lo >> sh) | (w[1] << (64u - sh)) : lo;
}
__device__ __forceinline__ uint64_t keep_bytes(uint64_t c, uint32_t nb) {  // the low nb bytes of c (nb <= 8)
  return nb >= 8 ? c : (c & ((1ull << (8u * nb)) - 1ull));
}
__device__ __forceinline__ uint32_t first_slash(const uint8_t* t, uint32_t from, uint32_t len) {
  for (uint32_t i = from; i < len; i += 8) {
    const uint64_t x = ld8(t, i) ^ 0x2F2F2F2F2F2F2F2Full;  // '/' -> 0x00
    const uint64_t z = (x - 0x0101010101010101ull) & ~x & 0x8080808080808080ull;
    if (z) {
      const uint32_t at = i + uint32_t(__builtin_ctzll(z) >> 3);
      return at < len ? at : len;
    }
  }
  return len;
}
__device__ uint32_t rt_route_dev(const RouteSlot* slots, uint32_t mask, const uint8_t* arena, uint32_t n_shards,
                                 const uint8_t* t, uint32_t len) {
  auto hash = [&](uint32_t klen) {
    uint32_t h = DICT_HASH_SEED;
    for (uint32_t i = 0; i < klen; i += 8) h = dict_hash_step(h, keep_bytes(ld8(t, i), klen - i));
    return dict_hash_final(h, klen);
  };
  auto find = [&](uint32_t klen) -> uint32_t {
    const uint32_t h = hash(klen);
    for (uint32_t s = h & mask;; s = (s + 1) & mask) {
      const RouteSlot r = slots[s];
      if (r.len == RT_EMPTY) return RT_EMPTY;
      if (r.hash == h && r.len == klen) {
        bool eq = true;
        for (uint32_t i = 0; i < klen && eq; i += 8)
          eq = keep_bytes(ld8(arena, r.off + i) ^ ld8(t, i), klen - i) == 0;
        if (eq) return r.shard;
      }
    }
  };
  const uint32_t e0 = first_slash(t, 0, len);
  const uint32_t fallback = fmix32(hash(e0) ^ 0x2545F491u) % n_shards;
  uint32_t s = find(e0);
  if (s == RT_EMPTY) return fallback;
  if (!(s & RT_SPLIT)) return s;
  if (e0 == len) return fallback;  // a one-word topic under a split word: only replicated filters match it
  const uint32_t e1 = first_slash(t, e0 + 1, len);
  s = find(e1);
  return s == RT_EMPTY || (s & RT_SPLIT) ? fallback : s;
}

__global__ __launch_bounds__(256) void k_route(const RouteSlot* __restrict__ slots, uint32_t mask,
                                               const uint8_t* __restrict__ arena, uint32_t n_shards,
                                               const uint8_t* __restrict__ tb, const uint64_t* __restrict__ to,
                                               uint64_t n, uint32_t* __restrict__ dest) {
  const uint64_t i = uint64_t(blockIdx.x) * 256u + threadIdx.x;
  if (i >= n) return;
  const uint64_t a = to[i], b = to[i + 1];
  dest[i] = rt_route_dev(slots, mask, arena, n_shards, tb + a, uint32_t(b - a));
}

// ---- the send order in one pass pair (emqx_gm_route_partition): a counting
// sort of the batch by shard, stable in batch order.  A block takes RP_B
// consecutive topics; pass 1 routes them (dest kept for pass 2) and writes the
// block's topic and byte counts per shard, shard-major ([s][block]) so ONE
// exclusive scan of each array gives every (shard, block) its first position;
// pass 2 ranks each topic among the block's earlier topics of its shard (wave
// ballots over the shard's 8 bits, then the 16 (round, wave) slots in order)
// and writes perm / plen at its position.  Replaces a stable radix sort of
// the shard numbers, a gather of the lengths and two prefix sums.
constexpr int RP_B = 1024;  // topics per block: 4 rounds of 256
__global__ __launch_bounds__(256) void k_part_count(const RouteSlot* __restrict__ slots, uint32_t mask,
                                                    const uint8_t* __restrict__ arena, uint32_t n_shards,
                                                    const uint8_t* __restrict__ tb, const uint64_t* __restrict__ to,
                                                    uint64_t n, uint64_t nblk, uint8_t* __restrict__ dest,
                                                    uint64_t* __restrict__ cnt, uint64_t* __restrict__ bytes) {
  __shared__ uint32_t s_c[256];
  __shared__ unsigned long long s_b[256];
  const int tid = threadIdx.x;
  s_c[tid] = 0;
  s_b[tid] = 0;
  __syncthreads();
  const uint64_t b = blockIdx.x;
  for (int v = 0; v < RP_B / 256; ++v) {
    const uint64_t i = b * RP_B + uint64_t(v) * 256 + tid;
    const bool ok = i < n;
    uint32_t d = 0xFFFFFFFFu, len = 0;
    if (ok) {
      const uint64_t a = to[i], e = to[i + 1];
      len = uint32_t(e - a);
      d = rt_route_dev(slots, mask, arena, n_shards, tb + a, len);
      d = d < n_shards ? d : d % n_shards;  // (rt_route returns a shard < n_shards; the LDS tables hold 256)
      dest[i] = uint8_t(d);
    }
    // the wave's counts per shard: one LDS atomic per distinct shard in the wave,
    // not one per topic (a wave's topics mostly share few shards -- at one shard
    // all of them: 1,024 same-address atomics per block were most of the kernel)
    unsigned long long left = __ballot(ok);
    while (left) {
      const int leader = __builtin_ctzll(left);
      const uint32_t dl = uint32_t(__shfl(int(d), leader, 64));
      const unsigned long long m = __ballot(ok && d == dl);
      uint64_t x = (ok && d == dl) ? len : 0u;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) x += uint64_t(__shfl_xor((long long)x, o, 64));
      if ((tid & 63) == leader) {
        atomicAdd(&s_c[dl], uint32_t(__popcll(m)));
        atomicAdd(&s_b[dl], (unsigned long long)x);
      }
      left &= ~m;
    }
  }
  __syncthreads();
  if (uint32_t(tid) < n_shards) {
    cnt[uint64_t(tid) * nblk + b] = s_c[tid];
    bytes[uint64_t(tid) * nblk + b] = s_b[tid];
  }
}
__global__ __launch_bounds__(256) void k_part_scatter(const uint8_t* __restrict__ dest, const uint64_t* __restrict__ to,
                                                      uint64_t n, uint64_t nblk, uint32_t n_shards,
                                                      const uint64_t* __restrict__ pos, uint32_t* __restrict__ perm,
                                                      uint32_t* __restrict__ plen) {
  constexpr int SLOTS = RP_B / 64;  // (round, wave) in batch order
  __shared__ uint32_t s_n[SLOTS][256];
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  for (int k = tid; k < SLOTS * 256; k += 256) (&s_n[0][0])[k] = 0;
  __syncthreads();
  const uint64_t b = blockIdx.x;
  uint32_t d[RP_B / 256], r[RP_B / 256];
  const uint64_t lt = (1ull << lane) - 1ull;
  for (int v = 0; v < RP_B / 256; ++v) {
    const uint64_t i = b * RP_B + uint64_t(v) * 256 + tid;
    const bool ok = i < n;
    d[v] = ok ? dest[i] : 0xFFu;
    uint64_t peers = __ballot(ok);
#pragma unroll
    for (int bit = 0; bit < 8; ++bit) {
      const uint64_t m = __ballot((d[v] >> bit) & 1u);
      peers &= ((d[v] >> bit) & 1u) ? m : ~m;
    }
    r[v] = uint32_t(__popcll(peers & lt));
    if (ok && r[v] == 0) s_n[v * 4 + wv][d[v]] = uint32_t(__popcll(peers));  // the shard's first lane in the wave
  }
  __syncthreads();
  // exclusive prefix over the slots, per shard (thread = shard)
  if (uint32_t(tid) < n_shards) {
    uint32_t run = 0;
    for (int k = 0; k < SLOTS; ++k) {
      const uint32_t c = s_n[k][tid];
      s_n[k][tid] = run;
      run += c;
    }
  }
  __syncthreads();
  for (int v = 0; v < RP_B / 256; ++v) {
    const uint64_t i = b * RP_B + uint64_t(v) * 256 + tid;
    if (i >= n) continue;
    const uint64_t p = pos[uint64_t(d[v]) * nblk + b] + s_n[v * 4 + wv][d[v]] + r[v];
    perm[p] = uint32_t(i);
    plen[p] = uint32_t(to[i + 1] - to[i]);
  }
}
__global__ void k_part_split(const uint64_t* __restrict__ pos, const uint64_t* __restrict__ bpos, uint64_t nblk,
                             uint32_t n_shards, uint64_t* __restrict__ split) {
  const uint32_t s = threadIdx.x;
  if (s < n_shards) {
    split[2 * s] = pos[uint64_t(s + 1) * nblk] - pos[uint64_t(s) * nblk];
    split[2 * s + 1] = bpos[uint64_t(s + 1) * nblk] - bpos[uint64_t(s) * nblk];
  }
}

// out topic i = input topic perm[i]: lengths, then (after a scan) the bytes
__global__ __launch_bounds__(256) void k_perm_lens(const uint64_t* __restrict__ to, const uint32_t* __restrict__ perm,
                                                   uint64_t n, uint64_t* __restrict__ lens) {
  const uint64_t i = uint64_t(blockIdx.x) * 256u + threadIdx.x;
  if (i < n) lens[i] = to[perm[i] + 1] - to[perm[i]];
}
// segment i of the permuted batch = topic perm[i] (k_gather_segs)
struct PermSeg {
  const uint64_t* to;
  const uint32_t* perm;
  __device__ __forceinline__ SegSpan at(uint64_t i) const {
    const uint64_t a = to[perm[i]];
    return {a, to[perm[i] + 1] - a};
  }
};
}  // namespace

int route_plan(const uint8_t* fb, const uint64_t* fo, uint64_t n, uint32_t n_shards, uint32_t* shard_out,
               emqx_gm_route** out) {
  // ---- first words and their counts
  std::vector<uint32_t> e0(n), e1(n);
  std::unordered_map<std::string_view, uint64_t> cnt0;
  uint64_t nonroot = 0;
  auto sv = [&](uint64_t i, uint64_t len) {
    return std::string_view(reinterpret_cast<const char*>(fb + fo[i]), len);
  };
  auto is_wild = [&](uint64_t i, uint64_t a, uint64_t b) {
    return b - a == 1 && (fb[fo[i] + a] == '+' || fb[fo[i] + a] == '#');
  };
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t len = fo[i + 1] - fo[i];
    if (len >= (1ull << 31)) throw std::length_error("prefix_plan: filter too long");
    uint64_t a = 0;
    while (a < len && fb[fo[i] + a] != '/') ++a;
    uint64_t b = a < len ? a + 1 : a;
    while (b < len && fb[fo[i] + b] != '/') ++b;
    e0[i] = uint32_t(a);
    e1[i] = uint32_t(b);
    if (is_wild(i, 0, a)) continue;
    ++cnt0[sv(i, a)];
    ++nonroot;
  }
  // ---- hot first words are split by their second word
  std::unordered_map<std::string_view, uint64_t> parts;  // partition key -> filters
  std::unordered_map<std::string_view, bool> hot;
  for (const auto& kv : cnt0) hot[kv.first] = n_shards > 1 && kv.second * 2 * n_shards > nonroot;
  std::vector<uint8_t> repl(n, 0);  // 1: every shard
  std::vector<std::string_view> key(n);
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t len = fo[i + 1] - fo[i];
    if (is_wild(i, 0, e0[i])) {
      repl[i] = 1;
      continue;
    }
    std::string_view w0 = sv(i, e0[i]);
    if (!hot[w0]) {
      key[i] = w0;
    } else if (e0[i] == len || is_wild(i, e0[i] + 1, e1[i])) {
      repl[i] = 1;  // 'w', 'w/#', 'w/+/...': every topic under w may match it
      continue;
    } else {
      key[i] = sv(i, e1[i]);
    }
    ++parts[key[i]];
  }
  // ---- greedy assignment: largest partition first, to the least loaded shard
  std::vector<std::pair<uint64_t, std::string_view>> order;
  order.reserve(parts.size());
  for (const auto& kv : parts) order.emplace_back(kv.second, kv.first);
  std::sort(order.begin(), order.end(), [](const auto& x, const auto& y) {
    return x.first != y.first ? x.first > y.first : x.second < y.second;
  });
  std::vector<uint64_t> load(n_shards, 0);
  std::unordered_map<std::string_view, uint32_t> owner;
  for (const auto& p : order) {
    const uint32_t s = uint32_t(std::min_element(load.begin(), load.end()) - load.begin());
    owner[p.second] = s;
    load[s] += p.first;
  }
  for (uint64_t i = 0; i < n; ++i) shard_out[i] = repl[i] ? EMQX_GM_ALL_SHARDS : owner[key[i]];
  // ---- the route table: every partition key, plus each hot first word marked split
  auto* r = new emqx_gm_route;
  r->n_shards = n_shards;
  std::vector<std::pair<std::string_view, uint32_t>> keys;
  for (const auto& kv : owner) keys.emplace_back(kv.first, kv.second);
  for (const auto& kv : hot)
    if (kv.second) keys.emplace_back(kv.first, RT_SPLIT);
  std::sort(keys.begin(), keys.end());  // deterministic layout
  uint64_t cap = 16;
  while (cap < keys.size() * 4) cap <<= 1;
  r->slots.assign(cap, RouteSlot{0, RT_EMPTY, 0, 0});
  for (const auto& k : keys) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(k.first.data());
    const uint32_t len = uint32_t(k.first.size());
    const uint32_t h = rt_hash(p, len);
    uint64_t s = h & (cap - 1);
    while (r->slots[s].len != RT_EMPTY) s = (s + 1) & (cap - 1);
    r->slots[s] = RouteSlot{h, len, uint32_t(r->arena.size()), k.second};
    r->arena.insert(r->arena.end(), p, p + len);
    if (r->arena.size() >= 0xFFFFFFF0ull) throw std::length_error("prefix_plan: route keys exceed 4 GiB");
  }
  r->arena.resize(r->arena.size() + 16, 0);  // (rt_route_dev reads whole aligned u64 words)
  *out = r;
  return EMQX_GM_OK;
}

int route_topics_host(const emqx_gm_route* r, const uint8_t* tb, const uint64_t* to, uint64_t n, uint32_t* dest) {
  const uint32_t mask = uint32_t(r->slots.size() - 1);
  for (uint64_t i = 0; i < n; ++i)
    dest[i] = rt_route(r->slots.data(), mask, r->arena.data(), r->n_shards, tb + to[i], uint32_t(to[i + 1] - to[i]));
  return EMQX_GM_OK;
}

int route_topics_device(emqx_gm_ctx* ctx, emqx_gm_route* r, const uint8_t* d_tb, const uint64_t* d_to, uint64_t n,
                        uint32_t* d_dest) {
  void* dev = nullptr;
  const size_t o_arena = (r->slots.size() * sizeof(RouteSlot) + 255) & ~size_t(255);
  {
    std::lock_guard<std::mutex> lk(r->mu);
    auto it = r->dev.find(ctx->device);
    if (it == r->dev.end()) {
      GM_HIP(ctx, hipMalloc(&dev, o_arena + r->arena.size()));
      GM_HIP(ctx, hipMemcpy(dev, r->slots.data(), r->slots.size() * sizeof(RouteSlot), hipMemcpyHostToDevice));
      GM_HIP(ctx, hipMemcpy(static_cast<uint8_t*>(dev) + o_arena, r->arena.data(), r->arena.size(),
                            hipMemcpyHostToDevice));
      r->dev[ctx->device] = dev;
    } else {
      dev = it->second;
    }
  }
  if (!n) return EMQX_GM_OK;
  hipLaunchKernelGGL(k_route, dim3(uint32_t((n + 255) / 256)), dim3(256), 0, ctx->stream,
                     static_cast<const RouteSlot*>(dev), uint32_t(r->slots.size() - 1),
                     static_cast<const uint8_t*>(dev) + o_arena, r->n_shards, d_tb, d_to, n, d_dest);
  GM_HIP(ctx, hipGetLastError());
  return EMQX_GM_OK;
}

int route_partition(emqx_gm_ctx* ctx, emqx_gm_route* r, const uint8_t* d_tb, const uint64_t* d_to, uint64_t n,
                    uint32_t* d_perm, uint32_t* d_plen, uint64_t* d_split) {
  const uint32_t W = r->n_shards;
  if (W == 0 || W > 256) return set_err(ctx, EMQX_GM_EUNSUPPORTED, "route_partition: more than 256 shards");
  if (int rc = route_topics_device(ctx, r, d_tb, d_to, 0, nullptr)) return rc;  // (uploads the route table)
  const void* dev = nullptr;
  {
    std::lock_guard<std::mutex> lk(r->mu);
    dev = r->dev[ctx->device];
  }
  const size_t o_arena = (r->slots.size() * sizeof(RouteSlot) + 255) & ~size_t(255);
  hipStream_t st = ctx->stream;
  if (!n) {
    GM_HIP(ctx, hipMemsetAsync(d_split, 0, 16 * W, st));
    return EMQX_GM_OK;
  }
  const uint64_t nblk = (n + RP_B - 1) / RP_B;
  PoolBuf dest(ctx->pool, n + 16), cnt(ctx->pool, W * nblk * 8 + 8), byt(ctx->pool, W * nblk * 8 + 8),
      pos(ctx->pool, (W * nblk + 1) * 8), bpos(ctx->pool, (W * nblk + 1) * 8);
  if (!dest.p || !cnt.p || !byt.p || !pos.p || !bpos.p) return set_err(ctx, EMQX_GM_ENOMEM, "route_partition: workspace");
  hipLaunchKernelGGL(k_part_count, dim3(uint32_t(nblk)), dim3(256), 0, st, static_cast<const RouteSlot*>(dev),
                     uint32_t(r->slots.size() - 1), static_cast<const uint8_t*>(dev) + o_arena, W, d_tb, d_to, n, nblk,
                     dest.as<uint8_t>(), cnt.as<uint64_t>(), byt.as<uint64_t>());
  GM_HIP(ctx, hipGetLastError());
  if (int rc = scan_lengths(ctx, cnt.as<uint64_t>(), W * nblk, pos.as<uint64_t>())) return rc;
  if (int rc = scan_lengths(ctx, byt.as<uint64_t>(), W * nblk, bpos.as<uint64_t>())) return rc;
  hipLaunchKernelGGL(k_part_scatter, dim3(uint32_t(nblk)), dim3(256), 0, st, dest.as<uint8_t>(), d_to, n, nblk, W,
                     pos.as<uint64_t>(), d_perm, d_plen);
  GM_HIP(ctx, hipGetLastError());
  hipLaunchKernelGGL(k_part_split, dim3(1), dim3(256), 0, st, pos.as<uint64_t>(), bpos.as<uint64_t>(), nblk, W, d_split);
  GM_HIP(ctx, hipGetLastError());
  return EMQX_GM_OK;
}

void free_route(emqx_gm_route* r) {
  for (auto& kv : r->dev) {
    hipSetDevice(kv.first);
    hipFree(kv.second);
  }
  delete r;
}

int scan_lengths(emqx_gm_ctx* ctx, const uint64_t* len, uint64_t n, uint64_t* out);

int permute_topics(emqx_gm_ctx* ctx, const uint8_t* d_tb, const uint64_t* d_to, uint64_t n, const uint32_t* d_perm,
                   uint8_t* d_out, uint64_t* d_out_off) {
  if (!n) {
    GM_HIP(ctx, hipMemsetAsync(d_out_off, 0, 8, ctx->stream));
    return EMQX_GM_OK;
  }
  PoolBuf lens(ctx->pool, n * 8 + 8);
  if (!lens.p) return set_err(ctx, EMQX_GM_ENOMEM, "permute_topics: workspace");
  hipLaunchKernelGGL(k_perm_lens, dim3(uint32_t((n + 255) / 256)), dim3(256), 0, ctx->stream, d_to, d_perm, n,
                     lens.as<uint64_t>());
  GM_HIP(ctx, hipGetLastError());
  if (int rc = scan_lengths(ctx, lens.as<uint64_t>(), n, d_out_off)) return rc;
  hipLaunchKernelGGL((k_gather_segs<uint8_t, PermSeg>), dim3(gather_blocks(n)), dim3(256), 0, ctx->stream, d_tb,
                     PermSeg{d_to, d_perm}, n, d_out_off, d_out);
  GM_HIP(ctx, hipGetLastError());
  GM_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return EMQX_GM_OK;
}

}  // namespace gm
