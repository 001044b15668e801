// gm_overlay.cpp — incremental index maintenance.
//
// The reference mutates its trie in place inside mria transactions:
// emqx_router:do_add_route/2 -> emqx_router_utils:insert_trie_route/2 ->
// emqx_trie:insert/1, and do_delete_route/2 -> delete_trie_route ->
// emqx_trie:delete/1 (apps/emqx/src/emqx_router.erl:112-125, 164-172;
// emqx_router_utils.erl:33-70; emqx_trie.erl:107-136): insert is idempotent per
// topic key, delete only acts on a present key.  Here a device snapshot is
// immutable (readers may hold it, RCU): emqx_gm_index_update returns a NEW
// snapshot = the shared base snapshot minus tombstones plus a small delta
// index, and rebuilds a flat snapshot once the delta passes 1/8 of the base.
// Result rows use the ids of the updated set (lexicographic rank), exactly
// what a full rebuild would return.
#include <algorithm>
#include <cstring>
#include <set>
#include <string>

#include "gm_internal.h"

namespace gm {
namespace {

int cmp_bytes(const uint8_t* a, uint64_t la, const uint8_t* b, uint64_t lb) {
  const int c = std::memcmp(a, b, std::min(la, lb));
  if (c) return c;
  return la < lb ? -1 : la > lb ? 1 : 0;
}

// Number of base filters sorting strictly before f; *found = exact hit.
uint64_t base_rank(const emqx_gm_index* base, const uint8_t* f, uint64_t len, bool* found) {
  uint64_t lo = 0, hi = base->info.n_filters;
  while (lo < hi) {
    const uint64_t m = (lo + hi) / 2;
    const uint64_t a = base->foff[m], b = base->foff[m + 1];
    if (cmp_bytes(base->fbytes.data() + a, b - a, f, len) < 0) lo = m + 1;
    else hi = m;
  }
  *found = false;
  if (lo < base->info.n_filters) {
    const uint64_t a = base->foff[lo], b = base->foff[lo + 1];
    *found = cmp_bytes(base->fbytes.data() + a, b - a, f, len) == 0;
  }
  return lo;
}

// emqx_topic:wildcard/1 on the filter bytes
bool wildcard(const uint8_t* p, uint64_t len) {
  uint64_t ws = 0;
  for (uint64_t i = 0; i <= len; ++i) {
    if (i < len && p[i] != '/') continue;
    if (i - ws == 1 && (p[ws] == '+' || p[ws] == '#')) return true;
    ws = i + 1;
  }
  return false;
}

}  // namespace

int update_index(emqx_gm_ctx* ctx, emqx_gm_index* prev, const uint8_t* fb, const uint64_t* fo, const uint8_t* ops,
                 uint64_t n_ops, emqx_gm_index** out) {
  if (!prev || !out) return set_err(ctx, EMQX_GM_EINVAL, "index_update: NULL argument");
  if (n_ops && (!fb || !fo || !ops)) return set_err(ctx, EMQX_GM_EINVAL, "index_update: NULL op buffers");
  if (!prev->gmap.empty()) return set_err(ctx, EMQX_GM_EUNSUPPORTED, "index_update: shard index");
  emqx_gm_index* base = prev->ov ? prev->ov->base : prev;
  if (base->info.n_subs) return set_err(ctx, EMQX_GM_EUNSUPPORTED, "index_update: index with subscriber lists");
  std::set<uint32_t> tomb;
  std::set<std::string> dset;
  if (prev->ov) {
    tomb.insert(prev->ov->tomb.begin(), prev->ov->tomb.end());
    for (size_t k = 0; k + 1 < prev->ov->doff.size(); ++k)
      dset.emplace(reinterpret_cast<const char*>(prev->ov->dbytes.data() + prev->ov->doff[k]),
                   prev->ov->doff[k + 1] - prev->ov->doff[k]);
  }
  for (uint64_t i = 0; i < n_ops; ++i) {
    if (fo[i + 1] < fo[i]) return set_err(ctx, EMQX_GM_EINVAL, "index_update: offsets not monotone");
    const uint8_t* f = fb + fo[i];
    const uint64_t len = fo[i + 1] - fo[i];
    bool found;
    const uint64_t b = base_rank(base, f, len, &found);
    if (ops[i]) {  // insert (idempotent)
      if (found) tomb.erase(uint32_t(b));
      else dset.emplace(reinterpret_cast<const char*>(f), len);
    } else {  // delete (only if present)
      if (found) tomb.insert(uint32_t(b));
      else dset.erase(std::string(reinterpret_cast<const char*>(f), len));
    }
  }
  const uint64_t nb = base->info.n_filters;
  if (tomb.empty() && dset.empty()) {
    base->refs.fetch_add(1);
    *out = base;
    return EMQX_GM_OK;
  }
  if (tomb.size() + dset.size() > std::max<uint64_t>(4096, nb / 8)) {
    // compaction: a flat snapshot of the updated set
    std::vector<uint8_t> bytes;
    std::vector<uint64_t> offs{0};
    auto dit = dset.begin();
    auto tit = tomb.begin();
    for (uint64_t b = 0; b <= nb; ++b) {
      const uint8_t* bp = b < nb ? base->fbytes.data() + base->foff[b] : nullptr;
      const uint64_t bl = b < nb ? base->foff[b + 1] - base->foff[b] : 0;
      while (dit != dset.end() &&
             (b == nb || cmp_bytes(reinterpret_cast<const uint8_t*>(dit->data()), dit->size(), bp, bl) < 0)) {
        bytes.insert(bytes.end(), dit->begin(), dit->end());
        offs.push_back(bytes.size());
        ++dit;
      }
      if (b == nb) break;
      if (tit != tomb.end() && *tit == b) {
        ++tit;
        continue;
      }
      bytes.insert(bytes.end(), bp, bp + bl);
      offs.push_back(bytes.size());
    }
    bytes.resize(bytes.size() + 64, 0);
    return build_index(ctx, bytes.data(), offs.data(), offs.size() - 1, nullptr, nullptr, nullptr, out);
  }
  auto* idx = new emqx_gm_index;
  idx->device = base->device;
  auto* ov = new OverlayState;
  idx->ov = ov;
  base->refs.fetch_add(1);
  ov->base = base;
  ov->tomb.assign(tomb.begin(), tomb.end());
  ov->doff.push_back(0);
  uint64_t dwild = 0;
  for (const std::string& d : dset) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(d.data());
    bool found;
    const uint32_t ip = uint32_t(base_rank(base, p, d.size(), &found));
    const uint32_t k = uint32_t(ov->ins.size());
    const uint32_t dead_below = uint32_t(std::lower_bound(ov->tomb.begin(), ov->tomb.end(), ip) - ov->tomb.begin());
    ov->ins.push_back(ip);
    ov->dgid.push_back(k + ip - dead_below);
    ov->dbytes.insert(ov->dbytes.end(), d.begin(), d.end());
    ov->doff.push_back(ov->dbytes.size());
    dwild += wildcard(p, d.size());
  }
  const uint64_t K = ov->ins.size();
  if (K) {
    std::vector<uint8_t> padded(ov->dbytes);
    padded.resize(padded.size() + 64, 0);
    const int rc = build_index(ctx, padded.data(), ov->doff.data(), K, nullptr, nullptr, nullptr, &ov->delta, nullptr,
                               ov->dgid.data());
    if (rc) {
      free_index(idx);
      return rc;
    }
  }
  // device: tombstone bitmap over base ids, its exclusive word prefix counts, insertion points
  const uint64_t words = nb / 32 + 1;
  std::vector<uint32_t> tbm(words, 0), tpre(words, 0);
  uint64_t twild = 0;
  for (uint32_t b : ov->tomb) {
    tbm[b >> 5] |= 1u << (b & 31);
    twild += wildcard(base->fbytes.data() + base->foff[b], base->foff[b + 1] - base->foff[b]);
  }
  for (uint64_t w = 1; w < words; ++w) tpre[w] = tpre[w - 1] + uint32_t(__builtin_popcount(tbm[w - 1]));
  const size_t bytes = (2 * words + K + 1) * 4;
  hipError_t e = hipMalloc(&ov->dev, bytes);
  uint32_t* D = static_cast<uint32_t*>(ov->dev);
  if (e == hipSuccess) e = hipMemcpy(D, tbm.data(), words * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(D + words, tpre.data(), words * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess && K) e = hipMemcpy(D + 2 * words, ov->ins.data(), K * 4, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    free_index(idx);
    return set_err(ctx, EMQX_GM_ENOMEM, std::string("index_update: device tables: ") + hipGetErrorString(e));
  }
  ov->d_tbm = D;
  ov->d_tpre = D + words;
  ov->d_ins = D + 2 * words;
  emqx_gm_index_info_t& in = idx->info;
  in = base->info;
  in.n_filters = nb - ov->tomb.size() + K;
  in.n_wildcard = base->info.n_wildcard - twild + dwild;
  in.trie_empty = in.n_wildcard == 0;
  in.device_bytes = base->info.device_bytes + bytes;
  if (ov->delta) {
    in.n_nodes += ov->delta->info.n_nodes;
    in.n_edges += ov->delta->info.n_edges;
    in.n_words += ov->delta->info.n_words;
    in.device_bytes += ov->delta->info.device_bytes;
    in.max_depth = std::max(in.max_depth, ov->delta->info.max_depth);
  }
  *out = idx;
  return EMQX_GM_OK;
}

// Bytes of final id `id`: a delta filter, or the surviving base filter b with
// b - tombstones_below(b) + delta_before(b) == id.
int overlay_filter(const emqx_gm_index* idx, uint32_t id, const uint8_t** bytes, uint64_t* len) {
  const OverlayState& ov = *idx->ov;
  if (id >= idx->info.n_filters) return EMQX_GM_EINVAL;
  auto dg = std::lower_bound(ov.dgid.begin(), ov.dgid.end(), id);
  if (dg != ov.dgid.end() && *dg == id) {
    const size_t k = size_t(dg - ov.dgid.begin());
    *bytes = ov.dbytes.data() + ov.doff[k];
    *len = ov.doff[k + 1] - ov.doff[k];
    return EMQX_GM_OK;
  }
  const emqx_gm_index* base = ov.base;
  auto final_id = [&](uint64_t b) -> uint64_t {
    const uint64_t dead = uint64_t(std::lower_bound(ov.tomb.begin(), ov.tomb.end(), uint32_t(b)) - ov.tomb.begin());
    const uint64_t before = uint64_t(std::upper_bound(ov.ins.begin(), ov.ins.end(), uint32_t(b)) - ov.ins.begin());
    return b - dead + before;
  };
  uint64_t lo = 0, hi = base->info.n_filters;  // smallest live b with final_id(b) >= id
  while (lo < hi) {
    const uint64_t m = (lo + hi) / 2;
    if (final_id(m) < id) lo = m + 1;
    else hi = m;
  }
  while (lo < base->info.n_filters && std::binary_search(ov.tomb.begin(), ov.tomb.end(), uint32_t(lo))) ++lo;
  if (lo >= base->info.n_filters || final_id(lo) != id) return EMQX_GM_EINVAL;
  *bytes = base->fbytes.data() + base->foff[lo];
  *len = base->foff[lo + 1] - base->foff[lo];
  return EMQX_GM_OK;
}

void free_overlay(emqx_gm_index* idx) {
  OverlayState* ov = idx->ov;
  idx->ov = nullptr;
  if (ov->dev) {
    hipSetDevice(idx->device);
    hipFree(ov->dev);
  }
  if (ov->delta && ov->delta->refs.fetch_sub(1) == 1) free_index(ov->delta);
  if (ov->base && ov->base->refs.fetch_sub(1) == 1) free_index(ov->base);
  delete ov;
}

}  // namespace gm
