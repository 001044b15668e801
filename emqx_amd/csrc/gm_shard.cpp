// gm_shard.cpp — a prefix-sharded index behind the C ABI (emqx_gm_index_build_sharded):
// SURVEY.md §8e C5's sharded form for a filter set too large for one GPU,
// reachable from ONE multi-device context -- the NIF's form -- instead of
// only from Python over torch.distributed (emqx_amd/sharded.py).
//
// The reference keeps one routing table per node and has no sharded trie
// (apps/emqx/src/emqx_router.erl:75-84); what makes sharding exact here is
// emqx_topic:match/2 (apps/emqx/src/emqx_topic.erl:65-87): a topic can only
// match filters whose first word is its own first word, '+' or '#'.  So
// emqx_gm_prefix_plan (gm_route.hip) partitions the filters by first word (a
// hot first word by its first two) over the context's devices, puts the
// filters beginning with '+' / '#' on every device, and routes each topic to
// the ONE device that holds every filter it can match:
//   build   the shards compiled at once (one host thread and one device each),
//           each with the global ids of its filters (rows come out in global
//           order: a shard's local order is the global one);
//   match   host buffers: every topic routed (all threads), each device's
//           topics gathered into a batch of its own, matched there (the
//           host-buffer pipeline of gm_host.cpp, all devices at once), and every
//           row put back at its topic's place in ONE result CSR -- nothing is
//           merged: a row comes from one shard whole;
//   fan-out host rows: each row goes to the shard of its filters (all on the
//           row's topic's shard, or on every shard), its global ids mapped to
//           that shard's local ones, fanned out there, and put back in order.
// Updates, images and device-buffer calls on a sharded index are refused
// (EMQX_GM_EUNSUPPORTED): a global id shifts on every shard when any filter
// is added, so a sharded set is rebuilt.
#include <algorithm>
#include <cstring>
#include <memory>
#include <numeric>
#include <thread>

#include "gm_internal.h"

namespace gm {

namespace {

unsigned host_threads() { return std::max(1u, std::min(16u, std::thread::hardware_concurrency())); }

// f(a, b) over [0, n) in up to host_threads() ranges at once
template <class F> void parallel_ranges(uint64_t n, uint64_t min_per, F f) {
  const unsigned T = n < 2 * min_per ? 1u : unsigned(std::min<uint64_t>(host_threads(), n / min_per));
  std::vector<std::thread> th;
  for (unsigned r = 1; r < T; ++r) th.emplace_back([&, r] { f(n * r / T, n * (r + 1) / T); });
  f(0, n / T);
  for (auto& t : th) t.join();
}

// emqx_topic:wildcard/1 on the filter bytes
bool is_wild(const uint8_t* p, uint64_t len) {
  uint64_t ws = 0;
  for (uint64_t i = 0; i <= len; ++i) {
    if (i < len && p[i] != '/') continue;
    if (i - ws == 1 && (p[ws] == '+' || p[ws] == '#')) return true;
    ws = i + 1;
  }
  return false;
}

std::vector<emqx_gm_ctx*> devices_of(emqx_gm_ctx* ctx) {
  std::vector<emqx_gm_ctx*> mem{ctx};
  for (emqx_gm_ctx* m : ctx->members) mem.push_back(m);
  return mem;
}

// a device's lock while its shard works (the first device's is the caller's)
struct MemberLock {
  std::unique_lock<std::recursive_mutex> lk;
  explicit MemberLock(emqx_gm_ctx* c) : lk(c->mu, std::defer_lock) {
    if (c->parent) lk.lock();
    hipSetDevice(c->device);
  }
};

}  // namespace

int build_sharded(emqx_gm_ctx* ctx, const uint8_t* fb, const uint64_t* fo, uint64_t n, const uint64_t* sub_off,
                  const uint32_t* sub_ids, uint32_t* perm_out, emqx_gm_index** out) {
  if (!out) return set_err(ctx, EMQX_GM_EINVAL, "index_build_sharded: out is NULL");
  if (n && (!fb || !fo)) return set_err(ctx, EMQX_GM_EINVAL, "index_build_sharded: NULL filter buffers");
  if (n >= 0x7FFFFFFFull) return set_err(ctx, EMQX_GM_EINVAL, "index_build_sharded: too many filters");
  if (sub_off && !sub_ids && n && sub_off[n] > 0)
    return set_err(ctx, EMQX_GM_EINVAL, "index_build_sharded: sub_ids is NULL");
  for (uint64_t i = 0; i < n; ++i)
    if (fo[i + 1] < fo[i] || (sub_off && sub_off[i + 1] < sub_off[i]))
      return set_err(ctx, EMQX_GM_EINVAL, "index_build_sharded: offsets not monotone");
  const std::vector<emqx_gm_ctx*> mem = devices_of(ctx);
  const int K = int(mem.size());
  // ---- global ids: the rank of each unique filter (what an unsharded build assigns)
  std::vector<uint32_t> ord(n);
  std::iota(ord.begin(), ord.end(), 0u);
  sort_filters(ord, fb, fo);
  std::vector<uint32_t> gid(n);
  auto sf = std::make_shared<SortedFilters>();  // (off starts as {0})
  for (uint64_t k = 0; k < n; ++k) {
    const uint32_t i = ord[k];
    const uint64_t li = fo[i + 1] - fo[i];
    bool dup = false;
    if (k) {
      const uint32_t p = ord[k - 1];
      dup = fo[p + 1] - fo[p] == li && std::memcmp(fb + fo[p], fb + fo[i], li) == 0;
    }
    if (!dup) {
      sf->bytes.insert(sf->bytes.end(), fb + fo[i], fb + fo[i] + li);
      sf->off.push_back(sf->bytes.size());
    }
    gid[i] = uint32_t(sf->off.size() - 2);
  }
  const uint64_t nf = sf->off.size() - 1;
  std::vector<uint32_t>().swap(ord);
  if (perm_out)
    for (uint64_t i = 0; i < n; ++i) perm_out[i] = gid[i];
  // ---- the plan: each filter's device (EMQX_GM_ALL_SHARDS: every one)
  std::vector<uint32_t> shard(n ? n : 1);
  emqx_gm_route* route = nullptr;
  if (const int rc = route_plan(fb, fo, n, uint32_t(K), shard.data(), &route)) return set_err(ctx, rc, "index_build_sharded: prefix plan");
  std::unique_ptr<emqx_gm_index> idx(new emqx_gm_index);
  idx->device = ctx->device;
  idx->route = route;
  idx->fshard.assign(nf, 0);
  for (uint64_t i = 0; i < n; ++i) idx->fshard[gid[i]] = shard[i];
  // ---- the shards, compiled and placed at once (each its own host thread and device)
  idx->shards.assign(K, nullptr);
  const int rc = run_all(K, [&](int k) -> int {
    MemberLock lk(mem[k]);
    std::vector<uint8_t> b;
    std::vector<uint64_t> o{0}, so{0};
    std::vector<uint32_t> g, si;
    for (uint64_t i = 0; i < n; ++i) {
      if (shard[i] != uint32_t(k) && shard[i] != EMQX_GM_ALL_SHARDS) continue;
      b.insert(b.end(), fb + fo[i], fb + fo[i + 1]);
      o.push_back(b.size());
      g.push_back(gid[i]);
      if (sub_off) {
        si.insert(si.end(), sub_ids + sub_off[i], sub_ids + sub_off[i + 1]);
        so.push_back(si.size());
      }
    }
    b.resize(b.size() + 64, 0);
    if (si.empty()) si.push_back(0);
    std::vector<uint32_t> perm(g.size() + 1);
    return build_index(mem[k], b.data(), o.data(), g.size(), sub_off ? so.data() : nullptr, sub_off ? si.data() : nullptr,
                       perm.data(), &idx->shards[k], nullptr, g.empty() ? nullptr : g.data());
  });
  hipSetDevice(ctx->device);
  if (rc) {
    free_index(idx.release());
    return rc;
  }
  // ---- the host side: the global filter table and counts
  idx->ft.set_base(sf);
  emqx_gm_index_info_t& in = idx->info;
  in.n_filters = nf;
  for (uint64_t f = 0; f < nf; ++f) in.n_wildcard += is_wild(sf->bytes.data() + sf->off[f], sf->off[f + 1] - sf->off[f]);
  in.trie_empty = in.n_wildcard == 0;
  for (emqx_gm_index* s : idx->shards) {
    in.n_nodes += s->info.n_nodes;
    in.n_edges += s->info.n_edges;
    in.n_words = std::max(in.n_words, s->info.n_words);
    in.device_bytes += s->info.device_bytes;
    in.max_depth = std::max(in.max_depth, s->info.max_depth);
  }
  if (sub_off) {  // per global id: its subscribers (duplicates' lists concatenated), as a build counts them
    std::vector<uint64_t> so(nf + 1, 0);
    for (uint64_t i = 0; i < n; ++i) so[gid[i] + 1] += sub_off[i + 1] - sub_off[i];
    for (uint64_t f = 0; f < nf; ++f) so[f + 1] += so[f];
    in.n_subs = so[nf];
    idx->subs = SubTable(std::move(so), {});
  }
  *out = idx.release();
  return EMQX_GM_OK;
}

int run_match_sharded(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const uint8_t* tb, const uint64_t* to, uint64_t n,
                      uint32_t flags, emqx_gm_csr* out) {
  const std::vector<emqx_gm_ctx*> mem = devices_of(ctx);
  const int K = int(idx->shards.size());
  if (K > int(mem.size())) return set_err(ctx, EMQX_GM_EINVAL, "match: a sharded index of another context");
  // ---- every topic's device (offsets checked first: the route reads each topic)
  std::atomic<int> bad{0};
  parallel_ranges(n, 1 << 16, [&](uint64_t a, uint64_t b) {
    for (uint64_t i = a; i < b; ++i)
      if (to[i + 1] < to[i]) bad.store(1);
  });
  if (bad.load()) return set_err(ctx, EMQX_GM_EINVAL, "match: topic offsets not monotone");
  std::vector<uint32_t> dest(n);
  parallel_ranges(n, 1 << 16, [&](uint64_t a, uint64_t b) { route_topics_host(idx->route, tb, to + a, b - a, dest.data() + a); });
  // ---- each device's topics, in batch order (a stable counting sort)
  std::vector<uint64_t> cnt(K + 1, 0);
  for (uint64_t i = 0; i < n; ++i) ++cnt[dest[i] + 1];
  for (int k = 0; k < K; ++k) cnt[k + 1] += cnt[k];
  std::vector<uint64_t> pos(n), fill(cnt.begin(), cnt.end() - 1);
  std::vector<uint32_t> order(n);
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t p = fill[dest[i]]++;
    order[p] = uint32_t(i);
    pos[i] = p - cnt[dest[i]];  // its row in its device's result
  }
  // ---- each device gathers and matches its batch (all at once)
  struct Part {
    std::vector<uint8_t> b;
    std::vector<uint64_t> o;
    emqx_gm_csr res{};
    emqx_gm_match_stats st{};
  };
  std::vector<Part> P(K);
  const int rc = run_all(K, [&](int k) -> int {
    MemberLock lk(mem[k]);
    Part& p = P[k];
    const uint64_t a = cnt[k], m = cnt[k + 1] - a;
    p.o.resize(m + 1);
    p.o[0] = 0;
    for (uint64_t j = 0; j < m; ++j) p.o[j + 1] = p.o[j] + (to[order[a + j] + 1] - to[order[a + j]]);
    p.b.resize(p.o[m] + 64);
    for (uint64_t j = 0; j < m; ++j) {
      const uint32_t i = order[a + j];
      if (to[i + 1] > to[i]) std::memcpy(p.b.data() + p.o[j], tb + to[i], to[i + 1] - to[i]);
    }
    const int r = run_match_host(mem[k], idx->shards[k], p.b.data(), p.o.data(), m, flags & ~EMQX_GM_DEVICE_IO, &p.res);
    p.st = mem[k]->stats;
    return r;
  });
  hipSetDevice(ctx->device);
  auto drop = [&]() {
    for (int k = 0; k < K; ++k)
      if (P[k].res.row_off || P[k].res.ids) {
        MemberLock lk(mem[k]);
        mem[k]->hpool->release(P[k].res.row_off);
        mem[k]->hpool->release(P[k].res.ids);
      }
    hipSetDevice(ctx->device);
  };
  if (rc) {
    drop();
    return rc;
  }
  // ---- every row back at its topic's place
  uint64_t total = 0;
  for (auto& p : P) total += p.res.nnz;
  uint64_t* r_off = static_cast<uint64_t*>(ctx->hpool->alloc((n + 1) * 8));
  uint32_t* r_ids = static_cast<uint32_t*>(ctx->hpool->alloc(total * 4 + 16));
  if (!r_off || !r_ids) {
    ctx->hpool->release(r_off);
    ctx->hpool->release(r_ids);
    drop();
    return set_err(ctx, EMQX_GM_ENOMEM, "match: host result");
  }
  r_off[0] = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t* ro = P[dest[i]].res.row_off;
    r_off[i + 1] = r_off[i] + (ro[pos[i] + 1] - ro[pos[i]]);
  }
  parallel_ranges(n, 1 << 16, [&](uint64_t a, uint64_t b) {
    for (uint64_t i = a; i < b; ++i) {
      const emqx_gm_csr& s = P[dest[i]].res;
      const uint64_t l = r_off[i + 1] - r_off[i];
      if (l) std::memcpy(r_ids + r_off[i], s.ids + s.row_off[pos[i]], l * 4);
    }
  });
  drop();
  emqx_gm_match_stats tot{};
  tot.n_topics = n;
  tot.nnz = total;
  for (auto& p : P) {
    tot.n_overflow += p.st.n_overflow;
    tot.n_wildcard_topics += p.st.n_wildcard_topics;
    tot.probes += p.st.probes;
    tot.match_kernel_ms = std::max(tot.match_kernel_ms, p.st.match_kernel_ms);
    tot.total_device_ms = std::max(tot.total_device_ms, p.st.total_device_ms);
  }
  ctx->stats = tot;
  out->n_rows = n;
  out->nnz = total;
  out->row_off = r_off;
  out->ids = r_ids;
  out->on_device = 0;
  out->priv = ctx;
  return EMQX_GM_OK;
}

int run_fanout_sharded(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const emqx_gm_csr* m, uint32_t flags,
                       emqx_gm_csr* out) {
  const std::vector<emqx_gm_ctx*> mem = devices_of(ctx);
  const int K = int(idx->shards.size());
  if (K > int(mem.size())) return set_err(ctx, EMQX_GM_EINVAL, "fanout: a sharded index of another context");
  const uint64_t n = m->n_rows, nnz = m->nnz, nf = idx->info.n_filters;
  if (m->row_off[0] != 0 || m->row_off[n] != nnz) return set_err(ctx, EMQX_GM_EINVAL, "fanout: row offsets");
  for (uint64_t i = 0; i < n; ++i)
    if (m->row_off[i + 1] < m->row_off[i]) return set_err(ctx, EMQX_GM_EINVAL, "fanout: row offsets not monotone");
  for (uint64_t j = 0; j < nnz; ++j)
    if (m->ids[j] >= nf) return set_err(ctx, EMQX_GM_EINVAL, "fanout: filter id out of range");
  // ---- each row's shard: that of its first filter held by one shard (a row's
  // filters all live on its topic's shard, or on every shard)
  std::vector<uint32_t> dest(n);
  for (uint64_t i = 0; i < n; ++i) {
    uint32_t s = 0;
    for (uint64_t j = m->row_off[i]; j < m->row_off[i + 1]; ++j)
      if (idx->fshard[m->ids[j]] != EMQX_GM_ALL_SHARDS) {
        s = idx->fshard[m->ids[j]];
        break;
      }
    dest[i] = s;
  }
  std::vector<uint64_t> cnt(K + 1, 0);
  for (uint64_t i = 0; i < n; ++i) ++cnt[dest[i] + 1];
  for (int k = 0; k < K; ++k) cnt[k + 1] += cnt[k];
  std::vector<uint64_t> pos(n), fill(cnt.begin(), cnt.end() - 1);
  std::vector<uint32_t> order(n);
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t p = fill[dest[i]]++;
    order[p] = uint32_t(i);
    pos[i] = p - cnt[dest[i]];
  }
  struct Part {
    std::vector<uint64_t> o;
    std::vector<uint32_t> ids;
    emqx_gm_csr res{};
  };
  std::vector<Part> P(K);
  const int rc = run_all(K, [&](int k) -> int {
    MemberLock lk(mem[k]);
    Part& p = P[k];
    const emqx_gm_index* s = idx->shards[k];
    const uint64_t a = cnt[k], r = cnt[k + 1] - a;
    p.o.assign(1, 0);
    for (uint64_t q = 0; q < r; ++q) {
      const uint32_t i = order[a + q];
      for (uint64_t j = m->row_off[i]; j < m->row_off[i + 1]; ++j) {  // global id -> the shard's local id
        auto it = std::lower_bound(s->gmap.begin(), s->gmap.end(), m->ids[j]);
        if (it == s->gmap.end() || *it != m->ids[j])
          return set_err(mem[k], EMQX_GM_EINVAL, "fanout: a row's filters are not on one shard");
        p.ids.push_back(uint32_t(it - s->gmap.begin()));
      }
      p.o.push_back(p.ids.size());
    }
    if (p.ids.empty()) p.ids.push_back(0);
    emqx_gm_csr sub{};
    sub.n_rows = r;
    sub.nnz = p.o.back();
    sub.row_off = p.o.data();
    sub.ids = p.ids.data();
    sub.on_device = 0;
    return run_fanout(mem[k], s, &sub, flags & EMQX_GM_WITH_EXACT, &p.res);
  });
  hipSetDevice(ctx->device);
  auto drop = [&]() {
    for (int k = 0; k < K; ++k)
      if (P[k].res.row_off || P[k].res.ids) {
        MemberLock lk(mem[k]);
        mem[k]->hpool->release(P[k].res.row_off);
        mem[k]->hpool->release(P[k].res.ids);
      }
    hipSetDevice(ctx->device);
  };
  if (rc) {
    drop();
    return rc;
  }
  uint64_t total = 0;
  for (auto& p : P) total += p.res.nnz;
  uint64_t* r_off = static_cast<uint64_t*>(ctx->hpool->alloc((n + 1) * 8));
  uint32_t* r_ids = static_cast<uint32_t*>(ctx->hpool->alloc(total * 4 + 16));
  if (!r_off || !r_ids) {
    ctx->hpool->release(r_off);
    ctx->hpool->release(r_ids);
    drop();
    return set_err(ctx, EMQX_GM_ENOMEM, "fanout: host result");
  }
  r_off[0] = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t* ro = P[dest[i]].res.row_off;
    r_off[i + 1] = r_off[i] + (ro[pos[i] + 1] - ro[pos[i]]);
  }
  parallel_ranges(n, 1 << 16, [&](uint64_t a, uint64_t b) {
    for (uint64_t i = a; i < b; ++i) {
      const emqx_gm_csr& s = P[dest[i]].res;
      const uint64_t l = r_off[i + 1] - r_off[i];
      if (l) std::memcpy(r_ids + r_off[i], s.ids + s.row_off[pos[i]], l * 4);
    }
  });
  drop();
  emqx_gm_match_stats tot{};
  tot.n_topics = n;
  tot.nnz = total;
  ctx->stats = tot;
  out->n_rows = n;
  out->nnz = total;
  out->row_off = r_off;
  out->ids = r_ids;
  out->on_device = 0;
  out->priv = ctx;
  return EMQX_GM_OK;
}

}  // namespace gm
