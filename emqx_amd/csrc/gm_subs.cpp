// gm_subs.cpp — subscriber maintenance on an index with subscriber lists
// (SURVEY.md §8a a10 writes, §8f rank 1).
//
// The reference: emqx_broker:subscribe/2 inserts {Topic, SubPid} into the
// emqx_subscriber bag (sharded past 1,024 subscribers) and, for a topic's
// first subscriber, adds its route (emqx_router:do_add_route/2);
// unsubscribe/1 deletes the pair and, after the last one, the route
// (apps/emqx/src/emqx_broker.erl:147-165, 445-454; emqx_broker_helper.erl:
// 82-91; emqx_router.erl:112-125, 164-172).  Here one call applies a batch of
// (filter, subscriber, subscribe | unsubscribe) ops and returns a NEW snapshot
// (RCU, like emqx_gm_index_update):
//   * each touched filter's list is read back, edited on the host (a pair is
//     present at most once; a subscribe appends, an unsubscribe removes the
//     pair and keeps the others' order);
//   * route changes (first subscriber / last one gone) go through the in-place
//     trie patch (gm_overlay.cpp, patch_update);
//   * the new snapshot gets a subscriber CSR of its own, written on the device
//     (gm_match.hip, rebuild_subs_device): untouched filters' lists copied from
//     the previous CSR through the id renumbering, touched ones from the host.
// Anything the patch cannot take (no room, a filter with '#' inside, a
// snapshot that is no longer the newest) rebuilds the index from the full
// lists.
#include <algorithm>
#include <cstring>
#include <functional>
#include <map>
#include <string>
#include <unordered_map>

#include "gm_internal.h"

namespace gm {
namespace {

struct FilterEdit {
  uint32_t old_id = NONE;  // the filter's id in prev, or NONE
  bool had_subs = false;
  bool was_pinned = false;  // prev holds the filter's route for another destination
  int pin = -1;             // route_add (1) / route_delete (0) ops seen; -1: unchanged
  std::vector<uint32_t> list;                    // prev's list, then appended subscribers
  std::vector<uint8_t> dead;                     // per list entry: unsubscribed
  std::unordered_map<uint32_t, uint64_t> where;  // subscriber -> its live entry

  void subscribe(uint32_t s) {
    auto it = where.find(s);
    if (it != where.end() && !dead[it->second]) return;  // already subscribed (bag: one pair)
    where[s] = list.size();
    list.push_back(s);
    dead.push_back(0);
  }
  void unsubscribe(uint32_t s) {
    auto it = where.find(s);
    if (it == where.end() || dead[it->second]) return;  // only if present
    dead[it->second] = 1;
  }
  bool pinned() const { return pin < 0 ? was_pinned : pin != 0; }
  bool live() const {
    for (uint8_t d : dead)
      if (!d) return true;
    return false;
  }
  // the filter stays a route while a local subscriber or another destination holds it
  bool present() const { return live() || pinned(); }
  std::vector<uint32_t> final_list() const {
    std::vector<uint32_t> o;
    o.reserve(list.size());
    for (size_t i = 0; i < list.size(); ++i)
      if (!dead[i]) o.push_back(list[i]);
    return o;
  }
};


// Fallback: the updated set rebuilt from full host lists.
int rebuild(emqx_gm_ctx* ctx, const emqx_gm_index* prev, const std::map<std::string, FilterEdit>& ed,
            emqx_gm_index** out) {
  std::vector<uint8_t> pin_in;  // per input filter, in the order they are added below
  const uint64_t nb = prev->info.n_filters;
  std::vector<uint32_t> all(prev->subs.total());
  if (!all.empty())
    GM_HIP(ctx, hipMemcpy(all.data(), prev->view.sub_ids, all.size() * 4, hipMemcpyDeviceToHost));
  std::vector<const FilterEdit*> edit_of(nb, nullptr);
  for (const auto& kv : ed)
    if (kv.second.old_id != NONE) edit_of[kv.second.old_id] = &kv.second;
  std::vector<uint8_t> fb;
  std::vector<uint64_t> fo{0}, so{0};
  std::vector<uint32_t> si;
  auto add = [&](const uint8_t* p, uint64_t len, const uint32_t* l, uint64_t cnt, bool pinned) {
    pin_in.push_back(pinned ? 1 : 0);
    fb.insert(fb.end(), p, p + len);
    fo.push_back(fb.size());
    si.insert(si.end(), l, l + cnt);
    so.push_back(si.size());
  };
  prev->ft.for_each([&](uint64_t f, const uint8_t* p, uint64_t len) {
    if (const FilterEdit* e = edit_of[f]) {
      if (!e->present()) return;  // the last subscriber left and no other destination: the route goes
      const std::vector<uint32_t> l = e->final_list();
      add(p, len, l.data(), l.size(), e->pinned());
    } else {
      add(p, len, all.data() + prev->subs.off(f), prev->subs.count(f), is_pinned(prev, f));
    }
  });
  for (const auto& kv : ed)
    if (kv.second.old_id == NONE && kv.second.present()) {
      const std::vector<uint32_t> l = kv.second.final_list();
      add(reinterpret_cast<const uint8_t*>(kv.first.data()), kv.first.size(), l.data(), l.size(), kv.second.pinned());
    }
  fb.resize(fb.size() + 64, 0);
  if (si.empty()) si.push_back(0);
  std::vector<uint32_t> perm(pin_in.size() + 1);
  const int rc = build_index(ctx, fb.data(), fo.data(), fo.size() - 1, so.data(), si.data(), perm.data(), out);
  if (rc) return rc;
  std::vector<uint8_t> marks((*out)->info.n_filters, 0);
  for (size_t i = 0; i < pin_in.size(); ++i) marks[perm[i]] = pin_in[i];
  (*out)->subs = SubTable((*out)->subs.offsets(), std::move(marks));
  return 0;
}

}  // namespace

bool is_pinned(const emqx_gm_index* idx, uint64_t f) {
  // (built: a filter without subscribers is route-only; gm_filters.h SubTable)
  return idx->subs.empty() || idx->subs.pinned(f);
}

int update_subs(emqx_gm_ctx* ctx, emqx_gm_index* prev, const uint8_t* fb, const uint64_t* fo, const uint32_t* subs,
                const uint8_t* ops, uint64_t n_ops, emqx_gm_index** out) {
  if (!prev || !out) return set_err(ctx, EMQX_GM_EINVAL, "index_update_subs: NULL argument");
  if (n_ops && (!fb || !fo || !subs || !ops)) return set_err(ctx, EMQX_GM_EINVAL, "index_update_subs: NULL op buffers");
  if (prev->ov) return set_err(ctx, EMQX_GM_EUNSUPPORTED, "index_update_subs: overlay snapshot");
  if (!prev->gmap.empty()) return set_err(ctx, EMQX_GM_EUNSUPPORTED, "index_update_subs: shard index");
  if (prev->subs.empty())
    return set_err(ctx, EMQX_GM_EUNSUPPORTED,
                   "index_update_subs: index without subscriber lists (route updates: emqx_gm_index_update)");
  for (uint64_t i = 0; i < n_ops; ++i)
    if (fo[i + 1] < fo[i]) return set_err(ctx, EMQX_GM_EINVAL, "index_update_subs: offsets not monotone");
  // ---- the touched filters, their current lists read back in one device gather
  std::map<std::string, FilterEdit> ed;  // filter bytes -> edit (byte order: the new filters' order)
  std::vector<FilterEdit*> by_op(n_ops);
  for (uint64_t i = 0; i < n_ops; ++i) {
    const uint8_t* f = fb + fo[i];
    const uint64_t len = fo[i + 1] - fo[i];
    auto ins = ed.try_emplace(std::string(reinterpret_cast<const char*>(f), len));
    if (ins.second) {
      bool found;
      const uint64_t r = filter_rank(prev, f, len, &found);
      if (found) ins.first->second.old_id = uint32_t(r);
    }
    by_op[i] = &ins.first->second;
  }
  {
    std::vector<FilterEdit*> touched;
    std::vector<uint64_t> src_off, dst_off{0};
    for (auto& kv : ed)
      if (kv.second.old_id != NONE) {
        const uint32_t id = kv.second.old_id;
        touched.push_back(&kv.second);
        src_off.push_back(prev->subs.off(id));
        dst_off.push_back(dst_off.back() + prev->subs.count(id));
      }
    std::vector<uint32_t> all(dst_off.back());
    if (!all.empty()) {
      const int rc = gather_segments(ctx, prev->view.sub_ids, src_off, dst_off, all.data());
      if (rc) return rc;
    }
    for (size_t j = 0; j < touched.size(); ++j) {
      FilterEdit& e = *touched[j];
      e.list.assign(all.begin() + dst_off[j], all.begin() + dst_off[j + 1]);
      e.had_subs = !e.list.empty();
      e.was_pinned = is_pinned(prev, e.old_id);
      e.dead.assign(e.list.size(), 0);
      for (uint64_t k = 0; k < e.list.size(); ++k) e.where[e.list[k]] = k;
    }
  }
  // ---- the ops, in order
  for (uint64_t i = 0; i < n_ops; ++i) {
    switch (ops[i]) {
      case EMQX_GM_SUB_UNSUBSCRIBE: by_op[i]->unsubscribe(subs[i]); break;
      case EMQX_GM_SUB_SUBSCRIBE: by_op[i]->subscribe(subs[i]); break;
      case EMQX_GM_SUB_ROUTE_ADD: by_op[i]->pin = 1; break;
      case EMQX_GM_SUB_ROUTE_DELETE: by_op[i]->pin = 0; break;
      default: return set_err(ctx, EMQX_GM_EINVAL, "index_update_subs: op kind");
    }
  }
  // ---- route changes: a first subscriber adds the route, the last one leaving deletes it
  std::set<uint32_t> tomb;
  std::set<std::string> dset;
  bool wf = true;
  for (const auto& kv : ed) {
    const bool present = kv.second.present();
    if (kv.second.old_id == NONE && present) {
      dset.insert(kv.first);
      wf = wf && well_formed_filter(reinterpret_cast<const uint8_t*>(kv.first.data()), kv.first.size());
    } else if (kv.second.old_id != NONE && !present) {
      tomb.insert(kv.second.old_id);
    }
  }
  const uint64_t nb = prev->info.n_filters;
  emqx_gm_index* idx = nullptr;
  std::vector<uint32_t> rmap;
  int rc = 1;
  bool same_routes = false;
  // a multi-device context: every member applies the same batch to its replica
  // of prev, on its own device, at the same time as the first device
  std::vector<RepTarget> reps = rep_targets(ctx, prev);
  auto locked = [](emqx_gm_ctx* c, const std::function<int()>& f) {
    std::unique_lock<std::recursive_mutex> lk(c->mu, std::defer_lock);
    if (c->parent) lk.lock();  // (a member: small calls hold only its lock)
    hipSetDevice(c->device);
    return f();
  };
  auto drop_reps = [&]() {
    for (auto& t : reps)
      if (t.out) {
        free_index(t.out);
        t.out = nullptr;
      }
  };
  {
    std::unique_lock<std::mutex> lk(prev->mirror_mu);
    if (tomb.empty() && dset.empty()) {
      // No route changed (a subscriber-only batch): the new snapshot shares
      // prev's tables (retained; the mirror, if any, moves on with it) and its
      // filter ids; only the subscriber CSR is new.  O(delta) on the host.
      idx = new emqx_gm_index;
      idx->device = prev->device;
      idx->dev_base = prev->dev_base;
      idx->dev_bytes = prev->dev_bytes;
      emqx_gm_index* owner = prev->blob_owner ? prev->blob_owner : prev;
      owner->refs.fetch_add(1);
      idx->blob_owner = owner;
      idx->view = prev->view;
      idx->info = prev->info;
      idx->info.device_bytes = prev->dev_bytes;  // the tables; the new CSR is added below
      idx->ft = prev->ft;
      idx->gmap = prev->gmap;
      idx->dev_flen = prev->dev_flen;
      idx->flen_stale = prev->flen_stale.load();
      idx->level_nodes = prev->level_nodes;
      idx->mirror = prev->mirror;
      prev->mirror = nullptr;
      for (auto& t : reps) {  // each replica shares its predecessor replica's tables the same way
        emqx_gm_index* r = replica_shell(t.m, idx);
        emqx_gm_index* rown = t.prev->blob_owner ? t.prev->blob_owner : t.prev;
        rown->refs.fetch_add(1);
        r->blob_owner = rown;
        r->dev_base = t.prev->dev_base;
        r->dev_bytes = t.prev->dev_bytes;
        r->view = t.prev->view;
        r->dev_flen = t.prev->dev_flen;
        t.out = r;
      }
      same_routes = true;
      rc = 0;
    } else if (prev->mirror && wf && tomb.size() + dset.size() <= std::max<uint64_t>(4096, nb / 8)) {
      rc = patch_update(ctx, prev, tomb, dset, &idx, &rmap, /*trie_only=*/true, &reps);
    }
  }
  if (rc < 0) return rc;
  if (rc == 1) {
    const int rb = rebuild(ctx, prev, ed, out);
    tl_ustats.kind = EMQX_GM_UPD_REBUILD;
    return rb;
  }
  if (same_routes) {
    // the touched filters' counts and marks (ids ascending = byte order: ed's order)
    std::vector<std::pair<uint32_t, uint64_t>> cnt;
    std::vector<std::pair<uint32_t, uint8_t>> pin;
    std::vector<uint32_t> aff_ids, aff_buf;
    std::vector<uint64_t> aff_off{0};
    for (const auto& kv : ed) {
      if (kv.second.old_id == NONE) continue;  // (an absent filter that stays absent)
      const std::vector<uint32_t> l = kv.second.final_list();
      cnt.emplace_back(kv.second.old_id, l.size());
      pin.emplace_back(kv.second.old_id, kv.second.pinned() ? 1 : 0);
      aff_ids.push_back(kv.second.old_id);
      aff_buf.insert(aff_buf.end(), l.begin(), l.end());
      aff_off.push_back(aff_buf.size());
    }
    idx->subs = prev->subs.apply(cnt, pin);
    rc = run_all(int(1 + reps.size()), [&](int k) {
      if (k == 0) return shift_subs_device(ctx, prev, idx, aff_ids, aff_off, aff_buf);
      RepTarget& t = reps[k - 1];
      return locked(t.m, [&] { return shift_subs_device(t.m, t.prev, t.out, aff_ids, aff_off, aff_buf); });
    });
    hipSetDevice(ctx->device);
    if (rc) {
      drop_reps();
      free_index(idx);
      return rc;
    }
    idx->info.n_subs = idx->subs.total();
    for (auto& t : reps) {
      t.out->subs = idx->subs;
      t.out->info.n_subs = idx->info.n_subs;
    }
    if (!reps.empty()) {
      tl_ustats.replicas = uint32_t(reps.size());
      tl_ustats.replica_mode = EMQX_GM_REP_SHARED;
    }
    tl_ustats.kind = EMQX_GM_UPD_SUBS_ONLY;
    if (const int ra = attach_replicas(idx, reps, 0)) {
      free_index(idx);
      return ra;
    }
    *out = idx;
    return EMQX_GM_OK;
  }
  // ---- route changes (ids renumbered): the new CSR from new id -> old id, the touched filters' final lists
  const uint64_t nf = idx->info.n_filters;
  std::vector<uint32_t> inv(nf, NONE);
  for (uint64_t f = 0; f < nb; ++f)
    if (rmap[f] != NONE) inv[rmap[f]] = uint32_t(f);
  std::vector<std::pair<uint32_t, std::vector<uint32_t>>> aff;
  {
    uint64_t k = 0;  // dset's filters in byte order: ids nb + k before renumbering
    for (const auto& kv : ed) {
      uint32_t nid = NONE;
      if (kv.second.old_id != NONE) nid = rmap[kv.second.old_id];
      else if (dset.count(kv.first)) nid = rmap[nb + k++];
      if (nid != NONE) aff.emplace_back(nid, kv.second.final_list());
    }
  }
  std::sort(aff.begin(), aff.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  std::vector<uint32_t> aff_ids, aff_buf;
  std::vector<uint64_t> aff_off{0};
  std::vector<uint64_t> cnt(nf, 0);
  for (uint64_t f = 0; f < nf; ++f)
    if (inv[f] != NONE) cnt[f] = prev->subs.count(inv[f]);
  for (auto& a : aff) {
    aff_ids.push_back(a.first);
    aff_buf.insert(aff_buf.end(), a.second.begin(), a.second.end());
    aff_off.push_back(aff_buf.size());
    cnt[a.first] = a.second.size();
  }
  std::vector<uint64_t> new_soff(nf + 1, 0);
  for (uint64_t f = 0; f < nf; ++f) new_soff[f + 1] = new_soff[f] + cnt[f];
  rc = run_all(int(1 + reps.size()), [&](int k) {
    if (k == 0) return rebuild_subs_device(ctx, prev, idx, new_soff, inv, aff_ids, aff_off, aff_buf);
    RepTarget& t = reps[k - 1];
    return locked(t.m, [&] { return rebuild_subs_device(t.m, t.prev, t.out, new_soff, inv, aff_ids, aff_off, aff_buf); });
  });
  hipSetDevice(ctx->device);
  if (rc) {
    drop_reps();
    free_index(idx);  // (its mirror goes too: later updates of this line rebuild)
    return rc;
  }
  idx->info.n_subs = new_soff.back();
  // the route-only marks of the new ids: untouched filters keep prev's, touched ones their final state
  std::vector<uint8_t> marks(nf, 0);
  for (uint64_t f = 0; f < nf; ++f)
    if (inv[f] != NONE) marks[f] = is_pinned(prev, inv[f]) ? 1 : 0;
  {
    uint64_t k = 0;
    for (const auto& kv : ed) {
      uint32_t nid = NONE;
      if (kv.second.old_id != NONE) nid = rmap[kv.second.old_id];
      else if (dset.count(kv.first)) nid = rmap[nb + k++];
      if (nid != NONE) marks[nid] = kv.second.pinned() ? 1 : 0;
    }
  }
  idx->subs = SubTable(std::move(new_soff), std::move(marks));
  for (auto& t : reps) {
    t.out->subs = idx->subs;
    t.out->info.n_subs = idx->info.n_subs;
  }
  if (const int ra = attach_replicas(idx, reps, 0)) {
    free_index(idx);
    return ra;
  }
  *out = idx;
  return EMQX_GM_OK;
}

}  // namespace gm
