// gm_multi.cpp — multi-device contexts (emqx_gm_opts.n_devices, SURVEY.md §8b:
// the open options "select the device list (1-8)").
//
// The reference's match_routes/1 runs in every publisher process, on all of a
// node's schedulers at once, against one routing table that mria replicates to
// every node (apps/emqx/src/emqx_router.erl:75-84, 128-145; emqx_trie.erl:
// 66-70).  A BEAM node loads a NIF once, so the MI355X analogue is ONE library
// context over all of the node's GPUs:
//   * every index snapshot made through the context is compiled once on the
//     host, on the first device, and REPLICATED to the others: the device
//     tables go device to device (a peer copy over xGMI between GPUs, a D2D
//     copy for a second replica on one GPU), the host tables are shared or
//     copied; nothing is recompiled (the replicated plan of SURVEY §8e C3);
//   * an update replicates its result the same way: an in-place patch result
//     is copied; a subscriber-only update_subs result, which shares its
//     predecessor's tables, shares the predecessor's replica's tables and
//     copies only its new subscriber CSR; an overlay result (no mirror, a
//     filter with '#' inside) repeats the same update on each replica;
//   * a host-buffer emqx_gm_match runs its chunks on every device at once
//     (gm_host.cpp) and returns ONE CSR in batch order.
#include <algorithm>
#include <chrono>
#include <cstring>
#include <memory>
#include <thread>

#include "gm_internal.h"

namespace gm {

namespace {

// the view's device pointers into the blob (the same set gm_image.cpp rebases)
template <class F> void for_blob_ptrs(IndexView& v, F f) {
  f(reinterpret_cast<const void**>(&v.nodes));
  f(reinterpret_cast<const void**>(&v.dict));
  f(reinterpret_cast<const void**>(&v.edges));
  f(reinterpret_cast<const void**>(&v.hot));
  f(reinterpret_cast<const void**>(&v.arena));
  f(reinterpret_cast<const void**>(&v.sub_off));
  f(reinterpret_cast<const void**>(&v.sub_ids));
  f(reinterpret_cast<const void**>(&v.gmap));
  f(reinterpret_cast<const void**>(&v.efilt));
  f(reinterpret_cast<const void**>(&v.mph_word));
  f(reinterpret_cast<const void**>(&v.d0_root));
}

// dst (on m's device) = src (on src_dev), `bytes` bytes, on m's stream
int copy_device(emqx_gm_ctx* m, void* dst, const void* src, int src_dev, size_t bytes) {
  if (!bytes) return 0;
  GM_HIP(m, hipSetDevice(m->device));
  if (src_dev == m->device) GM_HIP(m, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, m->stream));
  else GM_HIP(m, hipMemcpyPeerAsync(dst, m->device, src, src_dev, bytes, m->stream));
  GM_HIP(m, hipStreamSynchronize(m->stream));
  return 0;
}

}  // namespace

extern thread_local std::string tl_err;  // gm_api.cpp
thread_local emqx_gm_update_stats tl_ustats{};

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int run_all(int K, const std::function<int(int)>& f) {
  if (K <= 0) return 0;
  if (K == 1) return f(0);
  std::vector<int> rc(K, 0);
  std::vector<std::string> msg(K);
  auto one = [&](int k) {
    rc[k] = f(k);
    if (rc[k]) msg[k] = tl_err;
  };
  std::vector<std::thread> th;
  th.reserve(K - 1);
  for (int k = 1; k < K; ++k) th.emplace_back(one, k);
  one(0);
  for (auto& t : th) t.join();
  for (int k = 0; k < K; ++k)
    if (rc[k]) return set_err(nullptr, rc[k], msg[k]);
  return 0;
}

std::vector<RepTarget> rep_targets(emqx_gm_ctx* ctx, emqx_gm_index* prev) {
  std::vector<RepTarget> t;
  const size_t K = ctx->members.size();
  if (!K || !prev || prev->ov || prev->reps.size() != K) return t;
  for (size_t k = 0; k < K; ++k)
    if (!prev->reps[k] || prev->reps[k]->device != ctx->members[k]->device) return {};  // (another context's)
  for (size_t k = 0; k < K; ++k) t.push_back(RepTarget{ctx->members[k], prev->reps[k], nullptr});
  return t;
}

emqx_gm_index* replica_shell(emqx_gm_ctx* m, const emqx_gm_index* src) {
  auto* r = new emqx_gm_index;
  r->device = m->device;
  r->dev_bytes = src->dev_bytes;
  r->view = src->view;
  r->ft = src->ft;  // (a shared base + a small delta: cheap)
  r->gmap = src->gmap;
  r->subs = src->subs;  // (a shared base + a small delta: cheap)
  r->level_nodes = src->level_nodes;
  r->flen_stale = src->flen_stale.load();
  r->info = src->info;
  return r;
}

int attach_replicas(emqx_gm_index* out, std::vector<RepTarget>& t, int rc) {
  for (auto& x : t)
    if (!x.out) rc = rc ? rc : EMQX_GM_EDEVICE;
  if (rc) {
    for (auto& x : t) {
      if (x.out) free_index(x.out);
      x.out = nullptr;
    }
    return rc;
  }
  for (auto& x : t) {
    out->reps.push_back(x.out);
    x.out = nullptr;
  }
  return EMQX_GM_OK;
}

int replicate_index(emqx_gm_ctx* m, const emqx_gm_index* src, emqx_gm_index* share, emqx_gm_index** out) {
  if (src->ov) return set_err(m, EMQX_GM_EUNSUPPORTED, "replicate: overlay snapshot");
  // (a member's stream and pools are also used by small calls that hold only its lock)
  std::unique_lock<std::recursive_mutex> lk(m->mu, std::defer_lock);
  if (m->parent) lk.lock();
  std::unique_ptr<emqx_gm_index> r(replica_shell(m, src));
  struct Undo {  // a half-made replica's device memory and owner reference
    emqx_gm_index* r;
    ~Undo() {
      if (!r) return;
      (void)hipSetDevice(r->device);
      if (r->dev_base && !r->blob_owner) (void)hipFree(r->dev_base);
      if (r->dev_subs) (void)hipFree(r->dev_subs);
      if (r->blob_owner && r->blob_owner->refs.fetch_sub(1) == 1) free_index(r->blob_owner);
    }
  } undo{r.get()};
  if (src->dev_base) {
    if (share) {
      emqx_gm_index* owner = share->blob_owner ? share->blob_owner : share;
      owner->refs.fetch_add(1);
      r->blob_owner = owner;
      r->dev_base = share->dev_base;
    } else {
      GM_HIP(m, hipSetDevice(m->device));
      // the blob of a released snapshot of this size, when the device keeps one
      // (a fresh multi-GB hipMalloc after a few update cycles stalls)
      if ((r->dev_base = take_spare_blob(m->device, src->dev_bytes))) {
        r->reused_blob = true;
      } else {
        const hipError_t e = hipMalloc(&r->dev_base, src->dev_bytes);
        if (e != hipSuccess) {
          r->dev_base = nullptr;
          return set_err(m, EMQX_GM_ENOMEM, std::string("replicate: hipMalloc: ") + hipGetErrorString(e));
        }
      }
      if (const int rc = copy_device(m, r->dev_base, src->dev_base, src->device, src->dev_bytes)) return rc;
    }
  }
  const uint8_t* SB = static_cast<const uint8_t*>(src->dev_base);
  uint8_t* RB = static_cast<uint8_t*>(r->dev_base);
  const uint8_t* SS = static_cast<const uint8_t*>(src->dev_subs);
  if (src->dev_subs) {
    GM_HIP(m, hipSetDevice(m->device));
    const hipError_t e = hipMalloc(&r->dev_subs, src->subs_bytes);
    if (e != hipSuccess)
      return set_err(m, EMQX_GM_ENOMEM, std::string("replicate: hipMalloc (subscribers): ") + hipGetErrorString(e));
    r->subs_bytes = src->subs_bytes;
    if (const int rc = copy_device(m, r->dev_subs, src->dev_subs, src->device, src->subs_bytes)) return rc;
  }
  uint8_t* RS = static_cast<uint8_t*>(r->dev_subs);
  bool stray = false;
  for_blob_ptrs(r->view, [&](const void** p) {
    const uint8_t* q = static_cast<const uint8_t*>(*p);
    if (!q) return;
    if (SB && q >= SB && q < SB + src->dev_bytes) *p = RB + (q - SB);
    else if (SS && q >= SS && q < SS + src->subs_bytes) *p = RS + (q - SS);
    else stray = true;
  });
  if (stray) return set_err(m, EMQX_GM_EUNSUPPORTED, "replicate: a table outside the snapshot's allocations");
  if (src->dev_flen)
    r->dev_flen = reinterpret_cast<uint16_t*>(RB + (reinterpret_cast<const uint8_t*>(src->dev_flen) - SB));
  undo.r = nullptr;
  *out = r.release();
  return EMQX_GM_OK;
}

int replicate_result(emqx_gm_ctx* ctx, emqx_gm_index* prev, emqx_gm_index** out_p) {
  emqx_gm_index* out = *out_p;
  const size_t K = ctx->members.size();
  if (!K || !out || out->reps.size() == K) return EMQX_GM_OK;  // single device, or replicated by the update itself
  auto fail = [&](int rc) {
    if (out->refs.fetch_sub(1) == 1) free_index(out);
    *out_p = nullptr;
    return rc;
  };
  if (out->reps.size()) return fail(set_err(ctx, EMQX_GM_EINVAL, "replicate: a snapshot of another context"));
  // an overlay (a filter with '#' inside, or an update of a superseded
  // snapshot) stays on the first device: it is matched there, as its base is
  if (out->ov) return EMQX_GM_OK;
  // the snapshot whose device tables `out` shares (update_subs without a route
  // change) and, when prev is that one or shares it too, prev's replica of it
  const emqx_gm_index* own = out->blob_owner;
  const bool share = own && prev && prev->reps.size() == K && (prev == own || prev->blob_owner == own);
  const double t0 = now_ms();
  std::vector<emqx_gm_index*> reps(K, nullptr);
  int rc = 0;
  if (share) {
    rc = run_all(int(K), [&](int k) { return replicate_index(ctx->members[k], out, prev->reps[k], &reps[k]); });
  } else {
    // a tree of device-to-device copies: every replica made is the source of
    // one more in the next round (rounds: 1, 2, 4, ... copies at once), so the
    // first device's links are not the only ones that carry the tables
    std::vector<const emqx_gm_index*> src{out};
    size_t next = 0;
    while (!rc && next < K) {
      std::vector<std::pair<size_t, const emqx_gm_index*>> jobs;
      for (const emqx_gm_index* s : src)
        if (next < K) jobs.emplace_back(next++, s);
      rc = run_all(int(jobs.size()), [&](int j) {
        return replicate_index(ctx->members[jobs[j].first], jobs[j].second, nullptr, &reps[jobs[j].first]);
      });
      for (const auto& j : jobs)
        if (reps[j.first]) src.push_back(reps[j.first]);
    }
  }
  hipSetDevice(ctx->device);
  if (rc) {
    for (emqx_gm_index* r : reps)
      if (r) free_index(r);
    return fail(rc);
  }
  for (const emqx_gm_index* r : reps) {
    if (r->blob_owner) continue;
    if (r->reused_blob) ++tl_ustats.blobs_reused;
    else ++tl_ustats.blobs_fresh;
  }
  out->reps = std::move(reps);
  tl_ustats.replicas = uint32_t(K);
  tl_ustats.replica_mode = share ? EMQX_GM_REP_SHARED : EMQX_GM_REP_COPIED;
  tl_ustats.replicate_ms = now_ms() - t0;
  return EMQX_GM_OK;
}

}  // namespace gm

namespace gm {

// emqx_gm_fanout on host rows through a multi-device context: the rows are cut
// into one contiguous slice per device, balanced by matches; each device (a
// thread of its own, its own stream and pools) fans its slice out against its
// replica's subscriber CSR; then, in slice order, each slice's delivery
// offsets are rebased on its device and its rows DMA'd into their final place
// of ONE page-locked result.  The reference's dispatch runs in every publisher
// process at once (emqx_broker.erl:296-322, 506-530); a node's publish batch
// thus fans out over all its GPUs' PCIe links.  Small batches (fewer than
// GM_FANOUT_MULTI_MIN rows, default 65,536) take the first device alone.
int run_fanout_multi(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const emqx_gm_csr* m, uint32_t flags,
                     emqx_gm_csr* out) {
  std::vector<emqx_gm_ctx*> mem{ctx};
  std::vector<const emqx_gm_index*> rix{idx};
  for (size_t k = 0; k < ctx->members.size() && k < idx->reps.size(); ++k) {
    mem.push_back(ctx->members[k]);
    rix.push_back(idx->reps[k]);
  }
  const uint64_t n = m->n_rows, nnz = m->nnz;
  const char* me = knob("GM_FANOUT_MULTI_MIN");
  const uint64_t min_rows = me ? strtoull(me, nullptr, 10) : 65536;
  if (mem.size() < 2 || n < min_rows) return run_fanout(ctx, idx, m, flags, out);
  for (uint64_t i = 0; i < nnz; ++i)
    if (m->ids[i] >= idx->view.n_filters) return set_err(ctx, EMQX_GM_EINVAL, "fanout: filter id out of range");
  if (m->row_off[0] != 0 || m->row_off[n] != nnz) return set_err(ctx, EMQX_GM_EINVAL, "fanout: row offsets");
  for (uint64_t i = 0; i < n; ++i)
    if (m->row_off[i + 1] < m->row_off[i]) return set_err(ctx, EMQX_GM_EINVAL, "fanout: row offsets not monotone");
  const int K = int(mem.size());
  struct Part {
    uint64_t r0 = 0, r1 = 0, o0 = 0, o1 = 0;
    PoolBuf d_off, d_ids;
    emqx_gm_csr res{};
    int rc = 0;
    std::string err;
    emqx_gm_match_stats st{};
  };
  std::vector<Part> P(K);
  for (int k = 0; k < K; ++k) {  // row bounds: the first row at or past the k-th share of the matches
    P[k].r0 = k == 0 ? 0 : uint64_t(std::lower_bound(m->row_off, m->row_off + n, nnz * uint64_t(k) / K) - m->row_off);
    if (k) P[k - 1].r1 = P[k].r0;
  }
  P[K - 1].r1 = n;
  for (auto& p : P) p.o0 = m->row_off[p.r0], p.o1 = m->row_off[p.r1];
  const uint32_t fl = (flags & EMQX_GM_WITH_EXACT) | EMQX_GM_DEVICE_IO;
  auto work = [&](int k) {
    Part& p = P[k];
    emqx_gm_ctx* mc = mem[k];
    hipSetDevice(mc->device);
    std::unique_lock<std::recursive_mutex> lk(mc->mu, std::defer_lock);
    if (mc != ctx) lk.lock();  // (the caller holds the first device's lock)
    const uint64_t rows = p.r1 - p.r0, cnt = p.o1 - p.o0;
    p.d_off = PoolBuf(mc->pool, (rows + 1) * 8);
    p.d_ids = PoolBuf(mc->pool, cnt * 4 + 16);
    if (!p.d_off.p || !p.d_ids.p) {
      p.rc = EMQX_GM_ENOMEM;
      p.err = "fanout: slice workspace";
      return;
    }
    hipError_t e = hipMemcpyAsync(p.d_off.p, m->row_off + p.r0, (rows + 1) * 8, hipMemcpyHostToDevice, mc->stream);
    if (e == hipSuccess && cnt)
      e = hipMemcpyAsync(p.d_ids.p, m->ids + p.o0, cnt * 4, hipMemcpyHostToDevice, mc->stream);
    if (e != hipSuccess || launch_add_u64(mc->stream, p.d_off.as<uint64_t>(), rows + 1, uint64_t(0) - p.o0)) {
      p.rc = EMQX_GM_EDEVICE;
      p.err = "fanout: slice upload";
      return;
    }
    emqx_gm_csr sub{};
    sub.n_rows = rows;
    sub.nnz = cnt;
    sub.row_off = p.d_off.as<uint64_t>();
    sub.ids = p.d_ids.as<uint32_t>();
    sub.on_device = 1;
    p.rc = run_fanout(mc, rix[k], &sub, fl, &p.res);
    if (p.rc) p.err = std::string(emqx_gm_last_error(mc));
    p.st = mc->stats;
  };
  {
    std::vector<std::thread> th;
    for (int k = 1; k < K; ++k) th.emplace_back(work, k);
    work(0);
    for (auto& t : th) t.join();
  }
  // the rows' copy-out and the slices' buffers use every member's stream and
  // pools: their locks from here on (small calls hold only a member's lock)
  std::vector<std::unique_lock<std::recursive_mutex>> held;
  for (int k = 1; k < K; ++k) held.emplace_back(mem[k]->mu);
  auto drop = [&]() {
    for (int k = 0; k < K; ++k) {
      hipSetDevice(mem[k]->device);
      hipStreamSynchronize(mem[k]->stream);
      if (P[k].res.row_off || P[k].res.ids) {
        mem[k]->pool->release(P[k].res.row_off);
        mem[k]->pool->release(P[k].res.ids);
      }
      P[k].d_off.reset();
      P[k].d_ids.reset();
    }
    hipSetDevice(ctx->device);
  };
  for (int k = 0; k < K; ++k)
    if (P[k].rc) {
      const int rc = P[k].rc;
      const std::string msg = P[k].err;
      drop();
      return set_err(ctx, rc, msg);
    }
  uint64_t total = 0;
  for (auto& p : P) total += p.res.nnz;
  uint64_t* r_off = static_cast<uint64_t*>(ctx->hpool->alloc((n + 1) * 8, true));
  uint32_t* r_ids = static_cast<uint32_t*>(ctx->hpool->alloc(total * 4 + 16, true));
  if (!r_off || !r_ids) {
    ctx->hpool->release(r_off);
    ctx->hpool->release(r_ids);
    drop();
    return set_err(ctx, EMQX_GM_ENOMEM, "fanout: host result");
  }
  uint64_t base = 0;
  int rc = 0;
  for (int k = 0; k < K && !rc; ++k) {  // each slice's rows into place, rebased on its device
    Part& p = P[k];
    emqx_gm_ctx* mc = mem[k];
    hipSetDevice(mc->device);
    const uint64_t rows = p.r1 - p.r0;
    hipError_t e = launch_add_u64(mc->stream, p.res.row_off, rows, base) ? hipErrorLaunchFailure : hipSuccess;
    if (e == hipSuccess && rows)
      e = hipMemcpyAsync(r_off + p.r0, p.res.row_off, rows * 8, hipMemcpyDeviceToHost, mc->stream);
    if (e == hipSuccess && p.res.nnz)
      e = hipMemcpyAsync(r_ids + base, p.res.ids, p.res.nnz * 4, hipMemcpyDeviceToHost, mc->stream);
    if (e != hipSuccess) rc = set_err(ctx, EMQX_GM_EDEVICE, "fanout: rows to host");
    base += p.res.nnz;
  }
  drop();  // (waits for every copy)
  if (rc) {
    ctx->hpool->release(r_off);
    ctx->hpool->release(r_ids);
    return rc;
  }
  r_off[n] = total;
  emqx_gm_match_stats tot{};
  tot.n_topics = n;
  tot.nnz = total;
  for (auto& p : P) {
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

}  // namespace gm
