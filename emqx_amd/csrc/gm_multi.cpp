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
#include <cstring>
#include <memory>

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

int replicate_index(emqx_gm_ctx* m, const emqx_gm_index* src, emqx_gm_index* share, emqx_gm_index** out) {
  if (src->ov) return set_err(m, EMQX_GM_EUNSUPPORTED, "replicate: overlay snapshot");
  std::unique_ptr<emqx_gm_index> r(new emqx_gm_index);
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
  r->device = m->device;
  r->dev_bytes = src->dev_bytes;
  r->view = src->view;
  r->ft = src->ft;  // (a shared base + a small delta: cheap)
  r->gmap = src->gmap;
  r->subs = src->subs;  // (a shared base + a small delta: cheap)
  r->ov = nullptr;
  r->level_nodes = src->level_nodes;
  r->flen_stale = src->flen_stale.load();
  r->info = src->info;
  if (src->dev_base) {
    if (share) {
      emqx_gm_index* owner = share->blob_owner ? share->blob_owner : share;
      owner->refs.fetch_add(1);
      r->blob_owner = owner;
      r->dev_base = share->dev_base;
    } else {
      GM_HIP(m, hipSetDevice(m->device));
      const hipError_t e = hipMalloc(&r->dev_base, src->dev_bytes);
      if (e != hipSuccess)
        return set_err(m, EMQX_GM_ENOMEM, std::string("replicate: hipMalloc: ") + hipGetErrorString(e));
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

int replicate_result(emqx_gm_ctx* ctx, emqx_gm_index* prev, emqx_gm_index** out_p,
                     const std::function<int(emqx_gm_ctx*, emqx_gm_index*, emqx_gm_index**)>& redo) {
  emqx_gm_index* out = *out_p;
  const size_t K = ctx->members.size();
  if (!K || !out || out->reps.size() == K) return EMQX_GM_OK;  // single device, or a snapshot already replicated
  auto fail = [&](int rc) {
    if (out->refs.fetch_sub(1) == 1) free_index(out);
    *out_p = nullptr;
    return rc;
  };
  if (out->reps.size()) return fail(set_err(ctx, EMQX_GM_EINVAL, "replicate: a snapshot of another context"));
  // an overlay made from a snapshot without replicas (one made through another
  // context) stays on the first device: it is matched there, as its base is
  if (out->ov && (!prev || prev->reps.size() != K)) return EMQX_GM_OK;
  // the snapshot whose device tables `out` shares (update_subs without a route
  // change) and, when prev is that one or shares it too, prev's replica of it
  const emqx_gm_index* own = out->blob_owner;
  const bool share = own && prev && prev->reps.size() == K && (prev == own || prev->blob_owner == own);
  for (size_t k = 0; k < K; ++k) {
    emqx_gm_ctx* m = ctx->members[k];
    emqx_gm_index* rep = nullptr;
    int rc;
    if (out->ov) {
      rc = redo(m, prev->reps[k], &rep);
    } else {
      rc = replicate_index(m, out, share ? prev->reps[k] : nullptr, &rep);
    }
    if (rc) {
      hipSetDevice(ctx->device);
      return fail(rc);
    }
    out->reps.push_back(rep);
  }
  hipSetDevice(ctx->device);
  return EMQX_GM_OK;
}

}  // namespace gm
