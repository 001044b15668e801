// gm_api.cpp — extern "C" boundary of libemqx_gpu_match.so (include/emqx_gpu_match.h).
// No C++ exception crosses the ABI; every failure is an EMQX_GM_E* code with
// the message in emqx_gm_last_error().
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <new>
#include <stdexcept>

#include <sys/mman.h>

#include "gm_internal.h"
#include "../../include/emqx_gm_ext.h"

namespace gm {

// The message of the calling thread's last failing call.  Per thread, not per
// context: a context is shared by concurrent callers (e.g. NIF calls on
// several dirty schedulers), and a call runs start to end on one thread, so a
// caller reading emqx_gm_last_error() right after its own failure always gets
// its own message and the pointer stays valid until that thread's next call.
thread_local std::string tl_err;

int set_err(emqx_gm_ctx* ctx, int code, const std::string& msg) {
  (void)ctx;
  tl_err = msg;
  return code;
}

DevPool::~DevPool() {
  hipSetDevice(device_);
  reclaim(true);
  for (auto& kv : free_) hipFree(kv.second);
  for (auto& kv : live_) hipFree(kv.first);
  for (hipEvent_t e : ev_idle_) hipEventDestroy(e);
}

void DevPool::release_after(void* p, hipStream_t s) { release_after(&p, 1, s); }
// (one event for all the buffers: each event record is a marker packet on the
// stream, ~5 us of idle GPU between the kernels around it)
void DevPool::release_after(void* const* ps, int np, hipStream_t s) {
  void* q[4];
  int nq = 0;
  for (int i = 0; i < np && nq < 4; ++i)
    if (ps[i] && live_.count(ps[i])) q[nq++] = ps[i];
  if (!nq) return;
  hipEvent_t e = nullptr;
  if (!ev_idle_.empty()) {
    e = ev_idle_.back();
    ev_idle_.pop_back();
  } else if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
    e = nullptr;
  }
  if (!e || hipEventRecord(e, s) != hipSuccess) {  // no event: the old way, wait for the stream
    if (e) ev_idle_.push_back(e);
    hipStreamSynchronize(s);
    for (int i = 0; i < nq; ++i) release(q[i]);
    return;
  }
  for (int i = 0; i < nq; ++i) deferred_.emplace_back(q[i], i + 1 == nq ? e : nullptr);
}

void DevPool::reclaim(bool wait) {
  // a group of buffers freed together is consecutive, the event on its last
  size_t keep = 0;
  for (size_t i = 0; i < deferred_.size();) {
    size_t j = i;
    while (j < deferred_.size() && !deferred_[j].second) ++j;  // the group's event entry
    if (j == deferred_.size()) {  // (not expected: an unterminated group stays)
      while (i < j) deferred_[keep++] = deferred_[i++];
      break;
    }
    hipEvent_t e = deferred_[j].second;
    const bool done = wait ? (hipEventSynchronize(e), true) : hipEventQuery(e) == hipSuccess;
    if (done) {
      ev_idle_.push_back(e);
      for (size_t k = i; k <= j; ++k) release(deferred_[k].first);
    } else {
      for (size_t k = i; k <= j; ++k) deferred_[keep++] = deferred_[k];
    }
    i = j + 1;
  }
  deferred_.resize(keep);
}

// Buffers still handed out (live_) are NOT freed: a caller may hold a host CSR
// past emqx_gm_close, so they are detached and leak as plain malloc'd memory
// (what the CSRs were before the pool existed).
HostPool::~HostPool() {
  for (int k = 0; k < 2; ++k)
    for (auto& kv : free_[k]) drop(kv.second, k != 0);
}
void HostPool::drop(void* p, bool pinned) {
  if (pinned) (void)hipHostFree(p);
  else free(p);
}
void* HostPool::alloc(size_t bytes, bool pinned) {
  constexpr size_t HUGE_PAGE = 2u << 20;
  const size_t r = bytes < HUGE_PAGE ? ((bytes + 4095) & ~size_t(4095)) : ((bytes + HUGE_PAGE - 1) & ~(HUGE_PAGE - 1));
  auto& fl = free_[pinned ? 1 : 0];
  auto it = fl.lower_bound(r);
  if (it != fl.end() && it->first <= r + r / 4) {
    void* p = it->second;
    cached_ -= it->first;
    live_[p] = Buf{it->first, pinned};
    fl.erase(it);
    return p;
  }
  void* p = nullptr;
  if (pinned) {
    if (hipHostMalloc(&p, r, hipHostMallocPortable) != hipSuccess) return nullptr;
  } else {
    if (posix_memalign(&p, r >= HUGE_PAGE ? HUGE_PAGE : 64, r) != 0) return nullptr;
    if (r >= HUGE_PAGE) (void)madvise(p, r, MADV_HUGEPAGE);
  }
  live_[p] = Buf{r, pinned};  // overwrite: an address freed behind the pool's back may come back
  return p;
}
void HostPool::release(void* p) {
  if (!p) return;
  auto it = live_.find(p);
  if (it == live_.end()) {
    free(p);
    return;
  }
  const size_t r = it->second.bytes;
  const bool pinned = it->second.pinned;
  live_.erase(it);
  for (;;) {  // the largest cached ones go first
    auto* big = &free_[0];
    if (free_[0].empty() || (!free_[1].empty() && std::prev(free_[1].end())->first > std::prev(free_[0].end())->first))
      big = &free_[1];
    if (cached_ + r <= kCap || big->empty()) break;
    auto last = std::prev(big->end());
    cached_ -= last->first;
    drop(last->second, big == &free_[1]);
    big->erase(last);
  }
  if (r > kCap) {
    drop(p, pinned);
    return;
  }
  free_[pinned ? 1 : 0].emplace(r, p);
  cached_ += r;
}

PinPool::~PinPool() {
  for (auto& kv : size_) (void)hipHostFree(kv.first);
}
void* PinPool::get(size_t bytes) {
  size_t r = 64 << 10;  // powers of two from 64 KiB
  while (r < bytes) r <<= 1;
  {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = free_.find(r);
    if (it != free_.end()) {
      void* p = it->second;
      free_.erase(it);
      cached_ -= r;
      return p;
    }
  }
  void* p = nullptr;
  if (hipHostMalloc(&p, r, hipHostMallocPortable) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(mu_);
  size_[p] = r;
  return p;
}
void PinPool::put(void* p) {
  if (!p) return;
  std::lock_guard<std::mutex> lk(mu_);
  auto it = size_.find(p);
  if (it == size_.end()) return;
  if (cached_ + it->second > kCap) {  // (over the cap: freed)
    (void)hipHostFree(p);
    size_.erase(it);
    return;
  }
  free_.emplace(it->second, p);
  cached_ += it->second;
}

namespace {
std::mutex g_pin_mu;
std::map<uintptr_t, size_t> g_pinned;  // emqx_gm_host_alloc buffers: start -> bytes
}  // namespace
bool host_pinned_range(const void* p, size_t bytes) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  std::lock_guard<std::mutex> lk(g_pin_mu);
  auto it = g_pinned.upper_bound(a);
  if (it == g_pinned.begin()) return false;
  --it;
  return a >= it->first && a - it->first <= it->second && bytes <= it->second - (a - it->first);
}
void host_pinned_add(void* p, size_t bytes) {
  std::lock_guard<std::mutex> lk(g_pin_mu);
  g_pinned[reinterpret_cast<uintptr_t>(p)] = bytes;
}
bool host_pinned_remove(void* p) {
  std::lock_guard<std::mutex> lk(g_pin_mu);
  return g_pinned.erase(reinterpret_cast<uintptr_t>(p)) != 0;
}

static size_t round_size(size_t b) {
  if (b < 4096) return 4096;
  if (b < (64u << 20)) {  // powers of two below 64 MiB
    size_t p = 4096;
    while (p < b) p <<= 1;
    return p;
  }
  return (b + (2u << 20) - 1) & ~size_t((2u << 20) - 1);  // 2 MiB granules above
}

void* DevPool::alloc(size_t bytes) {
  if (!deferred_.empty()) reclaim(false);
  size_t r = round_size(bytes);
  auto it = free_.lower_bound(r);
  if (it != free_.end() && it->first <= r + r / 4) {
    void* p = it->second;
    live_[p] = it->first;
    cached_ -= it->first;
    free_.erase(it);
    return p;
  }
  void* p = nullptr;
  hipSetDevice(device_);
  if (hipMalloc(&p, r) != hipSuccess) {
    trim();
    if (!deferred_.empty()) {  // memory is short: wait for the deferred frees, then try once more
      reclaim(true);
      trim();
      if (hipMalloc(&p, r) == hipSuccess) {
        live_[p] = r;
        return p;
      }
    }
    if (hipMalloc(&p, r) != hipSuccess) return nullptr;
  }
  live_[p] = r;
  return p;
}

void DevPool::release(void* p) {
  auto it = live_.find(p);
  if (it == live_.end()) return;
  free_.emplace(it->second, p);
  cached_ += it->second;
  live_.erase(it);
}

void DevPool::trim() {
  hipSetDevice(device_);
  hipDeviceSynchronize();
  reclaim(false);  // (every event has passed now)
  for (auto& kv : free_) hipFree(kv.second);
  free_.clear();
  cached_ = 0;
}

int sum_filter_lengths(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const uint32_t* d_ids, uint64_t nnz,
                       uint64_t* out);

}  // namespace gm

#define GM_GUARD_BEGIN try {
#define GM_GUARD_END(ctx)                                                  \
  }                                                                        \
  catch (const std::bad_alloc&) {                                          \
    return gm::set_err((ctx), EMQX_GM_ENOMEM, "host allocation failed");   \
  }                                                                        \
  catch (const std::exception& e) {                                        \
    return gm::set_err((ctx), EMQX_GM_EINVAL, e.what());                   \
  }                                                                        \
  catch (...) {                                                            \
    return gm::set_err((ctx), EMQX_GM_EINVAL, "unknown error");            \
  }

extern "C" {

int emqx_gm_abi_version(void) { return EMQX_GM_ABI_VERSION; }

static int open_one(int dev, uint32_t flags, emqx_gm_ctx** out) {
  if (hipSetDevice(dev) != hipSuccess) return EMQX_GM_EDEVICE;
  auto* ctx = new emqx_gm_ctx;
  ctx->device = dev;
  ctx->open_flags = flags;
  if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
    delete ctx;
    return EMQX_GM_EDEVICE;
  }
  ctx->own_stream = true;
  gm::note_ctx_open(dev);
  ctx->pool = new gm::DevPool(dev);
  ctx->hpool = new gm::HostPool;
  ctx->pins = new gm::PinPool;
  for (auto& e : ctx->ev) {
    if (hipEventCreate(&e) != hipSuccess) {
      emqx_gm_close(ctx);
      return EMQX_GM_EDEVICE;
    }
  }
  *out = ctx;
  return EMQX_GM_OK;
}

int emqx_gm_open(const emqx_gm_opts* opts, emqx_gm_ctx** out) {
  if (!out) return EMQX_GM_EINVAL;
  *out = nullptr;
  GM_GUARD_BEGIN
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return EMQX_GM_EDEVICE;
  if (opts && (opts->flags & ~(EMQX_GM_OPEN_MIRROR_EAGER | EMQX_GM_OPEN_MIRROR_LAZY))) return EMQX_GM_EINVAL;
  if (opts && (opts->flags & EMQX_GM_OPEN_MIRROR_EAGER) && (opts->flags & EMQX_GM_OPEN_MIRROR_LAZY))
    return EMQX_GM_EINVAL;
  std::vector<int> devs;
  if (opts && opts->n_devices) {
    if (opts->n_devices > EMQX_GM_MAX_DEVICES) return EMQX_GM_EINVAL;
    devs.assign(opts->devices, opts->devices + opts->n_devices);
  } else {
    devs.push_back(opts ? opts->device : 0);
  }
  for (int d : devs)
    if (d < 0 || d >= count) return EMQX_GM_EINVAL;
  const uint32_t flags = opts ? opts->flags : 0;
  emqx_gm_ctx* ctx = nullptr;
  if (int rc = open_one(devs[0], flags, &ctx)) return rc;
  for (size_t k = 1; k < devs.size(); ++k) {
    emqx_gm_ctx* m = nullptr;
    if (int rc = open_one(devs[k], flags, &m)) {
      emqx_gm_close(ctx);
      return rc;
    }
    m->parent = ctx;
    ctx->members.push_back(m);
  }
  // replicas are copied GPU to GPU, in a tree (any listed device may be a
  // copy's source): peer access between every pair lets the copy engines go
  // over xGMI directly (already enabled, or unsupported: the runtime stages it)
  for (int a : devs)
    for (int b : devs) {
      int can = 0;
      if (a == b || hipDeviceCanAccessPeer(&can, a, b) != hipSuccess || !can) continue;
      hipSetDevice(a);
      (void)hipDeviceEnablePeerAccess(b, 0);
      (void)hipGetLastError();  // (hipErrorPeerAccessAlreadyEnabled is fine)
    }
  hipSetDevice(devs[0]);
  *out = ctx;
  return EMQX_GM_OK;
  GM_GUARD_END(nullptr)
}

int emqx_gm_devices(const emqx_gm_ctx* ctx, int32_t* devices, uint32_t* n) {
  if (!ctx || !n) return EMQX_GM_EINVAL;
  *n = uint32_t(1 + ctx->members.size());
  if (devices) {
    devices[0] = ctx->device;
    for (size_t k = 0; k < ctx->members.size(); ++k) devices[k + 1] = ctx->members[k]->device;
  }
  return EMQX_GM_OK;
}

int emqx_gm_host_alloc(emqx_gm_ctx* ctx, uint64_t bytes, void** p) {
  if (!ctx || !p) return EMQX_GM_EINVAL;
  *p = nullptr;
  hipSetDevice(ctx->device);
  void* q = nullptr;
  const hipError_t e = hipHostMalloc(&q, bytes ? bytes : 1, hipHostMallocPortable);
  if (e != hipSuccess) return gm::set_err(ctx, EMQX_GM_ENOMEM, std::string("host_alloc: ") + hipGetErrorString(e));
  GM_GUARD_BEGIN
  gm::host_pinned_add(q, bytes);
  *p = q;
  return EMQX_GM_OK;
  GM_GUARD_END(ctx)
}

int emqx_gm_host_free(emqx_gm_ctx* ctx, void* p) {
  if (!ctx) return EMQX_GM_EINVAL;
  if (!p) return EMQX_GM_OK;
  if (!gm::host_pinned_remove(p)) return gm::set_err(ctx, EMQX_GM_EINVAL, "host_free: not an emqx_gm_host_alloc buffer");
  // (a match call in flight on another thread may still read it: the caller's
  // business, as for any input buffer)
  GM_HIP(ctx, hipHostFree(p));
  return EMQX_GM_OK;
}

int emqx_gm_close(emqx_gm_ctx* ctx) {
  if (!ctx) return EMQX_GM_EINVAL;
  for (emqx_gm_ctx* m : ctx->members) emqx_gm_close(m);
  ctx->members.clear();
  {
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    hipSetDevice(ctx->device);
    if (ctx->stream) hipStreamSynchronize(ctx->stream);
    gm::note_ctx_close(ctx->device);
    gm::trim_spare_blob(ctx->device);
    gm::free_host_pipe(ctx);
    delete ctx->pool;
    delete ctx->hpool;
    delete ctx->pins;
    for (auto& e : ctx->ev)
      if (e) hipEventDestroy(e);
    if (ctx->own_stream && ctx->stream) hipStreamDestroy(ctx->stream);
    if (ctx->stream2) {
      hipStreamSynchronize(ctx->stream2);
      hipStreamDestroy(ctx->stream2);
    }
    if (ctx->stream_asm) {
      hipStreamSynchronize(ctx->stream_asm);
      hipStreamDestroy(ctx->stream_asm);
    }
    for (auto& e : ctx->ov_ev)
      if (e) hipEventDestroy(e);
    for (hipEvent_t e : ctx->ev_free) hipEventDestroy(e);
    for (void* p : ctx->pin_all) hipHostFree(p);
    if (ctx->ctr_ring) hipFree(ctx->ctr_ring);
  }
  delete ctx;
  return EMQX_GM_OK;
}

const char* emqx_gm_last_error(const emqx_gm_ctx* ctx) {
  (void)ctx;
  return gm::tl_err.c_str();
}

int emqx_gm_set_stream(emqx_gm_ctx* ctx, void* s) {
  if (!ctx) return EMQX_GM_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  hipSetDevice(ctx->device);
  hipStreamSynchronize(ctx->stream);
  if (ctx->stream_asm) hipStreamSynchronize(ctx->stream_asm);
  if (s) {
    if (ctx->own_stream) hipStreamDestroy(ctx->stream);
    ctx->stream = static_cast<hipStream_t>(s);
    ctx->own_stream = false;
  } else if (!ctx->own_stream) {
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess)
      return gm::set_err(ctx, EMQX_GM_EDEVICE, "set_stream: hipStreamCreate");
    ctx->own_stream = true;
  }
  return EMQX_GM_OK;
}

int emqx_gm_synchronize(emqx_gm_ctx* ctx) {
  if (!ctx) return EMQX_GM_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  for (emqx_gm_ctx* m : ctx->members) {
    std::lock_guard<std::recursive_mutex> ml(m->mu);
    hipSetDevice(m->device);
    GM_HIP(ctx, hipStreamSynchronize(m->stream));
  }
  hipSetDevice(ctx->device);
  GM_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (ctx->stream_asm) GM_HIP(ctx, hipStreamSynchronize(ctx->stream_asm));
  return EMQX_GM_OK;
}

// A snapshot made on a multi-device context gets its replicas (gm_multi.cpp)
// unless the update made them itself; the call's update stats are closed.
static int replicated(emqx_gm_ctx* ctx, int rc, emqx_gm_index* prev, emqx_gm_index** out, double t0) {
  if (!rc && !ctx->members.empty() && out && *out) rc = gm::replicate_result(ctx, prev, out);
  gm::tl_ustats.total_ms = gm::now_ms() - t0;
  return rc;
}
static double begin_index_call(uint32_t kind) {
  gm::tl_ustats = emqx_gm_update_stats{};
  gm::tl_ustats.kind = kind;
  return gm::now_ms();
}

int emqx_gm_index_build(emqx_gm_ctx* ctx, const uint8_t* fb, const uint64_t* fo, uint64_t n,
                        const uint64_t* sub_off, const uint32_t* sub_ids, uint32_t* perm_out,
                        emqx_gm_index** out) {
  if (!ctx) return EMQX_GM_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  GM_GUARD_BEGIN
  const double t0 = begin_index_call(EMQX_GM_UPD_BUILD);
  hipSetDevice(ctx->device);
  return replicated(ctx, gm::build_index(ctx, fb, fo, n, sub_off, sub_ids, perm_out, out), nullptr, out, t0);
  GM_GUARD_END(ctx)
}

int emqx_gm_index_build_sharded(emqx_gm_ctx* ctx, const uint8_t* fb, const uint64_t* fo, uint64_t n,
                                const uint64_t* sub_off, const uint32_t* sub_ids, uint32_t* perm_out,
                                emqx_gm_index** out) {
  if (!ctx) return EMQX_GM_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  GM_GUARD_BEGIN
  const double t0 = begin_index_call(EMQX_GM_UPD_BUILD);
  hipSetDevice(ctx->device);
  const int rc = gm::build_sharded(ctx, fb, fo, n, sub_off, sub_ids, perm_out, out);
  gm::tl_ustats.total_ms = gm::now_ms() - t0;
  return rc;
  GM_GUARD_END(ctx)
}

int emqx_gm_index_update(emqx_gm_ctx* ctx, emqx_gm_index* prev, const uint8_t* fb, const uint64_t* fo,
                         const uint8_t* ops, uint64_t n_ops, emqx_gm_index** out) {
  if (!ctx) return EMQX_GM_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  if (prev && prev->device != ctx->device)
    return gm::set_err(ctx, EMQX_GM_EINVAL, "index_update: index lives on another device");
  if (prev && prev->route)
    return gm::set_err(ctx, EMQX_GM_EUNSUPPORTED, "index_update: sharded index (rebuild it)");
  GM_GUARD_BEGIN
  const double t0 = begin_index_call(EMQX_GM_UPD_NONE);
  hipSetDevice(ctx->device);
  return replicated(ctx, gm::update_index(ctx, prev, fb, fo, ops, n_ops, out), prev, out, t0);
  GM_GUARD_END(ctx)
}

int emqx_gm_index_update_subs(emqx_gm_ctx* ctx, emqx_gm_index* prev, const uint8_t* fb, const uint64_t* fo,
                              const uint32_t* subs, const uint8_t* ops, uint64_t n_ops, emqx_gm_index** out) {
  if (!ctx) return EMQX_GM_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  if (prev && prev->device != ctx->device)
    return gm::set_err(ctx, EMQX_GM_EINVAL, "index_update_subs: index lives on another device");
  if (prev && prev->route)
    return gm::set_err(ctx, EMQX_GM_EUNSUPPORTED, "index_update_subs: sharded index (rebuild it)");
  GM_GUARD_BEGIN
  const double t0 = begin_index_call(EMQX_GM_UPD_NONE);
  hipSetDevice(ctx->device);
  return replicated(ctx, gm::update_subs(ctx, prev, fb, fo, subs, ops, n_ops, out), prev, out, t0);
  GM_GUARD_END(ctx)
}

int emqx_gm_index_export(emqx_gm_ctx* ctx, const emqx_gm_index* idx, uint32_t flags, uint8_t* buf, uint64_t* size) {
  if (!ctx) return EMQX_GM_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  if (idx && idx->route) return gm::set_err(ctx, EMQX_GM_EUNSUPPORTED, "index_export: sharded index");
  GM_GUARD_BEGIN
  return gm::index_export(ctx, idx, flags, buf, size);
  GM_GUARD_END(ctx)
}

int emqx_gm_index_device_blob(const emqx_gm_index* idx, const void** d_blob, uint64_t* bytes) {
  if (!idx || !d_blob || !bytes) return EMQX_GM_EINVAL;
  if (idx->ov || idx->dev_subs || !idx->dev_base) return EMQX_GM_EUNSUPPORTED;
  *d_blob = idx->dev_base;
  *bytes = idx->dev_bytes;
  return EMQX_GM_OK;
}

int emqx_gm_index_import(emqx_gm_ctx* ctx, const uint8_t* image, uint64_t size, const void* d_blob,
                         emqx_gm_index** out) {
  if (!ctx) return EMQX_GM_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  GM_GUARD_BEGIN
  const double t0 = begin_index_call(EMQX_GM_UPD_IMPORT);
  hipSetDevice(ctx->device);
  return replicated(ctx, gm::index_import(ctx, image, size, d_blob, out), nullptr, out, t0);
  GM_GUARD_END(ctx)
}

int emqx_gm_index_retain(emqx_gm_index* idx) {
  if (!idx) return EMQX_GM_EINVAL;
  idx->refs.fetch_add(1);
  return EMQX_GM_OK;
}

int emqx_gm_index_release(emqx_gm_index* idx) {
  if (!idx) return EMQX_GM_EINVAL;
  if (idx->refs.fetch_sub(1) == 1) gm::free_index(idx);
  return EMQX_GM_OK;
}

int emqx_gm_index_info(const emqx_gm_index* idx, emqx_gm_index_info_t* info) {
  if (!idx || !info) return EMQX_GM_EINVAL;
  *info = idx->info;
  return EMQX_GM_OK;
}

int emqx_gm_index_filter(const emqx_gm_index* idx, uint32_t id, const uint8_t** bytes, uint64_t* len) {
  if (!idx || !bytes || !len) return EMQX_GM_EINVAL;
  if (idx->ov) return gm::overlay_filter(idx, id, bytes, len);
  if (!idx->gmap.empty()) {  // shard index: ids are global
    auto it = std::lower_bound(idx->gmap.begin(), idx->gmap.end(), id);
    if (it == idx->gmap.end() || *it != id) return EMQX_GM_EINVAL;
    id = uint32_t(it - idx->gmap.begin());
  }
  if (id >= idx->info.n_filters) return EMQX_GM_EINVAL;
  *bytes = idx->ft.at(id, len);
  return EMQX_GM_OK;
}

int emqx_gm_index_subscriber_count(const emqx_gm_index* idx, uint32_t id, uint64_t* n) {
  if (!idx || !n || idx->ov || !idx->gmap.empty()) return EMQX_GM_EINVAL;
  if (id >= idx->info.n_filters) return EMQX_GM_EINVAL;
  *n = idx->subs.empty() ? 0 : idx->subs.count(id);
  return EMQX_GM_OK;
}

// The stats of the calling thread's last match / fan-out call and the
// context it ran on (emqx_gm_last_stats): concurrent callers of one context
// each read their own call's.
static thread_local emqx_gm_match_stats tl_stats;
static thread_local const emqx_gm_ctx* tl_stats_ctx = nullptr;
static int noted(const emqx_gm_ctx* api_ctx, const emqx_gm_ctx* ran, int rc) {
  if (rc == EMQX_GM_OK) {
    tl_stats = ran->stats;
    tl_stats_ctx = api_ctx;
  }
  return rc;
}

// A host-buffer call of at most one chunk (a publish window): ONE device serves
// it whole -- on a multi-device context the next one round-robin -- and the
// call holds that device's lock only while it queues its work and collects
// its rows (gm_host.cpp run_host_small), so concurrent callers (a NIF's dirty
// schedulers) overlap on one device and run on different GPUs at once, as the
// reference's publishers match in their own processes at once
// (apps/emqx/src/emqx_trie.erl:66-70, emqx_router.erl:128-145).  Larger calls
// are cut into chunks spread over every device (gm_host.cpp run_host_pipe).
static int match_small(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const uint8_t* tb, const uint64_t* to, uint64_t n,
                       uint32_t flags, emqx_gm_csr* out, gm::SmallFan* fan = nullptr) {
  const size_t K = 1 + (idx->reps.size() == ctx->members.size() ? ctx->members.size() : 0);
  const size_t pick = K > 1 ? ctx->rr.fetch_add(1, std::memory_order_relaxed) % K : 0;
  emqx_gm_ctx* mc = pick ? ctx->members[pick - 1] : ctx;
  const emqx_gm_index* rix = pick ? idx->reps[pick - 1] : idx;
  hipSetDevice(mc->device);
  emqx_gm_match_stats st{};
  const int rc = gm::run_host_small(mc, rix, tb, to, n, flags, out, &st, fan);
  if (rc == EMQX_GM_OK) {
    tl_stats = st;
    tl_stats_ctx = ctx;
  }
  hipSetDevice(ctx->device);
  return rc;
}

// a host-buffer call that runs whole on one device (run_host_small)
static bool small_call(const emqx_gm_index* idx, const uint64_t* to, uint64_t n, uint32_t flags) {
  return !(flags & EMQX_GM_DEVICE_IO) && !idx->ov && !idx->route && n <= gm::host_chunk_topics() &&
         (n == 0 || to[n] - to[0] <= (uint64_t(64) << 20)) && !gm::knob("GM_HOST_SIMPLE") && !gm::knob("GM_HOST_PIPE");
}

int emqx_gm_match(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const uint8_t* tb, const uint64_t* to,
                  uint64_t n, uint32_t flags, emqx_gm_csr* out) {
  if (!ctx) return EMQX_GM_EINVAL;
  if (!idx || !out || (n && (!tb || !to))) return gm::set_err(ctx, EMQX_GM_EINVAL, "match: NULL argument");
  if (flags & ~(EMQX_GM_WITH_EXACT | EMQX_GM_DEVICE_IO | EMQX_GM_NO_TIMING))
    return gm::set_err(ctx, EMQX_GM_EINVAL, "match: flags");
  if ((flags & EMQX_GM_NO_TIMING) && !(flags & EMQX_GM_DEVICE_IO))
    return gm::set_err(ctx, EMQX_GM_EINVAL, "match: EMQX_GM_NO_TIMING needs EMQX_GM_DEVICE_IO");
  if (n >= 0xFFFFFFF0ull) return gm::set_err(ctx, EMQX_GM_EINVAL, "match: batch too large (>= 2^32 topics)");
  if (idx->device != ctx->device) return gm::set_err(ctx, EMQX_GM_EINVAL, "match: index lives on another device");
  std::memset(out, 0, sizeof(*out));
  GM_GUARD_BEGIN
  if (idx->route) {  // a sharded index: each topic to its one device's shard (gm_shard.cpp)
    if (flags & EMQX_GM_DEVICE_IO)
      return gm::set_err(ctx, EMQX_GM_EUNSUPPORTED, "match: sharded index takes host buffers");
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    hipSetDevice(ctx->device);
    return noted(ctx, ctx, gm::run_match_sharded(ctx, idx, tb, to, n, flags, out));
  }
  if (small_call(idx, to, n, flags)) return match_small(ctx, idx, tb, to, n, flags, out);
  std::unique_lock<std::recursive_mutex> lk(ctx->mu);
  hipSetDevice(ctx->device);
  if (idx->ov) return noted(ctx, ctx, gm::run_match_overlay(ctx, idx, tb, to, n, flags, out));
  if (!(flags & EMQX_GM_DEVICE_IO) && !gm::knob("GM_HOST_SIMPLE"))  // host buffers: chunked, pipelined
    return noted(ctx, ctx, gm::run_match_host(ctx, idx, tb, to, n, flags, out));
  if (!(flags & EMQX_GM_DEVICE_IO)) return noted(ctx, ctx, gm::run_match(ctx, idx, tb, to, n, flags, out));
  // device buffers: the call is queued under the lock and waited for outside
  // it, so concurrent callers' batches queue behind this one meanwhile
  void* t = nullptr;
  const int rc = gm::match_submit(ctx, idx, tb, to, n, flags, &t);
  if (rc) return rc;
  lk.unlock();
  return noted(ctx, ctx, gm::match_wait(ctx, t, out));
  GM_GUARD_END(ctx)
}

int emqx_gm_match_submit(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const uint8_t* tb, const uint64_t* to,
                         uint64_t n, uint32_t flags, emqx_gm_call** call) {
  if (!ctx) return EMQX_GM_EINVAL;
  if (!call) return gm::set_err(ctx, EMQX_GM_EINVAL, "match_submit: NULL call");
  *call = nullptr;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  if (!idx || (n && (!tb || !to))) return gm::set_err(ctx, EMQX_GM_EINVAL, "match_submit: NULL argument");
  if (flags & ~(EMQX_GM_WITH_EXACT | EMQX_GM_DEVICE_IO | EMQX_GM_NO_TIMING))
    return gm::set_err(ctx, EMQX_GM_EINVAL, "match_submit: flags");
  if (!(flags & EMQX_GM_DEVICE_IO))
    return gm::set_err(ctx, EMQX_GM_EINVAL, "match_submit: device buffers only (EMQX_GM_DEVICE_IO)");
  if (n >= 0xFFFFFFF0ull) return gm::set_err(ctx, EMQX_GM_EINVAL, "match_submit: batch too large (>= 2^32 topics)");
  if (idx->device != ctx->device) return gm::set_err(ctx, EMQX_GM_EINVAL, "match_submit: index lives on another device");
  if (idx->ov) return gm::set_err(ctx, EMQX_GM_EUNSUPPORTED, "match_submit: overlay snapshot (use emqx_gm_match)");
  if (idx->route) return gm::set_err(ctx, EMQX_GM_EUNSUPPORTED, "match_submit: sharded index (use emqx_gm_match)");
  GM_GUARD_BEGIN
  hipSetDevice(ctx->device);
  void* t = nullptr;
  const int rc = gm::match_submit(ctx, idx, tb, to, n, flags, &t);
  if (rc == EMQX_GM_OK) *call = static_cast<emqx_gm_call*>(t);
  return rc;
  GM_GUARD_END(ctx)
}

int emqx_gm_match_wait(emqx_gm_ctx* ctx, emqx_gm_call* call, emqx_gm_csr* out) {
  if (!ctx || !call) return EMQX_GM_EINVAL;
  if (!out) return gm::set_err(ctx, EMQX_GM_EINVAL, "match_wait: NULL out");
  std::memset(out, 0, sizeof(*out));
  GM_GUARD_BEGIN
  hipSetDevice(ctx->device);
  return noted(ctx, ctx, gm::match_wait(ctx, call, out));
  GM_GUARD_END(ctx)
}

// A host-row fan-out of a publish window (fewer than 65,536 rows, at most 16M
// deliveries): like match_small, ONE device serves it whole, round-robin over a
// multi-device context's replicas, holding that device's lock only to queue
// its work (gm_host.cpp run_fanout_small).  1: not small, take the ordinary path.
static int fanout_small(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const emqx_gm_csr* m, emqx_gm_csr* out) {
  const size_t K = 1 + (idx->reps.size() == ctx->members.size() ? ctx->members.size() : 0);
  const size_t pick = K > 1 ? ctx->rr.fetch_add(1, std::memory_order_relaxed) % K : 0;
  emqx_gm_ctx* mc = pick ? ctx->members[pick - 1] : ctx;
  const emqx_gm_index* rix = pick ? idx->reps[pick - 1] : idx;
  hipSetDevice(mc->device);
  emqx_gm_match_stats st{};
  const int rc = gm::run_fanout_small(mc, rix, idx, m, out, &st);
  if (rc == EMQX_GM_OK) {
    tl_stats = st;
    tl_stats_ctx = ctx;
  }
  hipSetDevice(ctx->device);
  return rc;
}

int emqx_gm_fanout(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const emqx_gm_csr* m, uint32_t flags,
                   emqx_gm_csr* out) {
  if (!ctx) return EMQX_GM_EINVAL;
  if (idx && m && out && flags == (flags & EMQX_GM_WITH_EXACT) && !m->on_device && m->row_off && (!m->nnz || m->ids) &&
      m->n_rows < 65536 && !idx->view.gmap && !idx->ov && !idx->route && !idx->subs.empty() &&
      idx->device == ctx->device && !gm::knob("GM_FANOUT_SIMPLE")) {
    std::memset(out, 0, sizeof(*out));
    GM_GUARD_BEGIN
    const int rc = fanout_small(ctx, idx, m, out);
    if (rc != 1) return rc;
    GM_GUARD_END(ctx)
  }
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  if (!idx || !m || !out || (m->nnz && !m->ids) || !m->row_off)
    return gm::set_err(ctx, EMQX_GM_EINVAL, "fanout: NULL argument");
  if (flags & ~(EMQX_GM_WITH_EXACT | EMQX_GM_DEVICE_IO)) return gm::set_err(ctx, EMQX_GM_EINVAL, "fanout: flags");
  if (idx->view.gmap) return gm::set_err(ctx, EMQX_GM_EUNSUPPORTED, "fanout: shard index (fan out before merging)");
  if (idx->ov) return gm::set_err(ctx, EMQX_GM_EUNSUPPORTED, "fanout: overlay snapshot (subscribers need a rebuild)");
  std::memset(out, 0, sizeof(*out));
  GM_GUARD_BEGIN
  hipSetDevice(ctx->device);
  if (idx->route) {  // a sharded index: each row on the shard of its filters (gm_shard.cpp)
    if ((flags & EMQX_GM_DEVICE_IO) || m->on_device)
      return gm::set_err(ctx, EMQX_GM_EUNSUPPORTED, "fanout: sharded index takes host rows");
    if (idx->subs.empty()) return gm::set_err(ctx, EMQX_GM_EINVAL, "fanout: index without subscriber lists");
    return noted(ctx, ctx, gm::run_fanout_sharded(ctx, idx, m, flags, out));
  }
  if (!ctx->members.empty() && !(flags & EMQX_GM_DEVICE_IO) && !m->on_device)
    return noted(ctx, ctx, gm::run_fanout_multi(ctx, idx, m, flags, out));
  return noted(ctx, ctx, gm::run_fanout(ctx, idx, m, flags, out));
  GM_GUARD_END(ctx)
}

int emqx_gm_match_fanout(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const uint8_t* tb, const uint64_t* to, uint64_t n,
                         uint32_t flags, emqx_gm_csr* matches, emqx_gm_csr* deliveries) {
  if (!ctx) return EMQX_GM_EINVAL;
  if (!idx || !matches || !deliveries || (n && (!tb || !to)))
    return gm::set_err(ctx, EMQX_GM_EINVAL, "match_fanout: NULL argument");
  if (flags & ~EMQX_GM_WITH_EXACT) return gm::set_err(ctx, EMQX_GM_EINVAL, "match_fanout: flags (host buffers only)");
  if (n >= 0xFFFFFFF0ull) return gm::set_err(ctx, EMQX_GM_EINVAL, "match_fanout: batch too large (>= 2^32 topics)");
  if (idx->device != ctx->device) return gm::set_err(ctx, EMQX_GM_EINVAL, "match_fanout: index lives on another device");
  std::memset(matches, 0, sizeof(*matches));
  std::memset(deliveries, 0, sizeof(*deliveries));
  int rc = EMQX_GM_OK;
  bool fused = false;
  gm::SmallFan fan;
  GM_GUARD_BEGIN
  // a publish window: the fan-out rides the match's one device round trip
  // (gm_host.cpp run_host_small); otherwise, or when its speculation did not
  // hold, the two calls one after the other
  if (small_call(idx, to, n, flags) && !idx->view.gmap && !idx->subs.empty() && !gm::knob("GM_FANOUT_SIMPLE")) {
    rc = match_small(ctx, idx, tb, to, n, flags, matches, &fan);
    if (rc != EMQX_GM_OK) return rc;
    if (fan.ok) {
      *deliveries = fan.out;
      fused = true;
    }
  } else {
    rc = emqx_gm_match(ctx, idx, tb, to, n, flags, matches);
    if (rc != EMQX_GM_OK) return rc;
  }
  GM_GUARD_END(ctx)
  if (fused) return EMQX_GM_OK;
  if (gm::knob("GM_FANOUT_FUSED_ONLY")) {  // (tests: the fused form must have held)
    emqx_gm_csr_free(ctx, matches);
    return gm::set_err(ctx, EMQX_GM_EUNSUPPORTED,
                       "match_fanout: not fused (queued " + std::to_string(fan.queued) + ", speculative rows " +
                           std::to_string(fan.rows_spec) + ", deliveries " + std::to_string(fan.total) + " of " +
                           std::to_string(fan.cap) + ")");
  }
  rc = emqx_gm_fanout(ctx, idx, matches, 0, deliveries);
  if (rc != EMQX_GM_OK) emqx_gm_csr_free(ctx, matches);  // (the error message stays the fan-out's)
  return rc;
}

int emqx_gm_fanout_part(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const emqx_gm_csr* m, uint32_t part,
                        uint32_t n_parts, uint32_t flags, emqx_gm_csr* out, uint64_t* first) {
  if (!ctx) return EMQX_GM_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  if (!idx || !m || !out || (m->nnz && !m->ids) || !m->row_off)
    return gm::set_err(ctx, EMQX_GM_EINVAL, "fanout_part: NULL argument");
  if (!n_parts || part >= n_parts) return gm::set_err(ctx, EMQX_GM_EINVAL, "fanout_part: part out of range");
  if (flags & ~(EMQX_GM_WITH_EXACT | EMQX_GM_DEVICE_IO))
    return gm::set_err(ctx, EMQX_GM_EINVAL, "fanout_part: flags");
  if (idx->view.gmap) return gm::set_err(ctx, EMQX_GM_EUNSUPPORTED, "fanout_part: shard index");
  if (idx->ov) return gm::set_err(ctx, EMQX_GM_EUNSUPPORTED, "fanout_part: overlay snapshot");
  if (idx->route) return gm::set_err(ctx, EMQX_GM_EUNSUPPORTED, "fanout_part: sharded index");
  std::memset(out, 0, sizeof(*out));
  GM_GUARD_BEGIN
  hipSetDevice(ctx->device);
  return noted(ctx, ctx, gm::run_fanout(ctx, idx, m, flags, out, part, n_parts, first));
  GM_GUARD_END(ctx)
}

int emqx_gm_csr_free(emqx_gm_ctx* ctx, emqx_gm_csr* csr) {
  if (!ctx || !csr) return EMQX_GM_EINVAL;
  // a result CSR records its context (priv): its buffers belong to that
  // context's pools, and handing them to another one would corrupt both; a
  // small call's rows belong to the member device that served it
  if (csr->priv && csr->priv != static_cast<void*>(ctx)) {
    emqx_gm_ctx* owner = nullptr;
    for (emqx_gm_ctx* m : ctx->members)
      if (csr->priv == static_cast<void*>(m)) owner = m;
    if (!owner) return gm::set_err(ctx, EMQX_GM_EINVAL, "csr_free: the CSR belongs to another context");
    ctx = owner;
  }
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  if (csr->on_device) {
    // back to the pool once the work queued so far (which may still read the
    // rows: a fan-out, a later call's inputs) is done -- no wait here, so a
    // caller with the next call in flight keeps it in flight
    hipSetDevice(ctx->device);
    void* const bufs[2] = {csr->row_off, csr->ids};
    ctx->pool->release_after(bufs, 2, ctx->stream);
  } else {
    ctx->hpool->release(csr->row_off);
    ctx->hpool->release(csr->ids);
  }
  std::memset(csr, 0, sizeof(*csr));
  return EMQX_GM_OK;
}

int emqx_gm_last_stats(const emqx_gm_ctx* ctx, emqx_gm_match_stats* stats) {
  if (!ctx || !stats) return EMQX_GM_EINVAL;
  *stats = tl_stats_ctx == ctx ? tl_stats : ctx->stats;
  return EMQX_GM_OK;
}

int emqx_gm_last_update_stats(const emqx_gm_ctx* ctx, emqx_gm_update_stats* stats) {
  if (!ctx || !stats) return EMQX_GM_EINVAL;
  *stats = gm::tl_ustats;
  return EMQX_GM_OK;
}

int emqx_gm_index_replica_digest(emqx_gm_ctx* ctx, const emqx_gm_index* idx, uint32_t k, uint64_t* tables,
                                 uint64_t* subs) {
  if (!ctx || !idx || !tables || !subs) return EMQX_GM_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  if (k > idx->reps.size()) return gm::set_err(ctx, EMQX_GM_EINVAL, "replica_digest: no such replica");
  const emqx_gm_index* r = k ? idx->reps[k - 1] : idx;
  GM_GUARD_BEGIN
  auto fnv = [](uint64_t h, const std::vector<uint8_t>& b) {
    for (uint8_t x : b) h = (h ^ x) * 0x100000001B3ull;
    return h;
  };
  hipSetDevice(r->device);
  std::vector<uint8_t> b(r->dev_bytes);
  if (!b.empty()) GM_HIP(ctx, hipMemcpy(b.data(), r->dev_base, b.size(), hipMemcpyDeviceToHost));
  *tables = fnv(0xCBF29CE484222325ull, b);
  *subs = 0;
  if (r->view.sub_off) {
    const uint64_t nf = r->info.n_filters;
    std::vector<uint8_t> o((nf + 1) * 8);
    GM_HIP(ctx, hipMemcpy(o.data(), r->view.sub_off, o.size(), hipMemcpyDeviceToHost));
    uint64_t total = 0;
    std::memcpy(&total, o.data() + nf * 8, 8);
    std::vector<uint8_t> ids(total * 4);
    if (total) GM_HIP(ctx, hipMemcpy(ids.data(), r->view.sub_ids, ids.size(), hipMemcpyDeviceToHost));
    *subs = fnv(fnv(0xCBF29CE484222325ull, o), ids);
  }
  hipSetDevice(ctx->device);
  return EMQX_GM_OK;
  GM_GUARD_END(ctx)
}

// ---- extensions used by the bench / Python host layer (emqx_gm_ext.h) ----
int emqx_gm_matched_filter_bytes(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const emqx_gm_csr* csr,
                                 uint64_t* out) {
  if (!ctx || !idx || !csr || !out || !csr->on_device) return EMQX_GM_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  if (idx->ov || idx->route) return gm::set_err(ctx, EMQX_GM_EUNSUPPORTED, "matched_filter_bytes: overlay or sharded");
  GM_GUARD_BEGIN
  hipSetDevice(ctx->device);
  return gm::sum_filter_lengths(ctx, idx, csr->ids, csr->nnz, out);
  GM_GUARD_END(ctx)
}

int emqx_gm_index_compile_host(const uint8_t* fb, const uint64_t* fo, uint64_t n, const uint64_t* sub_off,
                               const uint32_t* sub_ids, uint32_t* perm_out, emqx_gm_index_info_t* info) {
  if (!info) return EMQX_GM_EINVAL;
  GM_GUARD_BEGIN
  return gm::build_index(nullptr, fb, fo, n, sub_off, sub_ids, perm_out, nullptr, info);
  GM_GUARD_END(nullptr)
}

// ---- sharded index ----
int emqx_gm_filter_ranks(const uint8_t* fb, const uint64_t* fo, uint64_t n, uint32_t* rank_out, uint64_t* n_unique) {
  if (n && (!fb || !fo || !rank_out)) return EMQX_GM_EINVAL;
  GM_GUARD_BEGIN
  std::vector<uint32_t> ord(n);
  for (uint64_t i = 0; i < n; ++i) ord[i] = uint32_t(i);
  gm::sort_filters(ord, fb, fo);
  uint32_t r = 0;
  for (uint64_t k = 0; k < n; ++k) {
    const uint32_t i = ord[k];
    if (k) {
      const uint32_t p = ord[k - 1];
      const uint64_t lp = fo[p + 1] - fo[p], li = fo[i + 1] - fo[i];
      if (lp != li || std::memcmp(fb + fo[p], fb + fo[i], li) != 0) ++r;
    }
    rank_out[i] = r;
  }
  if (n_unique) *n_unique = n ? uint64_t(r) + 1 : 0;
  return EMQX_GM_OK;
  GM_GUARD_END(nullptr)
}

int emqx_gm_shard_of(const uint8_t* fb, const uint64_t* fo, uint64_t n, uint32_t n_shards, uint32_t* out) {
  if (!n_shards || (n && (!fb || !fo || !out))) return EMQX_GM_EINVAL;
  for (uint64_t i = 0; i < n; ++i)
    out[i] = uint32_t(gm::fmix64(gm::hash_word_host(fb + fo[i], fo[i + 1] - fo[i]) ^ 0x5BD1E995ull) % n_shards);
  return EMQX_GM_OK;
}

int emqx_gm_select_filters(const uint8_t* fb, const uint64_t* fo, uint64_t n, const uint32_t* shard, uint32_t want,
                           uint8_t* out_b, uint64_t* out_o, uint64_t* n_out, uint64_t* bytes_out) {
  if (!n_out || !bytes_out || (n && (!fb || !fo || !shard))) return EMQX_GM_EINVAL;
  uint64_t k = 0, b = 0;
  for (uint64_t i = 0; i < n; ++i) {
    if (shard[i] != want) continue;
    const uint64_t len = fo[i + 1] - fo[i];
    if (out_b && out_o) {
      out_o[k] = b;
      std::memcpy(out_b + b, fb + fo[i], len);
    }
    ++k;
    b += len;
  }
  if (out_o) out_o[k] = b;
  *n_out = k;
  *bytes_out = b;
  return EMQX_GM_OK;
}

int emqx_gm_index_build_shard(emqx_gm_ctx* ctx, const uint8_t* fb, const uint64_t* fo, uint64_t n,
                              const uint32_t* global_ids, const uint64_t* sub_off, const uint32_t* sub_ids,
                              uint32_t* perm_out, emqx_gm_index** out) {
  if (!ctx) return EMQX_GM_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  if (n && !global_ids) return gm::set_err(ctx, EMQX_GM_EINVAL, "index_build_shard: global_ids is NULL");
  GM_GUARD_BEGIN
  const double t0 = begin_index_call(EMQX_GM_UPD_BUILD);
  hipSetDevice(ctx->device);
  return replicated(ctx, gm::build_index(ctx, fb, fo, n, sub_off, sub_ids, perm_out, out, nullptr, global_ids),
                    nullptr, out, t0);
  GM_GUARD_END(ctx)
}

int emqx_gm_csr_row_lengths(emqx_gm_ctx* ctx, const emqx_gm_csr* csr, uint32_t* d_lens) {
  if (!ctx) return EMQX_GM_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  if (!csr || !csr->on_device || !d_lens || !csr->row_off)
    return gm::set_err(ctx, EMQX_GM_EINVAL, "csr_row_lengths: needs a device CSR and a device output");
  GM_GUARD_BEGIN
  hipSetDevice(ctx->device);
  return gm::run_row_lengths(ctx, csr, d_lens);
  GM_GUARD_END(ctx)
}

int emqx_gm_merge_rows(emqx_gm_ctx* ctx, uint64_t n_rows, uint64_t stride, uint32_t n_pieces, const uint32_t* d_lens,
                       const uint32_t* d_ids, uint32_t flags, emqx_gm_csr* out) {
  if (!ctx) return EMQX_GM_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  if (!out || stride < n_rows || !n_pieces || (n_rows && (!d_lens || !d_ids)))
    return gm::set_err(ctx, EMQX_GM_EINVAL, "merge_rows: bad arguments");
  if (flags & ~EMQX_GM_DEVICE_IO) return gm::set_err(ctx, EMQX_GM_EINVAL, "merge_rows: flags");
  std::memset(out, 0, sizeof(*out));
  GM_GUARD_BEGIN
  hipSetDevice(ctx->device);
  return gm::run_merge_rows(ctx, n_rows, stride, n_pieces, d_lens, d_ids, flags, out);
  GM_GUARD_END(ctx)
}

// ---- prefix sharding ----
int emqx_gm_prefix_plan(const uint8_t* fb, const uint64_t* fo, uint64_t n, uint32_t n_shards, uint32_t* shard_out,
                        emqx_gm_route** route) {
  if (!route || !n_shards || (n && (!fb || !fo || !shard_out))) return EMQX_GM_EINVAL;
  *route = nullptr;
  GM_GUARD_BEGIN
  return gm::route_plan(fb, fo, n, n_shards, shard_out, route);
  GM_GUARD_END(nullptr)
}

int emqx_gm_route_topics_host(const emqx_gm_route* route, const uint8_t* tb, const uint64_t* to, uint64_t n,
                              uint32_t* dest) {
  if (!route || (n && (!tb || !to || !dest))) return EMQX_GM_EINVAL;
  return gm::route_topics_host(route, tb, to, n, dest);
}

int emqx_gm_route_topics(emqx_gm_ctx* ctx, emqx_gm_route* route, const uint8_t* d_tb, const uint64_t* d_to, uint64_t n,
                         uint32_t* d_dest) {
  if (!ctx) return EMQX_GM_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  if (!route || (n && (!d_tb || !d_to || !d_dest))) return gm::set_err(ctx, EMQX_GM_EINVAL, "route_topics: NULL argument");
  if (n >= 0xFFFFFFFFull)  // (u32 batch indices: perm, dest)
    return gm::set_err(ctx, EMQX_GM_EINVAL, "route_topics: batch too large (>= 2^32 topics)");
  GM_GUARD_BEGIN
  hipSetDevice(ctx->device);
  return gm::route_topics_device(ctx, route, d_tb, d_to, n, d_dest);
  GM_GUARD_END(ctx)
}

int emqx_gm_route_partition(emqx_gm_ctx* ctx, emqx_gm_route* route, const uint8_t* d_tb, const uint64_t* d_to,
                            uint64_t n, uint32_t* d_perm, uint32_t* d_plen, uint64_t* d_split) {
  if (!ctx) return EMQX_GM_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  if (!route || !d_split || (n && (!d_tb || !d_to || !d_perm || !d_plen)))
    return gm::set_err(ctx, EMQX_GM_EINVAL, "route_partition: NULL argument");
  if (n >= 0xFFFFFFFFull)  // (u32 batch indices: perm, dest)
    return gm::set_err(ctx, EMQX_GM_EINVAL, "route_partition: batch too large (>= 2^32 topics)");
  GM_GUARD_BEGIN
  hipSetDevice(ctx->device);
  return gm::route_partition(ctx, route, d_tb, d_to, n, d_perm, d_plen, d_split);
  GM_GUARD_END(ctx)
}

int emqx_gm_route_release(emqx_gm_route* route) {
  if (!route) return EMQX_GM_EINVAL;
  gm::free_route(route);
  return EMQX_GM_OK;
}

int emqx_gm_permute_topics(emqx_gm_ctx* ctx, const uint8_t* d_tb, const uint64_t* d_to, uint64_t n,
                           const uint32_t* d_perm, uint8_t* d_out, uint64_t* d_out_off) {
  if (!ctx) return EMQX_GM_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  if (!d_out_off || (n && (!d_tb || !d_to || !d_perm || !d_out)))
    return gm::set_err(ctx, EMQX_GM_EINVAL, "permute_topics: NULL argument");
  if (n >= 0xFFFFFFFFull)  // (u32 batch indices: perm, dest)
    return gm::set_err(ctx, EMQX_GM_EINVAL, "permute_topics: batch too large (>= 2^32 topics)");
  GM_GUARD_BEGIN
  hipSetDevice(ctx->device);
  return gm::permute_topics(ctx, d_tb, d_to, n, d_perm, d_out, d_out_off);
  GM_GUARD_END(ctx)
}

int emqx_gm_unpermute_rows(emqx_gm_ctx* ctx, uint64_t n, const uint32_t* d_perm, const uint32_t* d_lens,
                           const uint32_t* d_ids, uint32_t flags, emqx_gm_csr* out) {
  if (!ctx) return EMQX_GM_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  if (!out || (n && (!d_perm || !d_lens || !d_ids)))
    return gm::set_err(ctx, EMQX_GM_EINVAL, "unpermute_rows: NULL argument");
  if (n >= 0xFFFFFFFFull)  // (u32 batch indices: perm, dest)
    return gm::set_err(ctx, EMQX_GM_EINVAL, "unpermute_rows: batch too large (>= 2^32 topics)");
  if (flags & ~EMQX_GM_DEVICE_IO) return gm::set_err(ctx, EMQX_GM_EINVAL, "unpermute_rows: flags");
  std::memset(out, 0, sizeof(*out));
  GM_GUARD_BEGIN
  hipSetDevice(ctx->device);
  return gm::unpermute_rows(ctx, n, d_perm, d_lens, d_ids, flags, out);
  GM_GUARD_END(ctx)
}

int emqx_gm_pool_trim(emqx_gm_ctx* ctx) {
  if (!ctx) return EMQX_GM_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  ctx->pool->trim();
  gm::trim_spare_blob(ctx->device);
  for (emqx_gm_ctx* m : ctx->members) {
    std::lock_guard<std::recursive_mutex> ml(m->mu);  // (small calls hold only a member's lock)
    m->pool->trim();
    gm::trim_spare_blob(m->device);
  }
  return EMQX_GM_OK;
}

}  // extern "C"
