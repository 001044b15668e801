// gm_api.cpp — extern "C" boundary of libemqx_gpu_match.so (include/emqx_gpu_match.h).
// No C++ exception crosses the ABI; every failure is an EMQX_GM_E* code with
// the message in emqx_gm_last_error().
#include <cstring>
#include <new>
#include <stdexcept>

#include "gm_internal.h"

namespace gm {

int set_err(emqx_gm_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  return code;
}

DevPool::~DevPool() {
  hipSetDevice(device_);
  for (auto& kv : free_) hipFree(kv.second);
  for (auto& kv : live_) hipFree(kv.first);
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

int emqx_gm_open(const emqx_gm_opts* opts, emqx_gm_ctx** out) {
  if (!out) return EMQX_GM_EINVAL;
  *out = nullptr;
  GM_GUARD_BEGIN
  int dev = opts ? opts->device : 0;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return EMQX_GM_EDEVICE;
  if (dev < 0 || dev >= count) return EMQX_GM_EINVAL;
  if (hipSetDevice(dev) != hipSuccess) return EMQX_GM_EDEVICE;
  auto* ctx = new emqx_gm_ctx;
  ctx->device = dev;
  if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
    delete ctx;
    return EMQX_GM_EDEVICE;
  }
  ctx->own_stream = true;
  for (auto& e : ctx->ev) {
    if (hipEventCreate(&e) != hipSuccess) {
      delete ctx;
      return EMQX_GM_EDEVICE;
    }
  }
  ctx->pool = new gm::DevPool(dev);
  *out = ctx;
  return EMQX_GM_OK;
  GM_GUARD_END(nullptr)
}

int emqx_gm_close(emqx_gm_ctx* ctx) {
  if (!ctx) return EMQX_GM_EINVAL;
  {
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    hipSetDevice(ctx->device);
    if (ctx->stream) hipStreamSynchronize(ctx->stream);
    delete ctx->pool;
    for (auto& e : ctx->ev)
      if (e) hipEventDestroy(e);
    if (ctx->own_stream && ctx->stream) hipStreamDestroy(ctx->stream);
  }
  delete ctx;
  return EMQX_GM_OK;
}

const char* emqx_gm_last_error(const emqx_gm_ctx* ctx) { return ctx ? ctx->err.c_str() : "no context"; }

int emqx_gm_set_stream(emqx_gm_ctx* ctx, void* s) {
  if (!ctx) return EMQX_GM_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  hipSetDevice(ctx->device);
  hipStreamSynchronize(ctx->stream);
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
  hipSetDevice(ctx->device);
  GM_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return EMQX_GM_OK;
}

int emqx_gm_index_build(emqx_gm_ctx* ctx, const uint8_t* fb, const uint64_t* fo, uint64_t n,
                        const uint64_t* sub_off, const uint32_t* sub_ids, uint32_t* perm_out,
                        emqx_gm_index** out) {
  if (!ctx) return EMQX_GM_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  GM_GUARD_BEGIN
  hipSetDevice(ctx->device);
  return gm::build_index(ctx, fb, fo, n, sub_off, sub_ids, perm_out, out);
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
  if (!idx || !bytes || !len || id >= idx->info.n_filters) return EMQX_GM_EINVAL;
  *bytes = idx->fbytes.data() + idx->foff[id];
  *len = idx->foff[id + 1] - idx->foff[id];
  return EMQX_GM_OK;
}

int emqx_gm_match(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const uint8_t* tb, const uint64_t* to,
                  uint64_t n, uint32_t flags, emqx_gm_csr* out) {
  if (!ctx) return EMQX_GM_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  if (!idx || !out || (n && (!tb || !to))) return gm::set_err(ctx, EMQX_GM_EINVAL, "match: NULL argument");
  if (flags & ~(EMQX_GM_WITH_EXACT | EMQX_GM_DEVICE_IO)) return gm::set_err(ctx, EMQX_GM_EINVAL, "match: flags");
  if (n >= 0xFFFFFFF0ull) return gm::set_err(ctx, EMQX_GM_EINVAL, "match: batch too large (>= 2^32 topics)");
  if (idx->device != ctx->device) return gm::set_err(ctx, EMQX_GM_EINVAL, "match: index lives on another device");
  std::memset(out, 0, sizeof(*out));
  GM_GUARD_BEGIN
  hipSetDevice(ctx->device);
  return gm::run_match(ctx, idx, tb, to, n, flags, out);
  GM_GUARD_END(ctx)
}

int emqx_gm_fanout(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const emqx_gm_csr* m, uint32_t flags,
                   emqx_gm_csr* out) {
  if (!ctx) return EMQX_GM_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  if (!idx || !m || !out || (m->nnz && !m->ids) || !m->row_off)
    return gm::set_err(ctx, EMQX_GM_EINVAL, "fanout: NULL argument");
  if (flags & ~(EMQX_GM_WITH_EXACT | EMQX_GM_DEVICE_IO)) return gm::set_err(ctx, EMQX_GM_EINVAL, "fanout: flags");
  std::memset(out, 0, sizeof(*out));
  GM_GUARD_BEGIN
  hipSetDevice(ctx->device);
  return gm::run_fanout(ctx, idx, m, flags, out);
  GM_GUARD_END(ctx)
}

int emqx_gm_csr_free(emqx_gm_ctx* ctx, emqx_gm_csr* csr) {
  if (!ctx || !csr) return EMQX_GM_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  if (csr->on_device) {
    hipSetDevice(ctx->device);
    hipStreamSynchronize(ctx->stream);
    if (csr->row_off) ctx->pool->release(csr->row_off);
    if (csr->ids) ctx->pool->release(csr->ids);
  } else {
    free(csr->row_off);
    free(csr->ids);
  }
  std::memset(csr, 0, sizeof(*csr));
  return EMQX_GM_OK;
}

int emqx_gm_last_stats(const emqx_gm_ctx* ctx, emqx_gm_match_stats* stats) {
  if (!ctx || !stats) return EMQX_GM_EINVAL;
  *stats = ctx->stats;
  return EMQX_GM_OK;
}

// ---- extensions used by the bench / Python host layer (emqx_gm_ext.h) ----
int emqx_gm_matched_filter_bytes(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const emqx_gm_csr* csr,
                                 uint64_t* out) {
  if (!ctx || !idx || !csr || !out || !csr->on_device) return EMQX_GM_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
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

int emqx_gm_pool_trim(emqx_gm_ctx* ctx) {
  if (!ctx) return EMQX_GM_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  ctx->pool->trim();
  return EMQX_GM_OK;
}

}  // extern "C"
