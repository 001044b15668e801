// gm_workload.hip — seeded synthetic workloads of SURVEY.md §8d (spec in
// DESIGN.md "Workload generator").  Topics are generated ON the device,
// counter-based (topic i depends only on (seed, i)), so a 100M-topic batch is
// resident in HBM before the timed region without a host round trip.  The
// oracle (oracle/emqx_oracle.cpp) restates the same spec independently and
// tests/test_gpu_parity.py checks the two agree byte-for-byte.
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/emqx_gm_ext.h"
#include "gm_internal.h"

namespace gm {
namespace {

constexpr int kLevels = 5;
__host__ __device__ __forceinline__ int vocab(int l) {
  return l == 0 ? 64 : l == 1 ? 1024 : l == 2 ? 1024 : l == 3 ? 64 : 16;
}
constexpr int16_t C_PLUS = -1, C_HASH = -2, C_END = -3;

struct Rng {
  uint64_t s;
  __host__ __device__ __forceinline__ uint64_t next() {
    s += 0x9E3779B97F4A7C15ull;
    uint64_t z = s;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
};
__host__ __device__ __forceinline__ uint64_t mix(uint64_t x) {
  Rng r{x};
  return r.next();
}

__host__ __device__ __forceinline__ void topic_codes(uint64_t seed, uint64_t idx, const int16_t* fc, uint64_t nf,
                                                     int16_t out[kLevels]) {
  Rng r{mix(mix(seed ^ 0x70C1Cull) ^ (idx * 0xD1B54A32D192ED03ull))};
  if (nf == 0 || (r.next() & 1) == 0) {
    for (int l = 0; l < kLevels; ++l) out[l] = int16_t(r.next() % vocab(l));
    return;
  }
  const int16_t* c = fc + (r.next() % nf) * kLevels;
  for (int l = 0; l < kLevels; ++l) {
    const int16_t x = c[l];
    if (x >= 0) {
      out[l] = x;
    } else if (x == C_PLUS) {
      out[l] = int16_t(r.next() % vocab(l));
    } else {
      for (int m = l; m < kLevels; ++m) out[m] = int16_t(r.next() % vocab(m));
      break;
    }
  }
}

__host__ __device__ __forceinline__ uint32_t ndigits(uint32_t v) {
  return v >= 1000 ? 4 : v >= 100 ? 3 : v >= 10 ? 2 : 1;
}

__global__ __launch_bounds__(256) void k_topic_len(uint64_t seed, uint64_t start, uint64_t n,
                                                   const int16_t* __restrict__ fc, uint64_t nf,
                                                   uint64_t* __restrict__ len) {
  const uint64_t i = uint64_t(blockIdx.x) * 256u + threadIdx.x;
  if (i >= n) return;
  int16_t c[kLevels];
  topic_codes(seed, start + i, fc, nf, c);
  uint32_t L = kLevels - 1;
  for (int l = 0; l < kLevels; ++l) L += 3 + ndigits(uint32_t(c[l]));
  len[i] = L;
}

__global__ __launch_bounds__(256) void k_topic_write(uint64_t seed, uint64_t start, uint64_t n,
                                                     const int16_t* __restrict__ fc, uint64_t nf,
                                                     const uint64_t* __restrict__ off, uint8_t* __restrict__ out) {
  const uint64_t i = uint64_t(blockIdx.x) * 256u + threadIdx.x;
  if (i >= n) return;
  int16_t c[kLevels];
  topic_codes(seed, start + i, fc, nf, c);
  uint8_t* p = out + off[i];
  for (int l = 0; l < kLevels; ++l) {
    if (l) *p++ = '/';
    *p++ = 'l';
    *p++ = uint8_t('0' + l);
    *p++ = 'w';
    const uint32_t v = uint32_t(c[l]);
    const uint32_t d = ndigits(v);
    uint32_t x = v;
    for (int k = int(d) - 1; k >= 0; --k) {
      p[k] = uint8_t('0' + x % 10);
      x /= 10;
    }
    p += d;
  }
}

struct LoadLen {
  const uint64_t* p;
  __device__ uint64_t operator()(uint64_t i) const { return p[i]; }
};

}  // namespace

// scan helper from gm_match.hip
int scan_lengths(emqx_gm_ctx* ctx, const uint64_t* len, uint64_t n, uint64_t* out);

}  // namespace gm

using namespace gm;

extern "C" {

int emqx_gm_gen_filter_codes(uint64_t seed, uint64_t n, int wildcard_only, int16_t* codes) {
  if (!codes && n) return EMQX_GM_EINVAL;
  try {
    Rng r{mix(seed ^ 0xF17E5ull)};
    // the filters drawn so far (a flat open-addressing set of their keys + 1:
    // C5 draws 100M, which a node-based set made the slowest part of the bench's setup)
    uint64_t cap = 64;
    while (cap < 2 * n + 16) cap <<= 1;
    std::vector<uint64_t> seen(cap, 0);
    const uint64_t mask = cap - 1;
    auto insert = [&](uint64_t key) {
      const uint64_t k1 = key + 1;
      for (uint64_t h = mix(key) & mask;; h = (h + 1) & mask) {
        if (seen[h] == k1) return false;
        if (!seen[h]) {
          seen[h] = k1;
          return true;
        }
      }
    };
    uint64_t got = 0;
    while (got < n) {
      int16_t c[kLevels];
      for (int l = 0; l < kLevels; ++l) c[l] = C_END;
      const uint64_t kind = wildcard_only ? 20 + r.next() % 80 : r.next() % 100;
      if (kind < 20) {  // exact
        for (int l = 0; l < kLevels; ++l) c[l] = int16_t(r.next() % vocab(l));
      } else if (kind < 60) {  // one '+'
        for (int l = 0; l < kLevels; ++l) c[l] = int16_t(r.next() % vocab(l));
        c[r.next() % kLevels] = C_PLUS;
      } else if (kind < 90) {  // depth-k '#'
        const int k = 2 + int(r.next() % 3);
        for (int l = 0; l < k; ++l) c[l] = int16_t(r.next() % vocab(l));
        c[k] = C_HASH;
      } else {  // '+' at a non-root level, then '#'
        const int p = 1 + int(r.next() % 3);
        for (int l = 0; l < p; ++l) c[l] = int16_t(r.next() % vocab(l));
        c[p] = C_PLUS;
        c[p + 1] = C_HASH;
      }
      uint64_t key = 0;
      for (int l = 0; l < kLevels; ++l) key = key * 1031 + uint64_t(c[l] + 3);
      if (!insert(key)) continue;
      std::memcpy(codes + got * kLevels, c, sizeof(c));
      ++got;
    }
  } catch (...) {
    return EMQX_GM_ENOMEM;
  }
  return EMQX_GM_OK;
}

// "l<level>w<code>" words joined by '/' ('+' / '#' for the wildcards), on all
// threads: each range of filters measured, then written at its prefix offset
uint64_t emqx_gm_render_codes(const int16_t* codes, uint64_t n, uint8_t* bytes, uint64_t* off) {
  auto len_of = [&](uint64_t i) {
    const int16_t* c = codes + i * kLevels;
    uint64_t L = 0;
    for (int l = 0; l < kLevels && c[l] != C_END; ++l)
      L += (l ? 1u : 0u) + ((c[l] == C_PLUS || c[l] == C_HASH) ? 1u : 3u + ndigits(uint32_t(c[l])));
    return L;
  };
  auto write = [&](uint64_t i, uint8_t* p) {
    const int16_t* c = codes + i * kLevels;
    for (int l = 0; l < kLevels && c[l] != C_END; ++l) {
      if (l) *p++ = '/';
      if (c[l] == C_PLUS || c[l] == C_HASH) {
        *p++ = c[l] == C_PLUS ? '+' : '#';
        continue;
      }
      *p++ = 'l';
      *p++ = uint8_t('0' + l);
      *p++ = 'w';
      const uint32_t v = uint32_t(c[l]), d = ndigits(v);
      for (uint32_t k = 0, x = v; k < d; ++k, x /= 10) p[d - 1 - k] = uint8_t('0' + x % 10);
      p += d;
    }
  };
  const unsigned T = n < (1u << 16) ? 1u : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  std::vector<uint64_t> part(T + 1, 0);
  auto ranges = [&](auto body) {
    std::vector<std::thread> th;
    for (unsigned r = 1; r < T; ++r) th.emplace_back([&, r] { body(r, n * r / T, n * (r + 1) / T); });
    body(0u, uint64_t(0), n / T);
    for (auto& t : th) t.join();
  };
  ranges([&](unsigned r, uint64_t a, uint64_t b) {
    uint64_t L = 0;
    for (uint64_t i = a; i < b; ++i) L += len_of(i);
    part[r + 1] = L;
  });
  for (unsigned r = 0; r < T; ++r) part[r + 1] += part[r];
  if (off || bytes)
    ranges([&](unsigned r, uint64_t a, uint64_t b) {
      uint64_t pos = part[r];
      for (uint64_t i = a; i < b; ++i) {
        if (off) off[i] = pos;
        if (bytes) write(i, bytes + pos);
        pos += len_of(i);
      }
    });
  if (off) off[n] = part[T];
  return part[T];
}

int emqx_gm_gen_topics(emqx_gm_ctx* ctx, const int16_t* fcodes, uint64_t nf, uint64_t seed, uint64_t start,
                       uint64_t n, uint8_t** d_bytes, uint64_t** d_off, uint64_t* total_bytes) {
  if (!ctx || !d_bytes || !d_off || (nf && !fcodes)) return EMQX_GM_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  hipSetDevice(ctx->device);
  hipStream_t st = ctx->stream;
  PoolBuf fc(ctx->pool, nf * kLevels * 2 + 16), len(ctx->pool, n * 8 + 8);
  PoolBuf off(ctx->pool, (n + 1) * 8);
  if (!fc.p || !len.p || !off.p) return set_err(ctx, EMQX_GM_ENOMEM, "gen_topics: workspace");
  if (nf) GM_HIP(ctx, hipMemcpyAsync(fc.p, fcodes, nf * kLevels * 2, hipMemcpyHostToDevice, st));
  const dim3 g((n + 255) / 256);
  if (n) {
    hipLaunchKernelGGL(k_topic_len, g, dim3(256), 0, st, seed, start, n, fc.as<int16_t>(), nf, len.as<uint64_t>());
    GM_HIP(ctx, hipGetLastError());
  }
  int rc = scan_lengths(ctx, len.as<uint64_t>(), n, off.as<uint64_t>());
  if (rc) return rc;
  uint64_t total = 0;
  GM_HIP(ctx, hipMemcpyAsync(&total, off.as<uint64_t>() + n, 8, hipMemcpyDeviceToHost, st));
  GM_HIP(ctx, hipStreamSynchronize(st));
  PoolBuf bytes(ctx->pool, total + 64);
  if (!bytes.p) return set_err(ctx, EMQX_GM_ENOMEM, "gen_topics: bytes");
  GM_HIP(ctx, hipMemsetAsync(bytes.p, 0, total + 64, st));
  if (n) {
    hipLaunchKernelGGL(k_topic_write, g, dim3(256), 0, st, seed, start, n, fc.as<int16_t>(), nf, off.as<uint64_t>(),
                       bytes.as<uint8_t>());
    GM_HIP(ctx, hipGetLastError());
  }
  GM_HIP(ctx, hipStreamSynchronize(st));
  *d_bytes = static_cast<uint8_t*>(bytes.release_ownership());
  *d_off = static_cast<uint64_t*>(off.release_ownership());
  if (total_bytes) *total_bytes = total;
  return EMQX_GM_OK;
}

int emqx_gm_dev_alloc(emqx_gm_ctx* ctx, uint64_t bytes, void** out) {
  if (!ctx || !out) return EMQX_GM_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  *out = ctx->pool->alloc(bytes ? bytes : 16);
  return *out ? EMQX_GM_OK : set_err(ctx, EMQX_GM_ENOMEM, "dev_alloc");
}

int emqx_gm_dev_free(emqx_gm_ctx* ctx, void* p) {
  if (!ctx) return EMQX_GM_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  hipSetDevice(ctx->device);
  hipStreamSynchronize(ctx->stream);
  ctx->pool->release(p);
  return EMQX_GM_OK;
}

int emqx_gm_memcpy(emqx_gm_ctx* ctx, void* dst, const void* src, uint64_t bytes, int kind) {
  if (!ctx) return EMQX_GM_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(ctx->mu);
  hipSetDevice(ctx->device);
  const hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice : kind == 1 ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
  GM_HIP(ctx, hipMemcpyAsync(dst, src, bytes, k, ctx->stream));
  GM_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return EMQX_GM_OK;
}

}  // extern "C"
