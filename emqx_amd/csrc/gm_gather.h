// gm_gather.h — one contiguous output range from n variable-length segments
// (the prefix plan's topic permute, gm_route.hip, and its row un-permute,
// gm_match.hip).  Segment i (SEG::at(i) = its first element and length in src)
// lands at dst + out_off[i]; out_off is the exclusive scan of the lengths.
//
// A block takes 256 consecutive segments = one contiguous output range.  Its
// 16-lane groups gather the segments into LDS at their output positions --
// the LDS image is aligned to the output's 16-B grid, and source bytes are
// read as aligned dwords (up to 3 bytes either side of a segment: an aligned
// dword never leaves its page, so never its allocation) -- and the block then
// writes its range once, with 16-B non-temporal stores, using element stores
// only for the partial 16-B chunks at its two ends (the neighbouring blocks
// own the other bytes of those chunks).  The byte-per-lane copy this replaces
// ran at ~0.4 TB/s (7.3 ms for a 100M-topic batch, profiles/r04_h).  A block
// whose range passes the LDS buffer (topics averaging > 96 B) copies element
// by element.  The 256 spans are loaded first, one per thread, so a group's
// chain of dependent loads (perm -> offsets -> data) is not serialised per
// segment; a 16-lane group then loads four segments' first dwords together.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace gm {

constexpr uint32_t GATHER_LDS = 24576;

struct SegSpan {
  uint64_t first, len;  // elements of src
};

template <class T, class SEG>
__global__ __launch_bounds__(256) void k_gather_segs(const T* __restrict__ src, SEG seg, uint64_t n,
                                                     const uint64_t* __restrict__ out_off, T* __restrict__ dst) {
  static_assert(sizeof(T) == 1 || sizeof(T) == 4, "bytes or 32-bit ids");
  __shared__ __align__(16) uint8_t s_buf[GATHER_LDS + 32];
  __shared__ uintptr_t s_src[256];  // a segment's first source byte
  __shared__ uint32_t s_len[256], s_lds[256];  // its length (elements), its LDS byte
  const uint64_t i0 = uint64_t(blockIdx.x) * 256u;
  if (i0 >= n) return;
  const uint64_t i1 = i0 + 256 < n ? i0 + 256 : n;
  const uint64_t o0 = out_off[i0], o1 = out_off[i1];
  const uintptr_t g0 = reinterpret_cast<uintptr_t>(dst + o0), g1 = reinterpret_cast<uintptr_t>(dst + o1);
  const uintptr_t base = g0 & ~uintptr_t(15);  // LDS byte 0 <-> this global address
  const int tid = threadIdx.x;
  const uint64_t i = i0 + tid;
  if (g1 - base > GATHER_LDS) {  // block-uniform: element by element, a thread per segment
    if (i < i1) {
      const SegSpan sl = seg.at(i);
      const uint64_t d = out_off[i];
      for (uint64_t k = 0; k < sl.len; ++k) dst[d + k] = src[sl.first + k];
    }
    return;
  }
  // ---- the 256 segments' spans, one per thread (their dependent loads in parallel)
  if (i < i1) {
    const SegSpan sl = seg.at(i);
    s_src[tid] = reinterpret_cast<uintptr_t>(src + sl.first);
    s_len[tid] = uint32_t(sl.len);  // < GATHER_LDS
    s_lds[tid] = uint32_t(reinterpret_cast<uintptr_t>(dst + out_off[i]) - base);
  } else {
    s_len[tid] = 0;
  }
  __syncthreads();
  // ---- gather: 16-lane group q takes segments q + 16 j, four at a time with
  // their first 16 units loaded together (a unit = an aligned source dword)
  const int q = tid >> 4, sub = tid & 15;
  constexpr int B = 4;
  for (int j0 = 0; j0 < 16; j0 += B) {
    uint32_t v[B];
#pragma unroll
    for (int b = 0; b < B; ++b) {
      const int k = q + 16 * (j0 + b);
      const uintptr_t a = s_src[k];
      const uint32_t len = s_len[k];
      if constexpr (sizeof(T) == 4) {
        v[b] = uint32_t(sub) < len ? *reinterpret_cast<const uint32_t*>(a + 4 * sub) : 0u;
      } else {
        const uintptr_t a4 = a & ~uintptr_t(3);
        const uint32_t nw = uint32_t((a - a4 + len + 3) >> 2);
        v[b] = len && uint32_t(sub) < nw ? *reinterpret_cast<const uint32_t*>(a4 + 4 * sub) : 0u;
      }
    }
#pragma unroll
    for (int b = 0; b < B; ++b) {
      const int k = q + 16 * (j0 + b);
      const uintptr_t a = s_src[k];
      const uint32_t len = s_len[k], l0 = s_lds[k];
      if (!len) continue;
      if constexpr (sizeof(T) == 4) {
        if (uint32_t(sub) < len) *reinterpret_cast<uint32_t*>(s_buf + l0 + 4 * sub) = v[b];
        for (uint32_t e = sub + 16; e < len; e += 16)  // rows longer than 16 ids
          *reinterpret_cast<uint32_t*>(s_buf + l0 + 4 * e) = *reinterpret_cast<const uint32_t*>(a + 4 * e);
      } else {
        const uintptr_t a4 = a & ~uintptr_t(3);
        const uint32_t nw = uint32_t((a - a4 + len + 3) >> 2);
        for (uint32_t w = sub; w < nw; w += 16) {  // topics longer than ~60 bytes: more dwords
          const uint32_t x = w == uint32_t(sub) ? v[b] : *reinterpret_cast<const uint32_t*>(a4 + 4 * w);
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const uintptr_t sa = a4 + 4 * w + c;
            if (sa >= a && sa < a + len) s_buf[l0 + (sa - a)] = uint8_t(x >> (8 * c));
          }
        }
      }
    }
  }
  __syncthreads();
  // ---- write: whole 16-B chunks inside [g0, g1) as 16-B stores, the ends per element
  const uintptr_t c0 = (g0 + 15) & ~uintptr_t(15), c1 = g1 & ~uintptr_t(15);
  if (c0 < c1) {
    for (uintptr_t c = c0 + 16 * uintptr_t(tid); c < c1; c += 16 * 256) {
      const uint4 v = *reinterpret_cast<const uint4*>(s_buf + (c - base));
      __builtin_nontemporal_store(v.x, reinterpret_cast<uint32_t*>(c));
      __builtin_nontemporal_store(v.y, reinterpret_cast<uint32_t*>(c) + 1);
      __builtin_nontemporal_store(v.z, reinterpret_cast<uint32_t*>(c) + 2);
      __builtin_nontemporal_store(v.w, reinterpret_cast<uint32_t*>(c) + 3);
    }
    // head [g0, c0) and tail [c1, g1): fewer than 16 bytes each
    const uintptr_t h = g0 + uintptr_t(tid) * sizeof(T);
    if (h < c0) *reinterpret_cast<T*>(h) = *reinterpret_cast<const T*>(s_buf + (h - base));
    const uintptr_t t = c1 + uintptr_t(tid) * sizeof(T);
    if (t < g1) *reinterpret_cast<T*>(t) = *reinterpret_cast<const T*>(s_buf + (t - base));
  } else {  // the whole range inside one 16-B chunk or two partial ones: per element
    const uintptr_t e = g0 + uintptr_t(tid) * sizeof(T);
    if (e < g1) *reinterpret_cast<T*>(e) = *reinterpret_cast<const T*>(s_buf + (e - base));
  }
}

inline uint32_t gather_blocks(uint64_t n) { return uint32_t((n + 255) / 256); }

}  // namespace gm
