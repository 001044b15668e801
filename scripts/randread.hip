// Random-read calibration for the walk's access pattern (experiment, not
// product code).  Every lane reads `iters` random 16-B records of a table of
// `mb` MiB, either independent (addresses from a counter hash: up to UNROLL
// loads in flight per lane) or dependent (each address hashes the previous
// record, like one probe chain).  Prints loads/s; run under rocprofv3 --pmc
// with TCC_EA0_RDREQ_sum / TCC_EA0_RDREQ_32B_sum to get the fabric requests
// per load, which tells whether k_match_fused's 3.9 requests per topic are
// bandwidth or latency bound.
//
//   hipcc -O3 --offload-arch=gfx950 -o randread randread.hip
//   ./randread <table MiB> <mode 0=indep 1=dep> <waves per SIMD 1..8> [iters] [width 16|4|64]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

template <int MODE, int WIDTH>
__global__ __launch_bounds__(256) void k_rand(const uint4* __restrict__ tab, uint32_t nrec, uint32_t iters,
                                              uint32_t* __restrict__ out) {
  const uint32_t gid = blockIdx.x * 256u + threadIdx.x;
  uint32_t acc = mix(gid * 0x9E3779B1u + 1u);
  if (MODE == 0) {
    uint32_t s = acc;
    for (uint32_t i = 0; i < iters; i += 8) {
      uint4 v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t r = __umulhi(mix(s + uint32_t(k) * 0x632BE5ABu), nrec);
        if (WIDTH == 4) {
          v[k] = make_uint4(reinterpret_cast<const uint32_t*>(tab + r)[0], 0u, 0u, 0u);
        } else if (WIDTH == 64) {
          const uint32_t r4 = r & ~3u;
          const uint4 a = tab[r4], b = tab[r4 + 1], c = tab[r4 + 2], d = tab[r4 + 3];
          v[k] = make_uint4(a.x ^ b.y, c.z ^ d.w, a.w ^ c.x, b.z ^ d.y);
        } else {
          v[k] = tab[r];
        }
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) acc += v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
      s += 8u * 0x632BE5ABu;
    }
  } else {
    for (uint32_t i = 0; i < iters; ++i) {
      const uint32_t r = __umulhi(mix(acc + i), nrec);
      const uint4 v = tab[r];
      acc += v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  out[gid] = acc;
}

int main(int argc, char** argv) {
  const uint64_t mb = argc > 1 ? strtoull(argv[1], nullptr, 10) : 2048;
  const int mode = argc > 2 ? atoi(argv[2]) : 0;
  const int wps = argc > 3 ? atoi(argv[3]) : 8;
  const uint32_t iters = argc > 4 ? uint32_t(strtoul(argv[4], nullptr, 10)) : 256;
  const int width = argc > 5 ? atoi(argv[5]) : 16;
  const uint64_t bytes = mb << 20;
  const uint32_t nrec = uint32_t(bytes / 16);
  uint4* tab;
  uint32_t* out;
  CK(hipMalloc(&tab, bytes));
  CK(hipMemset(tab, 0x5A, bytes));
  const uint32_t blocks = 256u * uint32_t(wps);  // 4 waves per block: wps waves per SIMD over 256 CUs
  CK(hipMalloc(&out, size_t(blocks) * 256 * 4));
  auto launch = [&]() {
    if (mode == 0 && width == 16) hipLaunchKernelGGL((k_rand<0, 16>), dim3(blocks), dim3(256), 0, 0, tab, nrec, iters, out);
    else if (mode == 0 && width == 4) hipLaunchKernelGGL((k_rand<0, 4>), dim3(blocks), dim3(256), 0, 0, tab, nrec, iters, out);
    else if (mode == 0) hipLaunchKernelGGL((k_rand<0, 64>), dim3(blocks), dim3(256), 0, 0, tab, nrec, iters, out);
    else hipLaunchKernelGGL((k_rand<1, 16>), dim3(blocks), dim3(256), 0, 0, tab, nrec, iters, out);
  };
  launch();
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int reps = 5;
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) launch();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= reps;
  const double loads = double(blocks) * 256 * iters;
  printf("{\"table_mb\": %llu, \"mode\": \"%s\", \"waves_per_simd\": %d, \"width\": %d, \"loads\": %.0f, \"ms\": %.4f, "
         "\"G_loads_per_s\": %.2f, \"GB_per_s_at_128B\": %.1f}\n",
         (unsigned long long)mb, mode ? "dep" : "indep", wps, width, loads, ms, loads / ms / 1e6,
         loads * 128.0 / ms / 1e6);
  CK(hipFree(tab));
  CK(hipFree(out));
  return 0;
}
