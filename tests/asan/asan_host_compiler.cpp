// tests/asan/asan_host_compiler.cpp — TEST ONLY: the host index compiler
// (emqx_amd/csrc/gm_index.cpp) and the overlay id mapping (gm_overlay.cpp)
// built with AddressSanitizer + UBSan and fed untrusted filter
// bytes: random bytes (NUL, '/', '+', '#', 0xFF), empty sets and empty
// filters, 65,535-byte filters, 5,000-level filters, duplicates.  Host-only:
// build_index(host_only) never touches a device.  Built and run by
// tests/test_host_cpu.py::test_host_compiler_under_asan (`make -C
// emqx_amd/csrc asan`).
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../emqx_amd/csrc/gm_internal.h"

namespace gm {
int set_err(emqx_gm_ctx*, int code, const std::string&) { return code; }  // gm_api.cpp's, minus the thread-local
// gm_match.hip's device step of an in-place update: never reached here (no
// context, so no snapshot keeps a mirror)
int apply_patch_device(emqx_gm_ctx*, void*, const void*, size_t, const std::vector<std::pair<uint64_t, uint32_t>>&,
                       const uint8_t*, const IndexView&, uint64_t, uint64_t, uint64_t, const std::vector<uint32_t>&) {
  return EMQX_GM_EDEVICE;
}
}

static int compile(const std::vector<std::string>& fs) {
  std::vector<uint8_t> b;
  std::vector<uint64_t> o{0};
  for (auto& f : fs) {
    b.insert(b.end(), f.begin(), f.end());
    o.push_back(b.size());
  }
  b.resize(b.size() + 64, 0);
  std::vector<uint32_t> perm(fs.size() + 1);
  emqx_gm_index_info_t info{};
  const int rc = gm::build_index(nullptr, b.data(), o.data(), fs.size(), nullptr, nullptr, perm.data(), nullptr,
                                 &info);
  if (rc) return rc;
  // ids are ranks of the unique filters: perm is a valid id for every input
  for (size_t i = 0; i < fs.size(); ++i)
    if (perm[i] >= info.n_filters) return -100;
  return 0;
}

int main() {
  std::mt19937_64 rng(42);
  const char alpha[] = {'a', 'b', '/', '+', '#', '\0', '\xff', '$', 'z'};
  int bad = 0;
  auto check = [&](const char* what, const std::vector<std::string>& fs) {
    const int rc = compile(fs);
    if (rc) {
      std::fprintf(stderr, "%s: rc %d\n", what, rc);
      ++bad;
    }
  };
  check("empty set", {});
  check("one empty filter", {""});
  check("separators only", {"/", "//", "///", "+", "#", "+/#", "/+/", "#/#"});
  for (int round = 0; round < 200; ++round) {
    std::vector<std::string> fs;
    const int n = int(rng() % 300);
    for (int i = 0; i < n; ++i) {
      std::string f;
      const int len = int(rng() % 40);
      for (int k = 0; k < len; ++k) f.push_back(alpha[rng() % sizeof(alpha)]);
      fs.push_back(f);
      if (rng() % 5 == 0) fs.push_back(f);  // duplicates
    }
    check("random", fs);
  }
  check("65535-byte filters", {std::string(65535, 'w'), std::string(65534, 'w') + "#",
                               std::string(32767, 'a') + "/" + std::string(32767, 'b')});
  std::string deep;
  for (int i = 0; i < 5000; ++i) deep += (i ? "/" : "") + std::string(1, char('a' + i % 26));
  check("5000 levels", {deep, deep + "/#", "+/" + deep});
  std::string nul_laden("a\0b/\0/+\0", 8);
  check("NUL-laden", {nul_laden, std::string("\0", 1), std::string("\0/#", 3)});

  // overlay id mapping over a host-only base (gm_overlay.cpp overlay_filter)
  {
    emqx_gm_index base;
    std::vector<std::string> fs = {"a", "a/+", "b/#", "c", "d/e/f", "x"};
    base.foff.push_back(0);
    for (auto& f : fs) {
      base.fbytes.insert(base.fbytes.end(), f.begin(), f.end());
      base.foff.push_back(base.fbytes.size());
    }
    base.info.n_filters = fs.size();
    emqx_gm_index ov;
    ov.ov = new gm::OverlayState;
    ov.ov->base = &base;
    ov.ov->tomb = {1, 4};          // "a/+" and "d/e/f" deleted
    ov.ov->ins = {3, 6};           // "bb" sorts before "c" (3 base filters before it), "y" after all
    ov.ov->dgid = {2, 5};          // final ids: a b/# bb c x y
    const std::string d = "bby";
    ov.ov->dbytes.assign(d.begin(), d.end());
    ov.ov->doff = {0, 2, 3};
    ov.info.n_filters = 6;
    const char* want[] = {"a", "b/#", "bb", "c", "x", "y"};
    for (uint32_t id = 0; id < 6; ++id) {
      const uint8_t* p = nullptr;
      uint64_t len = 0;
      if (gm::overlay_filter(&ov, id, &p, &len) || std::string(reinterpret_cast<const char*>(p), len) != want[id]) {
        std::fprintf(stderr, "overlay id %u\n", id);
        ++bad;
      }
    }
    const uint8_t* p = nullptr;
    uint64_t len = 0;
    if (gm::overlay_filter(&ov, 6, &p, &len) != EMQX_GM_EINVAL) ++bad;  // out of range
    ov.ov->base = nullptr;
    delete ov.ov;
    ov.ov = nullptr;
  }
  std::printf(bad ? "ASAN_HOST_CHECK_FAILED %d\n" : "ASAN_HOST_CHECK_OK\n", bad);
  return bad ? 1 : 0;
}
