// gm_image.cpp — index images: one snapshot compiled once, replicated to other
// devices and processes (emqx_gm_index_export / _device_blob / _import).
//
// The reference keeps ONE routing table that mria replicates to every node
// (emqx_route / emqx_trie as replicated mnesia tables, apps/emqx/src/
// emqx_router.erl:75-84, 136): a node that joins copies the table, it does not
// recompute it.  The MI355X analogue for the replicated plans (SURVEY.md §8e
// C3, C5 replicated): rank 0 compiles the filter set on the host ONCE, and every
// other rank receives
//   * the host part of the snapshot (this file's image: the layout of the
//     device tables, the sorted filter table, shard ids, subscriber offsets,
//     route marks and counts), a few bytes per filter, and
//   * the device blob itself, either inside the image (host buffer: a shared
//     file, gloo) or device to device (an RCCL broadcast of
//     emqx_gm_index_device_blob into every GPU over xGMI), which
//     emqx_gm_index_import copies into an allocation of its own.
// So N ranks do one host build instead of N, and no rank holds more than one
// host copy of anything.
//
// Image layout (all little-endian, sections 256-B aligned, sizes in the header):
//   ImageHeader | filter bytes | filter offsets u64[n+1] | gmap u32[] |
//   soff u64[] | pinned u8[] | [device blob]
// The header carries a layout signature (the sizes of every device record and
// of the view), so an image is only accepted by a library of the same layout.
#include <array>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>

#include <thread>

#include "gm_internal.h"

namespace gm {
namespace {

constexpr char kMagic[8] = {'E', 'M', 'Q', 'X', 'G', 'M', 'I', '1'};
constexpr uint32_t kVersion = 3;
constexpr int kPtrs = 11;  // the view's device pointers, in ptr_fields() order

uint64_t layout_signature() {
  uint64_t h = 0x9E3779B97F4A7C15ull;
  const uint64_t parts[] = {sizeof(IndexView), sizeof(Node), sizeof(DictSlot), sizeof(EdgeSlot), sizeof(HotSlot),
                            uint64_t(EDGE_DEPTHS), uint64_t(HOT_TABLES), sizeof(emqx_gm_index_info_t), kVersion};
  for (uint64_t p : parts) h = fmix64(h ^ (p + 0x632BE59BD9B4E019ull));
  return h;
}

// the device-pointer fields of a view (mutable view: import rebases them)
template <class V> auto ptr_fields(V& v) {
  return std::array<const void**, kPtrs>{
      reinterpret_cast<const void**>(&v.nodes),   reinterpret_cast<const void**>(&v.dict),
      reinterpret_cast<const void**>(&v.edges),   reinterpret_cast<const void**>(&v.hot),
      reinterpret_cast<const void**>(&v.arena),   reinterpret_cast<const void**>(&v.sub_off),
      reinterpret_cast<const void**>(&v.sub_ids), reinterpret_cast<const void**>(&v.gmap),
      reinterpret_cast<const void**>(&v.efilt),   reinterpret_cast<const void**>(&v.mph_word),
      reinterpret_cast<const void**>(&v.d0_root)};
}

struct MirrorMeta {  // gm::Mirror without its blob (an imported index loads it lazily)
  uint64_t present, blob_size, o_nodes, o_dict, o_edges, o_hot, o_arena, o_flen, o_efilt, o_mph;
  uint64_t nodes_n, nodes_cap, arena_n, arena_cap, flen_cap, dict_used;
  uint64_t edge_used[EDGE_DEPTHS], hot_used[HOT_TABLES], mph_ovf_used[HOT_TABLES];
};

struct ImageHeader {
  char magic[8];
  uint32_t version, header_bytes;
  uint64_t layout_sig;
  uint64_t dev_bytes, flen_off, level_nodes;
  uint64_t n_filters, ft_bytes, gmap_n, soff_n, pinned_n;
  uint64_t blob_in_image;
  uint64_t flen_stale;      // the blob's filter lengths predate an in-place update (rewritten when asked for)
  uint64_t ptr_off[kPtrs];  // offset of each view pointer in the blob; ~0: null
  IndexView view;           // (its pointer fields are meaningless here)
  emqx_gm_index_info_t info;
  MirrorMeta mirror;
  uint64_t sec_off[6];      // filter bytes, filter offsets, gmap, soff, pinned, blob
  uint64_t total_bytes;
  uint64_t checksum;        // over this header (with 0 here) and the host sections (validate_image)
};

constexpr uint64_t al(uint64_t x) { return (x + 255) & ~uint64_t(255); }

}  // namespace

namespace {

// a + b <= lim without wrapping
bool fits(uint64_t a, uint64_t b, uint64_t lim) { return a <= lim && b <= lim - a; }
// n * k, or ~0 when it wraps
uint64_t mul(uint64_t n, uint64_t k) { return k && n > ~0ull / k ? ~0ull : n * k; }

uint64_t image_checksum(const uint8_t* img, const ImageHeader& h) {
  // the header (checksum field zero) and every byte after it up to the blob: a
  // corrupted transfer is refused before anything is read through its counts
  ImageHeader z = h;
  z.checksum = 0;
  uint64_t x = 0x243F6A8885A308D3ull;
  auto eat = [&](const uint8_t* p, uint64_t n) {
    uint64_t w;
    for (; n >= 8; p += 8, n -= 8) {
      std::memcpy(&w, p, 8);
      x = fmix64(x ^ w) + 0x9E3779B97F4A7C15ull;
    }
    w = 0;
    std::memcpy(&w, p, n);
    x = fmix64(x ^ w ^ (n << 56)) + 0x9E3779B97F4A7C15ull;
  };
  eat(reinterpret_cast<const uint8_t*>(&z), sizeof z);
  eat(img + sizeof z, h.sec_off[5] - sizeof z);  // (the header's padding too: every byte up to the blob)
  return x;
}

}  // namespace

int index_export(emqx_gm_ctx* ctx, const emqx_gm_index* idx, uint32_t flags, uint8_t* buf, uint64_t* size) {
  if (!idx || !size) return set_err(ctx, EMQX_GM_EINVAL, "index_export: NULL argument");
  if (flags & ~EMQX_GM_IMAGE_NO_BLOB) return set_err(ctx, EMQX_GM_EINVAL, "index_export: flags");
  if (idx->ov) return set_err(ctx, EMQX_GM_EUNSUPPORTED, "index_export: overlay snapshot (update it to a flat one)");
  // (a host-only index -- the CPU tests' -- is its mirror: its tables are exported from there)
  const bool host_only = !idx->dev_base && idx->mirror && !idx->mirror->blob.empty();
  if (idx->dev_subs || (!idx->dev_base && !host_only))
    return set_err(ctx, EMQX_GM_EUNSUPPORTED, "index_export: a snapshot whose subscriber CSR lives apart "
                                              "(emqx_gm_index_update_subs result) or without device tables");
  const uint64_t blob_bytes = host_only ? idx->mirror->blob.size() : idx->dev_bytes;
  ImageHeader h;
  std::memset(&h, 0, sizeof h);
  std::memcpy(h.magic, kMagic, 8);
  h.version = kVersion;
  h.header_bytes = sizeof(ImageHeader);
  h.layout_sig = layout_signature();
  h.dev_bytes = blob_bytes;
  h.level_nodes = idx->level_nodes;
  h.view = idx->view;
  h.info = idx->info;
  const uint8_t* base = host_only ? idx->mirror->blob.data() : static_cast<const uint8_t*>(idx->dev_base);
  IndexView v = idx->view;
  auto pf = ptr_fields(v);
  for (int i = 0; i < kPtrs; ++i) {
    const uint8_t* p = static_cast<const uint8_t*>(*pf[i]);
    if (!p) {
      h.ptr_off[i] = ~0ull;
      continue;
    }
    if (p < base || p >= base + blob_bytes)
      return set_err(ctx, EMQX_GM_EUNSUPPORTED, "index_export: a table outside the snapshot's blob");
    h.ptr_off[i] = uint64_t(p - base);
  }
  h.flen_off = idx->dev_flen ? uint64_t(reinterpret_cast<const uint8_t*>(idx->dev_flen) - base) : ~0ull;
  if (const Mirror* m = idx->mirror) {
    MirrorMeta& mm = h.mirror;
    mm.present = 1;
    mm.blob_size = m->blob_size;
    mm.o_nodes = m->o_nodes, mm.o_dict = m->o_dict, mm.o_edges = m->o_edges, mm.o_hot = m->o_hot;
    mm.o_arena = m->o_arena, mm.o_flen = m->o_flen, mm.o_efilt = m->o_efilt, mm.o_mph = m->o_mph;
    mm.nodes_n = m->nodes_n, mm.nodes_cap = m->nodes_cap, mm.arena_n = m->arena_n, mm.arena_cap = m->arena_cap;
    mm.flen_cap = m->flen_cap, mm.dict_used = m->dict_used;
    for (int d = 0; d < EDGE_DEPTHS; ++d) mm.edge_used[d] = m->edge_used[d];
    for (int t = 0; t < HOT_TABLES; ++t) mm.hot_used[t] = m->hot_used[t], mm.mph_ovf_used[t] = m->mph_ovf_used[t];
  }
  h.n_filters = idx->ft.size();
  uint64_t fbytes = 0;
  idx->ft.for_each([&](uint64_t, const uint8_t*, uint64_t l) { fbytes += l; });
  h.ft_bytes = fbytes;
  h.gmap_n = idx->gmap.size();
  const std::vector<uint64_t> soff = idx->subs.empty() ? std::vector<uint64_t>() : idx->subs.offsets();
  const std::vector<uint8_t> marks = idx->subs.empty() ? std::vector<uint8_t>() : idx->subs.marks();
  h.soff_n = soff.size();
  h.pinned_n = marks.size();
  h.blob_in_image = (flags & EMQX_GM_IMAGE_NO_BLOB) ? 0 : 1;
  h.flen_stale = idx->flen_stale.load() ? 1 : 0;
  uint64_t o = al(sizeof(ImageHeader));
  const uint64_t secsz[6] = {fbytes, (h.n_filters + 1) * 8, h.gmap_n * 4, h.soff_n * 8, h.pinned_n,
                             h.blob_in_image ? h.dev_bytes : 0};
  for (int s = 0; s < 6; ++s) {
    h.sec_off[s] = o;
    o += al(secsz[s]);
  }
  h.total_bytes = o;
  if (!buf) {
    *size = o;
    return EMQX_GM_OK;
  }
  if (*size < o) return set_err(ctx, EMQX_GM_EINVAL, "index_export: buffer too small (size it with buf NULL)");
  std::memset(buf, 0, al(sizeof(ImageHeader)));
  std::memcpy(buf, &h, sizeof h);
  uint8_t* fb = buf + h.sec_off[0];
  uint64_t* fo = reinterpret_cast<uint64_t*>(buf + h.sec_off[1]);
  uint64_t at = 0;
  fo[0] = 0;
  idx->ft.for_each([&](uint64_t r, const uint8_t* p, uint64_t l) {
    std::memcpy(fb + at, p, l);
    at += l;
    fo[r + 1] = at;
  });
  if (h.gmap_n) std::memcpy(buf + h.sec_off[2], idx->gmap.data(), h.gmap_n * 4);
  if (h.soff_n) std::memcpy(buf + h.sec_off[3], soff.data(), h.soff_n * 8);
  if (h.pinned_n) std::memcpy(buf + h.sec_off[4], marks.data(), h.pinned_n);
  if (h.blob_in_image && host_only) {
    std::memcpy(buf + h.sec_off[5], base, h.dev_bytes);
  } else if (h.blob_in_image) {
    hipSetDevice(idx->device);
    if (ctx) GM_HIP(ctx, hipStreamSynchronize(ctx->stream));
    GM_HIP(ctx, hipMemcpy(buf + h.sec_off[5], idx->dev_base, h.dev_bytes, hipMemcpyDeviceToHost));
  }
  h.checksum = image_checksum(buf, h);
  std::memcpy(buf, &h, sizeof h);
  *size = o;
  return EMQX_GM_OK;
}


// Everything index_import reads through an image's own counts and offsets is
// checked here, host-side and with no device (tests/asan: truncations at every
// section boundary, byte flips, oversized counts): the header's identity and
// checksum; every section inside the image, in order, without overlap and
// aligned; the filter offsets monotone and ending at the filter bytes; the
// shard ids, subscriber offsets and route marks sized by the filter count; the
// view's every table extent inside the device blob; the mirror's metadata
// inside the blob it describes.  An image from another node (the NIF's
// import_index/1) can then not make the library read or write out of bounds.
int validate_image(const uint8_t* img, uint64_t size, bool have_blob, std::string* why) {
  auto bad = [&](const char* w) {
    *why = std::string("index_import: ") + w;
    return EMQX_GM_EINVAL;
  };
  if (!img || size < sizeof(ImageHeader)) return bad("truncated image");
  ImageHeader h;
  std::memcpy(&h, img, sizeof h);
  if (std::memcmp(h.magic, kMagic, 8) || h.version != kVersion || h.header_bytes != sizeof(ImageHeader))
    return bad("not an index image of this library");
  if (h.layout_sig != layout_signature()) return bad("image from a library with another table layout");
  if (h.total_bytes > size) return bad("truncated image");
  if (h.blob_in_image > 1 || h.flen_stale > 1 || h.mirror.present > 1) return bad("corrupt header");
  if (!have_blob && !h.blob_in_image) return bad("the image holds no device blob and none was given");
  const uint64_t nf = h.n_filters;
  if (nf != h.info.n_filters || nf != h.view.n_filters || nf >= HF_NONE) return bad("inconsistent filter count");
  if (!h.dev_bytes || h.dev_bytes > (1ull << 44)) return bad("corrupt device blob size");
  const uint64_t secsz[6] = {h.ft_bytes, mul(nf + 1, 8), mul(h.gmap_n, 4), mul(h.soff_n, 8), h.pinned_n,
                             h.blob_in_image ? h.dev_bytes : 0};
  uint64_t end = sizeof(ImageHeader);
  for (int k = 0; k < 6; ++k) {
    if (h.sec_off[k] < end || h.sec_off[k] % 8 || !fits(h.sec_off[k], secsz[k], h.total_bytes))
      return bad("truncated image or corrupt section table");
    end = h.sec_off[k] + secsz[k];
  }
  if (image_checksum(img, h) != h.checksum) return bad("checksum mismatch (corrupt image)");
  if ((h.gmap_n && h.gmap_n != nf) || (h.soff_n && h.soff_n != nf + 1) || (h.pinned_n && h.pinned_n != nf))
    return bad("inconsistent table sizes");
  const uint64_t* fo = reinterpret_cast<const uint64_t*>(img + h.sec_off[1]);
  if (fo[0] != 0 || fo[nf] != h.ft_bytes) return bad("inconsistent filter table");
  for (uint64_t i = 0; i < nf; ++i)
    if (fo[i + 1] < fo[i]) return bad("inconsistent filter table");
  if (h.gmap_n) {
    const uint32_t* g = reinterpret_cast<const uint32_t*>(img + h.sec_off[2]);
    for (uint64_t i = 1; i < nf; ++i)
      if (g[i] <= g[i - 1]) return bad("shard ids not ascending");
  }
  if (h.soff_n) {
    const uint64_t* so = reinterpret_cast<const uint64_t*>(img + h.sec_off[3]);
    if (so[0] != 0 || so[nf] != h.info.n_subs) return bad("inconsistent subscriber offsets");
    for (uint64_t i = 0; i < nf; ++i)
      if (so[i + 1] < so[i]) return bad("inconsistent subscriber offsets");
  }
  // the view: every table the kernels index (by masks, capacities and counts) inside the blob
  const IndexView& v = h.view;
  const uint64_t B = h.dev_bytes;
  auto within = [&](int p, uint64_t bytes) {  // table p's first `bytes` bytes lie in the blob
    return h.ptr_off[p] == ~0ull ? bytes == 0 : fits(h.ptr_off[p], bytes, B);
  };
  for (int i = 0; i < kPtrs; ++i)
    if (h.ptr_off[i] != ~0ull && (h.ptr_off[i] >= B || h.ptr_off[i] % 16)) return bad("inconsistent table layout");
  uint64_t edges = 0, hot = 0, efilt = 0, mph = 0;
  for (int d = 0; d < EDGE_DEPTHS; ++d) {
    if (v.etab_mask[d] >= (1ull << 40) || v.etab_off[d] >= (1ull << 40)) return bad("inconsistent table layout");
    edges = std::max(edges, (v.etab_off[d] + v.etab_mask[d] + 1) * sizeof(EdgeSlot));
  }
  for (int t = 0; t < HOT_TABLES; ++t) {
    if (v.hot_cap[t] > SLOT_MASK || v.hot_off[t] >= (1ull << 40) || v.mph_cap[t] > v.hot_cap[t] ||
        v.efilt_off[t] >= (1ull << 40) || v.mph_off[t] >= (1ull << 40) || (v.mph_cap[t] && !v.mph_nb[t]))
      return bad("inconsistent table layout");
    hot = std::max(hot, (v.hot_off[t] + v.hot_cap[t]) * sizeof(HotSlot));
    if (v.efilt_mask[t]) efilt = std::max(efilt, (v.efilt_off[t] + uint64_t(v.efilt_mask[t]) + 1) * 4);
    if (v.mph_cap[t]) mph = std::max(mph, (v.mph_off[t] + v.mph_nb[t]) * 8);
  }
  if (v.dict_mask >= (1ull << 40)) return bad("inconsistent table layout");
  const uint64_t dict = (v.dict_mask + 1) * sizeof(DictSlot);
  if (!within(0, uint64_t(v.n_nodes) * sizeof(Node)) || !within(1, dict) || !within(2, edges) || !within(3, hot) ||
      !within(8, efilt) || !within(9, mph) || (h.ptr_off[10] != ~0ull && !within(10, 16)) ||
      (h.ptr_off[5] != ~0ull && !within(5, (nf + 1) * 8)) || (h.ptr_off[6] != ~0ull && !within(6, h.info.n_subs * 4)) ||
      (h.ptr_off[7] != ~0ull && !within(7, nf * 4)) || h.ptr_off[0] == ~0ull || h.ptr_off[1] == ~0ull ||
      h.ptr_off[3] == ~0ull || h.ptr_off[4] == ~0ull)
    return bad("a table extends past the device blob");
  if (h.ptr_off[7] != ~0ull && h.gmap_n != nf) return bad("inconsistent shard ids");
  if ((v.flags & IX_D0) && h.ptr_off[10] == ~0ull) return bad("inconsistent table layout");
  if (h.flen_off != ~0ull && (h.flen_off % 2 || !fits(h.flen_off, (nf + 1) * 2, B)))
    return bad("inconsistent filter lengths");
  if (h.mirror.present) {  // the in-place patcher indexes the host copy of the blob by these
    const MirrorMeta& m = h.mirror;
    const uint64_t M = m.blob_size;
    if (M > B || m.nodes_n > m.nodes_cap || m.arena_n > m.arena_cap || m.flen_cap < nf ||
        m.dict_used > v.dict_mask + 1 || m.o_nodes != h.ptr_off[0] || m.o_dict != h.ptr_off[1] ||
        m.o_edges != h.ptr_off[2] || m.o_hot != h.ptr_off[3] || m.o_arena != h.ptr_off[4] ||
        (h.ptr_off[8] != ~0ull && m.o_efilt != h.ptr_off[8]) || (h.ptr_off[9] != ~0ull && m.o_mph != h.ptr_off[9]) ||
        m.o_flen != h.flen_off || !fits(m.o_nodes, mul(m.nodes_cap, sizeof(Node)), M) || !fits(m.o_dict, dict, M) ||
        !fits(m.o_edges, edges, M) || !fits(m.o_hot, hot, M) || !fits(m.o_arena, m.arena_cap, M) ||
        !fits(m.o_flen, mul(m.flen_cap, 2), M) || !fits(m.o_efilt, efilt, M) || !fits(m.o_mph, mph, M) ||
        m.nodes_n < v.n_nodes)
      return bad("inconsistent mirror metadata");
    for (int d = 0; d < EDGE_DEPTHS; ++d)
      if (m.edge_used[d] > v.etab_mask[d] + 1) return bad("inconsistent mirror metadata");
    for (int t = 0; t < HOT_TABLES; ++t)
      if (m.hot_used[t] > v.hot_cap[t] || m.mph_ovf_used[t] > v.hot_cap[t] - v.mph_cap[t])
        return bad("inconsistent mirror metadata");
  }
  return EMQX_GM_OK;
}

// The host half of an import (no device): the header, the filter table, shard
// ids, subscriber offsets, route marks and the mirror's metadata of a
// validated image into idx; its view's pointer fields hold blob OFFSETS
// (+1; 0 = null) for the caller to rebase.
int import_host_part(const uint8_t* img, uint64_t size, bool have_blob, emqx_gm_index* idx, std::string* why) {
  if (int rc = validate_image(img, size, have_blob, why)) return rc;
  ImageHeader h;
  std::memcpy(&h, img, sizeof h);
  const uint64_t* fo = reinterpret_cast<const uint64_t*>(img + h.sec_off[1]);
  idx->dev_bytes = h.dev_bytes;
  idx->view = h.view;
  auto pf = ptr_fields(idx->view);
  for (int i = 0; i < kPtrs; ++i)
    *pf[i] = h.ptr_off[i] == ~0ull ? nullptr : reinterpret_cast<const void*>(uintptr_t(h.ptr_off[i] + 1));
  idx->dev_flen = h.flen_off == ~0ull ? nullptr : reinterpret_cast<uint16_t*>(uintptr_t(h.flen_off + 1));
  idx->level_nodes = h.level_nodes;
  idx->info = h.info;
  idx->flen_stale = h.flen_stale != 0;
  auto sf = std::make_shared<SortedFilters>();
  sf->bytes.assign(img + h.sec_off[0], img + h.sec_off[0] + h.ft_bytes);
  sf->off.assign(fo, fo + h.n_filters + 1);
  idx->ft.set_base(std::move(sf));
  const uint32_t* gm = reinterpret_cast<const uint32_t*>(img + h.sec_off[2]);
  idx->gmap.assign(gm, gm + h.gmap_n);
  const uint64_t* so = reinterpret_cast<const uint64_t*>(img + h.sec_off[3]);
  if (h.soff_n)
    idx->subs = SubTable(std::vector<uint64_t>(so, so + h.soff_n),
                         std::vector<uint8_t>(img + h.sec_off[4], img + h.sec_off[4] + h.pinned_n));
  if (h.mirror.present) {  // the updatable line continues here; its host copy loads on the first update
    const MirrorMeta& mm = h.mirror;
    auto* m = new Mirror;
    m->blob_size = mm.blob_size;
    m->o_nodes = mm.o_nodes, m->o_dict = mm.o_dict, m->o_edges = mm.o_edges, m->o_hot = mm.o_hot;
    m->o_arena = mm.o_arena, m->o_flen = mm.o_flen, m->o_efilt = mm.o_efilt, m->o_mph = mm.o_mph;
    m->nodes_n = mm.nodes_n, m->nodes_cap = mm.nodes_cap, m->arena_n = mm.arena_n, m->arena_cap = mm.arena_cap;
    m->flen_cap = mm.flen_cap, m->dict_used = mm.dict_used;
    for (int d = 0; d < EDGE_DEPTHS; ++d) m->edge_used[d] = mm.edge_used[d];
    for (int t = 0; t < HOT_TABLES; ++t) m->hot_used[t] = mm.hot_used[t], m->mph_ovf_used[t] = mm.mph_ovf_used[t];
    idx->mirror = m;
  }
  return EMQX_GM_OK;
}

// Test support (tests/asan/asan_host_compiler.cpp fuzzes images): a named
// u64 field of an image's header, and the checksum recomputed after a change.
uint64_t* image_field(uint8_t* img, const std::string& name) {
  auto* h = reinterpret_cast<ImageHeader*>(img);
  static const char* const sec[6] = {"sec_off0", "sec_off1", "sec_off2", "sec_off3", "sec_off4", "sec_off5"};
  for (int k = 0; k < 6; ++k)
    if (name == sec[k]) return &h->sec_off[k];
  if (name.compare(0, 7, "ptr_off") == 0) {
    const int k = std::atoi(name.c_str() + 7);
    return k >= 0 && k < kPtrs ? &h->ptr_off[k] : nullptr;
  }
  const std::pair<const char*, uint64_t*> f[] = {
      {"dev_bytes", &h->dev_bytes},          {"flen_off", &h->flen_off},
      {"n_filters", &h->n_filters},          {"ft_bytes", &h->ft_bytes},
      {"gmap_n", &h->gmap_n},                {"soff_n", &h->soff_n},
      {"pinned_n", &h->pinned_n},            {"blob_in_image", &h->blob_in_image},
      {"total_bytes", &h->total_bytes},      {"info.n_filters", &h->info.n_filters},
      {"info.n_subs", &h->info.n_subs},      {"view.dict_mask", &h->view.dict_mask},
      {"view.hot_cap1", &h->view.hot_cap[1]}, {"view.hot_off2", &h->view.hot_off[2]},
      {"view.etab_mask0", &h->view.etab_mask[0]}, {"mirror.blob_size", &h->mirror.blob_size},
      {"mirror.nodes_cap", &h->mirror.nodes_cap}, {"mirror.arena_cap", &h->mirror.arena_cap},
      {"mirror.flen_cap", &h->mirror.flen_cap}, {"mirror.o_hot", &h->mirror.o_hot},
      {"mirror.hot_used1", &h->mirror.hot_used[1]}, {"mirror.edge_used0", &h->mirror.edge_used[0]}};
  for (auto& kv : f)
    if (name == kv.first) return kv.second;
  return nullptr;
}
void image_reseal(uint8_t* img, uint64_t size) {
  auto* h = reinterpret_cast<ImageHeader*>(img);
  if (h->sec_off[5] >= sizeof(ImageHeader) && h->sec_off[5] <= size) h->checksum = image_checksum(img, *h);
}
uint32_t image_view_u32(uint8_t* img, int which, int t) {  // (the harness's view counts: 0 n_nodes, 1 efilt_mask[t], 2 mph_nb[t])
  auto* h = reinterpret_cast<ImageHeader*>(img);
  return which == 0 ? h->view.n_nodes : which == 1 ? h->view.efilt_mask[t] : h->view.mph_nb[t];
}
void image_view_set_u32(uint8_t* img, int which, int t, uint32_t x) {
  auto* h = reinterpret_cast<ImageHeader*>(img);
  (which == 0 ? h->view.n_nodes : which == 1 ? h->view.efilt_mask[t] : h->view.mph_nb[t]) = x;
}

int index_import(emqx_gm_ctx* ctx, const uint8_t* img, uint64_t size, const void* d_blob, emqx_gm_index** out) {
  if (!img || !out) return set_err(ctx, EMQX_GM_EINVAL, "index_import: NULL argument");
  std::unique_ptr<emqx_gm_index> idx(new emqx_gm_index);
  std::string why;
  if (int rc = import_host_part(img, size, d_blob != nullptr, idx.get(), &why)) return set_err(ctx, rc, why);
  ImageHeader h;
  std::memcpy(&h, img, sizeof h);
  idx->device = ctx->device;
  GM_HIP(ctx, hipSetDevice(ctx->device));
  {
    hipError_t e = hipMalloc(&idx->dev_base, h.dev_bytes);
    if (e != hipSuccess)
      return set_err(ctx, EMQX_GM_ENOMEM, std::string("index_import: hipMalloc: ") + hipGetErrorString(e));
  }
  hipError_t e = d_blob ? hipMemcpyAsync(idx->dev_base, d_blob, h.dev_bytes, hipMemcpyDeviceToDevice, ctx->stream)
                        : hipMemcpyAsync(idx->dev_base, img + h.sec_off[5], h.dev_bytes, hipMemcpyHostToDevice,
                                         ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) {
    (void)hipFree(idx->dev_base);
    idx->dev_base = nullptr;
    return set_err(ctx, EMQX_GM_EDEVICE, std::string("index_import: blob copy: ") + hipGetErrorString(e));
  }
  uint8_t* B = static_cast<uint8_t*>(idx->dev_base);
  auto pf = ptr_fields(idx->view);
  for (int i = 0; i < kPtrs; ++i)
    if (*pf[i]) *pf[i] = B + (reinterpret_cast<uintptr_t>(*pf[i]) - 1);
  if (idx->dev_flen) idx->dev_flen = reinterpret_cast<uint16_t*>(B + (reinterpret_cast<uintptr_t>(idx->dev_flen) - 1));
  // The updatable line's host mirror, by the build's policy (gm_index.cpp): kept
  // for tables up to kEagerMirrorBytes unless EMQX_GM_OPEN_MIRROR_* says
  // otherwise, so a joining node's first update does not pay a silent download.
  // An image that carries the tables gives the mirror its bytes directly (the
  // device tables ARE those bytes); a device-blob import downloads them.
  if (Mirror* M = idx->mirror) {
    bool eager = M->blob_size <= kEagerMirrorBytes;
    if (const char* pol = knob("GM_MIRROR")) eager = !std::strcmp(pol, "eager");
    if (ctx->open_flags & EMQX_GM_OPEN_MIRROR_EAGER) eager = true;
    if (ctx->open_flags & EMQX_GM_OPEN_MIRROR_LAZY) eager = false;
    if (eager && M->blob_size <= h.dev_bytes) {
      if (!d_blob) {
        const double t0 = now_ms();
        M->blob.resize(M->blob_size);
        const uint8_t* src = img + h.sec_off[5];
        const size_t nb = M->blob_size;
        const unsigned T = nb < (size_t(1) << 24) ? 1u : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        std::vector<std::thread> th;
        for (unsigned r = 1; r < T; ++r)
          th.emplace_back([&, r] { std::memcpy(M->blob.data() + nb * r / T, src + nb * r / T, nb * (r + 1) / T - nb * r / T); });
        std::memcpy(M->blob.data(), src, nb / T);
        for (auto& t : th) t.join();
        tl_ustats.mirror_loaded = 1;
        tl_ustats.mirror_bytes = nb;
        tl_ustats.mirror_ms = now_ms() - t0;
      } else if (const int rc = load_mirror_blob(ctx, idx.get())) {
        free_index(idx.release());
        return rc;
      }
    }
  }
  *out = idx.release();
  return EMQX_GM_OK;
}

// The host copy of an index's device tables for an in-place update, loaded on
// the first update of a snapshot built without one (gm_index.cpp: indexes past
// kEagerMirrorBytes, EMQX_GM_OPEN_MIRROR_LAZY, imported snapshots).  The device
// tables ARE the current state (filter-id fields included), so one download
// up to the subscriber CSR gives exactly what an eager mirror would hold.
// dev[0, bytes) to host memory nothing has touched yet, through two page-locked
// buffers: one chunk crosses PCIe while all threads copy the previous one out
// (so the destination's pages are first touched in parallel too).  The C5
// mirror (38 GB): one pass instead of a serial zero-fill, a page-pinning of the
// whole destination and the copy (7.7 s for the first update, round 5).
hipError_t download_blob(uint8_t* host, const uint8_t* dev, size_t bytes) {
  if (!bytes) return hipSuccess;
  const size_t CH = std::min<size_t>(size_t(128) << 20, (bytes + 4095) & ~size_t(4095));
  hipStream_t st = nullptr;
  void* buf[2] = {nullptr, nullptr};
  hipEvent_t done[2] = {nullptr, nullptr};
  hipError_t e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  bool staged = e == hipSuccess;
  for (int k = 0; k < 2 && staged; ++k)
    staged = hipHostMalloc(&buf[k], CH, hipHostMallocDefault) == hipSuccess &&
             hipEventCreateWithFlags(&done[k], hipEventDisableTiming) == hipSuccess;
  auto copy_out = [&](uint8_t* dst, const uint8_t* src, size_t n) {
    const unsigned T = n < (size_t(1) << 22) ? 1u : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    for (unsigned r = 1; r < T; ++r)
      th.emplace_back([=] { std::memcpy(dst + n * r / T, src + n * r / T, n * (r + 1) / T - n * r / T); });
    std::memcpy(dst, src, n / T);
    for (auto& t : th) t.join();
  };
  if (e == hipSuccess && staged) {
    const size_t nch = (bytes + CH - 1) / CH;
    auto issue = [&](size_t c) {  // chunk c into buffer c & 1
      const size_t n = std::min(CH, bytes - c * CH);
      hipError_t r = hipMemcpyAsync(buf[c & 1], dev + c * CH, n, hipMemcpyDeviceToHost, st);
      if (r == hipSuccess) r = hipEventRecord(done[c & 1], st);
      return r;
    };
    e = issue(0);
    for (size_t c = 0; c < nch && e == hipSuccess; ++c) {
      if (c + 1 < nch) e = issue(c + 1);  // (the next chunk crosses while this one is copied out)
      if (e == hipSuccess) e = hipEventSynchronize(done[c & 1]);
      if (e != hipSuccess) break;
      copy_out(host + c * CH, static_cast<const uint8_t*>(buf[c & 1]), std::min(CH, bytes - c * CH));
      // (buffer c & 1 is free again: chunk c + 2 is issued next round, after this copy)
    }
  } else if (e == hipSuccess) {  // no page-locked memory to spare: one pageable copy
    (void)hipGetLastError();
    e = hipMemcpy(host, dev, bytes, hipMemcpyDeviceToHost);
  }
  if (st) {
    const hipError_t es = hipStreamSynchronize(st);
    if (e == hipSuccess) e = es;
    (void)hipStreamDestroy(st);
  }
  for (int k = 0; k < 2; ++k) {
    if (done[k]) (void)hipEventDestroy(done[k]);
    if (buf[k]) (void)hipHostFree(buf[k]);
  }
  return e;
}

int load_mirror_blob(emqx_gm_ctx* ctx, emqx_gm_index* idx) {
  Mirror& M = *idx->mirror;
  if (!M.blob.empty() || !idx->dev_base) return EMQX_GM_OK;
  const double t0 = now_ms();
  hipSetDevice(idx->device);
  if (ctx) GM_HIP(ctx, hipStreamSynchronize(ctx->stream));
  M.blob.resize(M.blob_size);  // (left unwritten: the download below fills every byte)
  const hipError_t e = download_blob(M.blob.data(), static_cast<const uint8_t*>(idx->dev_base), M.blob_size);
  if (e != hipSuccess) {
    HostBytes().swap(M.blob);
    return set_err(ctx, EMQX_GM_EDEVICE, std::string("index_update: mirror download: ") + hipGetErrorString(e));
  }
  tl_ustats.mirror_loaded = 1;  // (emqx_gm_last_update_stats: what this call did)
  tl_ustats.mirror_bytes = M.blob_size;
  tl_ustats.mirror_ms = now_ms() - t0;
  return EMQX_GM_OK;
}

}  // namespace gm
