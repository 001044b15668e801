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
#include <cstring>
#include <memory>
#include <string>

#include "gm_internal.h"

namespace gm {
namespace {

constexpr char kMagic[8] = {'E', 'M', 'Q', 'X', 'G', 'M', 'I', '1'};
constexpr uint32_t kVersion = 2;
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
};

constexpr uint64_t al(uint64_t x) { return (x + 255) & ~uint64_t(255); }

}  // namespace

int index_export(emqx_gm_ctx* ctx, const emqx_gm_index* idx, uint32_t flags, uint8_t* buf, uint64_t* size) {
  if (!idx || !size) return set_err(ctx, EMQX_GM_EINVAL, "index_export: NULL argument");
  if (flags & ~EMQX_GM_IMAGE_NO_BLOB) return set_err(ctx, EMQX_GM_EINVAL, "index_export: flags");
  if (idx->ov) return set_err(ctx, EMQX_GM_EUNSUPPORTED, "index_export: overlay snapshot (update it to a flat one)");
  if (idx->dev_subs || !idx->dev_base)
    return set_err(ctx, EMQX_GM_EUNSUPPORTED, "index_export: a snapshot whose subscriber CSR lives apart "
                                              "(emqx_gm_index_update_subs result) or without device tables");
  ImageHeader h;
  std::memset(&h, 0, sizeof h);
  std::memcpy(h.magic, kMagic, 8);
  h.version = kVersion;
  h.header_bytes = sizeof(ImageHeader);
  h.layout_sig = layout_signature();
  h.dev_bytes = idx->dev_bytes;
  h.level_nodes = idx->level_nodes;
  h.view = idx->view;
  h.info = idx->info;
  const uint8_t* base = static_cast<const uint8_t*>(idx->dev_base);
  IndexView v = idx->view;
  auto pf = ptr_fields(v);
  for (int i = 0; i < kPtrs; ++i) {
    const uint8_t* p = static_cast<const uint8_t*>(*pf[i]);
    if (!p) {
      h.ptr_off[i] = ~0ull;
      continue;
    }
    if (p < base || p >= base + idx->dev_bytes)
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
  h.soff_n = idx->soff.size();
  h.pinned_n = idx->pinned.size();
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
  if (h.soff_n) std::memcpy(buf + h.sec_off[3], idx->soff.data(), h.soff_n * 8);
  if (h.pinned_n) std::memcpy(buf + h.sec_off[4], idx->pinned.data(), h.pinned_n);
  if (h.blob_in_image) {
    hipSetDevice(idx->device);
    if (ctx) GM_HIP(ctx, hipStreamSynchronize(ctx->stream));
    GM_HIP(ctx, hipMemcpy(buf + h.sec_off[5], idx->dev_base, h.dev_bytes, hipMemcpyDeviceToHost));
  }
  *size = o;
  return EMQX_GM_OK;
}

int index_import(emqx_gm_ctx* ctx, const uint8_t* img, uint64_t size, const void* d_blob, emqx_gm_index** out) {
  if (!img || !out) return set_err(ctx, EMQX_GM_EINVAL, "index_import: NULL argument");
  ImageHeader h;
  if (size < sizeof h) return set_err(ctx, EMQX_GM_EINVAL, "index_import: truncated image");
  std::memcpy(&h, img, sizeof h);
  if (std::memcmp(h.magic, kMagic, 8) || h.version != kVersion || h.header_bytes != sizeof(ImageHeader))
    return set_err(ctx, EMQX_GM_EINVAL, "index_import: not an index image of this library");
  if (h.layout_sig != layout_signature())
    return set_err(ctx, EMQX_GM_EINVAL, "index_import: image from a library with another table layout");
  if (h.total_bytes > size || h.sec_off[5] > h.total_bytes)
    return set_err(ctx, EMQX_GM_EINVAL, "index_import: truncated image");
  if (!d_blob && !h.blob_in_image)
    return set_err(ctx, EMQX_GM_EINVAL, "index_import: the image holds no device blob and none was given");
  const uint64_t* fo = reinterpret_cast<const uint64_t*>(img + h.sec_off[1]);
  if (fo[0] != 0 || fo[h.n_filters] != h.ft_bytes || h.n_filters != h.info.n_filters)
    return set_err(ctx, EMQX_GM_EINVAL, "index_import: inconsistent filter table");
  for (int i = 0; i < kPtrs; ++i)
    if (h.ptr_off[i] != ~0ull && h.ptr_off[i] >= h.dev_bytes)
      return set_err(ctx, EMQX_GM_EINVAL, "index_import: inconsistent table layout");
  std::unique_ptr<emqx_gm_index> idx(new emqx_gm_index);
  idx->device = ctx->device;
  idx->dev_bytes = h.dev_bytes;
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
  idx->view = h.view;
  auto pf = ptr_fields(idx->view);
  for (int i = 0; i < kPtrs; ++i) *pf[i] = h.ptr_off[i] == ~0ull ? nullptr : B + h.ptr_off[i];
  idx->dev_flen = h.flen_off == ~0ull ? nullptr : reinterpret_cast<uint16_t*>(B + h.flen_off);
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
  idx->soff.assign(so, so + h.soff_n);
  idx->pinned.assign(img + h.sec_off[4], img + h.sec_off[4] + h.pinned_n);
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
  *out = idx.release();
  return EMQX_GM_OK;
}

// The host copy of an index's device tables for an in-place update, loaded on
// the first update of a snapshot built without one (gm_index.cpp: indexes past
// kEagerMirrorBytes, EMQX_GM_OPEN_MIRROR_LAZY, imported snapshots).  The device
// tables ARE the current state (filter-id fields included), so one download
// up to the subscriber CSR gives exactly what an eager mirror would hold.
int load_mirror_blob(emqx_gm_ctx* ctx, emqx_gm_index* idx) {
  Mirror& M = *idx->mirror;
  if (!M.blob.empty() || !idx->dev_base) return EMQX_GM_OK;
  M.blob.resize(M.blob_size);
  hipSetDevice(idx->device);
  if (ctx) GM_HIP(ctx, hipStreamSynchronize(ctx->stream));
  // pinned for the copy (several times the pageable rate), when the host allows it
  const bool reg = hipHostRegister(M.blob.data(), M.blob_size, hipHostRegisterDefault) == hipSuccess;
  const hipError_t e = hipMemcpy(M.blob.data(), idx->dev_base, M.blob_size, hipMemcpyDeviceToHost);
  if (reg) (void)hipHostUnregister(M.blob.data());
  if (e != hipSuccess) {
    std::vector<uint8_t>().swap(M.blob);
    return set_err(ctx, EMQX_GM_EDEVICE, std::string("index_update: mirror download: ") + hipGetErrorString(e));
  }
  return EMQX_GM_OK;
}

}  // namespace gm
