// gm_internal.h — context, index snapshot and device memory pool.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdlib>
#include <cstdint>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <functional>
#include <vector>

#include "../../include/emqx_gpu_match.h"
#include "../../include/emqx_gm_ext.h"
#include "gm_common.h"
#include "gm_filters.h"

namespace gm {

// An allocator that default-initialises: a vector of PODs is left unwritten
// by resize() until its owner fills it (GBs of index tables filled by all
// threads, or by a copy, instead of first zeroed by one).
template <class T> struct DefaultInit : std::allocator<T> {
  template <class U> struct rebind {
    using other = DefaultInit<U>;
  };
  DefaultInit() = default;
  template <class U> DefaultInit(const DefaultInit<U>&) {}
  template <class U> void construct(U* p) { ::new (static_cast<void*>(p)) U; }
  template <class U, class... A> void construct(U* p, A&&... a) { ::new (static_cast<void*>(p)) U(std::forward<A>(a)...); }
};
using HostBytes = std::vector<uint8_t, DefaultInit<uint8_t>>;

// Caching device allocator: buffers are returned to a size-keyed free list and
// reused, so steady-state batches do no hipMalloc/hipFree.
class DevPool {
 public:
  explicit DevPool(int device) : device_(device) {}
  ~DevPool();
  void* alloc(size_t bytes);           // nullptr on failure
  void release(void* p);
  // Release once the work queued on `s` so far is done (a result CSR the
  // caller frees while later calls may still be queued behind its readers):
  // an event marks the point, alloc() reclaims the buffer once it has passed,
  // and nothing waits.
  void release_after(void* p, hipStream_t s);
  void release_after(void* const* ps, int np, hipStream_t s);  // one event for up to 4 buffers
  void trim();
  size_t cached_bytes() const { return cached_; }

 private:
  int device_;
  std::multimap<size_t, void*> free_;  // rounded size -> ptr
  std::map<void*, size_t> live_;       // ptr -> rounded size
  std::vector<std::pair<void*, hipEvent_t>> deferred_;
  std::vector<hipEvent_t> ev_idle_;
  size_t cached_ = 0;
  void reclaim(bool wait);
};

// Host result buffers (the CSRs emqx_gm_match / emqx_gm_fanout return in host
// memory): emqx_gm_csr_free hands them back and the next call reuses them, so a
// steady stream of calls does no first-touch page faults on fresh pages (2 GB
// per 100M-topic call).  Large buffers are 2 MiB aligned and advised as huge
// pages.  At most kCap bytes stay cached.
// pinned: page-locked (hipHostMalloc, portable to every device) buffers that
// the device writes by DMA -- the multi-chunk host-buffer match copies its rows
// straight into them (gm_host.cpp) instead of through a bounce buffer.
class HostPool {
 public:
  ~HostPool();
  void* alloc(size_t bytes, bool pinned = false);  // nullptr on failure
  void release(void* p);      // a buffer of this pool (any other pointer: free())
  size_t cached_bytes() const { return cached_; }

 private:
  static constexpr size_t kCap = 8ull << 30;
  struct Buf {
    size_t bytes;
    bool pinned;
  };
  std::multimap<size_t, void*> free_[2];  // [pinned] rounded size -> ptr
  std::map<void*, Buf> live_;
  size_t cached_ = 0;
  void drop(void* p, bool pinned);
};

// Page-locked staging buffers of the small host-buffer calls (gm_host.cpp
// run_host_small): each call in flight owns its own, so concurrent calls on
// one context overlap; a thread-safe size-keyed free list (at most kCap cached).
class PinPool {
 public:
  ~PinPool();
  void* get(size_t bytes);  // nullptr on failure
  void put(void* p);
 private:
  static constexpr size_t kCap = 512ull << 20;
  std::mutex mu_;
  std::multimap<size_t, void*> free_;
  std::map<void*, size_t> size_;
  size_t cached_ = 0;
};

// Page-locked host buffers handed out by emqx_gm_host_alloc: the host-buffer
// match sends topic text that lies in one of them by DMA, without staging it
// (gm_host.cpp).  Process-wide, so a buffer is found from any context.
bool host_pinned_range(const void* p, size_t bytes);
void host_pinned_add(void* p, size_t bytes);
bool host_pinned_remove(void* p);

// RAII handle on a pool buffer.
struct PoolBuf {
  DevPool* pool = nullptr;
  void* p = nullptr;
  PoolBuf() = default;
  PoolBuf(DevPool* pl, size_t bytes) : pool(pl), p(pl->alloc(bytes)) {}
  PoolBuf(const PoolBuf&) = delete;
  PoolBuf& operator=(const PoolBuf&) = delete;
  PoolBuf(PoolBuf&& o) noexcept : pool(o.pool), p(o.p) { o.p = nullptr; }
  PoolBuf& operator=(PoolBuf&& o) noexcept {
    reset();
    pool = o.pool;
    p = o.p;
    o.p = nullptr;
    return *this;
  }
  ~PoolBuf() { reset(); }
  void reset() {
    if (p && pool) pool->release(p);
    p = nullptr;
  }
  void* release_ownership() {
    void* q = p;
    p = nullptr;
    return q;
  }
  template <class T> T* as() const { return static_cast<T*>(p); }
};

// Per-call scratch sizes of the match pipeline.
constexpr int FAST_FC = 8;    // frontier capacity per lane (LDS)
constexpr int FAST_MC = 16;   // match capacity per lane (LDS)
constexpr uint32_t OVF_BIT = 0x80000000u;
constexpr uint32_t LIST_BIT = 0x40000000u;  // compact staging: the row is listed-pass row (cnt & ~LIST_BIT)
constexpr uint32_t CNT_MASK = 0x7FFFFFFFu;

}  // namespace gm

namespace gm {
struct HostPipe;  // gm_host.cpp: pinned staging + copy streams + worker threads of the host-buffer path
}

struct emqx_gm_ctx {
  int device = 0;
  uint32_t open_flags = 0;  // emqx_gm_opts.flags (EMQX_GM_OPEN_*)
  gm::HostPipe* host = nullptr;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  hipStream_t stream2 = nullptr;  // tokenizer stream of the overlapped match (GM_OVERLAP)
  // assembly stream (gm_match.hip MatchCall): a large device-buffer call's
  // scan + assembly run here behind its main pass, so the next call's main
  // pass (context stream) overlaps them
  hipStream_t stream_asm = nullptr;
  hipEvent_t ov_ev[9] = {};
  std::recursive_mutex mu;
  gm::DevPool* pool = nullptr;
  gm::HostPool* hpool = nullptr;
  gm::PinPool* pins = nullptr;  // (thread safe: small host calls stage outside mu)
  emqx_gm_match_stats stats{};
  hipEvent_t ev[6]{};
  // per match call (gm_match.hip MatchCall, under mu): reusable events and
  // 64-B pinned read-back slots, so several calls can be in flight
  std::vector<hipEvent_t> ev_free;
  std::vector<void*> pin_free, pin_all;
  double ids_per_topic = 4.0;  // speculative ids capacity of a match call (run_match), from recent calls
  double subs_per_match = 16.0;  // speculative deliveries capacity of a small host fan-out, from recent calls
  // A ring of 64-B pass-counter blocks (gm_match.hip MatchCall): a call takes
  // the next block, already zeroed -- the previous call's assembly kernel zeroes
  // it -- so a call needs no zeroing launch of its own.  State per block: 0 ready
  // (zero, or zeroed by a kernel queued before any later use), 1 held by a call,
  // 2 dirty (its call is done).
  static constexpr int CTR_RING = 16;
  void* ctr_ring = nullptr;
  uint8_t ctr_state[CTR_RING] = {};
  int ctr_next = 0;
  // A multi-device context (emqx_gm_opts.n_devices > 1): this context is the
  // first listed device; members[k - 1] serves devices[k] (its own stream,
  // pools and host pipeline; used only under this context's lock).  Every
  // index made through this context carries a replica per member
  // (emqx_gm_index::reps).
  std::vector<emqx_gm_ctx*> members;
  emqx_gm_ctx* parent = nullptr;    // a member: its multi-device context
  std::atomic<uint32_t> rr{0};      // round-robin start of the next small host-buffer call (gm_api.cpp)
};

namespace gm {
struct OverlayState;

// The library's A/B and diagnostic knobs (GM_* environment variables: table
// layout, load factor, walk form, staging, update path, host pipeline) are
// read only when EMQX_GM_AB is set (non-empty, not "0"), so a library loaded
// into a BEAM runs its one default layout and walk whatever else the host's
// environment holds (the list: emqx_gpu_match.h).  Read per call, so a test
// or an A/B script sets it beside the knob.
inline const char* knob(const char* name) {
  const char* ab = getenv("EMQX_GM_AB");
  if (!ab || !*ab || (ab[0] == '0' && !ab[1])) return nullptr;
  return getenv(name);
}

// What the calling thread's last index call did (emqx_gm_last_update_stats):
// the entry points reset it, the update paths fill it in.
extern thread_local emqx_gm_update_stats tl_ustats;
double now_ms();

// The id change of an in-place update, from O(delta) lists: prev ids `dels`
// deleted (ascending), new filter k (byte order) inserted with addpos[k] prev
// filters sorting before it and temporary id nb + k.  map(): prev id -> new id
// (NONE: deleted) = id - (dels below it) + (inserts at or before it); a
// temporary nb + k -> addpos[k] - (dels below addpos[k]) + k.  The device
// builds the whole table with a kernel (apply_patch_device); table() is the
// host twin, materialized only where the host needs it.
struct IdShift {
  uint64_t nb = 0;
  std::vector<uint64_t> dels, addpos;
  uint32_t map(uint64_t id) const {
    if (id >= nb) {
      const uint64_t k = id - nb, p = addpos[k];
      return uint32_t(p - (std::lower_bound(dels.begin(), dels.end(), p) - dels.begin()) + k);
    }
    if (std::binary_search(dels.begin(), dels.end(), id)) return NONE;
    return uint32_t(id - (std::lower_bound(dels.begin(), dels.end(), id) - dels.begin()) +
                    (std::upper_bound(addpos.begin(), addpos.end(), id) - addpos.begin()));
  }
  // indexed like the table (renum_field): map() without materializing it
  uint32_t operator[](uint64_t id) const { return map(id); }
  std::vector<uint32_t> table() const {
    std::vector<uint32_t> r(nb + addpos.size());
    uint64_t d = 0, a = 0;
    for (uint64_t id = 0; id < nb; ++id) {
      while (a < addpos.size() && addpos[a] <= id) ++a;
      if (d < dels.size() && dels[d] == id) {
        r[id] = NONE;
        ++d;
        continue;
      }
      r[id] = uint32_t(id - d + a);
    }
    for (uint64_t k = 0; k < addpos.size(); ++k) r[nb + k] = map(nb + k);
    return r;
  }
};

// Host copy of a plain index's device blob (no shard ids, no subscriber
// lists), byte for byte, with the headroom an in-place update may use
// (gm_overlay.cpp, patch_update): appended trie nodes, new words in the
// arena, more filter lengths.  It belongs to the newest snapshot of its line:
// an update moves it from the old snapshot (which stays valid for its readers)
// to the new one.
struct Mirror {
  HostBytes blob;                        // empty until the first update when built lazily (load_mirror_blob)
  size_t blob_size = 0;                  // bytes of the blob: the device tables up to the subscriber CSR
  size_t o_nodes = 0, o_dict = 0, o_edges = 0, o_hot = 0, o_arena = 0, o_flen = 0, o_efilt = 0, o_mph = 0;
  uint64_t nodes_n = 0, nodes_cap = 0;   // v1 level-trie nodes used / capacity
  uint64_t arena_n = 0, arena_cap = 0;   // word bytes used / capacity
  uint64_t flen_cap = 0;                 // filter-length entries available
  uint64_t dict_used = 0;
  uint64_t edge_used[EDGE_DEPTHS] = {};
  uint64_t hot_used[HOT_TABLES] = {};
  uint64_t mph_ovf_used[HOT_TABLES] = {};  // keys in each MPH table's overflow region
};
}

struct emqx_gm_index {
  std::atomic<int> refs{1};
  int device = 0;
  void* dev_base = nullptr;     // one allocation holding every table
  void* dev_subs = nullptr;     // a subscriber CSR of its own (after emqx_gm_index_update_subs), or nullptr
  size_t subs_bytes = 0;        // ... its bytes
  emqx_gm_index* blob_owner = nullptr;  // set: dev_base is that (retained) snapshot's blob, shared
  size_t dev_bytes = 0;
  gm::IndexView view{};
  uint16_t* dev_flen = nullptr; // filter lengths (stats only), inside dev_base
  mutable std::atomic<bool> flen_stale{false};  // dev_flen not yet rewritten after an in-place update
  mutable std::mutex flen_mu;
  // host copies
  gm::FilterTable ft;           // the sorted unique filters (id = rank), gm_filters.h
  std::vector<uint32_t> gmap;   // shard index: global id of each local filter (ascending); empty otherwise
  gm::SubTable subs;            // per filter id: subscriber CSR offset and route mark (emqx_gm_index_update_subs
                                // ROUTE_ADD); empty without subscriber lists.  gm_filters.h
  gm::OverlayState* ov = nullptr;  // overlay snapshot (emqx_gm_index_update); tables above unused then
  uint64_t level_nodes = 0;        // an upper bound on the trie nodes of any one depth (the slow path's frontier); 0: unknown
  gm::Mirror* mirror = nullptr;    // host copy of the blob (updatable plain index), see gm::Mirror
  std::mutex mirror_mu;            // an in-place update holds it while it patches and hands the mirror on
  emqx_gm_index_info_t info{};
  // made through a multi-device context: reps[k - 1] = this snapshot on that
  // context's members[k - 1] (same rows; its own device tables, or the tables
  // of an older replica it shares as this snapshot shares its owner's).  Owned:
  // released with this snapshot.
  std::vector<emqx_gm_index*> reps;
  bool reused_blob = false;  // (replicate_index: dev_base was a released snapshot's blob)
  // a prefix-sharded index (emqx_gm_index_build_sharded, gm_shard.cpp): shards[k]
  // on the context's k-th device (a shard index with global ids), route sends a
  // topic to its one shard, fshard[global id] = a filter's shard (or
  // EMQX_GM_ALL_SHARDS).  This object holds only the host side (ft, subs, info).
  std::vector<emqx_gm_index*> shards;
  emqx_gm_route* route = nullptr;
  std::vector<uint32_t> fshard;
};

namespace gm {
// gm_index.cpp
int build_index(emqx_gm_ctx* ctx, const uint8_t* fb, const uint64_t* fo, uint64_t n, const uint64_t* sub_off,
                const uint32_t* sub_ids, uint32_t* perm_out, emqx_gm_index** out,
                emqx_gm_index_info_t* host_only = nullptr, const uint32_t* gids = nullptr);
void sort_filters(std::vector<uint32_t>& ord, const uint8_t* fb, const uint64_t* fo);
void free_index(emqx_gm_index* idx);
// gm_index.cpp: a freed snapshot's device blob kept, one per device, for the
// next in-place update of that size (a large fresh hipMalloc after a few
// update / free cycles stalls: C5's 38 GB blob took ~1 s from the 7th update on,
// 0.3 ms before).  take: a spare of at least `bytes` (at most 1.25x), or null;
// give: keeps p (the device synchronized first, as hipFree does) or frees it;
// trim: frees the device's spare (emqx_gm_pool_trim, emqx_gm_close).
void* take_spare_blob(int device, size_t bytes);
void give_spare_blob(int device, void* p, size_t bytes);
void trim_spare_blob(int device);
// open contexts per device (emqx_gm_open / _close): a blob freed while none is
// open on its device is not kept (nothing would trim it)
void note_ctx_open(int device);
void note_ctx_close(int device);
// gm_match.hip
// A caller's work queued on the context stream right behind the speculative
// assembly of a DEVICE_IO match, before run_match's one host round trip (the
// host path queues the rows' copy-out there).  enqueue(row_off, ids, cap) gets
// the device rows and the ids capacity; `used` says whether those rows are the
// call's result (no reassembly happened).
struct MatchTail {
  std::function<int(const uint64_t* row_off, const uint32_t* ids, uint64_t cap)> enqueue;
  bool used = false;
};
int run_match(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const uint8_t* tb, const uint64_t* to, uint64_t n,
              uint32_t flags, emqx_gm_csr* out, MatchTail* tail = nullptr);
// the two halves of run_match (emqx_gm_match_submit / _wait): submit under
// ctx->mu; wait without it (it takes the lock after the device wait)
// tail (optional): as run_match's, kept by the caller until match_wait;
// st_out (optional): the call's own stats (ctx->stats may belong to a later call by then)
int match_submit(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const uint8_t* tb, const uint64_t* to, uint64_t n,
                 uint32_t flags, void** ticket, MatchTail* tail = nullptr);
int match_wait(emqx_gm_ctx* ctx, void* ticket, emqx_gm_csr* out, MatchTail* tail = nullptr,
               emqx_gm_match_stats* st_out = nullptr);
int run_fanout(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const emqx_gm_csr* m, uint32_t flags,
               emqx_gm_csr* out, uint32_t part = 0, uint32_t n_parts = 1, uint64_t* first_out = nullptr);
int run_merge_rows(emqx_gm_ctx* ctx, uint64_t n_rows, uint64_t stride, uint32_t n_pieces, const uint32_t* d_lens,
                   const uint32_t* d_ids, uint32_t flags, emqx_gm_csr* out);
int run_row_lengths(emqx_gm_ctx* ctx, const emqx_gm_csr* csr, uint32_t* d_out);
// prefix sharding (gm_route.hip) and the exchange's device steps
int route_plan(const uint8_t* fb, const uint64_t* fo, uint64_t n, uint32_t n_shards, uint32_t* shard_out,
               emqx_gm_route** out);
int route_topics_host(const emqx_gm_route* r, const uint8_t* tb, const uint64_t* to, uint64_t n, uint32_t* dest);
int route_topics_device(emqx_gm_ctx* ctx, emqx_gm_route* r, const uint8_t* d_tb, const uint64_t* d_to, uint64_t n,
                        uint32_t* d_dest);
int route_partition(emqx_gm_ctx* ctx, emqx_gm_route* r, const uint8_t* d_tb, const uint64_t* d_to, uint64_t n,
                    uint32_t* d_perm, uint32_t* d_plen, uint64_t* d_split);
void free_route(emqx_gm_route* r);
int permute_topics(emqx_gm_ctx* ctx, const uint8_t* d_tb, const uint64_t* d_to, uint64_t n, const uint32_t* d_perm,
                   uint8_t* d_out, uint64_t* d_out_off);
int unpermute_rows(emqx_gm_ctx* ctx, uint64_t n, const uint32_t* d_perm, const uint32_t* d_lens, const uint32_t* d_ids,
                   uint32_t flags, emqx_gm_csr* out);
int scan_lengths(emqx_gm_ctx* ctx, const uint64_t* len, uint64_t n, uint64_t* out);

// A replica an update makes on member context m from prev's replica `prev`
// (gm_overlay.cpp patch_update, gm_subs.cpp update_subs): each member applies
// the same O(delta) plan to its own device copy at the same time as the first
// device -- the reference's every-node-applies-the-delta replication
// (apps/emqx/src/emqx_router_utils.erl:33-38, emqx_trie.erl:114-136).
struct RepTarget {
  emqx_gm_ctx* m = nullptr;
  emqx_gm_index* prev = nullptr;
  emqx_gm_index* out = nullptr;  // made by the update (owned by the caller until attached)
};
// gm_overlay.cpp — incremental index maintenance.  An
// overlay snapshot = an immutable base snapshot (shared, retained) minus
// tombstoned base filters plus a small delta index over the inserted filters.
// Final filter ids are ranks in the updated set: a surviving base id b maps to
// b + (delta filters sorting before b) - (tombstones below b); delta filters
// carry their final ids directly (shard-style global ids).
struct OverlayState {
  emqx_gm_index* base = nullptr;     // retained flat snapshot
  emqx_gm_index* delta = nullptr;    // flat snapshot over the inserted filters, or nullptr
  std::vector<uint32_t> tomb;        // deleted base ids, ascending
  std::vector<uint32_t> ins;         // per delta filter (byte order): base filters sorting before it
  std::vector<uint32_t> dgid;        // per delta filter: final id
  std::vector<uint8_t> dbytes;       // delta filters, byte order
  std::vector<uint64_t> doff;
  void* dev = nullptr;               // tomb bitmap | its word prefix counts | ins
  const uint32_t* d_tbm = nullptr;
  const uint32_t* d_tpre = nullptr;
  const uint32_t* d_ins = nullptr;
};
int update_index(emqx_gm_ctx* ctx, emqx_gm_index* prev, const uint8_t* fb, const uint64_t* fo, const uint8_t* ops,
                 uint64_t n_ops, emqx_gm_index** out);
// The in-place patch of update_index (prev must hold the mirror and a write
// lock on it): deletes base ids `tomb`, inserts the filters `dset`.  Returns 1
// when a table lacks room (nothing changed), <0 on error.  rmap_out (optional)
// receives old id -> new id for prev's filters (NONE: deleted) followed by the
// new ids of dset's filters in byte order.
// trie_only: the new blob holds the tables up to the subscriber CSR only (the
// caller gives the snapshot a CSR of its own).
// reps (optional): the member replicas to patch alongside (RepTarget::out set on success).
int patch_update(emqx_gm_ctx* ctx, emqx_gm_index* prev, const std::set<uint32_t>& tomb,
                 const std::set<std::string>& dset, emqx_gm_index** out, std::vector<uint32_t>* rmap_out = nullptr,
                 bool trie_only = false, std::vector<RepTarget>* reps = nullptr);
bool well_formed_filter(const uint8_t* p, uint64_t len);
// gm_image.cpp: index images (emqx_gm_index_export / _import) and the lazy host mirror
int index_export(emqx_gm_ctx* ctx, const emqx_gm_index* idx, uint32_t flags, uint8_t* buf, uint64_t* size);
int index_import(emqx_gm_ctx* ctx, const uint8_t* img, uint64_t size, const void* d_blob, emqx_gm_index** out);
int load_mirror_blob(emqx_gm_ctx* ctx, emqx_gm_index* idx);
// an image's every count and offset checked against its own bytes (no device);
// EMQX_GM_EINVAL with the reason in *why
int validate_image(const uint8_t* img, uint64_t size, bool have_blob, std::string* why);
// the host half of an import (validate_image, then the host tables into idx;
// its view's pointer fields hold blob offsets + 1, 0 = null)
int import_host_part(const uint8_t* img, uint64_t size, bool have_blob, emqx_gm_index* idx, std::string* why);
// test support (tests/asan): a named u64 header field of an image (nullptr:
// unknown name), a u32 count of its view (0 n_nodes, 1 efilt_mask[t], 2
// mph_nb[t]), and the checksum recomputed after a change
uint64_t* image_field(uint8_t* img, const std::string& name);
uint32_t image_view_u32(uint8_t* img, int which, int t);
void image_view_set_u32(uint8_t* img, int which, int t, uint32_t x);
void image_reseal(uint8_t* img, uint64_t size);
// gm_match.hip: write the root's '+' record (IndexView::d0_root) from view v's
// depth-1 hot table on the device; d0 is the region's device address (v's own
// pointer is const).  0: written (the caller sets IX_D0), 1: not wanted
// (GM_D0=0), <0: error.
int refresh_d0(emqx_gm_ctx* ctx, const IndexView& v, void* d0);
// a plain index's host mirror is kept from the build when its tables are at most this big
// (C3's 4.6 GB tables keep theirs: a lazy first update downloads the tables,
// 0.8 s at C3 over pageable copies; the 38 GB C5 index does not)
constexpr size_t kEagerMirrorBytes = size_t(8) << 30;
// rank of f among idx's filters; *found = exact hit
uint64_t filter_rank(const emqx_gm_index* idx, const uint8_t* f, uint64_t len, bool* found);
// gm_subs.cpp: emqx_gm_index_update_subs
int update_subs(emqx_gm_ctx* ctx, emqx_gm_index* prev, const uint8_t* fb, const uint64_t* fo, const uint32_t* subs,
                const uint8_t* ops, uint64_t n_ops, emqx_gm_index** out);
bool is_pinned(const emqx_gm_index* idx, uint64_t f);
// gm_match.hip: segments [src_off[j], src_off[j] + (dst_off[j+1] - dst_off[j])) of
// the device array src gathered into host `out` (dst_off[m] elements), one
// device gather + one copy back
int gather_segments(emqx_gm_ctx* ctx, const uint32_t* src, const std::vector<uint64_t>& src_off,
                    const std::vector<uint64_t>& dst_off, uint32_t* out);
// gm_match.hip: the new subscriber CSR of a subscriber-only update_subs batch
// (ids unchanged; O(delta) host work, see there)
int shift_subs_device(emqx_gm_ctx* ctx, const emqx_gm_index* prev, emqx_gm_index* idx,
                      const std::vector<uint32_t>& aff_ids, const std::vector<uint64_t>& aff_off,
                      const std::vector<uint32_t>& aff_buf);
// gm_match.hip: the new subscriber CSR of update_subs (see there)
int rebuild_subs_device(emqx_gm_ctx* ctx, const emqx_gm_index* prev, emqx_gm_index* idx,
                        const std::vector<uint64_t>& new_soff, const std::vector<uint32_t>& inv,
                        const std::vector<uint32_t>& aff_ids, const std::vector<uint64_t>& aff_off,
                        const std::vector<uint32_t>& aff_buf);
int overlay_filter(const emqx_gm_index* idx, uint32_t id, const uint8_t** bytes, uint64_t* len);
void free_overlay(emqx_gm_index* idx);
// An op of Patcher::orops whose offset carries PATCH_AND clears its bits
// instead of setting them (an op never sets a bit another op clears, so the
// device applies them in any order).
constexpr uint64_t PATCH_AND = 1ull << 63;
// gm_match.hip: the device side of an in-place update (patch_update): dst =
// src (bytes), then the host-patched byte ranges (offset, length) of `host`
// written over it, the OR / AND ops (offset of a word, bits) applied, then every
// filter-id field of the hot slots and of nodes [0, n_nodes) renumbered by
// the shift (its table built on the device).  Done in one pass over the blob:
// the hot slots and nodes are renumbered while copied and the patched ranges
// go up already renumbered (GM_UPDATE_UNFUSED: copy, patch, then renumber in
// place -- the A/B twin).
int apply_patch_device(emqx_gm_ctx* ctx, void* dst, const void* src, size_t bytes,
                       const std::vector<std::pair<uint64_t, uint32_t>>& ranges, const uint8_t* host,
                       const IndexView& v, uint64_t o_hot, uint64_t o_nodes, uint64_t n_nodes,
                       const IdShift& shift, const std::vector<std::pair<uint64_t, uint32_t>>& orops);
// gm_match.hip
int run_match_overlay(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const uint8_t* tb, const uint64_t* to, uint64_t n,
                      uint32_t flags, emqx_gm_csr* out);
int set_err(emqx_gm_ctx* ctx, int code, const std::string& msg);
// gm_match.hip: offset conversions of the host-buffer path (n1 = entries)
int launch_off32_to_64(hipStream_t st, const uint32_t* in, uint64_t n1, uint64_t* out);
int launch_off64_to_32(hipStream_t st, const uint64_t* in, uint64_t n1, uint32_t* out);
int launch_copy_u32x2(hipStream_t st, const uint32_t* s0, uint32_t* d0, uint64_t n0, const uint32_t* s1, uint32_t* d1,
                      uint64_t n1, const uint64_t* n1_max = nullptr);
int launch_add_u64(hipStream_t st, uint64_t* p, uint64_t n1, uint64_t add);
// the host path's u16 topic lengths -> u64 offsets (n + 1 entries, an exclusive scan) on stream st
int scan_len16(emqx_gm_ctx* ctx, hipStream_t st, const uint16_t* len, uint64_t n, uint64_t* out);
// gm_host.cpp: emqx_gm_match on host buffers, chunked and pipelined (H2D / match / D2H overlap)
int run_match_host(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const uint8_t* tb, const uint64_t* to, uint64_t n,
                   uint32_t flags, emqx_gm_csr* out);
void free_host_pipe(emqx_gm_ctx* ctx);
// the topics of one host-pipeline chunk at most (a call this small runs whole on one device)
uint64_t host_chunk_topics();
// A host-buffer call of at most one chunk, entered WITHOUT ctx->mu: staged into
// the call's own page-locked buffer outside the lock, queued under it (inputs
// up, the match, the rows' copy-out behind its speculative assembly straight
// into the page-locked result; copies up to 1 MiB as kernels over mapped
// memory), waited for outside it -- so concurrent small calls on one device
// overlap one another's host work and device round trips
// fan (optional, emqx_gm_match_fanout): the call's fan-out queued behind its
// speculative rows in the same round trip; fan->ok says whether it held (the
// match's rows and the deliveries both within their capacities)
struct SmallFan {
  emqx_gm_csr out{};
  bool ok = false;
  // (why not, for the tests' message: queued, the rows were the speculative ones, deliveries vs capacity)
  bool queued = false, rows_spec = false;
  uint64_t total = 0, cap = 0;
};
int run_host_small(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const uint8_t* tb, const uint64_t* to, uint64_t n,
                   uint32_t flags, emqx_gm_csr* out, emqx_gm_match_stats* st_out, SmallFan* fan = nullptr);
int queue_fanout_spec(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const uint64_t* d_ro, const uint32_t* d_ids,
                      uint64_t n, uint64_t cap_m, uint64_t cap_f, uint64_t* seg_dst, uint64_t* row_off, uint32_t* ids);
// A host-row fan-out of a publish window, the same way (entered WITHOUT
// ctx->mu): the rows staged outside the lock, the deliveries written into a
// speculative capacity, one device round trip.  idx: the snapshot on this
// device (a replica), host: the primary (its filter count).  Returns 1 --
// nothing delivered -- for rows that are not a plain CSR, a fan-out whose
// expected size is past kFanSmallDeliveries, or one past its capacity: the
// caller takes the ordinary path.
int run_fanout_small(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const emqx_gm_index* host, const emqx_gm_csr* m,
                     emqx_gm_csr* out, emqx_gm_match_stats* st_out);
int queue_fanout_small(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const uint64_t* d_off, const uint32_t* d_ids,
                       uint64_t n, uint64_t nnz, uint64_t total, uint64_t* seg_dst, uint64_t* row_off, uint32_t* ids);
// gm_multi.cpp: multi-device contexts (emqx_gm_opts.n_devices).
// A copy of flat snapshot `src` (any device) on member context m's device:
// the host tables shared or copied, the device tables copied device to device
// (peer copy across devices) -- or, with `share` (a replica on m whose device
// tables hold the bytes src's own tables hold: src shares its owner's blob and
// share is that owner's replica), those tables shared.  No host mirror (the
// primary snapshot's line owns it).
int replicate_index(emqx_gm_ctx* m, const emqx_gm_index* src, emqx_gm_index* share, emqx_gm_index** out);
// f(k) for k = 0..K-1 at once, one thread each (k = 0 on the calling thread);
// the first failure's code, its message set on the calling thread
int run_all(int K, const std::function<int(int)>& f);
// the targets of an update of `prev` through ctx: one per member when prev has
// its replicas there, else none (the result is copied by replicate_result)
std::vector<RepTarget> rep_targets(emqx_gm_ctx* ctx, emqx_gm_index* prev);
// a new replica on m carrying src's host fields (filter table, subscriber
// table, info; shared bases) and no device tables yet
emqx_gm_index* replica_shell(emqx_gm_ctx* m, const emqx_gm_index* src);
// attach the targets' replicas to out (all made), or free them (rc != 0)
int attach_replicas(emqx_gm_index* out, std::vector<RepTarget>& t, int rc);
// After an index call on a multi-device context made `out` from `prev` (NULL
// for a build / import): give `out` its replicas unless the update already
// made them (an in-place patch or update_subs applies its delta on every
// device, RepTarget).  A flat result is copied device to device in a tree
// (sharing prev's replica's tables when out shares prev's); an overlay stays
// on the first device.  On failure `out` is released and *out_p cleared.
int replicate_result(emqx_gm_ctx* ctx, emqx_gm_index* prev, emqx_gm_index** out_p);
// gm_shard.cpp: the prefix-sharded index of a multi-device context
int build_sharded(emqx_gm_ctx* ctx, const uint8_t* fb, const uint64_t* fo, uint64_t n, const uint64_t* sub_off,
                  const uint32_t* sub_ids, uint32_t* perm_out, emqx_gm_index** out);
int run_match_sharded(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const uint8_t* tb, const uint64_t* to, uint64_t n,
                      uint32_t flags, emqx_gm_csr* out);
int run_fanout_sharded(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const emqx_gm_csr* m, uint32_t flags,
                       emqx_gm_csr* out);
// emqx_gm_fanout of host rows over a multi-device context's replicas (one
// slice per device, one page-locked result); small batches: run_fanout
int run_fanout_multi(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const emqx_gm_csr* m, uint32_t flags,
                     emqx_gm_csr* out);
}  // namespace gm

#define GM_HIP(ctx, expr)                                                                     \
  do {                                                                                        \
    hipError_t _e = (expr);                                                                   \
    if (_e != hipSuccess)                                                                     \
      return gm::set_err((ctx), EMQX_GM_EDEVICE,                                              \
                         std::string(#expr) + ": " + hipGetErrorString(_e));                  \
  } while (0)
