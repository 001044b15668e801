/*
 * emqx_gm_ext.h — extensions of libemqx_gpu_match.so that are NOT part of the
 * reference-facing boundary (emqx_gpu_match.h): the seeded synthetic workload
 * of SURVEY.md §8d (generated on the device for the bench), device-buffer
 * helpers for the Python host layer and bench, and roofline accounting.
 */
#ifndef EMQX_GM_EXT_H
#define EMQX_GM_EXT_H

#include "emqx_gpu_match.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Workload generator (spec: DESIGN.md "Workload generator").  codes: n x 5
 * int16 per filter: word index, -1 '+', -2 '#', -3 absent level. */
int emqx_gm_gen_filter_codes(uint64_t seed, uint64_t n, int wildcard_only, int16_t *codes);
/* Render codes to bytes + offsets[n+1]; returns the byte count (pass NULL
 * buffers to size). */
uint64_t emqx_gm_render_codes(const int16_t *codes, uint64_t n, uint8_t *bytes, uint64_t *off);
/* Generate topics [start, start+n) on the device; buffers come from the
 * context pool (free with emqx_gm_dev_free).  The byte buffer is padded. */
int emqx_gm_gen_topics(emqx_gm_ctx *ctx, const int16_t *filter_codes, uint64_t n_filters, uint64_t seed,
                       uint64_t start, uint64_t n, uint8_t **d_bytes, uint64_t **d_off, uint64_t *total_bytes);

/* Device buffers from the context pool. kind: 0 H2D, 1 D2H, 2 D2D. */
int emqx_gm_dev_alloc(emqx_gm_ctx *ctx, uint64_t bytes, void **out);
int emqx_gm_dev_free(emqx_gm_ctx *ctx, void *p);
int emqx_gm_memcpy(emqx_gm_ctx *ctx, void *dst, const void *src, uint64_t bytes, int kind);
/* Returns the context's cached device buffers to the runtime, and the device
 * blob kept from the last released index snapshot of 256 MiB or more (reused
 * by the next in-place update of its size; emqx_gm_close frees it too). */
int emqx_gm_pool_trim(emqx_gm_ctx *ctx);

/* Host-only self check of the index compiler (no device needed): compiles the
 * filter set into the flat tables and reports their sizes; perm_out as in
 * emqx_gm_index_build. */
int emqx_gm_index_compile_host(const uint8_t *filter_bytes, const uint64_t *filter_off, uint64_t n_filters,
                               const uint64_t *sub_off, const uint32_t *sub_ids, uint32_t *perm_out,
                               emqx_gm_index_info_t *info);

/* The filters with shard[i] == want, packed (two-call sizing: pass NULL
 * out_bytes/out_off to get *n_out and *bytes_out). */
int emqx_gm_select_filters(const uint8_t *filter_bytes, const uint64_t *filter_off, uint64_t n_filters,
                           const uint32_t *shard, uint32_t want, uint8_t *out_bytes, uint64_t *out_off,
                           uint64_t *n_out, uint64_t *bytes_out);

/* Sum of the byte lengths of the filters referenced by a device CSR (the
 * Σ len(f) term of the algorithmic-bytes formula). */
int emqx_gm_matched_filter_bytes(emqx_gm_ctx *ctx, const emqx_gm_index *idx, const emqx_gm_csr *csr,
                                 uint64_t *out);

/* One part of a fan-out split over n_parts devices ("split
 * rows and split wide rows across GPUs").  The deliveries emqx_gm_fanout would
 * return are numbered 0..T-1 in its order; part p produces the contiguous range
 * [T*p/n_parts, T*(p+1)/n_parts), so every row -- a 1M-subscriber row too -- is
 * cut wherever a range ends and the parts are disjoint and cover all T.  out:
 * row_off = the n_rows+1 GLOBAL delivery offsets (as emqx_gm_fanout's), nnz =
 * the part's length, ids = its deliveries; *first = its first global number.
 * This mirrors the reference's own split of a hot topic's subscribers into
 * shards dispatched independently (emqx_broker_helper.erl:82-91,
 * emqx_broker.erl:526-530). */
int emqx_gm_fanout_part(emqx_gm_ctx *ctx, const emqx_gm_index *idx, const emqx_gm_csr *matches, uint32_t part,
                        uint32_t n_parts, uint32_t flags, emqx_gm_csr *out, uint64_t *first);

/* What the calling thread's last index call (build, import, update,
 * update_subs) did -- observed, not inferred from sizes: the path it took,
 * whether it had to download the snapshot line's host mirror first (a lazy
 * mirror's first update: its bytes and time), and how the replicas of a
 * multi-device context were made. */
#define EMQX_GM_UPD_NONE 0      /* no change (the same snapshot retained)              */
#define EMQX_GM_UPD_PATCH 1     /* in-place patch of a device copy, O(delta)           */
#define EMQX_GM_UPD_OVERLAY 2   /* base + tombstones + delta index                     */
#define EMQX_GM_UPD_REBUILD 3   /* the updated set recompiled                          */
#define EMQX_GM_UPD_SUBS_ONLY 4 /* update_subs without a route change: tables shared   */
#define EMQX_GM_UPD_BUILD 5
#define EMQX_GM_UPD_IMPORT 6
#define EMQX_GM_REP_NONE 0      /* no replicas (single device, or left on the first)   */
#define EMQX_GM_REP_PATCHED 1   /* every member applied the same delta to its replica  */
#define EMQX_GM_REP_COPIED 2    /* device tables copied device to device (tree order)  */
#define EMQX_GM_REP_SHARED 3    /* members share their replica's tables + own new CSR  */
typedef struct {
  uint32_t kind;          /* EMQX_GM_UPD_*                                        */
  uint32_t replica_mode;  /* EMQX_GM_REP_*                                        */
  uint32_t replicas;      /* member replicas made                                 */
  int32_t mirror_loaded;  /* 1: the host mirror was loaded by this call           */
  uint64_t mirror_bytes;  /* ... its bytes                                        */
  double mirror_ms;       /* ... its time                                         */
  double device_ms;       /* the device part (every device at once), wall         */
  double replicate_ms;    /* replica copies after the first device's result, wall */
  double total_ms;        /* the whole call, wall                                 */
  uint32_t blobs_reused;  /* device tables placed in a released snapshot's blob   */
  uint32_t blobs_fresh;   /* ... in a fresh allocation (every device counted)     */
} emqx_gm_update_stats;
int emqx_gm_last_update_stats(const emqx_gm_ctx *ctx, emqx_gm_update_stats *stats);

/* Test support: FNV-1a digests of replica k's device tables (k = 0: the
 * snapshot itself, k >= 1: its replica on the context's k-th member) and of
 * its subscriber CSR (offsets + ids; 0 without one).  Replicas of one snapshot
 * hold byte-identical tables. */
int emqx_gm_index_replica_digest(emqx_gm_ctx *ctx, const emqx_gm_index *idx, uint32_t k, uint64_t *tables,
                                 uint64_t *subs);

#ifdef __cplusplus
}
#endif
#endif /* EMQX_GM_EXT_H */
