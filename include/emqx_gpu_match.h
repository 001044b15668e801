/*
 * emqx_gpu_match.h — C ABI of libemqx_gpu_match.so, the MI355X batch
 * topic-matching engine for EMQX's publish routing hot path.
 *
 * This is the drop-in boundary that a thin Erlang NIF (`emqx_gpu_match`,
 * nif/emqx_gpu_match_nif.c) binds.  Each entry point replaces one reference
 * interface (paths relative to the reference repo root):
 *
 *   emqx_gm_index_build   <- the emqx_trie / emqx_route tables as maintained by
 *                            emqx_router:do_add_route/2 + emqx_trie:insert/1
 *                            (apps/emqx/src/emqx_router.erl:112-125,
 *                             apps/emqx/src/emqx_trie.erl:107-119) and the
 *                            emqx_subscriber bag written by
 *                            emqx_broker:do_subscribe/4 (emqx_broker.erl:147-165)
 *   emqx_gm_index_info    <- emqx_trie:empty/0 (emqx_trie.erl:165-170)
 *   emqx_gm_match         <- emqx_trie:match/1 (emqx_trie.erl:139-161) with
 *                            flags = 0, or emqx_router:match_routes/1
 *                            (emqx_router.erl:128-145) with
 *                            EMQX_GM_WITH_EXACT; batched over many topics
 *   emqx_gm_fanout        <- emqx_broker:dispatch/2 + do_dispatch/2,3 +
 *                            subscribers/1 (emqx_broker.erl:296-322, 506-530)
 *   emqx_gm_match_fanout  <- emqx_broker:publish/1's route/2 + dispatch/2 of a
 *                            batch (emqx_broker.erl:204-215, 245-322)
 *
 * Result semantics (bit-exact with the reference, compared as sets):
 *   - filter ids are the lexicographic rank of the filter bytes (Erlang binary
 *     order = unsigned bytewise, prefix first), so each result row, sorted
 *     ascending by id, is `lists:sort/1` of the reference's result list;
 *   - flags = 0: row = emqx_trie:match(Topic) over the indexed filters that the
 *     trie holds (wildcard filters; a single-word '$X' topic also returns a
 *     non-wildcard '$X' filter, emqx_trie.erl:271-278); a wildcard topic gives
 *     an empty row (emqx_trie.erl:149-158);
 *   - EMQX_GM_WITH_EXACT: row = the distinct filters whose routes
 *     match_routes(Topic) returns: the literal filter == Topic (also for a
 *     wildcard Topic) plus the trie matches;
 *   - fan-out rows are multisets: a subscriber of two matching filters is
 *     delivered twice (emqx_persistent_session_SUITE.erl:705).
 *
 * Ownership: input buffers are borrowed for the duration of a call.  Result
 * CSR buffers belong to the library until emqx_gm_csr_free().  Indexes are
 * immutable and reference counted (RCU-style snapshot swap by the caller).
 * Threading: a context may be used from several threads; calls on one context
 * are serialised onto its HIP stream.  Errors: every call returns 0 or a
 * negative EMQX_GM_E* code; nothing aborts the process; the message is in
 * emqx_gm_last_error(), which is kept per calling thread (a failing call's
 * message cannot be replaced by a concurrent call on another thread).
 *
 * Device topic buffers (EMQX_GM_DEVICE_IO): the tokenizer reads whole aligned
 * 8-byte words, so at least 64 readable bytes must follow topic_bytes[toff[n]]
 * (the library pads its own copies of host buffers the same way).
 *
 * Environment: the default library reads ONE variable, EMQX_GM_AB.  Unless it
 * is set (non-empty, not "0"), every GM_* knob below is ignored, so a library
 * loaded into a BEAM runs one table layout and one walk whatever else the
 * host's environment holds.  With EMQX_GM_AB set (A/B scripts, the test
 * suite) the library reads, per call:
 *   layout (at build):  GM_HOT_LOAD_PCT, GM_HOT_LOAD_PCT_UPPER, GM_HOT_FLAT,
 *     GM_HOT_SPARSE, GM_HOT_RH_INSERT, GM_NO_RH_EXIT, GM_NO_MPH, GM_MPH_TABLES,
 *     GM_MPH_SLACK, GM_MPH_LAMBDA, GM_MPH_MIN_KEYS, GM_MPH_MAX_KEYS,
 *     GM_MPH_NO_FILTERED, GM_CHAIN, GM_NO_CHAIN, GM_NO_EDGE_FILTER,
 *     GM_EFILT_ALL, GM_EFILT_DIV, GM_EFILT_MAX_KB, GM_DICT_MUL, GM_L1_BYPASS,
 *     GM_TRIE_RUNS, GM_MIRROR, GM_NO_MIRROR;
 *   walk and staging:   GM_MATCH_MAIN (the superseded split / coop / lds
 *     forms), GM_TOK_GROUP, GM_OVERLAP, GM_FUSED_PRIO, GM_HOT_POLICY, GM_NT,
 *     GM_D0, GM_STAGE_COMPACT, GM_STAGE_SC1, GM_LISTED_CAP, GM_LISTED_DEFER,
 *     GM_SCAN_SPLIT, GM_SCAN_SUMS, GM_NO_SPEC_IDS, GM_ASM_STREAM;
 *   host path:          GM_HOST_SIMPLE, GM_HOST_PIPE, GM_HOST_CHUNK,
 *     GM_HOST_THREADS, GM_HOST_BOUNCE, GM_HOST_WIDE_ROWS, GM_HOST_OFF32,
 *     GM_FANOUT_MULTI_MIN, GM_FANOUT_SIMPLE, GM_FANOUT_FUSED_ONLY;
 *   updates:            GM_UPDATE_OVERLAY, GM_UPDATE_UNFUSED, GM_SPARE_BLOB_MIN;
 *   diagnostics:        GM_UPDATE_TIMING, GM_INDEX_STATS, GM_INDEX_VERIFY.
 */
#ifndef EMQX_GPU_MATCH_H
#define EMQX_GPU_MATCH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EMQX_GM_ABI_VERSION 1

#define EMQX_GM_OK            0
#define EMQX_GM_EINVAL       -1 /* bad argument (badarg / function_clause)     */
#define EMQX_GM_ENOMEM       -2 /* host or device allocation failed            */
#define EMQX_GM_EDEVICE      -3 /* HIP runtime / device fault                  */
#define EMQX_GM_EOVERFLOW    -4 /* a row exceeded the device result capacity    */
#define EMQX_GM_EUNSUPPORTED -5 /* operation not available on this build       */

/* emqx_gm_match / emqx_gm_fanout flags */
#define EMQX_GM_WITH_EXACT 0x1u /* emqx_router:match_routes/1 semantics        */
#define EMQX_GM_DEVICE_IO  0x2u /* inputs are device pointers; result stays on
                                   the device (bench / multi-GPU path)         */
#define EMQX_GM_NO_TIMING  0x4u /* emqx_gm_match / _submit on device buffers:
                                   do not time this call's main pass
                                   (stats.match_kernel_ms and total_device_ms
                                   read 0).  A timed call puts the kernel's
                                   start/stop timestamps on the stream, which
                                   costs the device ~5 us of idle each; a
                                   serving loop times one call in a few      */

typedef struct emqx_gm_ctx emqx_gm_ctx;
typedef struct emqx_gm_index emqx_gm_index;
typedef struct emqx_gm_call emqx_gm_call;

/* Device list (the opts "select the device list (1-8)").  A BEAM
 * node loads its NIF once, so one context must be able to serve the whole
 * node's GPUs, as the reference's match_routes/1 runs in every publisher
 * process on all schedulers at once (apps/emqx/src/emqx_trie.erl:66-70,
 * emqx_router.erl:75-84, 128-145).  With n_devices = k > 0 the context owns
 * one replica of every index per listed device (a device may be listed more
 * than once: several replicas, e.g. a one-GPU rehearsal):
 *   - an index is compiled ONCE on the host and its device tables are copied
 *     to the other devices device to device (peer copies over xGMI, in a tree:
 *     every replica made is the source of another, so 8 devices take 3 rounds
 *     of copies and every device's links carry them);
 *   - an update is applied on every device at once, each from its own replica
 *     of the predecessor, as every EMQX node applies the same route delta to
 *     its own tables (emqx_router_utils.erl:33-38, emqx_trie.erl:114-136): the
 *     in-place patch's host plan is made once and each device runs its own
 *     one-pass patch; a subscriber-only emqx_gm_index_update_subs shares each
 *     replica's tables and writes each device's new subscriber CSR there;
 *     rebuilds and imports are copied as at a build; an overlay result (a
 *     filter with '#' inside) stays on the first device and is matched there;
 *   - emqx_gm_match on host buffers: a batch of more than one chunk (256K
 *     topics) is cut into chunks that run on all the devices at once (one host
 *     pipeline per device), the rows back in the caller's ONE CSR in batch
 *     order; a smaller batch runs whole on ONE device, the next one
 *     round-robin, so concurrent callers (dirty schedulers) run on different
 *     GPUs at once (on any context, such a call stages its topics into
 *     page-locked buffers of its own and waits for the device without the
 *     context lock: concurrent small calls overlap on one GPU too);
 *   - emqx_gm_fanout on host rows (65,536 rows or more) cuts them into one
 *     slice per device, balanced by matches, into the caller's ONE result;
 *     fewer rows (a publish window's, at most 16M deliveries) run whole on
 *     ONE device, round-robin like a small match, and -- on any context --
 *     hold its lock only to queue their work, so concurrent fan-outs overlap;
 *   - device-buffer calls (EMQX_GM_DEVICE_IO, emqx_gm_match_submit, a
 *     device-row fan-out), the sharding helpers, emqx_gm_set_stream and
 *     emqx_gm_index_device_blob / _export use the first listed device; so
 *     does any call on an index made through another context (it has no
 *     replicas here).
 * n_devices = 0 is the single-device context on `device`. */
#define EMQX_GM_MAX_DEVICES 8
typedef struct {
  int32_t device;        /* HIP device ordinal (n_devices == 0)                 */
  uint32_t flags;        /* EMQX_GM_OPEN_* (0: defaults)                        */
  uint32_t n_devices;    /* 0: `device` alone; 1..EMQX_GM_MAX_DEVICES: devices[] */
  int32_t devices[EMQX_GM_MAX_DEVICES];
  uint32_t reserved0;
  uint64_t reserved[2];
} emqx_gm_opts;

/* emqx_gm_opts.flags: the host copy of a plain index's device tables that an
 * in-place emqx_gm_index_update patches (host RAM ~ the tables' size).  By
 * default it is kept from the build for tables up to 8 GiB and downloaded from
 * the device on a snapshot line's first update above that (a 100M-filter index
 * holds no 53 GB host copy unless it is updated; an import follows the same
 * policy, its copy made from the image when it carries the tables). */
#define EMQX_GM_OPEN_MIRROR_EAGER 0x1u /* always keep it from the build            */
#define EMQX_GM_OPEN_MIRROR_LAZY  0x2u /* never at build: on the first update      */

/* CSR result: row i = ids[row_off[i] .. row_off[i+1]) */
typedef struct {
  uint64_t n_rows;
  uint64_t nnz;
  uint64_t *row_off;     /* n_rows + 1 entries                                 */
  uint32_t *ids;         /* nnz entries (filter ids or subscriber ids)          */
  int32_t on_device;     /* 1: device pointers, 0: host pointers                */
  int32_t reserved0;
  void *priv;            /* library bookkeeping; do not touch                   */
} emqx_gm_csr;

typedef struct {
  uint64_t n_filters;    /* unique filters; ids 0..n_filters-1                  */
  uint64_t n_wildcard;   /* filters the trie holds (emqx_topic:wildcard/1)      */
  uint64_t n_nodes;      /* level-trie nodes                                    */
  uint64_t n_edges;      /* exact/'+'/'#' edges                                 */
  uint64_t n_words;      /* distinct words                                      */
  uint64_t n_subs;       /* subscriber entries (fan-out CSR)                    */
  uint64_t device_bytes; /* resident index bytes in HBM                         */
  uint32_t max_depth;    /* deepest filter (levels)                             */
  int32_t trie_empty;    /* emqx_trie:empty/0 (no wildcard filter)              */
} emqx_gm_index_info_t;

typedef struct {
  uint64_t n_topics;
  uint64_t nnz;
  uint64_t n_overflow;       /* rows completed by the device slow path        */
  uint64_t n_wildcard_topics;
  double match_kernel_ms;    /* device time of the fast match kernel          */
  double total_device_ms;    /* device time of all kernels of the call         */
  uint64_t algo_bytes;       /* algorithmic bytes of the fast kernel */
  uint64_t probes;           /* NFA edge probes counted by the fast kernel     */
} emqx_gm_match_stats;

/* ---- context ---- */
int emqx_gm_open(const emqx_gm_opts *opts, emqx_gm_ctx **out);
int emqx_gm_close(emqx_gm_ctx *ctx);
/* Message of the calling thread's last failing call (valid until that
 * thread's next call into the library). */
const char *emqx_gm_last_error(const emqx_gm_ctx *ctx);
int emqx_gm_abi_version(void);
/* Use an external HIP stream (e.g. torch's current stream); NULL = own. */
int emqx_gm_set_stream(emqx_gm_ctx *ctx, void *hip_stream);
int emqx_gm_synchronize(emqx_gm_ctx *ctx);

/* ---- index (emqx_trie / emqx_route / emqx_subscriber snapshot) ---- */
/* filters in any order (duplicates allowed: one id, subscriber lists are
 * concatenated).  perm_out (optional, n_filters entries) receives the id of
 * each input filter.  sub_off/sub_ids (optional) give each input filter's
 * subscriber ids (CSR with n_filters+1 offsets). */
int emqx_gm_index_build(emqx_gm_ctx *ctx, const uint8_t *filter_bytes, const uint64_t *filter_off,
                        uint64_t n_filters, const uint64_t *sub_off, const uint32_t *sub_ids,
                        uint32_t *perm_out, emqx_gm_index **out);
/* Incremental maintenance (emqx_router:do_add_route/2 / do_delete_route/2 ->
 * emqx_trie:insert/1, delete/1, apps/emqx/src/emqx_router.erl:112-125,
 * 164-172, emqx_trie.erl:107-136).  Applies n_ops filter inserts (ops[i] = 1,
 * idempotent) and deletes (ops[i] = 0, only if present), in order, to `prev`
 * and returns a NEW snapshot; `prev` is unchanged (readers holding it keep
 * it: RCU).  The newest snapshot of a line is patched in place on a device
 * copy of its tables: the result is a flat snapshot, a match on it costs what
 * a match on a rebuilt index costs, and the update costs O(delta) host work +
 * one device pass over the index (read once, written once into the new
 * snapshot's tables; those of the last released snapshot of the same size are
 * reused when there are any -- emqx_gm_pool_trim frees them).  A plain index keeps a host copy of its device
 * tables for this (host RAM ~ emqx_gm_index_info().device_bytes), handed on
 * to each newer snapshot.  Otherwise -- a filter with '#' before its last
 * word, or an update of a snapshot that is no longer the newest -- the new
 * snapshot shares prev's tables (tombstones + a delta index; emqx_gm_fanout
 * refuses it).  Past 1/8 of the set, or when the tables run out of headroom,
 * the set is rebuilt.  Ids in rows of the new snapshot are ranks in the
 * updated set, as a full rebuild would give.  Not available for shard indexes
 * or indexes with subscriber lists (EMQX_GM_EUNSUPPORTED: rebuild those). */
int emqx_gm_index_update(emqx_gm_ctx *ctx, emqx_gm_index *prev, const uint8_t *filter_bytes,
                         const uint64_t *filter_off, const uint8_t *ops, uint64_t n_ops, emqx_gm_index **out);
/* Subscriber maintenance on an index built with subscriber lists
 * (emqx_broker:subscribe/2, unsubscribe/1 with the route added on a filter's
 * first subscriber and deleted after its last: apps/emqx/src/
 * emqx_broker.erl:147-165, 445-454, emqx_router.erl:112-125, 164-172).
 * Applies n_ops ops in order: ops[i] = EMQX_GM_SUB_SUBSCRIBE subscribes
 * sub_ids[i] to filter i (idempotent per pair), EMQX_GM_SUB_UNSUBSCRIBE
 * unsubscribes it (only if present).  A subscribe appends to the filter's
 * list, an unsubscribe keeps the others' order.  EMQX_GM_SUB_ROUTE_ADD /
 * ROUTE_DELETE (sub_ids[i] ignored) mark / unmark filter i as routed to
 * another destination (a remote node or a shared group: do_add_route/2 with
 * a dest other than the local node): a filter is in the index while it has a
 * local subscriber OR that mark, so its matches still come back (with an
 * empty subscriber segment) for the caller's lookup_routes/1.  In a built
 * index, a filter given no subscribers carries the mark.
 * Returns a NEW snapshot (RCU, as emqx_gm_index_update): route changes are
 * patched into a device copy of the newest snapshot's tables and the new
 * snapshot gets a subscriber CSR of its own; what the patch cannot take is
 * rebuilt.  EMQX_GM_EUNSUPPORTED for indexes without subscriber lists (use
 * emqx_gm_index_update), overlay snapshots and shard indexes. */
#define EMQX_GM_SUB_UNSUBSCRIBE 0u
#define EMQX_GM_SUB_SUBSCRIBE 1u
#define EMQX_GM_SUB_ROUTE_ADD 2u
#define EMQX_GM_SUB_ROUTE_DELETE 3u
int emqx_gm_index_update_subs(emqx_gm_ctx *ctx, emqx_gm_index *prev, const uint8_t *filter_bytes,
                              const uint64_t *filter_off, const uint32_t *sub_ids, const uint8_t *ops,
                              uint64_t n_ops, emqx_gm_index **out);
/* Index images: one snapshot compiled once and replicated (the reference's
 * routing tables are ONE copy that mria replicates to every node, not a
 * per-node recomputation: apps/emqx/src/emqx_router.erl:75-84, 136).
 * export: the snapshot as a self-contained host image -- the host tables
 * (layout, sorted filter table, shard ids, subscriber offsets, route marks)
 * and, unless EMQX_GM_IMAGE_NO_BLOB, the device tables; two-call sizing (buf
 * NULL sets *size).  device_blob: the device tables of a snapshot (read-only;
 * e.g. the source of an RCCL broadcast to the other GPUs).  import: a new
 * snapshot on ctx's device from an image, its device tables from the image or,
 * when d_blob is not NULL, copied from d_blob (device memory of ctx's device,
 * device_blob's bytes).  An imported plain index keeps its in-place update
 * line: its host mirror loads on the first update.  Overlay snapshots and
 * emqx_gm_index_update_subs results: EMQX_GM_EUNSUPPORTED (export a rebuilt
 * or emqx_gm_index_update'd snapshot).  An image is accepted only by a library
 * of the same table layout (EMQX_GM_EINVAL otherwise). */
#define EMQX_GM_IMAGE_NO_BLOB 0x1u
int emqx_gm_index_export(emqx_gm_ctx *ctx, const emqx_gm_index *idx, uint32_t flags, uint8_t *buf,
                         uint64_t *size);
int emqx_gm_index_device_blob(const emqx_gm_index *idx, const void **d_blob, uint64_t *bytes);
int emqx_gm_index_import(emqx_gm_ctx *ctx, const uint8_t *image, uint64_t size, const void *d_blob,
                         emqx_gm_index **out);
int emqx_gm_index_retain(emqx_gm_index *idx);
int emqx_gm_index_release(emqx_gm_index *idx);
int emqx_gm_index_info(const emqx_gm_index *idx, emqx_gm_index_info_t *info);
/* bytes of filter `id` (host memory owned by the index) */
int emqx_gm_index_filter(const emqx_gm_index *idx, uint32_t id, const uint8_t **bytes, uint64_t *len);
/* Number of subscribers of filter `id` (0 for an index built without
 * subscriber lists): the length of that filter's segment in a fan-out row,
 * which lets a caller split a row back into (filter, subscribers) groups --
 * do_dispatch/2 sends {deliver, Filter, Msg} per filter (emqx_broker.erl:
 * 506-525). */
int emqx_gm_index_subscriber_count(const emqx_gm_index *idx, uint32_t id, uint64_t *n);

/* ---- hot path ---- */
int emqx_gm_match(emqx_gm_ctx *ctx, const emqx_gm_index *idx, const uint8_t *topic_bytes,
                  const uint64_t *topic_off, uint64_t n_topics, uint32_t flags, emqx_gm_csr *out);
/* emqx_gm_match in two halves, for device buffers (EMQX_GM_DEVICE_IO
 * required): submit queues the call's kernels on the context stream and
 * returns at once; wait blocks until that call is done, hands out its rows
 * (exactly what emqx_gm_match returns) and frees the call.  Several calls may
 * be in flight on one context, from one thread or many (the reference matches
 * in every publisher's own process, lock-free: emqx_trie.erl:68-70,
 * emqx_router.erl:128-145): a batch's launches queue behind the previous
 * one's while the host still finishes that one, so the device does not idle
 * between small batches.  The inputs (and the index, which the call retains)
 * must stay valid until wait returns.  Overlay snapshots: EMQX_GM_EUNSUPPORTED
 * (use emqx_gm_match).  emqx_gm_match itself waits without the context lock
 * for device buffers. */
int emqx_gm_match_submit(emqx_gm_ctx *ctx, const emqx_gm_index *idx, const uint8_t *topic_bytes,
                         const uint64_t *topic_off, uint64_t n_topics, uint32_t flags, emqx_gm_call **call);
int emqx_gm_match_wait(emqx_gm_ctx *ctx, emqx_gm_call *call, emqx_gm_csr *out);
/* Pinned host buffers for the host-buffer emqx_gm_match: topic text (and
 * offsets) that a caller packs straight into memory from emqx_gm_host_alloc
 * crosses PCIe by DMA from where it lies, with no staging copy by the
 * library's workers (the NIF packs a publish batch's binaries here).  The
 * memory is page-locked and visible to every device of the context; free it
 * with emqx_gm_host_free on the same context. */
int emqx_gm_host_alloc(emqx_gm_ctx *ctx, uint64_t bytes, void **p);
int emqx_gm_host_free(emqx_gm_ctx *ctx, void *p);
/* The devices of a context, in emqx_gm_opts order (*n = 1 for a single-device
 * context); devices may be NULL to ask for the count. */
int emqx_gm_devices(const emqx_gm_ctx *ctx, int32_t *devices, uint32_t *n);
int emqx_gm_fanout(emqx_gm_ctx *ctx, const emqx_gm_index *idx, const emqx_gm_csr *matches,
                   uint32_t flags, emqx_gm_csr *out_subs);
/* emqx_broker:publish/1's route + dispatch of a batch in one call
 * (emqx_broker.erl:204-215, 245-322): the rows of emqx_gm_match(flags) into
 * *matches and their fan-out, as emqx_gm_fanout gives it, into *deliveries
 * (host buffers only; flags: EMQX_GM_WITH_EXACT or 0).  A publish window (a
 * batch of at most one chunk, 256K topics) makes ONE device round trip for
 * both: the fan-out is queued right behind the match's speculative rows and
 * kept when the rows and the deliveries fit their capacities (else the
 * fan-out runs after the match, as the two calls would).  On error nothing is
 * returned; both results are freed with emqx_gm_csr_free.  The NIF's
 * fanout_batch/2. */
int emqx_gm_match_fanout(emqx_gm_ctx *ctx, const emqx_gm_index *idx, const uint8_t *topic_bytes,
                         const uint64_t *topic_off, uint64_t n_topics, uint32_t flags, emqx_gm_csr *matches,
                         emqx_gm_csr *deliveries);
int emqx_gm_csr_free(emqx_gm_ctx *ctx, emqx_gm_csr *csr);
int emqx_gm_last_stats(const emqx_gm_ctx *ctx, emqx_gm_match_stats *stats);

/* ---- sharded index (BASELINE configs[4]) ----
 * For filter sets too large to replicate, filters are hash-partitioned over
 * devices (emqx_gm_shard_of), every device matches the whole publish batch
 * against its shard, rows are exchanged (RCCL all-to-all: device q receives
 * topic slice q from every shard) and merged by global filter id.  The
 * reference has no sharded trie (every node replicates emqx_route/emqx_trie
 * through mria, emqx_router.erl:75-84); the merged rows equal the unsharded
 * match_routes/1 rows. */
/* Global id of each filter: its lexicographic rank among the unique filters
 * (the id an unsharded emqx_gm_index_build would assign). */
int emqx_gm_filter_ranks(const uint8_t *filter_bytes, const uint64_t *filter_off, uint64_t n_filters,
                         uint32_t *rank_out, uint64_t *n_unique);
/* Shard of each filter: fmix64(word hash of the filter bytes) mod n_shards. */
int emqx_gm_shard_of(const uint8_t *filter_bytes, const uint64_t *filter_off, uint64_t n_filters,
                     uint32_t n_shards, uint32_t *shard_out);
/* Index over one shard whose result rows carry the given global ids (which
 * must ascend with the filter bytes).  emqx_gm_fanout is not available on a
 * shard index (subscribers live with their shard: fan out before merging). */
int emqx_gm_index_build_shard(emqx_gm_ctx *ctx, const uint8_t *filter_bytes, const uint64_t *filter_off,
                              uint64_t n_filters, const uint32_t *global_ids, const uint64_t *sub_off,
                              const uint32_t *sub_ids, uint32_t *perm_out, emqx_gm_index **out);
/* Row lengths of a device CSR into device memory (u32 per row). */
int emqx_gm_csr_row_lengths(emqx_gm_ctx *ctx, const emqx_gm_csr *csr, uint32_t *d_lens);
/* Merge n_pieces per-shard results for the same n_rows rows.  d_lens: device
 * u32 [n_pieces][stride] (stride >= n_rows, padding rows 0); d_ids: device
 * u32, the pieces' rows concatenated piece-major.  Rows are disjoint sorted
 * id lists; the result rows are their sorted unions (flags: DEVICE_IO keeps
 * the CSR on the device). */
int emqx_gm_merge_rows(emqx_gm_ctx *ctx, uint64_t n_rows, uint64_t stride, uint32_t n_pieces,
                       const uint32_t *d_lens, const uint32_t *d_ids, uint32_t flags, emqx_gm_csr *out);

/* ---- prefix sharding (gm_route.hip): each topic needs ONE shard ----
 * A topic can only match filters whose first word is its own first word, '+'
 * or '#' (emqx_topic:match/2, emqx_topic.erl:65-87).  emqx_gm_prefix_plan
 * partitions filters by first word (a hot first word -- over 1/(2N) of the
 * filters -- by its first two words) over n_shards, greedily by size; filters
 * whose first word is '+' / '#' (and a hot word's 'w', 'w/#', 'w/+/...') go to
 * every shard (shard_out = EMQX_GM_ALL_SHARDS).  The returned route maps each
 * topic to the one shard that holds every filter it can match, so a batch is
 * routed (all-to-all of topic bytes), each rank walks only its share, and the
 * rows go back to the topics' ranks (emqx_gm_unpermute_rows) -- no merge. */
#define EMQX_GM_ALL_SHARDS 0xFFFFFFFFu
typedef struct emqx_gm_route emqx_gm_route;
int emqx_gm_prefix_plan(const uint8_t *filter_bytes, const uint64_t *filter_off, uint64_t n_filters,
                        uint32_t n_shards, uint32_t *shard_out, emqx_gm_route **route);
/* The prefix-sharded index behind ONE multi-device context (the NIF's form of
 * this plan, for a filter set that does not fit one GPU): the filters are
 * partitioned as emqx_gm_prefix_plan does over the context's devices (one
 * shard per listed device; '+' / '#'-first filters on every one), each shard
 * compiled and placed on its device at once.  The returned index is used like
 * any other: emqx_gm_match on host buffers routes each topic to its one shard,
 * matches every device's topics there at the same time and returns the rows in
 * batch order (global ids, bit-exact with an unsharded index); emqx_gm_fanout
 * on host rows fans each row out on its shard; emqx_gm_index_info / _filter /
 * _subscriber_count answer for the whole set.  Device-buffer calls, updates and
 * images of a sharded index: EMQX_GM_EUNSUPPORTED (a global id shifts on every
 * shard when one filter is added: rebuild it).  Arguments as emqx_gm_index_build. */
int emqx_gm_index_build_sharded(emqx_gm_ctx *ctx, const uint8_t *filter_bytes, const uint64_t *filter_off,
                                uint64_t n_filters, const uint64_t *sub_off, const uint32_t *sub_ids,
                                uint32_t *perm_out, emqx_gm_index **out);
/* dest[i] = the shard of topic i (host buffers / device buffers, n_topics entries) */
int emqx_gm_route_topics_host(const emqx_gm_route *route, const uint8_t *topic_bytes, const uint64_t *topic_off,
                              uint64_t n_topics, uint32_t *dest);
int emqx_gm_route_topics(emqx_gm_ctx *ctx, emqx_gm_route *route, const uint8_t *d_topic_bytes,
                         const uint64_t *d_topic_off, uint64_t n_topics, uint32_t *d_dest);
int emqx_gm_route_release(emqx_gm_route *route);
/* The send order of a routed device batch in one call (the step's route, sort
 * and split sizes): d_perm[i] = the batch index of the i-th topic in order of
 * (shard, batch index), d_plen[i] = its length in bytes, d_split[2 s] / [2 s + 1]
 * = the topics / bytes bound for shard s (n_shards <= 256).  Device buffers:
 * n_topics u32 each, 2 * n_shards u64.  Stream-ordered like the other calls. */
int emqx_gm_route_partition(emqx_gm_ctx *ctx, emqx_gm_route *route, const uint8_t *d_topic_bytes,
                            const uint64_t *d_topic_off, uint64_t n_topics, uint32_t *d_perm, uint32_t *d_plen,
                            uint64_t *d_split);
/* (route_topics / route_partition / permute_topics / unpermute_rows index the
 * batch with u32: n_topics / n_rows < 2^32 - 1, else EMQX_GM_EINVAL) */
/* The exchange's device steps.  permute: out topic i = topic perm[i] (d_out
 * holds as many bytes as the input, d_out_off n+1 entries).  unpermute: row
 * perm[i] of the result = input row i, the input rows packed with u32 lengths
 * d_lens[i] (flags: EMQX_GM_DEVICE_IO keeps the CSR on the device). */
int emqx_gm_permute_topics(emqx_gm_ctx *ctx, const uint8_t *d_topic_bytes, const uint64_t *d_topic_off,
                           uint64_t n_topics, const uint32_t *d_perm, uint8_t *d_out, uint64_t *d_out_off);
int emqx_gm_unpermute_rows(emqx_gm_ctx *ctx, uint64_t n_rows, const uint32_t *d_perm, const uint32_t *d_lens,
                           const uint32_t *d_ids, uint32_t flags, emqx_gm_csr *out);

#ifdef __cplusplus
}
#endif
#endif /* EMQX_GPU_MATCH_H */
