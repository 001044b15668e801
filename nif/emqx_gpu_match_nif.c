/*
 * emqx_gpu_match_nif.c — thin Erlang NIF over libemqx_gpu_match.so.
 *
 * Erlang module `emqx_gpu_match` (nif/emqx_gpu_match.erl).  All calls run on
 * dirty CPU schedulers (a batch takes > 1 ms).  Non-binary input -> badarg;
 * device faults -> {error, Reason} so the Erlang wrapper can fall back to
 * emqx_trie:match/1.  An index is an enif resource whose
 * destructor releases the device snapshot (emqx_gm_index_release).
 *
 * Build (only where erl_nif.h exists; this container has no Erlang):
 *   cc -O2 -fPIC -shared -I$ERL_ROOT/usr/include -I../include \
 *      emqx_gpu_match_nif.c -L../emqx_amd -lemqx_gpu_match -o emqx_gpu_match_nif.so
 */
#include <erl_nif.h>
#include <stdlib.h>
#include <string.h>

#include "emqx_gpu_match.h"

/* An index snapshot.  Result rows are binaries that point straight into the
 * snapshot's host copy of the filter bytes (emqx_gm_index_filter) and keep
 * this resource -- hence the snapshot -- alive: no per-snapshot copy of the
 * filter set is made, so an incremental update_index costs O(delta), not
 * O(filters). */
typedef struct {
  emqx_gm_index *idx;
} gm_index_res;

static ErlNifResourceType *INDEX_RT;
static emqx_gm_ctx *CTX;
static ERL_NIF_TERM A_OK, A_ERROR, A_BADARG, A_INSERT, A_DELETE, A_SUBSCRIBE, A_UNSUBSCRIBE, A_ROUTE_ADD,
    A_ROUTE_DELETE;

static void index_dtor(ErlNifEnv *env, void *obj) {
  gm_index_res *r = (gm_index_res *)obj;
  (void)env;
  if (r->idx) emqx_gm_index_release(r->idx);
}

/* LoadInfo (erlang:load_nif/2): a device ordinal, or the node's device list
 * [D0, D1, ...] (1..EMQX_GM_MAX_DEVICES entries; repeats give several replicas
 * on one GPU).  With a list, the ONE context of this node replicates every
 * index to all listed GPUs and each match_*_batch / fanout_batch spreads its
 * batch over them (emqx_gm_opts.n_devices), as the reference's match_routes/1
 * runs on all schedulers at once (emqx_trie.erl:66-70, emqx_router.erl:128-145). */
static int load(ErlNifEnv *env, void **priv, ERL_NIF_TERM info) {
  int device = 0;
  unsigned nl = 0;
  emqx_gm_opts o;
  (void)priv;
  memset(&o, 0, sizeof(o));
  if (enif_get_list_length(env, info, &nl) && nl > 0) {
    ERL_NIF_TERM h, t = info;
    if (nl > EMQX_GM_MAX_DEVICES) return 1;
    while (enif_get_list_cell(env, t, &h, &t)) {
      if (!enif_get_int(env, h, &device)) return 1;
      o.devices[o.n_devices++] = device;
    }
  } else {
    enif_get_int(env, info, &device);
    o.device = device;
  }
  INDEX_RT = enif_open_resource_type(env, NULL, "emqx_gm_index", index_dtor, ERL_NIF_RT_CREATE, NULL);
  A_OK = enif_make_atom(env, "ok");
  A_ERROR = enif_make_atom(env, "error");
  A_BADARG = enif_make_atom(env, "badarg");
  A_INSERT = enif_make_atom(env, "insert");
  A_DELETE = enif_make_atom(env, "delete");
  A_SUBSCRIBE = enif_make_atom(env, "subscribe");
  A_UNSUBSCRIBE = enif_make_atom(env, "unsubscribe");
  A_ROUTE_ADD = enif_make_atom(env, "route_add");
  A_ROUTE_DELETE = enif_make_atom(env, "route_delete");
  return emqx_gm_open(&o, &CTX) == EMQX_GM_OK && INDEX_RT ? 0 : 1;
}

static void unload(ErlNifEnv *env, void *priv) {
  (void)env;
  (void)priv;
  if (CTX) emqx_gm_close(CTX);
}

/* The failing call's own message: emqx_gm_last_error() is per calling thread,
 * and this NIF call runs start to end on one dirty scheduler thread. */
static ERL_NIF_TERM error_tuple(ErlNifEnv *env, int rc) {
  const char *m = emqx_gm_last_error(CTX);
  (void)rc;
  return enif_make_tuple2(env, A_ERROR, enif_make_string(env, m && *m ? m : "device", ERL_NIF_LATIN1));
}

/* Pack a list of binaries into (bytes, offsets). */
static int pack_list(ErlNifEnv *env, ERL_NIF_TERM list, uint8_t **bytes, uint64_t **off, uint64_t *n) {
  unsigned len;
  ERL_NIF_TERM h, t = list;
  ErlNifBinary b;
  uint64_t total = 0, i = 0;
  if (!enif_get_list_length(env, list, &len)) return 0;
  while (enif_get_list_cell(env, t, &h, &t)) {
    if (!enif_inspect_binary(env, h, &b)) return 0;
    total += b.size;
  }
  *bytes = enif_alloc(total + 64);
  *off = enif_alloc((len + 1) * sizeof(uint64_t));
  (*off)[0] = 0;
  t = list;
  while (enif_get_list_cell(env, t, &h, &t)) {
    enif_inspect_binary(env, h, &b);
    memcpy(*bytes + (*off)[i], b.data, b.size);
    (*off)[i + 1] = (*off)[i] + b.size;
    ++i;
  }
  memset(*bytes + total, 0, 64);
  *n = len;
  return 1;
}

/* A publish batch packed straight into page-locked memory (emqx_gm_host_alloc):
 * the library then sends the text to the GPUs by DMA from here, with no
 * staging copy of its own.  One buffer per dirty scheduler thread, grown as
 * batches grow; the offsets stay in ordinary memory (the library validates and
 * rebases them anyway). */
static __thread uint8_t *PIN_BUF;
static __thread uint64_t PIN_CAP;

static int pack_topics(ErlNifEnv *env, ERL_NIF_TERM list, uint8_t **bytes, uint64_t **off, uint64_t *n) {
  unsigned len;
  ERL_NIF_TERM h, t = list;
  ErlNifBinary b;
  uint64_t total = 0, i = 0;
  if (!enif_get_list_length(env, list, &len)) return 0;
  while (enif_get_list_cell(env, t, &h, &t)) {
    if (!enif_inspect_binary(env, h, &b)) return 0;
    total += b.size;
  }
  if (PIN_CAP < total + 64) {
    void *p = NULL;
    uint64_t cap = PIN_CAP ? PIN_CAP : (1u << 20);
    while (cap < total + 64) cap *= 2;
    if (PIN_BUF) emqx_gm_host_free(CTX, PIN_BUF);
    PIN_BUF = NULL;
    PIN_CAP = 0;
    if (emqx_gm_host_alloc(CTX, cap, &p) == EMQX_GM_OK) {
      PIN_BUF = p;
      PIN_CAP = cap;
    }
  }
  if (!PIN_BUF) return pack_list(env, list, bytes, off, n);  /* (no page-locked memory: the plain way) */
  *bytes = PIN_BUF;
  *off = enif_alloc((len + 1) * sizeof(uint64_t));
  (*off)[0] = 0;
  t = list;
  while (enif_get_list_cell(env, t, &h, &t)) {
    enif_inspect_binary(env, h, &b);
    memcpy(*bytes + (*off)[i], b.data, b.size);
    (*off)[i + 1] = (*off)[i] + b.size;
    ++i;
  }
  memset(*bytes + total, 0, 64);
  *n = len;
  return 1;
}
static void free_topics(uint8_t *bytes, uint64_t *off) {
  if (bytes != PIN_BUF) enif_free(bytes);
  enif_free(off);
}

static ERL_NIF_TERM make_index_term(ErlNifEnv *env, emqx_gm_index *idx) {
  gm_index_res *r = enif_alloc_resource(INDEX_RT, sizeof(*r));
  ERL_NIF_TERM term;
  r->idx = idx;
  term = enif_make_resource(env, r);
  enif_release_resource(r);
  return enif_make_tuple2(env, A_OK, term);
}

/* Subscriber lists [[SubId :: non_neg_integer()]] -> CSR (n+1 offsets); one
 * list per filter. */
static int pack_subs(ErlNifEnv *env, ERL_NIF_TERM lists, uint64_t n, uint64_t **off, uint32_t **ids) {
  unsigned len, k;
  ERL_NIF_TERM h, t = lists, e, u;
  uint64_t total = 0, i = 0;
  if (!enif_get_list_length(env, lists, &len) || len != n) return 0;
  while (enif_get_list_cell(env, t, &h, &t)) {
    if (!enif_get_list_length(env, h, &k)) return 0;
    total += k;
  }
  *off = enif_alloc((n + 1) * sizeof(uint64_t));
  *ids = enif_alloc((total ? total : 1) * sizeof(uint32_t));
  (*off)[0] = 0;
  t = lists;
  while (enif_get_list_cell(env, t, &h, &t)) {
    uint64_t o = (*off)[i];
    u = h;
    while (enif_get_list_cell(env, u, &e, &u)) {
      unsigned v;
      if (!enif_get_uint(env, e, &v)) {
        enif_free(*off);
        enif_free(*ids);
        return 0;
      }
      (*ids)[o++] = v;
    }
    (*off)[++i] = o;
  }
  return 1;
}

/* load_index([Filter :: binary()]) -> {ok, Index} | {error, Reason}
 * load_index([Filter :: binary()], [[SubId :: non_neg_integer()]]) -> idem,
 *   with each filter's subscriber ids (the emqx_subscriber bag of
 *   emqx_broker.erl:147-165 with its {shard, I} buckets flattened), which
 *   fanout_batch/2 returns per topic. */
static ERL_NIF_TERM do_load(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[], int sharded) {
  uint8_t *fb;
  uint64_t *fo, n, *so = NULL;
  uint32_t *si = NULL;
  emqx_gm_index *idx = NULL;
  int rc;
  if (!pack_list(env, argv[0], &fb, &fo, &n)) return enif_make_badarg(env);
  if (argc == 2 && !pack_subs(env, argv[1], n, &so, &si)) {
    enif_free(fb);
    enif_free(fo);
    return enif_make_badarg(env);
  }
  rc = sharded ? emqx_gm_index_build_sharded(CTX, fb, fo, n, so, si, NULL, &idx)
               : emqx_gm_index_build(CTX, fb, fo, n, so, si, NULL, &idx);
  enif_free(fb);
  enif_free(fo);
  if (so) enif_free(so);
  if (si) enif_free(si);
  if (rc != EMQX_GM_OK) return error_tuple(env, rc);
  return make_index_term(env, idx);
}

static ERL_NIF_TERM load_index(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
  return do_load(env, argc, argv, 0);
}

/* load_index_sharded/1,2: as load_index/1,2, for a route table too large for
 * one GPU: the filters partitioned by first word over the context's devices
 * (emqx_gm_index_build_sharded), each topic matched on its one device.
 * match_batch/2, match_routes_batch/2 and fanout_batch/2 take the result like
 * any index; update_index/2, update_subs/2 and export_index/1 return
 * {error, Reason} for it (EMQX_GM_EUNSUPPORTED: rebuild it). */
static ERL_NIF_TERM load_index_sharded(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
  return do_load(env, argc, argv, 1);
}

/* update_index(Index, [{Filter :: binary(), insert | delete}]) -> {ok, NewIndex} | {error, Reason}
 * emqx_gm_index_update: a new snapshot; Index stays valid for its readers. */
static ERL_NIF_TERM update_index(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
  gm_index_res *r;
  unsigned len, i = 0;
  ERL_NIF_TERM h, t = argv[1], fl = enif_make_list(env, 0);
  uint8_t *fb, *ops;
  uint64_t *fo, n;
  emqx_gm_index *idx = NULL;
  int rc;
  (void)argc;
  if (!enif_get_resource(env, argv[0], INDEX_RT, (void **)&r) || !enif_get_list_length(env, argv[1], &len))
    return enif_make_badarg(env);
  ops = enif_alloc(len + 1);
  while (enif_get_list_cell(env, t, &h, &t)) {
    const ERL_NIF_TERM *tup;
    int arity;
    if (!enif_get_tuple(env, h, &arity, &tup) || arity != 2) {
      enif_free(ops);
      return enif_make_badarg(env);
    }
    if (!enif_is_identical(tup[1], A_INSERT) && !enif_is_identical(tup[1], A_DELETE)) {
      enif_free(ops);
      return enif_make_badarg(env);  /* only insert | delete */
    }
    fl = enif_make_list_cell(env, tup[0], fl);
    ops[i++] = enif_is_identical(tup[1], A_INSERT) ? 1 : 0;
  }
  /* fl was built by prepending: reverse it back to the ops' order */
  if (!enif_make_reverse_list(env, fl, &fl) || !pack_list(env, fl, &fb, &fo, &n)) {
    enif_free(ops);
    return enif_make_badarg(env);
  }
  rc = emqx_gm_index_update(CTX, r->idx, fb, fo, ops, n, &idx);
  enif_free(fb);
  enif_free(fo);
  enif_free(ops);
  if (rc != EMQX_GM_OK) return error_tuple(env, rc);
  return make_index_term(env, idx);
}

/* update_subs(Index, [{Filter :: binary(), SubId :: non_neg_integer(),
 *                       subscribe | unsubscribe | route_add | route_delete}])
 *   -> {ok, NewIndex} | {error, Reason}
 * emqx_gm_index_update_subs on an index from load_index/2: emqx_broker's
 * subscribe/unsubscribe, with the route added on a filter's first subscriber
 * and deleted after its last; route_add / route_delete (SubId ignored) mark a
 * filter routed to another destination (a remote node, a shared group), which
 * keeps it in the index without a local subscriber. */
static ERL_NIF_TERM update_subs(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
  gm_index_res *r;
  unsigned len, i = 0;
  ERL_NIF_TERM h, t = argv[1], fl = enif_make_list(env, 0);
  uint8_t *fb, *ops;
  uint32_t *subs;
  uint64_t *fo, n;
  emqx_gm_index *idx = NULL;
  int rc;
  (void)argc;
  if (!enif_get_resource(env, argv[0], INDEX_RT, (void **)&r) || !enif_get_list_length(env, argv[1], &len))
    return enif_make_badarg(env);
  ops = enif_alloc(len + 1);
  subs = enif_alloc((len + 1) * sizeof(uint32_t));
  while (enif_get_list_cell(env, t, &h, &t)) {
    const ERL_NIF_TERM *tup;
    int arity;
    unsigned s;
    uint8_t kind;
    if (!enif_get_tuple(env, h, &arity, &tup) || arity != 3 || !enif_get_uint(env, tup[1], &s)) goto bad;
    if (enif_is_identical(tup[2], A_SUBSCRIBE)) kind = EMQX_GM_SUB_SUBSCRIBE;
    else if (enif_is_identical(tup[2], A_UNSUBSCRIBE)) kind = EMQX_GM_SUB_UNSUBSCRIBE;
    else if (enif_is_identical(tup[2], A_ROUTE_ADD)) kind = EMQX_GM_SUB_ROUTE_ADD;
    else if (enif_is_identical(tup[2], A_ROUTE_DELETE)) kind = EMQX_GM_SUB_ROUTE_DELETE;
    else goto bad;
    fl = enif_make_list_cell(env, tup[0], fl);
    subs[i] = s;
    ops[i++] = kind;
    continue;
  bad:
    enif_free(ops);
    enif_free(subs);
    return enif_make_badarg(env);
  }
  if (!enif_make_reverse_list(env, fl, &fl) || !pack_list(env, fl, &fb, &fo, &n)) {
    enif_free(ops);
    enif_free(subs);
    return enif_make_badarg(env);
  }
  rc = emqx_gm_index_update_subs(CTX, r->idx, fb, fo, subs, ops, n, &idx);
  enif_free(fb);
  enif_free(fo);
  enif_free(ops);
  enif_free(subs);
  if (rc != EMQX_GM_OK) return error_tuple(env, rc);
  return make_index_term(env, idx);
}

static ERL_NIF_TERM do_match(ErlNifEnv *env, const ERL_NIF_TERM argv[], uint32_t flags) {
  gm_index_res *r;
  uint8_t *tb;
  uint64_t *to, n, i, k;
  emqx_gm_csr out;
  ERL_NIF_TERM bin, result, *rows;
  int rc;
  if (!enif_get_resource(env, argv[0], INDEX_RT, (void **)&r)) return enif_make_badarg(env);
  if (!pack_topics(env, argv[1], &tb, &to, &n)) return enif_make_badarg(env);
  rc = emqx_gm_match(CTX, r->idx, tb, to, n, flags, &out);
  free_topics(tb, to);
  if (rc != EMQX_GM_OK) return error_tuple(env, rc);
  /* each filter is a binary over the snapshot's own host bytes, kept alive by the resource */
  rows = enif_alloc(sizeof(ERL_NIF_TERM) * (n ? n : 1));
  for (i = 0; i < n; ++i) {
    ERL_NIF_TERM row = enif_make_list(env, 0);
    for (k = out.row_off[i + 1]; k > out.row_off[i]; --k) {
      const uint8_t *p;
      uint64_t l;
      emqx_gm_index_filter(r->idx, out.ids[k - 1], &p, &l);
      bin = enif_make_resource_binary(env, r, p, l);
      row = enif_make_list_cell(env, bin, row);
    }
    rows[i] = row;
  }
  result = enif_make_list_from_array(env, rows, (unsigned)n);
  enif_free(rows);
  emqx_gm_csr_free(CTX, &out);
  return result;
}

/* match_batch(Index, [Topic]) -> [[Filter]]   (emqx_trie:match/1 per topic) */
static ERL_NIF_TERM match_batch(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  return do_match(env, argv, 0);
}

/* match_routes_batch(Index, [Topic]) -> [[Filter]]  (emqx_router:match_routes/1 filters) */
static ERL_NIF_TERM match_routes_batch(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  return do_match(env, argv, EMQX_GM_WITH_EXACT);
}

/* fanout_batch(Index, [Topic]) -> [[{Filter, [SubId]}]]
 * emqx_broker:publish/1's route + dispatch for each topic: its matched filters
 * (match_routes/1) in ascending order, each with the subscribers do_dispatch/2
 * folds over (emqx_broker.erl:296-322, 506-530) -- the order of the GPU
 * fan-out row, cut back into one segment per filter so the caller can send
 * {deliver, Filter, Msg}.  The index must come from load_index/2. */
static ERL_NIF_TERM fanout_batch(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
  gm_index_res *r;
  uint8_t *tb;
  uint64_t *to, n, i, k, d_pos;
  emqx_gm_csr m, d;
  ERL_NIF_TERM result, *rows;
  int rc;
  (void)argc;
  if (!enif_get_resource(env, argv[0], INDEX_RT, (void **)&r)) return enif_make_badarg(env);
  if (!pack_topics(env, argv[1], &tb, &to, &n)) return enif_make_badarg(env);
  /* the match and its fan-out in one call: one device round trip per window */
  rc = emqx_gm_match_fanout(CTX, r->idx, tb, to, n, EMQX_GM_WITH_EXACT, &m, &d);
  free_topics(tb, to);
  if (rc != EMQX_GM_OK) return error_tuple(env, rc);
  rows = enif_alloc(sizeof(ERL_NIF_TERM) * (n ? n : 1));
  for (i = 0; i < n; ++i) {
    ERL_NIF_TERM row = enif_make_list(env, 0);
    d_pos = d.row_off[i + 1];
    for (k = m.row_off[i + 1]; k > m.row_off[i]; --k) {  /* filters back to front */
      const uint8_t *p;
      uint64_t l, c, j;
      ERL_NIF_TERM subs = enif_make_list(env, 0);
      const uint32_t f = m.ids[k - 1];
      if (emqx_gm_index_filter(r->idx, f, &p, &l) != EMQX_GM_OK ||
          emqx_gm_index_subscriber_count(r->idx, f, &c) != EMQX_GM_OK || c > d_pos - d.row_off[i]) {
        enif_free(rows);
        emqx_gm_csr_free(CTX, &m);
        emqx_gm_csr_free(CTX, &d);
        return error_tuple(env, EMQX_GM_EINVAL);
      }
      for (j = 0; j < c; ++j) subs = enif_make_list_cell(env, enif_make_uint(env, d.ids[d_pos - 1 - j]), subs);
      d_pos -= c;
      row = enif_make_list_cell(env, enif_make_tuple2(env, enif_make_resource_binary(env, r, p, l), subs), row);
    }
    rows[i] = row;
  }
  result = enif_make_list_from_array(env, rows, (unsigned)n);
  enif_free(rows);
  emqx_gm_csr_free(CTX, &m);
  emqx_gm_csr_free(CTX, &d);
  return result;
}

/* empty(Index) -> boolean()  (emqx_trie:empty/0) */
static ERL_NIF_TERM empty(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
  gm_index_res *r;
  emqx_gm_index_info_t info;
  (void)argc;
  if (!enif_get_resource(env, argv[0], INDEX_RT, (void **)&r)) return enif_make_badarg(env);
  emqx_gm_index_info(r->idx, &info);
  return enif_make_atom(env, info.trie_empty ? "true" : "false");
}

/* export_index(Index) -> {ok, Image :: binary()} | {error, Reason}
 * emqx_gm_index_export with the device tables: the snapshot as one binary a
 * joining node imports instead of recompiling the route table (the reference
 * replicates its routing tables through mria, emqx_router.erl:75-84). */
static ERL_NIF_TERM export_index(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
  gm_index_res *r;
  ErlNifBinary bin;
  uint64_t size = 0;
  int rc;
  (void)argc;
  if (!enif_get_resource(env, argv[0], INDEX_RT, (void **)&r)) return enif_make_badarg(env);
  rc = emqx_gm_index_export(CTX, r->idx, 0, NULL, &size);
  if (rc != EMQX_GM_OK) return error_tuple(env, rc);
  if (!enif_alloc_binary((size_t)size, &bin))
    return enif_make_tuple2(env, A_ERROR, enif_make_string(env, "enomem", ERL_NIF_LATIN1));
  rc = emqx_gm_index_export(CTX, r->idx, 0, bin.data, &size);
  if (rc != EMQX_GM_OK) {
    enif_release_binary(&bin);
    return error_tuple(env, rc);
  }
  return enif_make_tuple2(env, A_OK, enif_make_binary(env, &bin));
}

/* import_index(Image :: binary()) -> {ok, Index} | {error, Reason}
 * emqx_gm_index_import on this node's device (an image of another layout or
 * a truncated one: {error, _}). */
static ERL_NIF_TERM import_index(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
  ErlNifBinary bin;
  emqx_gm_index *idx = NULL;
  int rc;
  (void)argc;
  if (!enif_inspect_binary(env, argv[0], &bin)) return enif_make_badarg(env);
  rc = emqx_gm_index_import(CTX, bin.data, bin.size, NULL, &idx);
  if (rc != EMQX_GM_OK) return error_tuple(env, rc);
  return make_index_term(env, idx);
}

static ErlNifFunc funcs[] = {
    {"load_index", 1, load_index, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"load_index", 2, load_index, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"load_index_sharded", 1, load_index_sharded, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"load_index_sharded", 2, load_index_sharded, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"update_index", 2, update_index, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"update_subs", 2, update_subs, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"match_batch", 2, match_batch, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"match_routes_batch", 2, match_routes_batch, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"fanout_batch", 2, fanout_batch, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"empty", 1, empty, 0},
    {"export_index", 1, export_index, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"import_index", 1, import_index, ERL_NIF_DIRTY_JOB_CPU_BOUND},
};

ERL_NIF_INIT(emqx_gpu_match, funcs, load, NULL, NULL, unload)
