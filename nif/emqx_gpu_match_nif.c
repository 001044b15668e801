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

typedef struct {
  emqx_gm_index *idx;
  ErlNifBinary filters; /* concatenated sorted filters (sub-binaries are returned) */
  uint64_t *foff;
  uint64_t n;
} gm_index_res;

static ErlNifResourceType *INDEX_RT;
static emqx_gm_ctx *CTX;
static ERL_NIF_TERM A_OK, A_ERROR, A_BADARG, A_INSERT;

static void index_dtor(ErlNifEnv *env, void *obj) {
  gm_index_res *r = (gm_index_res *)obj;
  (void)env;
  if (r->idx) emqx_gm_index_release(r->idx);
  if (r->foff) enif_free(r->foff);
  enif_release_binary(&r->filters);
}

static int load(ErlNifEnv *env, void **priv, ERL_NIF_TERM info) {
  int device = 0;
  emqx_gm_opts o;
  (void)priv;
  enif_get_int(env, info, &device);
  memset(&o, 0, sizeof(o));
  o.device = device;
  INDEX_RT = enif_open_resource_type(env, NULL, "emqx_gm_index", index_dtor, ERL_NIF_RT_CREATE, NULL);
  A_OK = enif_make_atom(env, "ok");
  A_ERROR = enif_make_atom(env, "error");
  A_BADARG = enif_make_atom(env, "badarg");
  A_INSERT = enif_make_atom(env, "insert");
  return emqx_gm_open(&o, &CTX) == EMQX_GM_OK && INDEX_RT ? 0 : 1;
}

static void unload(ErlNifEnv *env, void *priv) {
  (void)env;
  (void)priv;
  if (CTX) emqx_gm_close(CTX);
}

static ERL_NIF_TERM error_tuple(ErlNifEnv *env, int rc) {
  const char *m = emqx_gm_last_error(CTX);
  (void)rc;
  return enif_make_tuple2(env, A_ERROR, enif_make_string(env, m ? m : "device", ERL_NIF_LATIN1));
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

/* Wrap an index snapshot in a resource that also owns the sorted filter
 * bytes (result rows are sub-binaries of them). */
static ERL_NIF_TERM make_index_term(ErlNifEnv *env, emqx_gm_index *idx) {
  emqx_gm_index_info_t info;
  gm_index_res *r;
  ERL_NIF_TERM term;
  uint64_t i;
  emqx_gm_index_info(idx, &info);
  r = enif_alloc_resource(INDEX_RT, sizeof(*r));
  memset(r, 0, sizeof(*r));
  r->idx = idx;
  r->n = info.n_filters;
  r->foff = enif_alloc((r->n + 1) * sizeof(uint64_t));
  r->foff[0] = 0;
  for (i = 0; i < r->n; ++i) {
    const uint8_t *p;
    uint64_t l;
    emqx_gm_index_filter(idx, (uint32_t)i, &p, &l);
    r->foff[i + 1] = r->foff[i] + l;
  }
  enif_alloc_binary(r->foff[r->n], &r->filters);
  for (i = 0; i < r->n; ++i) {
    const uint8_t *p;
    uint64_t l;
    emqx_gm_index_filter(idx, (uint32_t)i, &p, &l);
    memcpy(r->filters.data + r->foff[i], p, l);
  }
  term = enif_make_resource(env, r);
  enif_release_resource(r);
  return enif_make_tuple2(env, A_OK, term);
}

/* load_index([Filter :: binary()]) -> {ok, Index} | {error, Reason} */
static ERL_NIF_TERM load_index(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
  uint8_t *fb;
  uint64_t *fo, n;
  emqx_gm_index *idx = NULL;
  int rc;
  (void)argc;
  if (!pack_list(env, argv[0], &fb, &fo, &n)) return enif_make_badarg(env);
  rc = emqx_gm_index_build(CTX, fb, fo, n, NULL, NULL, NULL, &idx);
  enif_free(fb);
  enif_free(fo);
  if (rc != EMQX_GM_OK) return error_tuple(env, rc);
  return make_index_term(env, idx);
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

static ERL_NIF_TERM do_match(ErlNifEnv *env, const ERL_NIF_TERM argv[], uint32_t flags) {
  gm_index_res *r;
  uint8_t *tb;
  uint64_t *to, n, i, k;
  emqx_gm_csr out;
  ERL_NIF_TERM bin, result, *rows;
  int rc;
  if (!enif_get_resource(env, argv[0], INDEX_RT, (void **)&r)) return enif_make_badarg(env);
  if (!pack_list(env, argv[1], &tb, &to, &n)) return enif_make_badarg(env);
  rc = emqx_gm_match(CTX, r->idx, tb, to, n, flags, &out);
  enif_free(tb);
  enif_free(to);
  if (rc != EMQX_GM_OK) return error_tuple(env, rc);
  /* one binary term backed by the resource; rows are sub-binaries of it */
  bin = enif_make_resource_binary(env, r, r->filters.data, r->filters.size);
  rows = enif_alloc(sizeof(ERL_NIF_TERM) * (n ? n : 1));
  for (i = 0; i < n; ++i) {
    ERL_NIF_TERM row = enif_make_list(env, 0);
    for (k = out.row_off[i + 1]; k > out.row_off[i]; --k) {
      uint32_t f = out.ids[k - 1];
      row = enif_make_list_cell(env, enif_make_sub_binary(env, bin, r->foff[f], r->foff[f + 1] - r->foff[f]), row);
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

/* fanout_batch(Index, [Topic]) -> [[SubscriberId]]  (emqx_broker:dispatch/2 multiset) */
static ERL_NIF_TERM fanout_batch(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
  gm_index_res *r;
  uint8_t *tb;
  uint64_t *to, n, i, k;
  emqx_gm_csr m, d;
  ERL_NIF_TERM result, *rows;
  int rc;
  (void)argc;
  if (!enif_get_resource(env, argv[0], INDEX_RT, (void **)&r)) return enif_make_badarg(env);
  if (!pack_list(env, argv[1], &tb, &to, &n)) return enif_make_badarg(env);
  rc = emqx_gm_match(CTX, r->idx, tb, to, n, EMQX_GM_WITH_EXACT, &m);
  enif_free(tb);
  enif_free(to);
  if (rc != EMQX_GM_OK) return error_tuple(env, rc);
  rc = emqx_gm_fanout(CTX, r->idx, &m, 0, &d);
  emqx_gm_csr_free(CTX, &m);
  if (rc != EMQX_GM_OK) return error_tuple(env, rc);
  rows = enif_alloc(sizeof(ERL_NIF_TERM) * (n ? n : 1));
  for (i = 0; i < n; ++i) {
    ERL_NIF_TERM row = enif_make_list(env, 0);
    for (k = d.row_off[i + 1]; k > d.row_off[i]; --k)
      row = enif_make_list_cell(env, enif_make_uint(env, d.ids[k - 1]), row);
    rows[i] = row;
  }
  result = enif_make_list_from_array(env, rows, (unsigned)n);
  enif_free(rows);
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

static ErlNifFunc funcs[] = {
    {"load_index", 1, load_index, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"update_index", 2, update_index, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"match_batch", 2, match_batch, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"match_routes_batch", 2, match_routes_batch, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"fanout_batch", 2, fanout_batch, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"empty", 1, empty, 0},
};

ERL_NIF_INIT(emqx_gpu_match, funcs, load, NULL, NULL, unload)
