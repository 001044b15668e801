/*
 * c_abi_smoke.c -- the C-ABI boundary used from plain C, the way the Erlang NIF
 * (nif/emqx_gpu_match_nif.c) or any other native caller would: no Python, no
 * torch.  Builds an index over the reference's router-suite filters
 * (emqx_router_SUITE.erl:81-95 t_match_routes: exact + 'a/+/c' + 'a/b/#' + '#'),
 * matches a batch with match_routes semantics and with emqx_trie:match/1
 * semantics, fans out, replicates the snapshot through an image
 * (export / import) and checks every row against the expected filter sets.
 * Exit status 0 = all checks passed.  tests/test_gpu_parity.py builds it with
 * gcc against include/ and runs it on the GPU box.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "emqx_gpu_match.h"

#define CHECK(cond, msg)                                                          \
  do {                                                                            \
    if (!(cond)) {                                                                \
      fprintf(stderr, "FAIL %s:%d %s (%s)\n", __FILE__, __LINE__, msg,            \
              ctx ? emqx_gm_last_error(ctx) : "");                                \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

static void pack(const char *const *s, uint64_t n, uint8_t *bytes, uint64_t *off) {
  off[0] = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t l = strlen(s[i]);
    memcpy(bytes + off[i], s[i], l);
    off[i + 1] = off[i] + l;
  }
  memset(bytes + off[n], 0, 64);
}

/* row i of `csr` as filter strings, '|'-joined, into buf */
static void row_str(const emqx_gm_index *idx, const emqx_gm_csr *csr, uint64_t i, char *buf) {
  buf[0] = 0;
  for (uint64_t k = csr->row_off[i]; k < csr->row_off[i + 1]; ++k) {
    const uint8_t *b;
    uint64_t len;
    emqx_gm_index_filter(idx, csr->ids[k], &b, &len);
    if (k > csr->row_off[i]) strcat(buf, "|");
    strncat(buf, (const char *)b, (size_t)len);
  }
}

int main(void) {
  emqx_gm_ctx *ctx = NULL;
  emqx_gm_opts o;
  memset(&o, 0, sizeof o);
  if (emqx_gm_open(&o, &ctx) != EMQX_GM_OK) {
    fprintf(stderr, "FAIL emqx_gm_open (no device?)\n");
    return 1;
  }
  CHECK(emqx_gm_abi_version() == EMQX_GM_ABI_VERSION, "abi version");
  /* emqx_router_SUITE:t_match_routes plus a '$SYS' filter */
  static const char *filters[] = {"a/b/c", "a/+/c", "a/b/#", "#", "$SYS/#", "a/b/c"};
  static const char *topics[] = {"a/b/c", "a/x/c", "a/b/d/e", "x", "$SYS/broker", "a/+/c"};
  /* sorted filter sets (Erlang binary order) per topic, match_routes semantics */
  static const char *want_routes[] = {"#|a/+/c|a/b/#|a/b/c", "#|a/+/c", "#|a/b/#", "#", "$SYS/#", "a/+/c"};
  /* emqx_trie:match/1: wildcard filters only; a wildcard topic gives [] */
  static const char *want_trie[] = {"#|a/+/c|a/b/#", "#|a/+/c", "#|a/b/#", "#", "$SYS/#", ""};
  const uint64_t nf = 6, nt = 6;
  uint8_t fb[256], tb[256];
  uint64_t fo[7], to[7];
  pack(filters, nf, fb, fo);
  pack(topics, nt, tb, to);
  /* subscribers: filter i -> {10 * i, 10 * i + 1}; the duplicate a/b/c concatenates */
  uint64_t so[7];
  uint32_t si[12];
  for (uint64_t i = 0; i < nf; ++i) {
    so[i] = 2 * i;
    si[2 * i] = (uint32_t)(10 * i);
    si[2 * i + 1] = (uint32_t)(10 * i + 1);
  }
  so[nf] = 2 * nf;
  emqx_gm_index *idx = NULL;
  uint32_t perm[6];
  CHECK(emqx_gm_index_build(ctx, fb, fo, nf, so, si, perm, &idx) == EMQX_GM_OK, "index_build");
  emqx_gm_index_info_t info;
  CHECK(emqx_gm_index_info(idx, &info) == EMQX_GM_OK && info.n_filters == 5 && !info.trie_empty, "info");
  CHECK(perm[0] == perm[5], "duplicate filters share one id");

  char buf[512];
  emqx_gm_csr out;
  CHECK(emqx_gm_match(ctx, idx, tb, to, nt, EMQX_GM_WITH_EXACT, &out) == EMQX_GM_OK, "match_routes");
  for (uint64_t i = 0; i < nt; ++i) {
    row_str(idx, &out, i, buf);
    if (strcmp(buf, want_routes[i])) {
      fprintf(stderr, "FAIL match_routes row %llu: got '%s' want '%s'\n", (unsigned long long)i, buf, want_routes[i]);
      return 1;
    }
  }
  /* fan-out of the match_routes rows: each filter's subscribers, rows as multisets */
  emqx_gm_csr fan;
  CHECK(emqx_gm_fanout(ctx, idx, &out, 0, &fan) == EMQX_GM_OK, "fanout");
  CHECK(fan.row_off[1] - fan.row_off[0] == 10, "a/b/c: 4 filters, a/b/c with 4 subscribers, 2 each for the rest");
  emqx_gm_csr_free(ctx, &fan);
  emqx_gm_csr_free(ctx, &out);

  CHECK(emqx_gm_match(ctx, idx, tb, to, nt, 0, &out) == EMQX_GM_OK, "trie match");
  for (uint64_t i = 0; i < nt; ++i) {
    row_str(idx, &out, i, buf);
    if (strcmp(buf, want_trie[i])) {
      fprintf(stderr, "FAIL trie row %llu: got '%s' want '%s'\n", (unsigned long long)i, buf, want_trie[i]);
      return 1;
    }
  }
  emqx_gm_csr_free(ctx, &out);

  /* replicate through an image and match again on the copy */
  uint64_t sz = 0;
  CHECK(emqx_gm_index_export(ctx, idx, 0, NULL, &sz) == EMQX_GM_OK && sz > 0, "export size");
  uint8_t *img = malloc(sz);
  CHECK(img && emqx_gm_index_export(ctx, idx, 0, img, &sz) == EMQX_GM_OK, "export");
  emqx_gm_index *copy = NULL;
  CHECK(emqx_gm_index_import(ctx, img, sz, NULL, &copy) == EMQX_GM_OK, "import");
  img[0] ^= 0xFF;
  emqx_gm_index *bad = NULL;
  CHECK(emqx_gm_index_import(ctx, img, sz, NULL, &bad) == EMQX_GM_EINVAL && !bad, "a corrupt image is refused");
  free(img);
  CHECK(emqx_gm_match(ctx, copy, tb, to, nt, EMQX_GM_WITH_EXACT, &out) == EMQX_GM_OK, "match on the copy");
  for (uint64_t i = 0; i < nt; ++i) {
    row_str(copy, &out, i, buf);
    CHECK(!strcmp(buf, want_routes[i]), "imported rows");
  }
  emqx_gm_csr_free(ctx, &out);

  /* errors cross the ABI as codes: a bad flag, a NULL output */
  CHECK(emqx_gm_match(ctx, idx, tb, to, nt, 0x80u, &out) == EMQX_GM_EINVAL, "unknown flag");
  CHECK(emqx_gm_index_build(ctx, fb, fo, nf, NULL, NULL, NULL, NULL) == EMQX_GM_EINVAL, "NULL out");

  emqx_gm_index_release(copy);
  emqx_gm_index_release(idx);
  emqx_gm_close(ctx);

  /* a two-device context (device 0 listed twice: two replicas on one GPU, the
   * one-GPU rehearsal of a node's device list): one build replicated, a
   * 600k-topic host batch spread over both in 256K-topic chunks, from a
   * page-locked buffer (emqx_gm_host_alloc) and from plain memory, an update
   * replicated; every row as expected */
  ctx = NULL;
  memset(&o, 0, sizeof o);
  o.n_devices = 2;
  o.devices[0] = 0;
  o.devices[1] = 0;
  CHECK(emqx_gm_open(&o, &ctx) == EMQX_GM_OK, "open two devices");
  int32_t devs[EMQX_GM_MAX_DEVICES];
  uint32_t ndev = 0;
  CHECK(emqx_gm_devices(ctx, devs, &ndev) == EMQX_GM_OK && ndev == 2 && devs[0] == 0 && devs[1] == 0, "devices");
  CHECK(emqx_gm_index_build(ctx, fb, fo, nf, NULL, NULL, NULL, &idx) == EMQX_GM_OK, "two-device build");
  const uint64_t big = 600000;
  uint64_t bytes_big = 0;
  for (uint64_t i = 0; i < big; ++i) bytes_big += strlen(topics[i % nt]);
  uint8_t *pb = NULL;
  CHECK(emqx_gm_host_alloc(ctx, bytes_big + 64, (void **)&pb) == EMQX_GM_OK && pb, "host_alloc");
  uint8_t *plain = malloc(bytes_big + 64);
  uint64_t *bo = malloc((big + 1) * sizeof(uint64_t));
  CHECK(plain && bo, "malloc");
  bo[0] = 0;
  for (uint64_t i = 0; i < big; ++i) {
    const uint64_t l = strlen(topics[i % nt]);
    memcpy(pb + bo[i], topics[i % nt], l);
    bo[i + 1] = bo[i] + l;
  }
  memset(pb + bytes_big, 0, 64);
  memcpy(plain, pb, bytes_big + 64);
  for (int pass = 0; pass < 3; ++pass) {
    if (pass == 2) {  /* an update (filter 'x/#' added), replicated to both devices */
      static const char *nf_s[] = {"x/#"};
      uint8_t ub[80];
      uint64_t uo[2];
      uint8_t op = 1;
      emqx_gm_index *nidx = NULL;
      pack(nf_s, 1, ub, uo);
      CHECK(emqx_gm_index_update(ctx, idx, ub, uo, &op, 1, &nidx) == EMQX_GM_OK, "two-device update");
      emqx_gm_index_release(idx);
      idx = nidx;
    }
    CHECK(emqx_gm_match(ctx, idx, pass == 1 ? plain : pb, bo, big, EMQX_GM_WITH_EXACT, &out) == EMQX_GM_OK,
          "two-device match");
    CHECK(out.n_rows == big && !out.on_device, "two-device rows");
    for (uint64_t i = 0; i < big; i += 997) {
      row_str(idx, &out, i, buf);
      const char *w = want_routes[i % nt];
      if (pass == 2 && i % nt == 3) w = "#|x/#";
      if (strcmp(buf, w)) {
        fprintf(stderr, "FAIL two-device row %llu (pass %d): got '%s' want '%s'\n", (unsigned long long)i, pass, buf, w);
        return 1;
      }
    }
    row_str(idx, &out, big - 1, buf);
    CHECK(!strcmp(buf, want_routes[(big - 1) % nt]), "two-device last row");
    emqx_gm_csr_free(ctx, &out);
  }
  CHECK(emqx_gm_host_free(ctx, pb) == EMQX_GM_OK, "host_free");
  CHECK(emqx_gm_host_free(ctx, plain) == EMQX_GM_EINVAL, "host_free of a malloc'd buffer");
  free(plain);
  free(bo);
  emqx_gm_index_release(idx);
  emqx_gm_close(ctx);
  printf("C_ABI_SMOKE_OK\n");
  return 0;
}
