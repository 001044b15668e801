/* tests/nif_stub/erl_nif.h — TEST ONLY: declarations of the OTP NIF API
 * functions nif/emqx_gpu_match_nif.c uses, so that the shim can be
 * type-checked (gcc -fsyntax-only) in a container without Erlang
 * (no erl_nif.h on this image).  It is never linked or run;
 * the real header ships with OTP (erts/emulator/beam/erl_nif.h). */
#ifndef EMQX_TEST_ERL_NIF_STUB_H
#define EMQX_TEST_ERL_NIF_STUB_H
#include <stddef.h>

typedef unsigned long ERL_NIF_TERM;
typedef struct enif_environment_t ErlNifEnv;
typedef struct enif_resource_type_t ErlNifResourceType;
typedef void ErlNifResourceDtor(ErlNifEnv *, void *);
typedef enum { ERL_NIF_RT_CREATE = 1, ERL_NIF_RT_TAKEOVER = 2 } ErlNifResourceFlags;
typedef enum { ERL_NIF_LATIN1 = 1 } ErlNifCharEncoding;
typedef struct {
  size_t size;
  unsigned char *data;
  void *ref_bin;
  void *__spare__[2];
} ErlNifBinary;
typedef struct {
  const char *name;
  unsigned arity;
  ERL_NIF_TERM (*fptr)(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]);
  unsigned flags;
} ErlNifFunc;
#define ERL_NIF_DIRTY_JOB_CPU_BOUND 1

int enif_get_int(ErlNifEnv *, ERL_NIF_TERM, int *);
int enif_get_uint(ErlNifEnv *, ERL_NIF_TERM, unsigned *);
ErlNifResourceType *enif_open_resource_type(ErlNifEnv *, const char *, const char *, ErlNifResourceDtor *,
                                            ErlNifResourceFlags, ErlNifResourceFlags *);
ERL_NIF_TERM enif_make_atom(ErlNifEnv *, const char *);
ERL_NIF_TERM enif_make_tuple2(ErlNifEnv *, ERL_NIF_TERM, ERL_NIF_TERM);
ERL_NIF_TERM enif_make_string(ErlNifEnv *, const char *, ErlNifCharEncoding);
int enif_get_list_length(ErlNifEnv *, ERL_NIF_TERM, unsigned *);
int enif_get_list_cell(ErlNifEnv *, ERL_NIF_TERM, ERL_NIF_TERM *, ERL_NIF_TERM *);
int enif_inspect_binary(ErlNifEnv *, ERL_NIF_TERM, ErlNifBinary *);
int enif_alloc_binary(size_t, ErlNifBinary *);
void enif_release_binary(ErlNifBinary *);
ERL_NIF_TERM enif_make_binary(ErlNifEnv *, ErlNifBinary *);
void *enif_alloc(size_t);
void enif_free(void *);
void *enif_alloc_resource(ErlNifResourceType *, size_t);
ERL_NIF_TERM enif_make_resource(ErlNifEnv *, void *);
void enif_release_resource(void *);
ERL_NIF_TERM enif_make_badarg(ErlNifEnv *);
int enif_get_resource(ErlNifEnv *, ERL_NIF_TERM, ErlNifResourceType *, void **);
int enif_get_tuple(ErlNifEnv *, ERL_NIF_TERM, int *, const ERL_NIF_TERM **);
ERL_NIF_TERM enif_make_list(ErlNifEnv *, unsigned, ...);
ERL_NIF_TERM enif_make_list_cell(ErlNifEnv *, ERL_NIF_TERM, ERL_NIF_TERM);
int enif_make_reverse_list(ErlNifEnv *, ERL_NIF_TERM, ERL_NIF_TERM *);
int enif_is_identical(ERL_NIF_TERM, ERL_NIF_TERM);
ERL_NIF_TERM enif_make_resource_binary(ErlNifEnv *, void *, const void *, size_t);
ERL_NIF_TERM enif_make_list_from_array(ErlNifEnv *, const ERL_NIF_TERM[], unsigned);
ERL_NIF_TERM enif_make_uint(ErlNifEnv *, unsigned);

#define ERL_NIF_INIT(NAME, FUNCS, LOAD, RELOAD, UPGRADE, UNLOAD)                                       \
  const void *emqx_test_nif_entry(void) {                                                             \
    static const void *e[] = {FUNCS, (const void *)(LOAD), (const void *)(UNLOAD)};                    \
    (void)(RELOAD);                                                                                   \
    (void)(UPGRADE);                                                                                  \
    return e;                                                                                         \
  }
#endif
