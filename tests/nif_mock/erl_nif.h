/*
 * erl_nif.h (test mock) -- just enough of the erl_nif API for
 * emqx_amd/csrc/nif/emqx_tm_nif.c to compile and run outside an Erlang VM.
 * The OTP headers are not in this image; this is NOT them.  Terms are
 * immutable heap nodes that are never freed (tests are short), environments
 * carry the "process" they belong to, enif_send appends to a mailbox that
 * tests read back.  Implementation: mock_erts.c.
 */
#ifndef EMQX_TM_MOCK_ERL_NIF_H
#define EMQX_TM_MOCK_ERL_NIF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef uintptr_t ERL_NIF_TERM;
typedef struct mock_env ErlNifEnv;
typedef struct mock_rt ErlNifResourceType;
typedef struct { int id; } ErlNifPid;
typedef struct {
    size_t size;
    unsigned char* data;
} ErlNifBinary;
typedef void ErlNifResourceDtor(ErlNifEnv*, void*);
typedef enum { ERL_NIF_RT_CREATE = 1, ERL_NIF_RT_TAKEOVER = 2 } ErlNifResourceFlags;
typedef struct {
    const char* name;
    unsigned arity;
    ERL_NIF_TERM (*fptr)(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]);
    unsigned flags;
} ErlNifFunc;
typedef struct {
    const char* name;
    int num_of_funcs;
    ErlNifFunc* funcs;
    int (*load)(ErlNifEnv*, void**, ERL_NIF_TERM);
    void (*unload)(ErlNifEnv*, void*);
} ErlNifEntry;

#define ERL_NIF_DIRTY_JOB_CPU_BOUND 1
#define ERL_NIF_DIRTY_JOB_IO_BOUND 2

#define ERL_NIF_INIT(NAME, FUNCS, LOAD, RELOAD, UPGRADE, UNLOAD)                                      \
    ErlNifEntry* nif_init(void) {                                                                     \
        static ErlNifEntry entry = {#NAME, (int)(sizeof(FUNCS) / sizeof(FUNCS[0])), FUNCS, LOAD, UNLOAD}; \
        return &entry;                                                                                \
    }

void* enif_alloc(size_t size);
void enif_free(void* ptr);
ErlNifEnv* enif_alloc_env(void);
void enif_free_env(ErlNifEnv* env);
ErlNifPid* enif_self(ErlNifEnv* env, ErlNifPid* pid);
int enif_send(ErlNifEnv* caller_env, const ErlNifPid* to, ErlNifEnv* msg_env, ERL_NIF_TERM msg);
ERL_NIF_TERM enif_make_copy(ErlNifEnv* dst, ERL_NIF_TERM t);

ErlNifResourceType* enif_open_resource_type(ErlNifEnv* env, const char* module, const char* name,
                                            ErlNifResourceDtor* dtor, ErlNifResourceFlags flags,
                                            ErlNifResourceFlags* tried);
void* enif_alloc_resource(ErlNifResourceType* type, size_t size);
void enif_release_resource(void* obj);
void enif_keep_resource(void* obj);
ERL_NIF_TERM enif_make_resource(ErlNifEnv* env, void* obj);
int enif_get_resource(ErlNifEnv* env, ERL_NIF_TERM t, ErlNifResourceType* type, void** objp);

ERL_NIF_TERM enif_make_atom(ErlNifEnv* env, const char* name);
ERL_NIF_TERM enif_make_badarg(ErlNifEnv* env);
ERL_NIF_TERM enif_make_uint(ErlNifEnv* env, unsigned v);
ERL_NIF_TERM enif_make_uint64(ErlNifEnv* env, uint64_t v);
ERL_NIF_TERM enif_make_tuple2(ErlNifEnv* env, ERL_NIF_TERM a, ERL_NIF_TERM b);
ERL_NIF_TERM enif_make_tuple3(ErlNifEnv* env, ERL_NIF_TERM a, ERL_NIF_TERM b, ERL_NIF_TERM c);
ERL_NIF_TERM enif_make_tuple5(ErlNifEnv* env, ERL_NIF_TERM a, ERL_NIF_TERM b, ERL_NIF_TERM c, ERL_NIF_TERM d,
                              ERL_NIF_TERM e);
ERL_NIF_TERM enif_make_list(ErlNifEnv* env, unsigned cnt, ...);
ERL_NIF_TERM enif_make_list1(ErlNifEnv* env, ERL_NIF_TERM e1);
ERL_NIF_TERM enif_make_list_cell(ErlNifEnv* env, ERL_NIF_TERM head, ERL_NIF_TERM tail);
unsigned char* enif_make_new_binary(ErlNifEnv* env, size_t size, ERL_NIF_TERM* termp);

int enif_get_int(ErlNifEnv* env, ERL_NIF_TERM t, int* ip);
int enif_get_uint(ErlNifEnv* env, ERL_NIF_TERM t, unsigned* ip);
int enif_inspect_binary(ErlNifEnv* env, ERL_NIF_TERM t, ErlNifBinary* bin);
int enif_get_list_length(ErlNifEnv* env, ERL_NIF_TERM t, unsigned* len);
int enif_get_list_cell(ErlNifEnv* env, ERL_NIF_TERM list, ERL_NIF_TERM* head, ERL_NIF_TERM* tail);
int enif_get_tuple(ErlNifEnv* env, ERL_NIF_TERM t, int* arity, const ERL_NIF_TERM** array);
int enif_is_identical(ERL_NIF_TERM a, ERL_NIF_TERM b);
int enif_compare(ERL_NIF_TERM a, ERL_NIF_TERM b);
int enif_is_ref(ErlNifEnv* env, ERL_NIF_TERM t);

#ifdef __cplusplus
}
#endif
#endif
