/*
 * isal_hip_shim.c — the C-ABI boundary of the MI355X erasure-code engine.
 *
 * Exports the reference's data-path symbols (erasure_code.h, gf_vect_mul.h:
 * ec_encode_data, ec_encode_data_update, gf_vect_dot_prod, gf_vect_mad,
 * gf_vect_mul and their *_base twins) and the batched extension (isal_hip.h).
 * Replaces the reference's L2 dispatch + L3 glue (ec_multibinary.asm:79-93,
 * ec_highlevel_func.c:159-698): instead of picking a CPU ISA, calls are
 * routed to the GPU kernels in ec_kernels.hip (small host-resident calls: the
 * CPU route, ec_cpu.c).
 *
 * Per call (run_ec):
 *   1. classify every shard pointer (device/managed vs host) with
 *      hipPointerGetAttributes;
 *   2. route: host-resident calls of at most ISAL_HIP_CPU_MAX_BYTES run on the
 *      CPU route (ec_cpu.c) — the GPU round trip costs more than the work, as
 *      the reference's own short-length fallback recognises
 *      (ec_highlevel_func.c:159-194); ISAL_HIP_BACKEND=gpu|cpu|auto overrides;
 *   3. otherwise stage host-resident shards through a per-thread pinned or HBM
 *      buffer (zero-copy / packed / column-chunked), upload the pointer table +
 *      derived coefficient tables, launch, copy host-resident outputs back and
 *      synchronise — the reference API is synchronous.
 *
 * Failures: the reference API has no error return, so a host-resident call
 * must not fail where the reference would succeed. A failing HIP call hands
 * the columns that are not yet final to the CPU route (reported once on
 * stderr). Only a call with device-resident shards — which no CPU route can
 * serve — or one made under ISAL_HIP_BACKEND=gpu aborts.
 * Thread safety: all mutable state is per thread (pthread key) except the
 * atomic counters and the read-once knobs.
 */
#define _GNU_SOURCE /* dladdr */
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "crc.h"
#include "crc64.h"
#include "erasure_code.h"
#include "isal_hip.h"
#include "isal_hip_internal.h"

/* ---- errors, counters, routing log -------------------------------------- */

static void
die(const char *what, hipError_t e)
{
        fprintf(stderr,
                "isal_hip: %s failed: %s (%d) on a call with device-resident shards (or with "
                "ISAL_HIP_BACKEND=gpu); no CPU route can serve it, aborting\n",
                what, hipGetErrorString(e), (int) e);
        abort();
}

static unsigned long long g_launches, g_cpu_calls, g_fallbacks;

void
isal_hip_count_launch(void)
{
        __atomic_add_fetch(&g_launches, 1ull, __ATOMIC_RELAXED);
}

unsigned long long
isal_hip_kernel_launches(void)
{
        return __atomic_load_n(&g_launches, __ATOMIC_RELAXED);
}

unsigned long long
isal_hip_cpu_calls(void)
{
        return __atomic_load_n(&g_cpu_calls, __ATOMIC_RELAXED);
}

unsigned long long
isal_hip_fallbacks(void)
{
        return __atomic_load_n(&g_fallbacks, __ATOMIC_RELAXED);
}

/* ---- kernel registry --------------------------------------------------------
 * Filled while the library loads (static initialisers of the kernel objects,
 * ec_device.h KernelReg), read by isal_hip_selftest_kernels. */
#define KREG_MAX 4096
static int gpu_present(void);
static const void *kreg_fn[KREG_MAX];
static const char *kreg_name[KREG_MAX];
static int kreg_n, kreg_lost;

void
isal_hip_kreg_add(const void *fn, const char *name)
{
        const int i = __atomic_fetch_add(&kreg_n, 1, __ATOMIC_RELAXED);
        if (i >= KREG_MAX) {
                __atomic_add_fetch(&kreg_lost, 1, __ATOMIC_RELAXED);
                return;
        }
        kreg_fn[i] = fn;
        kreg_name[i] = name;
}

int
isal_hip_selftest_kernels(int *nkernels)
{
        int i, n = __atomic_load_n(&kreg_n, __ATOMIC_ACQUIRE), bad = 0;
        if (n > KREG_MAX)
                n = KREG_MAX;
        if (nkernels)
                *nkernels = n;
        if (__atomic_load_n(&kreg_lost, __ATOMIC_RELAXED))
                return ISAL_HIP_ENOMEM; /* the registry is too small to vouch for every kernel */
        if (!gpu_present())
                return ISAL_HIP_EHIP;
        for (i = 0; i < n; i++) {
                hipFuncAttributes a;
                const hipError_t e = hipFuncGetAttributes(&a, kreg_fn[i]);
                if (e != hipSuccess) {
                        Dl_info info;
                        const int found = dladdr(kreg_fn[i], &info) != 0;
                        (void) hipGetLastError();
                        fprintf(stderr,
                                "isal_hip: selftest: kernel with no usable device code: %s (handle %s+0x%lx): "
                                "%s\n",
                                kreg_name[i], found ? info.dli_fname : "?",
                                found ? (unsigned long) ((const char *) kreg_fn[i] - (const char *) info.dli_fbase)
                                      : 0ul,
                                hipGetErrorString(e));
                        bad++;
                }
        }
        return bad;
}

int
isal_hip_max_rows_per_pass(void)
{
        return EC_MAX_ROWS_PER_PASS;
}

const char *
isal_hip_target(void)
{
        return "gfx950";
}

static const char *const op_names[] = {"encode", "update", "verify"};

/* ISAL_HIP_LOG=1: one stderr line per drop-in call naming the route taken. */
static void
route_log(int op, int len, int k, int rows, const char *route, const char *why)
{
        if (isal_hip_knob(ISAL_HIP_KNOB_LOG) > 0)
                fprintf(stderr, "isal_hip: %s len=%d k=%d rows=%d -> %s (%s)\n", op_names[op], len,
                        k, rows, route, why);
}

/* A HIP failure under a host-resident call: reported once per process (every
 * time with ISAL_HIP_LOG=1), then the call finishes on the CPU route. */
static void
report_fallback(const char *what, hipError_t e)
{
        static int reported;
        __atomic_add_fetch(&g_fallbacks, 1ull, __ATOMIC_RELAXED);
        if (!__atomic_exchange_n(&reported, 1, __ATOMIC_RELAXED) ||
            isal_hip_knob(ISAL_HIP_KNOB_LOG) > 0)
                fprintf(stderr,
                        "isal_hip: %s failed: %s (%d); host-resident calls fall back to the CPU "
                        "route (reported once; ISAL_HIP_LOG=1 reports each)\n",
                        what, hipGetErrorString(e), (int) e);
}

enum { BACKEND_AUTO = 0, BACKEND_GPU = 1, BACKEND_CPU = 2 };

static int
backend(void)
{
        const long long v = isal_hip_knob(ISAL_HIP_KNOB_BACKEND);
        static int warned;
        if (v == -2 && !__atomic_exchange_n(&warned, 1, __ATOMIC_RELAXED))
                fprintf(stderr, "isal_hip: ISAL_HIP_BACKEND must be auto, gpu or cpu; using auto\n");
        return v == BACKEND_GPU || v == BACKEND_CPU ? (int) v : BACKEND_AUTO;
}

/* Host calls of at most this many shard bytes ((k + rows) * len) take the CPU
 * route under ISAL_HIP_BACKEND=auto (override: ISAL_HIP_CPU_MAX_BYTES). Below
 * it the ~30 us GPU round trip costs more than the arithmetic (DESIGN.md §3,
 * measured crossover in profiles/r02/r02_route_crossover.txt). */
#define DEFAULT_CPU_MAX_BYTES ((size_t) 8 << 20)

static size_t
cpu_max_bytes(void)
{
        const long long v = isal_hip_knob(ISAL_HIP_KNOB_CPU_MAX_BYTES);
        return v >= 0 ? (size_t) v : DEFAULT_CPU_MAX_BYTES;
}

/* The same limit for calls whose host shards are all page-locked and used in
 * place by the kernels (no staging copy): there the GPU wins from 1.8 MB
 * (k = 10, p = 4: 51.6 vs 59.1 us; 14.7 MB: 290 vs 497 us,
 * profiles/r03/r03_route_crossover_c.jsonl). Override: ISAL_HIP_CPU_MAX_BYTES_PINNED
 * (ISAL_HIP_CPU_MAX_BYTES also lowers it). */
#define DEFAULT_CPU_MAX_BYTES_PINNED ((size_t) 2 << 20)

static size_t
cpu_max_bytes_pinned(void)
{
        const long long v = isal_hip_knob(ISAL_HIP_KNOB_CPU_MAX_BYTES_PINNED);
        const size_t all = cpu_max_bytes();
        if (v >= 0)
                return (size_t) v;
        return all < DEFAULT_CPU_MAX_BYTES_PINNED ? all : DEFAULT_CPU_MAX_BYTES_PINNED;
}

/* Is a GPU usable at all? (Asked once: a host without one, or without a
 * working driver, serves every host-resident call on the CPU route.) */
static int gpu_ok;
static pthread_once_t gpu_once = PTHREAD_ONCE_INIT;

static void
gpu_probe(void)
{
        int n = 0;
        gpu_ok = hipGetDeviceCount(&n) == hipSuccess && n > 0;
        if (!gpu_ok)
                (void) hipGetLastError();
}

static int
gpu_present(void)
{
        pthread_once(&gpu_once, gpu_probe);
        return gpu_ok;
}

/* ---- per-thread context ------------------------------------------------- */

/* Host-resident shards are staged through HBM in chunks of at most this many
 * bytes in total (override: ISAL_HIP_STAGE_MB). */
#define DEFAULT_STAGE_BYTES (256u << 20)
/* Large host calls are cut into column chunks of this many bytes per shard
 * (override: ISAL_HIP_CHUNK_KB) that flow through PIPE_NBUF staging buffers:
 * the H2D copy of chunk i+1, the kernel of chunk i and the D2H copy of chunk
 * i-1 run at once on three streams. */
#define DEFAULT_CHUNK_BYTES ((size_t) 4 << 20)
#define PIPE_NBUF 3

typedef struct {
        int device;
        hipStream_t stream;
        void *d_args; /* device: pointer table + coefficient tables */
        void *h_args; /* pinned mirror of d_args (fine-grained, coherent) */
        void *h_args_dev; /* the same pinned buffer as seen by kernels (zero-copy) */
        size_t args_cap;
        unsigned char *d_stage; /* device scratch for host-resident shards */
        size_t stage_cap;
        /* pipelined column chunks (gpu_pipelined): copy-in / copy-out streams
         * and per-buffer events, created on first use */
        hipStream_t s_in, s_out;
        hipEvent_t ev_in[PIPE_NBUF], ev_k[PIPE_NBUF], ev_out[PIPE_NBUF];
        int pipe_ready;
        struct outq *oq; /* the call thread's copy-out worker (gpu_pipelined) */
        struct copyjob *jobs; /* [3]: worker's copies in / out, this thread's list */
        /* the last call's derived coefficient tables and 0/1 masks, reused
         * while its coefficients (byte 1 of each gftbls entry) repeat */
        int tk, trows;
        unsigned tgen;
        unsigned char *tcoef;
        uint32_t *ttbl;
        size_t tcap_coef, tcap_tbl;
        isal_hip_encmask tem;
        /* the same coefficients' LDS product tables on the device (drop-in
         * encodes of 7-8 rows, isal_hip_karg_ldsx), built on first use */
        uint64_t *d_ldsx;
        size_t ldsx_cap;
        int ldsx_ok;
        /* completion of kernel-argument calls (isal_hip_kdone): device words
         * {arrival counter, verify result}, the page-locked host mailbox
         * {seq, result} and its device view, the last sequence number, and
         * calls since the stream was last synchronised */
        void *d_done;
        volatile unsigned long long *h_mail;
        void *h_mail_dev;
        unsigned long long seq;
        int unsynced;
        /* checksum entry points on device buffers: kernel tables of the last
         * geometry per flavour (CRC32C, the eight CRC64) and the partials */
        struct crcc {
                long long len;
                int tt;
                void *d_tabs;
        } c32, c64[ISAL_HIP_CRC64_NVARIANTS];
        void *d_cpart;
        size_t cpart_cap;
} ctx_t;

/* Copy-out worker of a calling thread. The runtime serves a copy from or to
 * pageable memory synchronously on the thread that issues it (tools/
 * stage_probe.c: hipMemcpyAsync returns when the copy is done), so copies in
 * and out overlap only when two host threads issue them: the calling thread
 * stages chunks in and launches, this worker copies chunks out in order. */
typedef struct outq {
        pthread_t th;
        pthread_mutex_t mu;
        pthread_cond_t cv;
        int quit, active;
        long long posted, handled; /* chunks launched / whose output copies are enqueued */
        /* the call being served */
        int nsrc, nptr, len;
        const uint64_t *view;
        unsigned char *const *dst;
        size_t chunk, slot, set_bytes;
        /* the worker's first failure */
        hipError_t err;
        const char *what;
        long long fail_chunk;
        int rows_out;
        /* a one-off batch of copies (gpu_chunked's second issuing thread) */
        struct copyjob *job;
        int job_state; /* 0 none, 1 posted, 2 finished */
} outq_t;

/* Copies the worker issues on s_out for gpu_chunked: after `after` (if set,
 * a GPU-side wait), then `record` is recorded. */
#define COPYJOB_MAX 512
typedef struct copyjob {
        int n;
        struct {
                void *dst;
                const void *src;
                size_t bytes;
                hipMemcpyKind kind;
        } cp[COPYJOB_MAX];
        hipEvent_t after, record;
        hipError_t err;
        const char *what;
} copyjob_t;

static hipError_t outq_start(ctx_t *c);
static void copyjob_post(outq_t *q, copyjob_t *j);
static hipError_t copyjob_wait(outq_t *q, copyjob_t *j);

static void outq_stop(ctx_t *c);

static pthread_key_t ctx_key;
static pthread_once_t ctx_once = PTHREAD_ONCE_INIT;

/* A calling thread's contexts, one per device it has made calls on: a thread
 * that serves shards on several GPUs keeps each GPU's stream, buffers and
 * mailbox instead of rebuilding them on every device switch. */
#define CTX_MAX_DEV 64
typedef struct {
        ctx_t *dev[CTX_MAX_DEV];
} tctx_t;

static unsigned long long g_ctx_created;

unsigned long long
isal_hip_contexts_created(void)
{
        return __atomic_load_n(&g_ctx_created, __ATOMIC_RELAXED);
}

static void
ctx_free(ctx_t *c)
{
        if (!c)
                return;
        /* Best effort at thread exit: the runtime may already be shutting down. */
        if (c->stream)
                (void) hipStreamDestroy(c->stream);
        if (c->d_args)
                (void) hipFree(c->d_args);
        if (c->h_args)
                (void) hipHostFree(c->h_args);
        if (c->d_stage)
                (void) hipFree(c->d_stage);
        if (c->d_done)
                (void) hipFree(c->d_done);
        if (c->h_mail)
                (void) hipHostFree((void *) c->h_mail);
        if (c->oq)
                outq_stop(c);
        if (c->c32.d_tabs)
                (void) hipFree(c->c32.d_tabs);
        for (int v = 0; v < ISAL_HIP_CRC64_NVARIANTS; v++)
                if (c->c64[v].d_tabs)
                        (void) hipFree(c->c64[v].d_tabs);
        if (c->d_cpart)
                (void) hipFree(c->d_cpart);
        if (c->d_ldsx)
                (void) hipFree(c->d_ldsx);
        free(c->jobs);
        free(c->tcoef);
        free(c->ttbl);
        if (c->pipe_ready) {
                int b;
                (void) hipStreamDestroy(c->s_in);
                (void) hipStreamDestroy(c->s_out);
                for (b = 0; b < PIPE_NBUF; b++) {
                        (void) hipEventDestroy(c->ev_in[b]);
                        (void) hipEventDestroy(c->ev_k[b]);
                        (void) hipEventDestroy(c->ev_out[b]);
                }
        }
        free(c);
}

static void
tctx_release(void *p)
{
        tctx_t *t = (tctx_t *) p;
        int d;
        if (!t)
                return;
        for (d = 0; d < CTX_MAX_DEV; d++)
                ctx_free(t->dev[d]);
        free(t);
}

static void
ctx_key_init(void)
{
        if (pthread_key_create(&ctx_key, tctx_release) != 0) {
                fprintf(stderr, "isal_hip: pthread_key_create failed\n");
                abort();
        }
}

/* The calling thread's context on device dev — which must be the thread's
 * current device when the context is first made (its stream belongs to the
 * current device) — or NULL with *err set. */
static ctx_t *
ctx_get(int dev, hipError_t *err, const char **what)
{
        tctx_t *t;
        ctx_t *c;
        pthread_once(&ctx_once, ctx_key_init);
        if (dev < 0 || dev >= CTX_MAX_DEV) {
                *err = hipErrorInvalidDevice;
                *what = "device ordinal (at most 64 GPUs per process)";
                return NULL;
        }
        t = (tctx_t *) pthread_getspecific(ctx_key);
        if (!t) {
                t = (tctx_t *) calloc(1, sizeof(*t));
                if (!t || pthread_setspecific(ctx_key, t) != 0) {
                        fprintf(stderr, "isal_hip: out of host memory\n");
                        abort();
                }
        }
        if ((c = t->dev[dev]) != NULL)
                return c;
        c = (ctx_t *) calloc(1, sizeof(*c));
        if (!c) {
                fprintf(stderr, "isal_hip: out of host memory\n");
                abort();
        }
        c->device = dev;
        /* A BLOCKING stream: it is ordered after work already queued on the
         * legacy default stream (e.g. torch kernels that just wrote the
         * shards), as the synchronous reference API implies. */
        if ((*err = hipStreamCreate(&c->stream)) != hipSuccess) {
                *what = "hipStreamCreate";
                free(c);
                return NULL;
        }
        t->dev[dev] = c;
        __atomic_add_fetch(&g_ctx_created, 1ull, __ATOMIC_RELAXED);
        return c;
}

/* The call's device coefficient tables (isal_hip_build_tables layout) and 0/1
 * masks: rebuilt only when the coefficients differ from the thread's last
 * call (a storage caller encodes stripe after stripe with one matrix; the
 * rebuild is ~5k table lookups for k = 10, p = 4). NULL when out of memory. */
static const uint32_t *
ctx_tables(ctx_t *c, int k, int rows, const unsigned char *gftbls, const isal_hip_encmask **em)
{
        const size_t n = (size_t) k * (size_t) rows, nd = isal_hip_tables_dwords(k, rows);
        const unsigned gen = isal_hip_knob_generation();
        size_t i;
        int hit = c->ttbl && c->tk == k && c->trows == rows && c->tgen == gen;
        for (i = 0; hit && i < n; i++)
                hit = c->tcoef[i] == gftbls[i * 32 + 1];
        if (!hit) {
                if (n > c->tcap_coef) {
                        unsigned char *x = (unsigned char *) realloc(c->tcoef, n);
                        if (!x)
                                return NULL;
                        c->tcoef = x;
                        c->tcap_coef = n;
                }
                /* k = 0 (the empty sum: zero parity) has no tables at all; keep
                 * one dword so that only a failed allocation returns NULL */
                if (nd > c->tcap_tbl || !c->ttbl) {
                        const size_t cap = nd ? nd : 1;
                        uint32_t *x = (uint32_t *) realloc(c->ttbl, cap * 4);
                        if (!x)
                                return NULL;
                        c->ttbl = x;
                        c->tcap_tbl = cap;
                }
                c->tk = -1; /* not valid until rebuilt */
                c->ldsx_ok = 0;
                for (i = 0; i < n; i++)
                        c->tcoef[i] = gftbls[i * 32 + 1];
                isal_hip_build_tables(k, rows, gftbls, c->ttbl);
                isal_hip_enc_masks(k, rows, gftbls, &c->tem);
                c->tk = k;
                c->trows = rows;
                c->tgen = gen;
        }
        *em = &c->tem;
        return c->ttbl;
}

static hipError_t
ensure_args(ctx_t *c, size_t bytes)
{
        size_t cap;
        hipError_t e;
        if (bytes <= c->args_cap)
                return hipSuccess;
        cap = c->args_cap ? c->args_cap : 64 * 1024;
        while (cap < bytes)
                cap *= 2;
        if (c->d_args)
                (void) hipFree(c->d_args);
        if (c->h_args)
                (void) hipHostFree(c->h_args);
        c->d_args = c->h_args = c->h_args_dev = NULL;
        c->args_cap = 0;
        if ((e = hipMalloc(&c->d_args, cap)) != hipSuccess)
                return e;
        /* coherent: kernels of the zero-copy path read arguments and shards the
         * host just wrote, and the host reads what they wrote, with no cached
         * copies in between */
        if ((e = hipHostMalloc(&c->h_args, cap, hipHostMallocCoherent)) != hipSuccess ||
            (e = hipHostGetDevicePointer(&c->h_args_dev, c->h_args, 0)) != hipSuccess) {
                (void) hipFree(c->d_args);
                if (c->h_args)
                        (void) hipHostFree(c->h_args);
                c->d_args = c->h_args = c->h_args_dev = NULL;
                return e;
        }
        c->args_cap = cap;
        return hipSuccess;
}

static hipError_t
ensure_stage(ctx_t *c, size_t bytes)
{
        hipError_t e;
        if (bytes <= c->stage_cap)
                return hipSuccess;
        if (c->d_stage)
                (void) hipFree(c->d_stage);
        c->d_stage = NULL;
        c->stage_cap = 0;
        if ((e = hipMalloc((void **) &c->d_stage, bytes)) != hipSuccess)
                return e;
        c->stage_cap = bytes;
        return hipSuccess;
}

static hipError_t
ensure_pipe(ctx_t *c)
{
        hipError_t e;
        int b;
        if (c->pipe_ready)
                return hipSuccess;
        if ((e = hipStreamCreateWithFlags(&c->s_in, hipStreamNonBlocking)) != hipSuccess)
                return e;
        if ((e = hipStreamCreateWithFlags(&c->s_out, hipStreamNonBlocking)) != hipSuccess) {
                (void) hipStreamDestroy(c->s_in);
                return e;
        }
        for (b = 0; b < PIPE_NBUF; b++) {
                if ((e = hipEventCreateWithFlags(&c->ev_in[b], hipEventDisableTiming)) != hipSuccess ||
                    (e = hipEventCreateWithFlags(&c->ev_k[b], hipEventDisableTiming)) != hipSuccess ||
                    (e = hipEventCreateWithFlags(&c->ev_out[b], hipEventDisableTiming)) != hipSuccess) {
                        /* leak the few created events: this only happens when the
                         * runtime is failing anyway */
                        (void) hipStreamDestroy(c->s_in);
                        (void) hipStreamDestroy(c->s_out);
                        return e;
                }
        }
        c->pipe_ready = 1;
        return hipSuccess;
}

static size_t
stage_limit(void)
{
        const long long v = isal_hip_knob(ISAL_HIP_KNOB_STAGE_MB);
        return v > 0 ? (size_t) v << 20 : DEFAULT_STAGE_BYTES;
}

/* ---- pointer classification ------------------------------------------- */

/* Where a shard lives (kind; ISAL_HIP_MEM_*) and, for device and page-locked
 * memory, the device its attributes name (*dev; -1 otherwise). Returns what a
 * kernel would use for it: device (hipMalloc) and managed memory, the pointer
 * itself; page-locked host memory (hipHostMalloc, hipHostRegister — NIC / disk
 * DMA buffers usually are), the device's mapping of it, which kernels of THAT
 * device read and write in place over PCIe with no staging copy
 * (ISAL_HIP_PINNED_DIRECT=0 stages it like pageable memory) — but only when
 * the shard's LAST byte maps through the same registration too: a shard that
 * runs past the end of a partly registered buffer would make the kernel touch
 * unmapped memory (a GPU fault the CPU route could not recover from), so it is
 * staged (kind pageable). Pageable memory: 0 — it is copied through a staging
 * buffer. For device memory *rbase / *rsize receive its allocation's range. */
enum {
        CL_HOST = ISAL_HIP_MEM_PAGEABLE,
        CL_DEVICE = ISAL_HIP_MEM_DEVICE,
        CL_MANAGED = ISAL_HIP_MEM_MANAGED,
        CL_PINNED = ISAL_HIP_MEM_PINNED,
};

static uint64_t
classify(const void *p, size_t len, int *kind, int *dev, uintptr_t *rbase, size_t *rsize)
{
        hipPointerAttribute_t a, z;
        hipError_t e;
        *kind = CL_HOST;
        *dev = -1;
        *rsize = 0;
        if (!p)
                return 0;
        e = hipPointerGetAttributes(&a, p);
        if (e != hipSuccess) {
                (void) hipGetLastError(); /* unknown to HIP: plain host memory */
                return 0;
        }
        if (a.type == hipMemoryTypeDevice) {
                hipDeviceptr_t base;
                size_t size;
                *kind = CL_DEVICE;
                *dev = a.device;
                if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t) p) == hipSuccess) {
                        *rbase = (uintptr_t) base;
                        *rsize = size;
                } else {
                        (void) hipGetLastError();
                }
                return (uint64_t) (uintptr_t) p;
        }
        if (a.type == hipMemoryTypeManaged || a.type == hipMemoryTypeUnified) {
                *kind = CL_MANAGED;
                return (uint64_t) (uintptr_t) p;
        }
        if (a.type == hipMemoryTypeHost && a.devicePointer &&
            isal_hip_knob(ISAL_HIP_KNOB_PINNED_DIRECT) != 0) {
                /* attributes describe p itself (the mapping of the allocation
                 * base plus p's offset into it) */
                const char *last = (const char *) p + (len ? len - 1 : 0);
                if (len > 1) {
                        if (hipPointerGetAttributes(&z, last) != hipSuccess) {
                                (void) hipGetLastError();
                                return 0;
                        }
                        if (z.type != hipMemoryTypeHost || z.device != a.device ||
                            (const char *) z.devicePointer != (const char *) a.devicePointer + (len - 1))
                                return 0;
                }
                *kind = CL_PINNED;
                *dev = a.device;
                return (uint64_t) (uintptr_t) a.devicePointer;
        }
        return 0;
}

/* The device a drop-in call runs on (isal_hip.h). The reference API has no
 * device argument (erasure_code.h:108-110), so it comes from the shards: the
 * device that holds the call's device-resident (hipMalloc) shards — they must
 * all be on one; managed memory does not bind a device — else the caller's
 * current device. A page-locked host shard is used in place only through the
 * mapping made for the chosen device (its own); otherwise it is staged. */
int
isal_hip_route_device(int n, const int *kind, const int *dev, int cur, int *bad, int *in_place)
{
        int i, owner = -1;
        if (bad)
                *bad = -1;
        if (n < 0 || (n > 0 && (!kind || !dev)))
                return -3;
        for (i = 0; i < n; i++) {
                if (kind[i] != CL_DEVICE)
                        continue;
                if (owner < 0) {
                        owner = dev[i];
                } else if (dev[i] != owner) {
                        if (bad)
                                *bad = i;
                        return -2;
                }
        }
        if (owner < 0)
                owner = cur;
        if (in_place)
                for (i = 0; i < n; i++)
                        in_place[i] = kind[i] == CL_DEVICE || kind[i] == CL_MANAGED ||
                                      (kind[i] == CL_PINNED && owner >= 0 && dev[i] == owner);
        return owner;
}

/* Device allocations already seen by one call: a shard inside one of them is
 * device memory too, with no HIP query (a stripe's shards usually come from
 * one or two allocations: 14 queries of ~0.4 us become one or two). Only
 * within one call — a later call may find the memory freed and reused. */
#define SEEN_MAX 4
typedef struct {
        int n;
        uintptr_t lo[SEEN_MAX], hi[SEEN_MAX];
        int dev[SEEN_MAX];
} seen_t;

/* the device of the seen allocation holding [p, p + len), or -1 */
static int
seen_dev(const seen_t *sn, const void *p, size_t len)
{
        const uintptr_t a = (uintptr_t) p;
        int i;
        for (i = 0; i < sn->n; i++)
                if (a >= sn->lo[i] && a < sn->hi[i] && len <= sn->hi[i] - a)
                        return sn->dev[i];
        return -1;
}

static void
seen_add(seen_t *sn, uintptr_t base, size_t size, int dev)
{
        if (size && dev >= 0 && sn->n < SEEN_MAX) {
                sn->lo[sn->n] = base;
                sn->hi[sn->n] = base + size;
                sn->dev[sn->n] = dev;
                sn->n++;
        }
}

/* ---- the generic synchronous call --------------------------------------- */

enum { OP_ENCODE = ISAL_HIP_OP_ENCODE, OP_UPDATE = ISAL_HIP_OP_UPDATE, OP_VERIFY = ISAL_HIP_OP_VERIFY };

/*
 * Routes of one synchronous call:
 *   cpu        every shard host-resident and (k + rows) * len <= cpu_max_bytes
 *              (ISAL_HIP_BACKEND=auto), or ISAL_HIP_BACKEND=cpu, or no GPU:
 *              ec_cpu.c. The routing itself still asks HIP (once per process
 *              for the device count, then hipPointerGetAttributes per shard
 *              pointer, ~1 us each), so even ISAL_HIP_BACKEND=cpu initialises
 *              the HIP runtime when a GPU is present; the arithmetic makes no
 *              HIP call;
 *   zero-copy  len * (k + rows) <= ZC_BYTES: pointer table, coefficient tables,
 *              host-resident shards and verify slots all live in the pinned
 *              buffer and the kernel reads/writes them over PCIe — the call is
 *              one launch and one stream sync;
 *   packed     host-staged bytes <= PACK_BYTES: the same layout, moved with one
 *              H2D and one D2H DMA into/out of HBM;
 *   chunked    larger: shards staged per column chunk (gpu_chunked below).
 * A HIP failure in a host-resident call hands the columns not yet final to the
 * CPU route; with any device-resident shard (or ISAL_HIP_BACKEND=gpu) it aborts.
 */
#define ZC_BYTES ((size_t) 256 << 10)
#define PACK_BYTES ((size_t) 4 << 20)

/* Byte layout of the argument buffer of one call. */
typedef struct {
        size_t ptr_bytes, args_bytes, slots_off, slots_bytes, stage_off, slot, total;
} layout_t;

static layout_t
call_layout(int op, int len, int k, int rows, int nptr, int nstage)
{
        layout_t L;
        L.ptr_bytes = ((size_t) nptr * 8 + 15) & ~(size_t) 15;
        L.args_bytes = L.ptr_bytes + ((isal_hip_tables_dwords(k, rows) * 4 + 15) & ~(size_t) 15);
        L.slots_off = L.args_bytes;
        L.slots_bytes = op == OP_VERIFY ? (size_t) EC_VERIFY_SLOTS(rows) * 8 : 0;
        L.stage_off = (L.slots_off + L.slots_bytes + 255) & ~(size_t) 255;
        L.slot = ((size_t) len + 255) & ~(size_t) 255;
        L.total = L.stage_off + L.slot * (size_t) nstage;
        return L;
}

static unsigned long long
min_slot(const unsigned long long *slots, int n)
{
        unsigned long long m = ~0ull;
        int i;
        for (i = 0; i < n; i++)
                if (slots[i] < m)
                        m = slots[i];
        return m;
}

/* Enqueue one chunk's kernel(s) with the argument block at `args` (device or
 * zero-copy view). For OP_VERIFY *nslots receives the number of slots written
 * at args + L->slots_off. */
static hipError_t
launch_op(ctx_t *c, int op, char *args, const layout_t *L, int nptr, int nsrc, int clen,
          long long c0, int k, int rows, int vec_i, int vec16, const isal_hip_encmask *em, int *nslots)
{
        const uint64_t *ptrs = (const uint64_t *) args;
        const uint32_t *tbl = (const uint32_t *) (args + L->ptr_bytes);
        *nslots = 0;
        if (op == OP_VERIFY)
                return (hipError_t) isal_hip_launch_verify(
                        ptrs, nptr, 0, nsrc, tbl, clen, k, rows, c0,
                        (unsigned long long *) (args + L->slots_off), nslots, vec16, em, c->stream);
        if (op == OP_ENCODE)
                return (hipError_t) isal_hip_launch_encode(ptrs, nptr, 0, nsrc, tbl, clen, k, rows,
                                                           1, vec16, em, c->stream);
        return (hipError_t) isal_hip_launch_update(ptrs, nptr, 0, nsrc, tbl, clen, k, rows, vec_i,
                                                   1, vec16, c->stream);
}

/* Outcome of a GPU attempt: on failure `what`/`err` name the HIP call and
 * columns [0, done) are final, so a fallback redoes only [done, len). An
 * update (read-modify-write) that failed while copying a chunk's parity back
 * also reports how many output rows of [done, chunk_end) had their copy
 * enqueued (rows_out): those must not be folded twice. */
typedef struct {
        hipError_t err;
        const char *what;
        long long done, chunk_end;
        int rows_out;
        unsigned long long first_bad;
} gpu_res;

/* Fault injection (tests): ISAL_HIP_FAULT=<site> makes every GPU-routed call
 * fail at that site as if the HIP call there had returned an error, without
 * issuing it — the fallback paths then run for real. Sites: */
enum {
        FAULT_NONE = 0,
        FAULT_ALLOC = 1,  /* staging / argument buffer allocation */
        FAULT_H2D = 2,    /* a host-to-device copy */
        FAULT_LAUNCH = 3, /* the kernel launch */
        FAULT_D2H = 4,    /* the device-to-host copy of output row 1 (chunked) or of the outputs */
        FAULT_SYNC = 5,   /* the final stream synchronisation */
};

/* ISAL_HIP_FAULT_CHUNK=n narrows the fault to column chunk n of a call, so
 * the fallback also runs after earlier chunks finished on the GPU. */
static int
fault_at(int site, long long chunk)
{
        const long long fc = isal_hip_knob(ISAL_HIP_KNOB_FAULT_CHUNK);
        return site != FAULT_NONE && isal_hip_knob(ISAL_HIP_KNOB_FAULT) == site &&
               (fc < 0 || fc == chunk);
}

#define GPU_TRY_ATC(r, site, chunk, call)                                                          \
        do {                                                                                       \
                hipError_t e_ = fault_at(site, chunk) ? hipErrorOutOfMemory : (call);              \
                if (e_ != hipSuccess) {                                                            \
                        (r).err = e_;                                                              \
                        (r).what = #call;                                                          \
                        return (r);                                                                \
                }                                                                                  \
        } while (0)

#define GPU_TRY_AT(r, site, call) GPU_TRY_ATC(r, site, 0, call)

#define GPU_TRY(r, call)                                                                           \
        do {                                                                                       \
                hipError_t e_ = (call);                                                            \
                if (e_ != hipSuccess) {                                                            \
                        (r).err = e_;                                                              \
                        (r).what = #call;                                                          \
                        return (r);                                                                \
                }                                                                                  \
        } while (0)

/* zero-copy and packed modes (whole shards, one chunk). Host outputs are
 * written only after the stream completed, so a failure leaves them untouched. */
static gpu_res
gpu_small(ctx_t *c, int op, int len, int k, int rows, int vec_i, const unsigned char *gftbls,
          unsigned char *const *src, int nsrc, unsigned char *const *dst, const uint64_t *view,
          int nstage, int zero_copy, const uint32_t *tbl, const isal_hip_encmask *em)
{
        gpu_res r = {hipSuccess, NULL, 0, 0, 0, ~0ull};
        int nptr = nsrc + rows, i, s, first_out = -1, vec16 = 1, nslots;
        layout_t L = call_layout(op, len, k, rows, nptr, nstage);
        char *h, *dv;
        size_t upload;
        uint64_t *h_ptrs;

        GPU_TRY_AT(r, FAULT_ALLOC, ensure_args(c, L.total));
        h = (char *) c->h_args;
        dv = zero_copy ? (char *) c->h_args_dev : (char *) c->d_args; /* what kernels see */
        h_ptrs = (uint64_t *) h;
        memcpy(h + L.ptr_bytes, tbl, isal_hip_tables_dwords(k, rows) * 4);
        upload = L.args_bytes;
        for (i = 0, s = 0; i < nptr; i++) {
                unsigned char *host = i < nsrc ? src[i] : dst[i - nsrc];
                uint64_t d;
                if (view[i]) {
                        d = view[i];
                } else {
                        d = (uint64_t) (uintptr_t) (dv + L.stage_off + (size_t) s * L.slot);
                        if (i < nsrc || op != OP_ENCODE) {
                                memcpy(h + L.stage_off + (size_t) s * L.slot, host, (size_t) len);
                                upload = L.stage_off + (size_t) (s + 1) * L.slot;
                        }
                        if (i >= nsrc && first_out < 0)
                                first_out = s;
                        s++;
                }
                h_ptrs[i] = d;
                if (d & 15)
                        vec16 = 0;
        }
        if (!zero_copy)
                GPU_TRY_AT(r, FAULT_H2D, hipMemcpyAsync(c->d_args, h, upload, hipMemcpyHostToDevice, c->stream));
        GPU_TRY_AT(r, FAULT_LAUNCH, launch_op(c, op, dv, &L, nptr, nsrc, len, 0, k, rows, vec_i, vec16, em, &nslots));
        if (!zero_copy) {
                if (op == OP_VERIFY)
                        GPU_TRY(r, hipMemcpyAsync(h + L.slots_off, (char *) c->d_args + L.slots_off,
                                                  (size_t) nslots * 8, hipMemcpyDeviceToHost,
                                                  c->stream));
                else if (first_out >= 0)
                        GPU_TRY_AT(r, FAULT_D2H, hipMemcpyAsync(h + L.stage_off + (size_t) first_out * L.slot,
                                                  (char *) c->d_args + L.stage_off +
                                                          (size_t) first_out * L.slot,
                                                  (size_t) (nstage - first_out) * L.slot,
                                                  hipMemcpyDeviceToHost, c->stream));
        }
        GPU_TRY_AT(r, FAULT_SYNC, hipStreamSynchronize(c->stream));
        if (op == OP_VERIFY) {
                r.first_bad = min_slot((const unsigned long long *) (h + L.slots_off), nslots);
        } else {
                for (i = nsrc, s = first_out; i < nptr && s >= 0; i++)
                        if (!view[i])
                                memcpy(dst[i - nsrc], h + L.stage_off + (size_t) s++ * L.slot,
                                       (size_t) len);
        }
        r.done = len;
        return r;
}

/* Issue this thread's share of a chunk's copies on the call's stream (the
 * fault sites of the tests apply to them: an H2D list fails at its first
 * copy, a D2H list at its second). *enq: copies enqueued. */
static hipError_t
issue_copies(ctx_t *c, const copyjob_t *j, int fault_site, long long ci, const char **what, int *enq)
{
        int i;
        hipError_t e;
        *enq = 0;
        for (i = 0; i < j->n; i++) {
                e = fault_at(i == 1 || fault_site == FAULT_H2D ? fault_site : FAULT_NONE, ci)
                            ? hipErrorOutOfMemory
                            : hipMemcpyAsync(j->cp[i].dst, j->cp[i].src, j->cp[i].bytes, j->cp[i].kind,
                                             c->stream);
                if (e != hipSuccess) {
                        *what = j->cp[i].kind == hipMemcpyHostToDevice ? "hipMemcpyAsync(H2D chunk)"
                                                                        : "hipMemcpyAsync(D2H chunk)";
                        return e;
                }
                *enq = i + 1;
        }
        return hipSuccess;
}

static void
job_add(copyjob_t *j, void *dst, const void *src, size_t bytes, hipMemcpyKind kind)
{
        j->cp[j->n].dst = dst;
        j->cp[j->n].src = src;
        j->cp[j->n].bytes = bytes;
        j->cp[j->n].kind = kind;
        j->n++;
}

/* Column-chunked mode: whole shards when nothing is staged, else chunks of at
 * most stage_limit() bytes over all staged shards. r.done advances past every
 * chunk whose outputs are final.
 * With two or more staged shards the chunk's copies are shared with the
 * calling thread's worker (ISAL_HIP_PAR_COPY=0: not): a pageable copy runs
 * synchronously on the thread that issues it with a fixed cost of ~14 us,
 * and a second issuing thread hides part of it (H2D of 2 MiB shards:
 * 36 -> 41 GB/s, profiles/r03/r03_stage_probe_b.jsonl). The worker copies in on
 * s_out (the kernel waits for its event); for an encode it also copies half
 * the parity out after the kernel. An update's parity comes back from this
 * thread alone, in row order, so a failure leaves a known prefix of rows
 * updated (rows_out). */
static gpu_res
gpu_chunked(ctx_t *c, int op, int len, int k, int rows, int vec_i, const unsigned char *gftbls,
            unsigned char *const *src, int nsrc, unsigned char *const *dst, const uint64_t *view,
            int nstage, const uint32_t *tbl, const isal_hip_encmask *em)
{
        gpu_res r = {hipSuccess, NULL, 0, 0, 0, ~0ull};
        int nptr = nsrc + rows, i, nslots, par = 0;
        size_t chunk, slot;
        layout_t L;
        uint64_t *h_ptrs;
        long long c0;
        copyjob_t *win = NULL, *wout = NULL, *mine = NULL;

        if (nstage) {
                size_t per = stage_limit() / (size_t) nstage;
                per &= ~(size_t) 4095;
                if (per < 4096)
                        per = 4096;
                chunk = (size_t) len < per ? (size_t) len : per;
                slot = (chunk + 255) & ~(size_t) 255; /* keep every slot 256-B aligned */
                GPU_TRY_AT(r, FAULT_ALLOC, ensure_stage(c, slot * (size_t) nstage));
        } else {
                chunk = (size_t) len;
                slot = 0;
        }
        if (nstage >= 2 && nptr <= COPYJOB_MAX && isal_hip_knob(ISAL_HIP_KNOB_PAR_COPY) != 0) {
                if (!c->jobs)
                        c->jobs = (copyjob_t *) malloc(3 * sizeof(copyjob_t));
                /* no helper (no memory, no thread): one issuing thread, as before */
                par = c->jobs && ensure_pipe(c) == hipSuccess && outq_start(c) == hipSuccess;
                (void) hipGetLastError();
                if (par) {
                        win = &c->jobs[0];
                        wout = &c->jobs[1];
                        mine = &c->jobs[2];
                }
        }

        L = call_layout(op, len, k, rows, nptr, 0);
        GPU_TRY(r, ensure_args(c, L.stage_off));
        h_ptrs = (uint64_t *) c->h_args;
        memcpy((char *) c->h_args + L.ptr_bytes, tbl, isal_hip_tables_dwords(k, rows) * 4);

        for (c0 = 0; c0 < len; c0 += (long long) chunk) {
                int clen = (int) ((long long) len - c0 < (long long) chunk ? len - c0 : (long long) chunk);
                int s = 0, vec16 = 1, nin = 0, enq = 0;
                const long long ci = c0 / (long long) chunk;
                if (par) {
                        win->n = mine->n = 0;
                        win->after = NULL;
                        win->record = c->ev_in[0];
                }
                for (i = 0; i < nptr; i++) {
                        unsigned char *host = i < nsrc ? src[i] : dst[i - nsrc];
                        uint64_t d;
                        if (view[i]) {
                                d = view[i] + (uint64_t) c0;
                        } else {
                                unsigned char *st = c->d_stage + (size_t) s++ * slot;
                                d = (uint64_t) (uintptr_t) st;
                                /* sources, and outputs of a read-modify-write update or
                                 * of a verify, go in */
                                if (i < nsrc || op != OP_ENCODE) {
                                        if (!par)
                                                GPU_TRY_ATC(r, FAULT_H2D, ci,
                                                            hipMemcpyAsync(st, host + c0, (size_t) clen,
                                                                           hipMemcpyHostToDevice, c->stream));
                                        else
                                                job_add(nin++ & 1 ? win : mine, st, host + c0, (size_t) clen,
                                                        hipMemcpyHostToDevice);
                                }
                        }
                        h_ptrs[i] = d;
                        if (d & 15)
                                vec16 = 0;
                }
                if (par) {
                        hipError_t e, ew;
                        const char *what = NULL;
                        if (win->n)
                                copyjob_post(c->oq, win);
                        e = issue_copies(c, mine, FAULT_H2D, ci, &what, &enq);
                        ew = win->n ? copyjob_wait(c->oq, win) : hipSuccess;
                        if (e == hipSuccess && ew != hipSuccess) {
                                e = ew;
                                what = win->what;
                        }
                        if (e == hipSuccess && win->n)
                                e = hipStreamWaitEvent(c->stream, c->ev_in[0], 0);
                        if (e != hipSuccess) {
                                r.err = e;
                                r.what = what ? what : "hipStreamWaitEvent(helper copies in)";
                                return r;
                        }
                }
                GPU_TRY(r, hipMemcpyAsync(c->d_args, c->h_args, L.args_bytes,
                                          hipMemcpyHostToDevice, c->stream));
                GPU_TRY_ATC(r, FAULT_LAUNCH, ci, launch_op(c, op, (char *) c->d_args, &L, nptr, nsrc, clen, c0, k, rows,
                                     vec_i, vec16, em, &nslots));
                if (op == OP_VERIFY) {
                        GPU_TRY(r, hipMemcpyAsync((char *) c->h_args + L.slots_off,
                                                  (char *) c->d_args + L.slots_off,
                                                  (size_t) nslots * 8, hipMemcpyDeviceToHost,
                                                  c->stream));
                        GPU_TRY(r, hipStreamSynchronize(c->stream));
                        r.first_bad = min_slot(
                                (const unsigned long long *) ((char *) c->h_args + L.slots_off),
                                nslots);
                        r.done = c0 + clen;
                        if (r.first_bad != ~0ull)
                                break;
                        continue;
                }
                s = 0; /* staged slots are in pointer order: outputs follow sources */
                r.chunk_end = c0 + clen;
                r.rows_out = 0;
                if (par && op == OP_ENCODE) {
                        /* encode: half the parity rows leave through the worker */
                        hipError_t e, ew;
                        const char *what = NULL;
                        int nout = 0;
                        wout->n = mine->n = 0;
                        wout->after = c->ev_k[0];
                        wout->record = c->ev_out[0];
                        GPU_TRY(r, hipEventRecord(c->ev_k[0], c->stream));
                        for (i = 0; i < nptr; i++) {
                                if (view[i])
                                        continue;
                                if (i >= nsrc)
                                        job_add(nout++ & 1 ? wout : mine, dst[i - nsrc] + c0,
                                                c->d_stage + (size_t) s * slot, (size_t) clen,
                                                hipMemcpyDeviceToHost);
                                s++;
                        }
                        if (wout->n)
                                copyjob_post(c->oq, wout);
                        e = issue_copies(c, mine, FAULT_D2H, ci, &what, &enq);
                        ew = wout->n ? copyjob_wait(c->oq, wout) : hipSuccess;
                        /* some parity copies may be under way: a failed drain must abort */
                        r.rows_out = enq || wout->n ? 1 : 0;
                        if (e == hipSuccess && ew != hipSuccess) {
                                e = ew;
                                what = wout->what;
                        }
                        if (e == hipSuccess && wout->n)
                                e = fault_at(FAULT_SYNC, ci) ? hipErrorOutOfMemory
                                                             : hipStreamSynchronize(c->s_out);
                        if (e != hipSuccess) {
                                r.err = e;
                                r.what = what ? what : "hipStreamSynchronize(helper copies out)";
                                return r;
                        }
                } else {
                        for (i = 0; i < nptr; i++) {
                                if (view[i])
                                        continue;
                                if (i >= nsrc) {
                                        GPU_TRY_ATC(r, i - nsrc == 1 ? FAULT_D2H : FAULT_NONE, ci,
                                                    hipMemcpyAsync(dst[i - nsrc] + c0,
                                                                   c->d_stage + (size_t) s * slot,
                                                                   (size_t) clen, hipMemcpyDeviceToHost,
                                                                   c->stream));
                                        r.rows_out = i - nsrc + 1;
                                }
                                s++;
                        }
                }
                GPU_TRY_ATC(r, FAULT_SYNC, ci, hipStreamSynchronize(c->stream));
                r.done = c0 + clen;
                r.rows_out = 0;
        }
        r.done = len;
        return r;
}

/* Column-chunk bytes per shard of a pipelined call: ISAL_HIP_CHUNK_KB, else
 * DEFAULT_CHUNK_BYTES. Every chunk costs one copy per staged shard each way,
 * and a copy from or to pageable memory has a fixed cost of ~14 us beside its
 * bytes (profiles/r03/r03_calltrace.txt), so chunks must be large: at 16 MiB
 * shards 4 MiB chunks beat one chunk by 4-9 %, 1 MiB chunks lose 50 %
 * (profiles/r03/r03_chunk_sweep*.jsonl). */
static size_t
chunk_bytes(void)
{
        const long long kb = isal_hip_knob(ISAL_HIP_KNOB_CHUNK_KB);
        return kb > 0 ? (size_t) kb << 10 : DEFAULT_CHUNK_BYTES;
}

/* Output copies of chunk ci (staging set ci % PIPE_NBUF) on s_out, after its
 * kernel. *rows_out: output rows whose copy was enqueued. */
static hipError_t
copy_out_chunk(ctx_t *c, const outq_t *q, long long ci, const char **what, int *rows_out)
{
        const long long p0 = ci * (long long) q->chunk;
        const int plen = (int) ((long long) q->len - p0 < (long long) q->chunk ? q->len - p0
                                                                                : (long long) q->chunk);
        const int b = (int) (ci % PIPE_NBUF);
        unsigned char *stage = c->d_stage + (size_t) b * q->set_bytes;
        hipError_t e;
        int i, s = 0;
        *rows_out = 0;
        if ((e = hipStreamWaitEvent(c->s_out, c->ev_k[b], 0)) != hipSuccess) {
                *what = "hipStreamWaitEvent(copy-out)";
                return e;
        }
        for (i = 0; i < q->nptr; i++) {
                if (q->view[i])
                        continue;
                if (i >= q->nsrc) {
                        e = fault_at(i - q->nsrc == 1 ? FAULT_D2H : FAULT_NONE, ci)
                                    ? hipErrorOutOfMemory
                                    : hipMemcpyAsync(q->dst[i - q->nsrc] + p0, stage + (size_t) s * q->slot,
                                                     (size_t) plen, hipMemcpyDeviceToHost, c->s_out);
                        if (e != hipSuccess) {
                                *what = "hipMemcpyAsync(D2H chunk)";
                                return e;
                        }
                        *rows_out = i - q->nsrc + 1;
                }
                s++;
        }
        if ((e = hipEventRecord(c->ev_out[b], c->s_out)) != hipSuccess)
                *what = "hipEventRecord(copy-out)";
        return e;
}

static void
run_copyjob(ctx_t *c, copyjob_t *j)
{
        int i;
        j->err = hipSuccess;
        j->what = NULL;
        if (j->after && (j->err = hipStreamWaitEvent(c->s_out, j->after, 0)) != hipSuccess) {
                j->what = "hipStreamWaitEvent(helper copies)";
                return;
        }
        for (i = 0; i < j->n; i++)
                if ((j->err = hipMemcpyAsync(j->cp[i].dst, j->cp[i].src, j->cp[i].bytes, j->cp[i].kind,
                                             c->s_out)) != hipSuccess) {
                        j->what = "hipMemcpyAsync(helper copies)";
                        return;
                }
        if (j->record && (j->err = hipEventRecord(j->record, c->s_out)) != hipSuccess)
                j->what = "hipEventRecord(helper copies)";
}

static void
copyjob_post(outq_t *q, copyjob_t *j)
{
        pthread_mutex_lock(&q->mu);
        q->job = j;
        q->job_state = 1;
        pthread_cond_broadcast(&q->cv);
        pthread_mutex_unlock(&q->mu);
}

/* Wait until the worker has issued the posted job's copies (pageable ones
 * are complete by then); its error. */
static hipError_t
copyjob_wait(outq_t *q, copyjob_t *j)
{
        pthread_mutex_lock(&q->mu);
        while (q->job_state == 1)
                pthread_cond_wait(&q->cv, &q->mu);
        q->job_state = 0;
        q->job = NULL;
        pthread_mutex_unlock(&q->mu);
        return j->err;
}

static void *
outq_main(void *arg)
{
        ctx_t *c = (ctx_t *) arg;
        outq_t *q = c->oq;
        (void) hipSetDevice(c->device);
        pthread_mutex_lock(&q->mu);
        for (;;) {
                long long ci;
                const char *what = NULL;
                int rows_out;
                hipError_t e;
                while (!q->quit && q->job_state != 1 &&
                       !(q->active && q->err == hipSuccess && q->handled < q->posted))
                        pthread_cond_wait(&q->cv, &q->mu);
                if (q->quit)
                        break;
                if (q->job_state == 1) {
                        copyjob_t *j = q->job;
                        pthread_mutex_unlock(&q->mu);
                        run_copyjob(c, j);
                        pthread_mutex_lock(&q->mu);
                        q->job_state = 2;
                        pthread_cond_broadcast(&q->cv);
                        continue;
                }
                ci = q->handled;
                pthread_mutex_unlock(&q->mu);
                e = copy_out_chunk(c, q, ci, &what, &rows_out);
                pthread_mutex_lock(&q->mu);
                if (e != hipSuccess) {
                        q->err = e;
                        q->what = what;
                        q->fail_chunk = ci;
                        q->rows_out = rows_out;
                } else {
                        q->handled = ci + 1;
                }
                pthread_cond_broadcast(&q->cv);
        }
        pthread_mutex_unlock(&q->mu);
        return NULL;
}

/* Copy-out helpers alive in the process, at most max_helpers(): each is a
 * thread with two streams of its own, and they all share the process's few
 * hardware queues (isal_hip.h, "routing"). */
static int g_helpers;
#define DEFAULT_MAX_HELPERS 8

static int
max_helpers(void)
{
        const long long v = isal_hip_knob(ISAL_HIP_KNOB_MAX_HELPERS);
        return v >= 0 ? (int) v : DEFAULT_MAX_HELPERS;
}

static hipError_t
outq_start(ctx_t *c)
{
        outq_t *q;
        if (c->oq)
                return hipSuccess;
        if (__atomic_add_fetch(&g_helpers, 1, __ATOMIC_ACQ_REL) > max_helpers()) {
                __atomic_sub_fetch(&g_helpers, 1, __ATOMIC_ACQ_REL);
                return hipErrorNotSupported; /* over the cap: issue copies alone */
        }
        q = (outq_t *) calloc(1, sizeof(*q));
        if (!q) {
                __atomic_sub_fetch(&g_helpers, 1, __ATOMIC_ACQ_REL);
                return hipErrorOutOfMemory;
        }
        pthread_mutex_init(&q->mu, NULL);
        pthread_cond_init(&q->cv, NULL);
        c->oq = q;
        if (pthread_create(&q->th, NULL, outq_main, c) != 0) {
                pthread_mutex_destroy(&q->mu);
                pthread_cond_destroy(&q->cv);
                free(q);
                c->oq = NULL;
                __atomic_sub_fetch(&g_helpers, 1, __ATOMIC_ACQ_REL);
                return hipErrorOutOfMemory;
        }
        return hipSuccess;
}

static void
outq_stop(ctx_t *c)
{
        outq_t *q = c->oq;
        pthread_mutex_lock(&q->mu);
        q->quit = 1;
        pthread_cond_broadcast(&q->cv);
        pthread_mutex_unlock(&q->mu);
        pthread_join(q->th, NULL);
        pthread_mutex_destroy(&q->mu);
        pthread_cond_destroy(&q->cv);
        free(q);
        c->oq = NULL;
        __atomic_sub_fetch(&g_helpers, 1, __ATOMIC_ACQ_REL);
}

/* Wait until the worker has enqueued the copies of chunks [0, n) or failed;
 * returns its error. */
static hipError_t
outq_wait(outq_t *q, long long n)
{
        hipError_t e;
        pthread_mutex_lock(&q->mu);
        while (q->err == hipSuccess && q->handled < n)
                pthread_cond_wait(&q->cv, &q->mu);
        e = q->err;
        pthread_mutex_unlock(&q->mu);
        return e;
}

/*
 * Pipelined column chunks: large host-resident encode / update calls. Chunk i
 * flows through staging set i % PIPE_NBUF in HBM: H2D of its sources (and of
 * its parity, for an update) on s_in, argument upload + kernel on the call's
 * stream, D2H of its outputs on s_out, chained by events. The calling thread
 * stages in and launches; the copy-out worker (outq) issues the D2H copies,
 * so that the H2D of chunk i + 1, the kernel of chunk i and the D2H of chunk
 * i - 1 run at once even for pageable host buffers. Host memory is written
 * only by the D2H copies, in chunk order: r.done is the end of the last chunk
 * whose output copies were all enqueued, rows_out counts the rows of the next
 * chunk whose copy was enqueued when an enqueue failed (as gpu_chunked). The
 * caller quiesces every stream before it trusts either.
 */
static gpu_res
gpu_pipelined(ctx_t *c, int op, int len, int k, int rows, int vec_i, const unsigned char *gftbls,
              unsigned char *const *src, int nsrc, unsigned char *const *dst, const uint64_t *view,
              int nstage, const uint32_t *tbl, const isal_hip_encmask *em)
{
        gpu_res r = {hipSuccess, NULL, 0, 0, 0, ~0ull};
        const int nptr = nsrc + rows;
        size_t chunk = chunk_bytes(), per, slot, set_bytes, astride;
        long long nchunks, ci, launched = 0;
        layout_t L;
        outq_t *q;
        int b, i;

        per = stage_limit() / ((size_t) nstage * PIPE_NBUF) & ~(size_t) 4095;
        if (chunk > per)
                chunk = per < 4096 ? 4096 : per;
        if (chunk >= (size_t) len) /* one chunk: nothing to overlap */
                return gpu_chunked(c, op, len, k, rows, vec_i, gftbls, src, nsrc, dst, view, nstage, tbl, em);
        if (!c->oq && outq_start(c) != hipSuccess) {
                /* no helper for this thread (the process cap, or no thread):
                 * one chunk at a time, copies issued by this thread alone */
                (void) hipGetLastError();
                return gpu_chunked(c, op, len, k, rows, vec_i, gftbls, src, nsrc, dst, view, nstage, tbl, em);
        }
        slot = (chunk + 255) & ~(size_t) 255;
        set_bytes = slot * (size_t) nstage;
        GPU_TRY_AT(r, FAULT_ALLOC, ensure_stage(c, set_bytes * PIPE_NBUF));
        GPU_TRY_AT(r, FAULT_ALLOC, ensure_pipe(c));
        GPU_TRY_AT(r, FAULT_ALLOC, outq_start(c));
        L = call_layout(op, len, k, rows, nptr, 0);
        astride = (L.args_bytes + 255) & ~(size_t) 255;
        GPU_TRY_AT(r, FAULT_ALLOC, ensure_args(c, astride * PIPE_NBUF));
        /* one argument region per staging set: pointer table + coefficient tables */
        memcpy((char *) c->h_args + L.ptr_bytes, tbl, isal_hip_tables_dwords(k, rows) * 4);
        for (b = 1; b < PIPE_NBUF; b++)
                memcpy((char *) c->h_args + b * astride + L.ptr_bytes, (char *) c->h_args + L.ptr_bytes,
                       L.args_bytes - L.ptr_bytes);
        nchunks = ((long long) len + (long long) chunk - 1) / (long long) chunk;

        q = c->oq;
        pthread_mutex_lock(&q->mu);
        q->nsrc = nsrc;
        q->nptr = nptr;
        q->len = len;
        q->view = view;
        q->dst = dst;
        q->chunk = chunk;
        q->slot = slot;
        q->set_bytes = set_bytes;
        q->posted = q->handled = 0;
        q->err = hipSuccess;
        q->active = 1;
        pthread_mutex_unlock(&q->mu);

        for (ci = 0; ci < nchunks && r.err == hipSuccess; ci++) {
                const long long c0 = ci * (long long) chunk;
                const int clen = (int) ((long long) len - c0 < (long long) chunk ? len - c0 : (long long) chunk);
                char *h, *dargs;
                unsigned char *stage;
                uint64_t *h_ptrs;
                int s = 0, vec16 = 1, nslots;
                hipError_t e = hipSuccess;
                const char *what = NULL;
                b = (int) (ci % PIPE_NBUF);
                h = (char *) c->h_args + b * astride;
                dargs = (char *) c->d_args + b * astride;
                stage = c->d_stage + b * set_bytes;
                h_ptrs = (uint64_t *) h;
#define PIPE_STEP(site, call)                                                                      \
        do {                                                                                       \
                if (e == hipSuccess) {                                                             \
                        e = fault_at(site, ci) ? hipErrorOutOfMemory : (call);                     \
                        if (e != hipSuccess)                                                       \
                                what = #call;                                                      \
                }                                                                                  \
        } while (0)
                if (ci >= PIPE_NBUF) {
                        /* staging set b is free once chunk ci - NBUF's parity has left it
                         * (its copy-out event recorded), and argument region b once that
                         * chunk's upload ran */
                        if ((e = outq_wait(q, ci - PIPE_NBUF + 1)) != hipSuccess)
                                break; /* the worker's failure, reported below */
                        PIPE_STEP(FAULT_SYNC, hipEventSynchronize(c->ev_k[b]));
                        PIPE_STEP(FAULT_NONE, hipStreamWaitEvent(c->s_in, c->ev_out[b], 0));
                }
                for (i = 0; i < nptr && e == hipSuccess; i++) {
                        unsigned char *host = i < nsrc ? src[i] : dst[i - nsrc];
                        uint64_t d;
                        if (view[i]) {
                                d = view[i] + (uint64_t) c0;
                        } else {
                                unsigned char *st = stage + (size_t) s++ * slot;
                                d = (uint64_t) (uintptr_t) st;
                                if (i < nsrc || op != OP_ENCODE)
                                        PIPE_STEP(FAULT_H2D, hipMemcpyAsync(st, host + c0, (size_t) clen,
                                                                            hipMemcpyHostToDevice, c->s_in));
                        }
                        h_ptrs[i] = d;
                        if (d & 15)
                                vec16 = 0;
                }
                PIPE_STEP(FAULT_NONE, hipEventRecord(c->ev_in[b], c->s_in));
                PIPE_STEP(FAULT_NONE, hipStreamWaitEvent(c->stream, c->ev_in[b], 0));
                PIPE_STEP(FAULT_NONE, hipMemcpyAsync(dargs, h, L.args_bytes, hipMemcpyHostToDevice, c->stream));
                PIPE_STEP(FAULT_LAUNCH, (hipError_t) launch_op(c, op, dargs, &L, nptr, nsrc, clen, c0, k, rows,
                                                               vec_i, vec16, em, &nslots));
                PIPE_STEP(FAULT_NONE, hipEventRecord(c->ev_k[b], c->stream));
#undef PIPE_STEP
                if (e != hipSuccess) {
                        r.err = e;
                        r.what = what;
                        break;
                }
                launched = ci + 1;
                pthread_mutex_lock(&q->mu);
                q->posted = launched;
                pthread_cond_signal(&q->cv);
                pthread_mutex_unlock(&q->mu);
        }
        /* let the worker finish the chunks that were launched (or fail) */
        (void) outq_wait(q, launched);
        pthread_mutex_lock(&q->mu);
        q->active = 0;
        if (q->err != hipSuccess) { /* the first failure in chunk order is the worker's */
                r.err = q->err;
                r.what = q->what;
                r.done = q->fail_chunk * (long long) chunk;
                r.chunk_end = r.done + (long long) chunk < len ? r.done + (long long) chunk : len;
                r.rows_out = q->rows_out;
        } else {
                r.done = q->handled * (long long) chunk < len ? q->handled * (long long) chunk : len;
                r.rows_out = 0;
        }
        pthread_mutex_unlock(&q->mu);
        if (r.err != hipSuccess)
                return r;
        GPU_TRY_ATC(r, FAULT_SYNC, nchunks - 1, hipStreamSynchronize(c->s_out));
        r.done = len;
        return r;
}

/* Wait for everything a call queued; the first error, if any. */
static hipError_t
quiesce(ctx_t *c)
{
        hipError_t e = hipStreamSynchronize(c->stream), e2;
        if (c->pipe_ready) {
                if ((e2 = hipStreamSynchronize(c->s_in)) != hipSuccess && e == hipSuccess)
                        e = e2;
                if ((e2 = hipStreamSynchronize(c->s_out)) != hipSuccess && e == hipSuccess)
                        e = e2;
        }
        return e;
}

/* Kernel-argument encode (isal_hip_launch_encode_karg): one launch, no
 * argument upload — for device-resident, 16-byte aligned shards of a
 * one-pass stripe that fits the 2 KiB argument block. */
static int
karg_fits(int op, int len, int k, int rows, const uint64_t *view, int nptr)
{
        int i;
        if (len < 16 || rows > EC_MAX_ROWS_PER_PASS || nptr > ISAL_HIP_KARG_PTRS ||
            isal_hip_tables_dwords(op == OP_UPDATE ? 1 : k, rows) > ISAL_HIP_KARG_TBL ||
            isal_hip_knob(ISAL_HIP_KNOB_KARG) == 0)
                return 0;
        for (i = 0; i < nptr; i++)
                if (view[i] & 15)
                        return 0;
        return 1;
}

/* The completion words of kernel-argument calls, allocated on a thread's
 * first such call: device {counters = 0 (isal_hip_kdone), verify result = ~0}, host mailbox
 * (page-locked, coherent: the kernel's system-scope stores land in it with no
 * cached copy in between). */
#define KDONE_CNT_BYTES ((size_t) ISAL_HIP_KDONE_WORDS * 4)
static hipError_t
ensure_done(ctx_t *c)
{
        static const unsigned long long res_init = ~0ull;
        hipError_t e;
        void *h = NULL;
        if (c->d_done)
                return hipSuccess;
        if ((e = hipMalloc(&c->d_done, KDONE_CNT_BYTES + 64)) != hipSuccess)
                return e;
        if ((e = hipMemset(c->d_done, 0, KDONE_CNT_BYTES)) != hipSuccess ||
            (e = hipMemcpy((char *) c->d_done + KDONE_CNT_BYTES, &res_init, 8, hipMemcpyHostToDevice)) !=
                    hipSuccess ||
            (e = hipHostMalloc(&h, 64, hipHostMallocCoherent)) != hipSuccess ||
            (e = hipHostGetDevicePointer(&c->h_mail_dev, h, 0)) != hipSuccess) {
                (void) hipFree(c->d_done);
                if (h)
                        (void) hipHostFree(h);
                c->d_done = NULL;
                return e;
        }
        memset(h, 0, 64);
        c->h_mail = (volatile unsigned long long *) h;
        return hipSuccess;
}

static double
now_s(void)
{
        struct timespec t;
        clock_gettime(CLOCK_MONOTONIC, &t);
        return (double) t.tv_sec + 1e-9 * (double) t.tv_nsec;
}

/* Wait for call `seq` of this thread: spin on the mailbox the kernel's last
 * workgroup writes (the runtime's completion signal and wake-up cost ~9 us
 * more). Bounded: after SPIN_S seconds without it the stream is
 * synchronised, so a kernel that faulted is reported through the runtime and
 * a slow one is simply waited for. The stream is still synchronised every
 * SYNC_EVERY calls (the kernels have long ended by then) so the runtime
 * retires its launch records. */
static unsigned long long g_slow_waits;

unsigned long long
isal_hip_slow_waits(void)
{
        return __atomic_load_n(&g_slow_waits, __ATOMIC_RELAXED);
}

#define DONE_SPIN_S 0.02
#define DONE_YIELD_S 50e-6 /* then yield the CPU between polls: callers may outnumber cores */
#define DONE_SYNC_EVERY 64
static hipError_t
wait_done(ctx_t *c, unsigned long long seq)
{
        hipError_t e;
        unsigned spins = 0;
        int yield = 0;
        double t0 = 0;
        while (c->h_mail[0] != seq) {
                if (yield)
                        sched_yield();
                else
                        __builtin_ia32_pause();
                if ((++spins & 63) == 0) {
                        const double t = now_s();
                        if (t0 == 0)
                                t0 = t;
                        else if (t - t0 > DONE_SPIN_S)
                                break;
                        else
                                yield = t - t0 > DONE_YIELD_S;
                }
        }
        if (c->h_mail[0] != seq) {
                __atomic_add_fetch(&g_slow_waits, 1ull, __ATOMIC_RELAXED);
                if ((e = hipStreamSynchronize(c->stream)) != hipSuccess)
                        return e;
                c->unsynced = 0;
                if (c->h_mail[0] != seq)
                        return hipErrorUnknown; /* the kernel ended without writing its completion word */
                return hipSuccess;
        }
        __atomic_thread_fence(__ATOMIC_ACQUIRE); /* the result word was written before seq */
        if (++c->unsynced >= DONE_SYNC_EVERY) {
                c->unsynced = 0;
                return hipStreamSynchronize(c->stream);
        }
        return hipSuccess;
}

/* The LDS product tables of the thread's cached coefficients (ctx_tables) on
 * the device, uploaded when the coefficients change; NULL (the call then
 * keeps the v_perm kernel) when memory runs out. The upload is synchronous and
 * no kernel of this context is in flight: every drop-in call has completed
 * before the next one starts. */
static const uint64_t *
ctx_ldsx(ctx_t *c, int k, int rows)
{
        const size_t nw = isal_hip_ldsx_words(k, rows);
        uint64_t *h;
        if (c->ldsx_ok)
                return c->d_ldsx;
        if (nw > c->ldsx_cap) {
                if (c->d_ldsx)
                        (void) hipFree(c->d_ldsx);
                c->d_ldsx = NULL;
                c->ldsx_cap = 0;
                if (hipMalloc((void **) &c->d_ldsx, nw * 8) != hipSuccess) {
                        c->d_ldsx = NULL;
                        return NULL;
                }
                c->ldsx_cap = nw;
        }
        if (!(h = (uint64_t *) malloc(nw * 8)))
                return NULL;
        isal_hip_build_ldsx_tables_coef(k, rows, c->tcoef, h);
        if (hipMemcpy(c->d_ldsx, h, nw * 8, hipMemcpyHostToDevice) == hipSuccess)
                c->ldsx_ok = 1;
        free(h);
        return c->ldsx_ok ? c->d_ldsx : NULL;
}

/* A kernel-argument call's arguments, in the 2 KiB block the kernels read
 * from their kernarg segment. mail: the completion mailbox is used (every
 * shard is hipMalloc memory: managed memory the host may read directly is
 * left to hipStreamSynchronize, which also makes the host's view coherent;
 * ISAL_HIP_KARG_DONE=0 turns the mailbox off). A verify needs the mailbox. */
static gpu_res
gpu_karg(ctx_t *c, int op, int len, int k, int rows, int vec_i, const uint64_t *view, const uint32_t *tbl,
         const isal_hip_encmask *em, int mail)
{
        static int inflight; /* kernel-argument calls of the process in flight (lane width) */
        static const char *const launch_what[] = {"encode launch (kernel arguments)",
                                                  "update launch (kernel arguments)",
                                                  "verify launch (kernel arguments)"};
        static const char *const wait_what[] = {"encode completion (kernel arguments)",
                                                "update completion (kernel arguments)",
                                                "verify completion (kernel arguments)"};
        gpu_res r = {hipSuccess, NULL, 0, 0, 0, ~0ull};
        const int nsrc = op == OP_UPDATE ? 1 : k;
        isal_hip_kdone d = {NULL, NULL, NULL, 0ull};
        isal_hip_karg a;
        hipError_t e;
        int busy;
        memset(&a, 0, sizeof(a));
        memcpy(a.ptrs, view, sizeof(uint64_t) * (size_t) (nsrc + rows));
        if (mail) {
                GPU_TRY_AT(r, FAULT_ALLOC, ensure_done(c));
                d.cnt = (unsigned *) c->d_done;
                d.res = op == OP_VERIFY ? (unsigned long long *) ((char *) c->d_done + KDONE_CNT_BYTES) : NULL;
                d.mail = (unsigned long long *) c->h_mail_dev;
        }
        /* an injected launch failure (tests) launches nothing, as a failed launch */
        if (fault_at(FAULT_LAUNCH, 0)) {
                r.err = hipErrorOutOfMemory;
                r.what = launch_what[op];
                return r;
        }
        if (mail)
                d.seq = ++c->seq;
        if (op == OP_UPDATE) {
                /* one pass: source vec_i's tables for every row are contiguous */
                memcpy(a.tbl, tbl + isal_hip_tables_dwords(vec_i, rows), isal_hip_tables_dwords(1, rows) * 4);
                e = (hipError_t) isal_hip_launch_update_karg(&a, &d, len, rows, c->stream);
        } else {
                memcpy(a.tbl, tbl, isal_hip_tables_dwords(k, rows) * 4);
                busy = __atomic_add_fetch(&inflight, 1, __ATOMIC_RELAXED);
                e = (hipError_t) (op == OP_VERIFY
                                          ? isal_hip_launch_verify_karg(&a, &d, len, k, rows, em, c->stream)
                                          : isal_hip_launch_encode_karg(
                                                    &a, &d, len, k, rows, em, busy,
                                                    isal_hip_karg_ldsx(k, rows) ? ctx_ldsx(c, k, rows) : NULL,
                                                    c->stream));
        }
        if (e == hipSuccess) {
                r.what = wait_what[op];
                e = fault_at(FAULT_SYNC, 0) ? hipErrorOutOfMemory
                    : mail                  ? wait_done(c, d.seq)
                                            : hipStreamSynchronize(c->stream);
        } else {
                r.what = launch_what[op];
        }
        if (op != OP_UPDATE) /* this call is no longer in flight, whatever failed */
                __atomic_sub_fetch(&inflight, 1, __ATOMIC_RELAXED);
        if ((r.err = e) != hipSuccess)
                return r;
        r.what = NULL;
        if (op == OP_VERIFY)
                r.first_bad = c->h_mail[1];
        r.done = len;
        return r;
}

static unsigned long long
cpu_route(int op, long long c0, int len, int k, int rows, int vec_i, const unsigned char *gftbls,
          unsigned char *const *src, int nsrc, unsigned char *const *dst)
{
        __atomic_add_fetch(&g_cpu_calls, 1ull, __ATOMIC_RELAXED);
        return isal_cpu_run(op, c0, len, k, rows, vec_i, gftbls, src, nsrc, dst);
}

/* A call whose device-resident shards sit on two GPUs: no one kernel can
 * reach both (and no CPU route can read either). */
static void
die_mixed(const char *fn, int i0, int d0, int i1, int d1)
{
        fprintf(stderr,
                "isal_hip: %s: device-resident shards on two GPUs (shard %d on device %d, shard %d "
                "on device %d); one call runs on one GPU, aborting\n",
                fn, i0, d0, i1, d1);
        abort();
}

/*
 * OP_ENCODE: dst[l] = XOR_j c[l][j] * src[j], nsrc = k.
 * OP_UPDATE: dst[l] ^= c[l][vec_i] * src[0], nsrc = 1.
 * OP_VERIFY: compare dst[l] with XOR_j c[l][j] * src[j]; nothing is written.
 * Returns ~0 (no mismatch / not a verify) or the first mismatch as
 * column << 8 | row. fn names the entry point in abort messages.
 * The call runs on the device holding its device-resident shards
 * (isal_hip_route_device): the thread's current device is switched to it for
 * the call and restored before returning.
 */
static unsigned long long
run_ec(const char *fn, int op, int len, int k, int rows, int vec_i, const unsigned char *gftbls,
       unsigned char *const *src, int nsrc, unsigned char *const *dst)
{
        const int be = backend();
        const int nptr = nsrc + rows;
        uint64_t view_buf[512], *view;
        int kind_buf[512], dev_buf[512], *kind, *devs;
        static const isal_hip_encmask no_masks;
        const isal_hip_encmask *em = &no_masks;
        const uint32_t *tbl = NULL;
        seen_t sn;
        int i, nstage = 0, ndev = 0, nplain = 0, all_host, cur_dev, run_dev, bad, mail;
        size_t bytes;
        gpu_res r;
        ctx_t *c;

        if (len <= 0 || rows <= 0 || k < 0)
                return ~0ull;
        if (op == OP_UPDATE && (vec_i < 0 || vec_i >= k)) {
                /* Out-of-range vec_i is undefined in the reference (it reads past
                 * gftbls); here it must not become an out-of-bounds GPU access. */
                fprintf(stderr, "isal_hip: ec update with vec_i=%d outside [0,%d): ignored\n",
                        vec_i, k);
                return ~0ull;
        }
        bytes = (size_t) len * (size_t) nptr;
        if (!gpu_present()) {
                if (be == BACKEND_GPU) {
                        fprintf(stderr, "isal_hip: ISAL_HIP_BACKEND=gpu but no GPU is usable\n");
                        abort();
                }
                /* no HIP runtime to ask: every pointer is a host pointer */
                route_log(op, len, k, rows, "cpu", "no GPU");
                return cpu_route(op, 0, len, k, rows, vec_i, gftbls, src, nsrc, dst);
        }

        if (nptr <= 512) {
                view = view_buf;
                kind = kind_buf;
                devs = dev_buf;
        } else {
                view = (uint64_t *) malloc((sizeof(uint64_t) + 2 * sizeof(int)) * (size_t) nptr);
                if (!view) {
                        fprintf(stderr, "isal_hip: out of host memory\n");
                        abort();
                }
                kind = (int *) (view + nptr);
                devs = kind + nptr;
        }
        if (hipGetDevice(&cur_dev) != hipSuccess) {
                (void) hipGetLastError();
                cur_dev = -1; /* no page-locked shard is used in place */
        }
        sn.n = 0;
        for (i = 0; i < nptr; i++) {
                const void *p = i < nsrc ? src[i] : dst[i - nsrc];
                uintptr_t rb = 0;
                size_t rs = 0;
                const int sd = seen_dev(&sn, p, (size_t) len);
                if (sd >= 0) {
                        view[i] = (uint64_t) (uintptr_t) p;
                        kind[i] = CL_DEVICE;
                        devs[i] = sd;
                } else {
                        view[i] = classify(p, (size_t) len, &kind[i], &devs[i], &rb, &rs);
                        if (kind[i] == CL_DEVICE)
                                seen_add(&sn, rb, rs, devs[i]);
                }
        }
        /* the device the call runs on (-1: none known, the caller's current
         * device could not be read) */
        run_dev = isal_hip_route_device(nptr, kind, devs, cur_dev, &bad, NULL);
        if (run_dev == -2) {
                int i0 = 0;
                while (kind[i0] != CL_DEVICE)
                        i0++;
                die_mixed(fn, i0, devs[i0], bad, devs[bad]);
        }
        for (i = 0; i < nptr; i++) {
                const int is_dev = kind[i] == CL_DEVICE || kind[i] == CL_MANAGED;
                /* page-locked memory is used in place only through the run
                 * device's own mapping */
                if (kind[i] == CL_PINNED && devs[i] != run_dev)
                        view[i] = 0;
                nplain += kind[i] == CL_DEVICE;
                /* An update's parity in page-locked host memory is staged, not
                 * written in place: a kernel that failed after it started could
                 * have folded some of it already, and the CPU fallback could not
                 * tell which bytes. (Encode overwrites, verify only reads.) */
                if (op == OP_UPDATE && i >= nsrc && view[i] && !is_dev)
                        view[i] = 0;
                ndev += is_dev;
                nstage += !view[i];
        }
        all_host = ndev == 0;

        if (all_host && (be == BACKEND_CPU ||
                         (be == BACKEND_AUTO &&
                          bytes <= (nstage == 0 ? cpu_max_bytes_pinned() : cpu_max_bytes())))) {
                if (view != view_buf)
                        free(view);
                route_log(op, len, k, rows, "cpu", be == BACKEND_CPU ? "ISAL_HIP_BACKEND=cpu" : "small host call");
                return cpu_route(op, 0, len, k, rows, vec_i, gftbls, src, nsrc, dst);
        }

        /* the shards' device, when the caller's current device is another one */
        if (run_dev != cur_dev && (r.err = hipSetDevice(run_dev)) != hipSuccess)
                die("hipSetDevice (to the device holding the shards)", r.err);
        c = ctx_get(run_dev, &r.err, &r.what);
        if (c && !(tbl = ctx_tables(c, k, rows, gftbls, &em))) {
                r.err = hipErrorOutOfMemory;
                r.what = "ctx_tables (host memory)";
                c = NULL;
        }
        if (c && op == OP_UPDATE)
                em = &no_masks;
        if (!c) {
                r.done = 0;
                r.first_bad = ~0ull;
        } else if (ndev == nptr && (mail = nplain == nptr && isal_hip_knob(ISAL_HIP_KNOB_KARG_DONE) != 0,
                                    op != OP_VERIFY || mail) &&
                   karg_fits(op, len, k, rows, view, nptr)) {
                route_log(op, len, k, rows, "gpu kernel-args", "device shards");
                r = gpu_karg(c, op, len, k, rows, vec_i, view, tbl, em, mail);
        } else if (bytes <= ZC_BYTES || (nstage && (size_t) len * (size_t) nstage <= PACK_BYTES)) {
                const int zc = bytes <= ZC_BYTES;
                route_log(op, len, k, rows, zc ? "gpu zero-copy" : "gpu packed",
                          all_host ? "host shards" : "device shards");
                r = gpu_small(c, op, len, k, rows, vec_i, gftbls, src, nsrc, dst, view, nstage, zc, tbl, em);
        } else {
                const int piped = nstage && op != OP_VERIFY && isal_hip_knob(ISAL_HIP_KNOB_PIPE_CHUNKS) != 0;
                route_log(op, len, k, rows,
                          piped ? "gpu pipelined chunks" : nstage ? "gpu chunked" : "gpu direct (no staging)",
                          all_host ? "host shards" : "device shards");
                r = piped ? gpu_pipelined(c, op, len, k, rows, vec_i, gftbls, src, nsrc, dst, view, nstage, tbl, em)
                          : gpu_chunked(c, op, len, k, rows, vec_i, gftbls, src, nsrc, dst, view, nstage, tbl, em);
        }
        if (view != view_buf)
                free(view);
        if (r.err == hipSuccess) {
                if (run_dev != cur_dev)
                        (void) hipSetDevice(cur_dev);
                return r.first_bad;
        }
        if (!all_host || be == BACKEND_GPU)
                die(r.what, r.err);
        /* all shards host-resident: the call ran on the caller's own device */
        (void) hipGetLastError();
        report_fallback(r.what, r.err);
        /* Nothing queued may still write our outputs: drain every stream of the
         * call. Output copies into host memory were enqueued for [0, done) (and
         * rows_out rows beyond); if the streams cannot be drained their state
         * is unknown and no CPU result may be written over them. */
        if (c && quiesce(c) != hipSuccess && (r.done > 0 || r.rows_out))
                die("draining the streams after a failed call (output state unknown)", r.err);
        if (op == OP_UPDATE && r.rows_out) {
                /* rows [0, rows_out) of [done, chunk_end) are already updated */
                unsigned char *s1 = src[0] + r.done, **d1;
                const int nr = rows - r.rows_out;
                d1 = (unsigned char **) malloc(sizeof(*d1) * (size_t) (nr > 0 ? nr : 1));
                if (!d1)
                        abort();
                for (i = 0; i < nr; i++)
                        d1[i] = dst[r.rows_out + i] + r.done;
                (void) cpu_route(op, 0, (int) (r.chunk_end - r.done), k, nr, vec_i,
                                 gftbls + (size_t) r.rows_out * k * 32, &s1, 1, d1);
                free(d1);
                r.done = r.chunk_end;
        }
        return cpu_route(op, r.done, len, k, rows, vec_i, gftbls, src, nsrc, dst);
}

unsigned long long
isal_hip_run(const char *fn, int op, int len, int k, int rows, int vec_i, const unsigned char *gftbls,
             unsigned char *const *src, int nsrc, unsigned char *const *dst)
{
        return run_ec(fn, op, len, k, rows, vec_i, gftbls, src, nsrc, dst);
}

/* ---- reference data-path ABI ------------------------------------------- */

void
ec_encode_data(int len, int k, int rows, unsigned char *gftbls, unsigned char **data,
               unsigned char **coding)
{
        run_ec("ec_encode_data", OP_ENCODE, len, k, rows, 0, gftbls, data, k, coding);
}

void
ec_encode_data_base(int len, int k, int rows, unsigned char *gftbls, unsigned char **data,
                    unsigned char **coding)
{
        run_ec("ec_encode_data_base", OP_ENCODE, len, k, rows, 0, gftbls, data, k, coding);
}

void
ec_encode_data_update(int len, int k, int rows, int vec_i, unsigned char *gftbls,
                      unsigned char *data, unsigned char **coding)
{
        run_ec("ec_encode_data_update", OP_UPDATE, len, k, rows, vec_i, gftbls, &data, 1, coding);
}

void
ec_encode_data_update_base(int len, int k, int rows, int vec_i, unsigned char *gftbls,
                           unsigned char *data, unsigned char **coding)
{
        run_ec("ec_encode_data_update_base", OP_UPDATE, len, k, rows, vec_i, gftbls, &data, 1, coding);
}

void
gf_vect_dot_prod(int len, int vlen, unsigned char *gftbls, unsigned char **src,
                 unsigned char *dest)
{
        run_ec("gf_vect_dot_prod", OP_ENCODE, len, vlen, 1, 0, gftbls, src, vlen, &dest);
}

void
gf_vect_dot_prod_base(int len, int vlen, unsigned char *gftbls, unsigned char **src,
                      unsigned char *dest)
{
        run_ec("gf_vect_dot_prod_base", OP_ENCODE, len, vlen, 1, 0, gftbls, src, vlen, &dest);
}

void
gf_vect_mad(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src,
            unsigned char *dest)
{
        run_ec("gf_vect_mad", OP_UPDATE, len, vec, 1, vec_i, gftbls, &src, 1, &dest);
}

void
gf_vect_mad_base(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src,
                 unsigned char *dest)
{
        run_ec("gf_vect_mad_base", OP_UPDATE, len, vec, 1, vec_i, gftbls, &src, 1, &dest);
}

/* dest = c * src with c = gftbl[1]; -1 (nothing touched) when len % 32 != 0,
 * as ec_base.c:350-353. */
int
gf_vect_mul(int len, unsigned char *gftbl, void *src, void *dest)
{
        unsigned char *s = (unsigned char *) src, *d = (unsigned char *) dest;
        if (len % 32)
                return -1;
        run_ec("gf_vect_mul", OP_ENCODE, len, 1, 1, 0, gftbl, &s, 1, &d);
        return 0;
}

int
gf_vect_mul_base(int len, unsigned char *gftbl, unsigned char *src, unsigned char *dest)
{
        return gf_vect_mul(len, gftbl, src, dest);
}

/* ---- device of an object's calls ------------------------------------------ */

/* Make dev the calling thread's current device for one call on an object that
 * belongs to it (a batch, a pipeline). Returns the device to restore with
 * isal_hip_dev_leave (-1: no switch was needed), or -2 when the switch failed. */
int
isal_hip_dev_enter(int dev)
{
        int cur;
        if (hipGetDevice(&cur) != hipSuccess) {
                (void) hipGetLastError();
                return -1;
        }
        if (cur == dev)
                return -1;
        if (hipSetDevice(dev) != hipSuccess) {
                (void) hipGetLastError();
                return -2;
        }
        return cur;
}

void
isal_hip_dev_leave(int prev)
{
        if (prev >= 0)
                (void) hipSetDevice(prev);
}

/* ---- batched extension (isal_hip.h) ------------------------------------ */

struct isal_hip_batch {
        int len, k, rows, nstripes, device, vec16;
        uint64_t *d_ptrs;
        uint32_t *d_tbl;
        isal_hip_xrows xr; /* 0/1 parity rows: CRCs derived, not computed */
        isal_hip_encmask em; /* 0/1 rows and columns: XORs instead of lookups */
        /* CRC32C state, allocated on first use: kernel tables + combine plan,
         * and the per-lane partials (crc_kernels.hip) */
        uint64_t *d_ldsx; /* LDS product tables of the wide passes (NULL: not used) */
        isal_hip_crc_geom crc;
        uint32_t *d_crc, *d_part, *d_tail;
        /* CRC64 state, allocated on first use: one table set per variant
         * and pass used (never overwritten, so switching variants needs no
         * device synchronisation) and the per-lane chains. The fused pass
         * (c64_tt tiles per block) and the checksum-only pass (c64_tt_ck)
         * have their own block geometry; the partials are sized for the
         * shorter blocks. */
        int c64_tt, c64_tt_ck;
        uint64_t *d_c64tab[ISAL_HIP_CRC64_NVARIANTS], *d_c64tab_ck[ISAL_HIP_CRC64_NVARIANTS], *d_c64part;
};

/* Every shard of a batch on device dev: hipMalloc memory of dev, managed
 * memory, or page-locked host memory whose device address is its host address.
 * A stripe's shards usually come from a few allocations, so a device range
 * already seen answers without a HIP query. */
static int
batch_check_ptrs(const uint64_t *ptrs, size_t n, size_t len, int dev)
{
        seen_t sn;
        size_t i;
        sn.n = 0;
        for (i = 0; i < n; i++) {
                const void *p = (const void *) (uintptr_t) ptrs[i];
                hipPointerAttribute_t a;
                int sd;
                if (!p)
                        return ISAL_HIP_EINVAL;
                if ((sd = seen_dev(&sn, p, len)) >= 0) {
                        if (sd != dev)
                                return ISAL_HIP_EDEVICE;
                        continue;
                }
                if (hipPointerGetAttributes(&a, p) != hipSuccess) {
                        (void) hipGetLastError();
                        return ISAL_HIP_EINVAL; /* pageable: no kernel can reach it */
                }
                if (a.type == hipMemoryTypeDevice) {
                        hipDeviceptr_t base;
                        size_t size;
                        if (a.device != dev)
                                return ISAL_HIP_EDEVICE;
                        if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t) p) == hipSuccess)
                                seen_add(&sn, (uintptr_t) base, size, a.device);
                        else
                                (void) hipGetLastError();
                } else if (a.type == hipMemoryTypeHost) {
                        if (a.devicePointer != p)
                                return ISAL_HIP_EINVAL;
                } else if (a.type != hipMemoryTypeManaged && a.type != hipMemoryTypeUnified) {
                        return ISAL_HIP_EINVAL;
                }
        }
        return ISAL_HIP_OK;
}

int
isal_hip_batch_create(isal_hip_batch **out, int len, int k, int rows, const unsigned char *gftbls,
                      int nstripes, unsigned char *const *data, unsigned char *const *coding)
{
        isal_hip_batch *b;
        uint64_t *h_ptrs;
        long long s, stride = (long long) k + rows;
        size_t nptr;
        int j, vec16 = 1;
        if (!out || len < 0 || k < 0 || rows <= 0 || nstripes <= 0 || !gftbls || !coding ||
            (k > 0 && !data))
                return ISAL_HIP_EINVAL;
        *out = NULL;
        b = (isal_hip_batch *) calloc(1, sizeof(*b));
        nptr = (size_t) nstripes * (size_t) stride;
        h_ptrs = (uint64_t *) malloc(nptr * 8);
        if (!b || !h_ptrs) {
                free(b);
                free(h_ptrs);
                return ISAL_HIP_ENOMEM;
        }
        for (s = 0; s < nstripes; s++) {
                for (j = 0; j < k; j++)
                        h_ptrs[s * stride + j] = (uint64_t) (uintptr_t) data[s * k + j];
                for (j = 0; j < rows; j++)
                        h_ptrs[s * stride + k + j] = (uint64_t) (uintptr_t) coding[s * rows + j];
        }
        for (s = 0; s < (long long) nptr; s++)
                if (h_ptrs[s] & 15)
                        vec16 = 0;
        b->len = len;
        b->k = k;
        b->rows = rows;
        b->nstripes = nstripes;
        b->vec16 = vec16;
        if (hipGetDevice(&b->device) != hipSuccess) {
                free(h_ptrs);
                isal_hip_batch_destroy(b);
                return ISAL_HIP_EHIP;
        }
        if (len > 0 && (j = batch_check_ptrs(h_ptrs, nptr, (size_t) len, b->device)) != ISAL_HIP_OK) {
                free(h_ptrs);
                isal_hip_batch_destroy(b);
                return j;
        }
        if (hipMalloc((void **) &b->d_ptrs, nptr * 8) != hipSuccess ||
            hipMemcpy(b->d_ptrs, h_ptrs, nptr * 8, hipMemcpyHostToDevice) != hipSuccess) {
                free(h_ptrs);
                isal_hip_batch_destroy(b);
                return ISAL_HIP_EHIP;
        }
        free(h_ptrs);
        if (isal_hip_batch_set_tables(b, gftbls) != 0) {
                isal_hip_batch_destroy(b);
                return ISAL_HIP_EHIP;
        }
        *out = b;
        return ISAL_HIP_OK;
}

static int
batch_set_tables_impl(isal_hip_batch *b, const unsigned char *gftbls)
{
        size_t n;
        uint32_t *h;
        hipError_t e;
        isal_hip_xrows xr;
        isal_hip_encmask em;
        if (!b || !gftbls)
                return ISAL_HIP_EINVAL;
        n = isal_hip_tables_dwords(b->k, b->rows);
        h = (uint32_t *) malloc(n * 4 + 4);
        if (!h)
                return ISAL_HIP_ENOMEM;
        isal_hip_build_tables(b->k, b->rows, gftbls, h);
        /* published with the device tables only: a failed update keeps the
         * old row masks beside the old coefficients */
        isal_hip_xor_rows(b->k, b->rows, gftbls, &xr);
        isal_hip_enc_masks(b->k, b->rows, gftbls, &em);
        if (!b->d_tbl) {
                if (hipMalloc((void **) &b->d_tbl, n * 4 + 4) != hipSuccess) {
                        free(h);
                        return ISAL_HIP_EHIP;
                }
                e = hipSuccess;
        } else {
                /* launches already queued on any (possibly non-blocking) stream may
                 * still read the old coefficients: let them finish first */
                e = hipDeviceSynchronize();
        }
        if (e == hipSuccess)
                e = hipMemcpy(b->d_tbl, h, n * 4, hipMemcpyHostToDevice);
        free(h);
        /* the wide passes' LDS product tables (ec_encode_ldsx): k <= 64, a
         * pass of at least 4 rows (4 only when ISAL_HIP_ENC_LDSX=1 forces it) */
        if (e == hipSuccess && b->k >= 1 && b->k <= 64 && b->rows >= 4) {
                const size_t nw = isal_hip_ldsx_words(b->k, b->rows);
                uint64_t *hx = (uint64_t *) malloc(nw * 8);
                if (!hx)
                        return ISAL_HIP_ENOMEM;
                isal_hip_build_ldsx_tables(b->k, b->rows, gftbls, hx);
                if (!b->d_ldsx && hipMalloc((void **) &b->d_ldsx, nw * 8) != hipSuccess)
                        b->d_ldsx = NULL;
                e = b->d_ldsx ? hipMemcpy(b->d_ldsx, hx, nw * 8, hipMemcpyHostToDevice) : hipSuccess;
                free(hx);
        }
        if (e != hipSuccess)
                return ISAL_HIP_EHIP;
        b->xr = xr;
        b->em = em;
        b->em.ldsx = b->d_ldsx;
        return ISAL_HIP_OK;
}

static int
batch_encode_impl(isal_hip_batch *b, void *stream)
{
        if (!b)
                return ISAL_HIP_EINVAL;
        return isal_hip_launch_encode(b->d_ptrs, b->k + b->rows, 0, b->k, b->d_tbl, b->len, b->k,
                                      b->rows, b->nstripes, b->vec16, &b->em, stream)
                       ? ISAL_HIP_EHIP
                       : ISAL_HIP_OK;
}

static int
batch_update_impl(isal_hip_batch *b, int vec_i, void *stream)
{
        if (!b || vec_i < 0 || vec_i >= b->k)
                return ISAL_HIP_EINVAL;
        return isal_hip_launch_update(b->d_ptrs, b->k + b->rows, vec_i, b->k, b->d_tbl, b->len,
                                      b->k, b->rows, vec_i, b->nstripes, b->vec16, stream)
                       ? ISAL_HIP_EHIP
                       : ISAL_HIP_OK;
}

static int
batch_check_impl(isal_hip_batch *b, unsigned long long *bad, void *stream)
{
        if (!b || !bad || !b->vec16)
                return ISAL_HIP_EINVAL;
        return isal_hip_launch_verify_batch(b->d_ptrs, b->k + b->rows, 0, b->k, b->d_tbl, b->len, b->k, b->rows,
                                            b->nstripes, &b->em, bad, stream)
                       ? ISAL_HIP_EHIP
                       : ISAL_HIP_OK;
}

int
isal_hip_batch_destroy(isal_hip_batch *b)
{
        if (!b)
                return ISAL_HIP_OK;
        if (b->d_ptrs)
                (void) hipFree(b->d_ptrs);
        if (b->d_tbl)
                (void) hipFree(b->d_tbl);
        if (b->d_ldsx)
                (void) hipFree(b->d_ldsx);
        if (b->d_crc)
                (void) hipFree(b->d_crc);
        if (b->d_part)
                (void) hipFree(b->d_part);
        for (int v = 0; v < ISAL_HIP_CRC64_NVARIANTS; v++) {
                if (b->d_c64tab[v])
                        (void) hipFree(b->d_c64tab[v]);
                if (b->d_c64tab_ck[v])
                        (void) hipFree(b->d_c64tab_ck[v]);
        }
        if (b->d_c64part)
                (void) hipFree(b->d_c64part);
        free(b);
        return ISAL_HIP_OK;
}

/* ---- CRC32C of the batch's shards (isal_hip.h) ---------------------------- */

/* Tiles per CRC workgroup: `def` (64 for both CRC32C and CRC64: 256 KiB of
 * each shard per block, partials 0.1 % (CRC32C) / 0.2 % (CRC64) of the bytes
 * — profiles/r02/r02_crc_tiles_sweep_b.jsonl, r03_crc_tiles_sweep.jsonl), halved
 * while the launch would have fewer than 2048 workgroups.
 * ISAL_HIP_CRC_TILES overrides. */
static int
crc_tiles(int len, int nstripes, int def)
{
        const long long knob = isal_hip_knob(ISAL_HIP_KNOB_CRC_TILES);
        long long ntiles = ((long long) len + ISAL_HIP_CRC_TILE - 1) / ISAL_HIP_CRC_TILE;
        int tt = knob >= 0 ? (int) knob : def;
        if (tt < 1)
                tt = 1;
        if (knob >= 0)
                return tt;
        while (tt > 1 && (long long) nstripes * ((ntiles + tt - 1) / tt) < 2048)
                tt /= 2;
        return tt;
}

static int
batch_crc_setup(isal_hip_batch *b)
{
        uint32_t *h;
        size_t tab = ISAL_HIP_CRC_TAB_DWORDS,
               plan = ISAL_HIP_CRC_PLAN_DWORDS + ISAL_HIP_CRC_EXT_DWORDS + ISAL_HIP_CRC_B16_DWORDS +
                      ISAL_HIP_CRC_FPRE_DWORDS,
               nsh, part, tail;
        hipError_t e;
        if (b->d_crc)
                return ISAL_HIP_OK;
        /* 64 tiles per block: the checksum-only pass is memory-side bound and runs
         * 12 % faster than at 16, the fused pass is flat from 16 to 64
         * (profiles/r02/r02_crc_tiles_sweep_b.jsonl) */
        isal_hip_crc_geometry(b->len, crc_tiles(b->len, b->nstripes, 64), &b->crc);
        nsh = (size_t) b->nstripes * (size_t) (b->k + b->rows);
        part = nsh * (size_t) b->crc.nblk * 256;
        tail = nsh * 256;
        h = (uint32_t *) malloc((tab + plan) * 4);
        if (!h)
                return ISAL_HIP_ENOMEM;
        isal_hip_crc32c_tables(h);
        isal_hip_crc32c_plan(b->len, b->crc.tt, h + tab);
        isal_hip_crc32c_ext_tables(h, h + ISAL_HIP_CRC_EXT_TAB);
        isal_hip_crc32c_byte_tables(h + ISAL_HIP_CRC_B16_TAB);
        isal_hip_crc32c_pre_tables(h, h + ISAL_HIP_CRC_FPRE_TAB);
        e = hipMalloc((void **) &b->d_crc, (tab + plan) * 4);
        if (e == hipSuccess)
                e = hipMemcpy(b->d_crc, h, (tab + plan) * 4, hipMemcpyHostToDevice);
        free(h);
        if (e == hipSuccess)
                e = hipMalloc((void **) &b->d_part, (part + tail) * 4);
        if (e != hipSuccess) {
                if (b->d_crc)
                        (void) hipFree(b->d_crc);
                b->d_crc = b->d_part = NULL;
                return e == hipErrorOutOfMemory ? ISAL_HIP_ENOMEM : ISAL_HIP_EHIP;
        }
        b->d_tail = b->d_part + part;
        return ISAL_HIP_OK;
}

static int
batch_crc_finish(isal_hip_batch *b, unsigned int init, unsigned int *crc, void *stream)
{
        const long long nsh = (long long) b->nstripes * (b->k + b->rows);
        return isal_hip_launch_crc_combine(b->d_part, b->d_tail, b->d_crc + ISAL_HIP_CRC_TAB_DWORDS,
                                           b->crc.nblk, b->crc.tail != 0, init, (uint32_t *) crc,
                                           nsh, stream)
                       ? ISAL_HIP_EHIP
                       : ISAL_HIP_OK;
}

static int
batch_crc_empty(isal_hip_batch *b, unsigned int init, unsigned int *crc, void *stream)
{
        /* crc32_iscsi of 0 bytes is init_crc */
        const size_t n = (size_t) b->nstripes * (size_t) (b->k + b->rows);
        return hipMemsetD32Async((hipDeviceptr_t) crc, (int) init, n, (hipStream_t) stream) ==
                               hipSuccess
                       ? ISAL_HIP_OK
                       : ISAL_HIP_EHIP;
}

static int
batch_crc_impl(isal_hip_batch *b, unsigned int init, unsigned int *crc, void *stream)
{
        int r;
        if (!b || !crc)
                return ISAL_HIP_EINVAL;
        if (b->len == 0)
                return batch_crc_empty(b, init, crc, stream);
        if ((r = batch_crc_setup(b)) != ISAL_HIP_OK)
                return r;
        if (isal_hip_launch_crc(b->d_ptrs, b->k + b->rows, 0, b->k + b->rows, b->nstripes, b->len,
                                b->vec16, b->crc.tt, b->d_crc, b->d_part, b->d_tail,
                                b->k + b->rows, 0, stream))
                return ISAL_HIP_EHIP;
        return batch_crc_finish(b, init, crc, stream);
}

/* ---- CRC64 of the batch's shards (isal_hip.h) ----------------------------- */

/* ck: the checksum-only pass (else the fused encode + CRC64 pass). */
static int
batch_crc64_setup(isal_hip_batch *b, int variant, int ck)
{
        isal_hip_crc64_geom g;
        uint64_t *h, *d = NULL;
        hipError_t e;
        const size_t tab = ISAL_HIP_CRC64_TAB_ENTRIES;
        uint64_t **slot = ck ? &b->d_c64tab_ck[variant] : &b->d_c64tab[variant];
        if (*slot)
                return ISAL_HIP_OK;
        if (!b->d_c64part && !b->c64_tt) {
                /* Tiles per block: the fused pass 64 (flat from 32 to 64,
                 * profiles/r03/r03_crc_tiles_sweep.jsonl; 128 is 1.2-1.6 %
                 * slower), the checksum-only pass with its two chains per lane
                 * 128 (+1.3-1.6 % over 64, profiles/r05/r05_crc64_tiles_ab.txt).
                 * crc_tiles halves both alike for small batches, so c64_tt_ck
                 * >= c64_tt and the partials sized for c64_tt hold either. */
                b->c64_tt = crc_tiles(b->len, b->nstripes, 64);
                b->c64_tt_ck = crc_tiles(b->len, b->nstripes, 128);
                isal_hip_crc64_geometry(b->len, b->c64_tt < b->c64_tt_ck ? b->c64_tt : b->c64_tt_ck, &g);
                if (g.nblk) {
                        e = hipMalloc((void **) &b->d_c64part, (size_t) b->nstripes *
                                                                       (size_t) (b->k + b->rows) *
                                                                       (size_t) g.nblk * 256 * 8);
                        if (e != hipSuccess) {
                                b->d_c64part = NULL;
                                b->c64_tt = b->c64_tt_ck = 0; /* retry the whole setup next time */
                                return e == hipErrorOutOfMemory ? ISAL_HIP_ENOMEM : ISAL_HIP_EHIP;
                        }
                }
        }
        h = (uint64_t *) malloc(tab * 8);
        if (!h)
                return ISAL_HIP_ENOMEM;
        isal_hip_crc64_tables(variant, b->len, ck ? b->c64_tt_ck : b->c64_tt, h);
        /* a fresh buffer per variant: launches of other variants queued on any
         * stream keep reading their own tables */
        e = hipMalloc((void **) &d, tab * 8);
        if (e == hipSuccess)
                e = hipMemcpy(d, h, tab * 8, hipMemcpyHostToDevice);
        free(h);
        if (e != hipSuccess) {
                if (d)
                        (void) hipFree(d);
                return e == hipErrorOutOfMemory ? ISAL_HIP_ENOMEM : ISAL_HIP_EHIP;
        }
        *slot = d; /* published only once filled */
        return ISAL_HIP_OK;
}

static int
batch_crc64_impl(isal_hip_batch *b, int variant, unsigned long long init,
                     unsigned long long *crc, void *stream)
{
        int r;
        if (!b || !crc || variant < 0 || variant >= ISAL_HIP_CRC64_NVARIANTS)
                return ISAL_HIP_EINVAL;
        if ((r = batch_crc64_setup(b, variant, 1)) != ISAL_HIP_OK)
                return r;
        return isal_hip_launch_crc64(b->d_ptrs, b->k + b->rows, b->k + b->rows, b->nstripes,
                                     b->len, b->vec16, isal_hip_crc64_is_refl(variant), b->c64_tt_ck,
                                     b->d_c64tab_ck[variant], b->d_c64part,
                                     isal_hip_crc64_init_term(variant, b->len, init),
                                     (uint64_t *) crc, stream)
                       ? ISAL_HIP_EHIP
                       : ISAL_HIP_OK;
}

static int
batch_encode_crc64_impl(isal_hip_batch *b, int variant, unsigned long long init,
                            unsigned long long *crc, void *stream)
{
        int r;
        isal_hip_crc64_geom g;
        if (!b || !crc || variant < 0 || variant >= ISAL_HIP_CRC64_NVARIANTS)
                return ISAL_HIP_EINVAL;
        if ((r = batch_crc64_setup(b, variant, 0)) != ISAL_HIP_OK)
                return r;
        isal_hip_crc64_geometry(b->len, b->c64_tt, &g);
        if (b->vec16 && b->len % 16 == 0 && g.nblk > 0 && b->rows <= EC_MAX_ROWS_PER_PASS &&
            b->k >= 1 && b->k <= ISAL_HIP_CRC64_MAX_FUSED_K)
                /* one pass over the stripe: encode + CRC64 of all k + rows shards */
                return isal_hip_launch_encode_crc64(
                               b->d_ptrs, b->k, b->rows, b->nstripes, b->len, b->d_tbl, &b->xr,
                               isal_hip_crc64_is_refl(variant), b->c64_tt, b->d_c64tab[variant],
                               b->d_c64part, isal_hip_crc64_init_term(variant, b->len, init),
                               (uint64_t *) crc, stream)
                       ? ISAL_HIP_EHIP
                       : ISAL_HIP_OK;
        /* unaligned shards, short or ragged len, wide stripes: encode, then CRC64 */
        if (isal_hip_batch_encode(b, stream) != ISAL_HIP_OK)
                return ISAL_HIP_EHIP;
        return isal_hip_batch_crc64(b, variant, init, crc, stream);
}

static int
batch_encode_crc_impl(isal_hip_batch *b, unsigned int init, unsigned int *crc, void *stream)
{
        int r;
        if (!b || !crc)
                return ISAL_HIP_EINVAL;
        if (b->len == 0)
                return batch_crc_empty(b, init, crc, stream);
        if ((r = batch_crc_setup(b)) != ISAL_HIP_OK)
                return r;
        if (b->vec16 && b->len % 16 == 0 && b->k >= 1 && b->k <= ISAL_HIP_CRC_MAX_FUSED_K) {
                /* one pass over the stripe: encode + CRC of all k + rows shards
                 * (row 0's chains formed from the sources' when it is a 0/1 row) */
                if (isal_hip_launch_encode_crc(b->d_ptrs, b->k + b->rows, 0, b->k, b->d_tbl, &b->xr,
                                               b->len, b->k, b->rows, b->nstripes, b->crc.tt,
                                               b->d_crc, b->d_part, b->d_tail, stream))
                        return ISAL_HIP_EHIP;
        } else {
                /* unaligned shards, ragged len or very wide k: encode, then CRC */
                if (isal_hip_batch_encode(b, stream) != ISAL_HIP_OK)
                        return ISAL_HIP_EHIP;
                if (isal_hip_launch_crc(b->d_ptrs, b->k + b->rows, 0, b->k + b->rows, b->nstripes,
                                        b->len, b->vec16, b->crc.tt, b->d_crc, b->d_part,
                                        b->d_tail, b->k + b->rows, 0, stream))
                        return ISAL_HIP_EHIP;
        }
        return batch_crc_finish(b, init, crc, stream);
}

/* ---- checksum entry points (crc.h, crc64.h) --------------------------------
 * The reference's crc32_iscsi (include/crc.h:136-150) and crc64_* flavours
 * (include/crc64.h:54-163, isa-l.def:75-122), routed like ec_encode_data: a
 * buffer in device memory (hipMalloc or managed) is checksummed by the GPU
 * kernels of the batch API (crc_kernels.hip, crc64_kernels.hip) on the device
 * that holds it — one shard, pointer table and result in the thread's pinned
 * argument buffer, one stream synchronisation — and a host buffer by the CPU
 * route (crc_cpu.c), where the PCIe copy would cost more than the arithmetic.
 * The kernel tables of each flavour are kept per thread and device for the
 * last length (they depend on it); a storage caller checksums fragment after
 * fragment of one length. A failing HIP call on a device buffer aborts (no
 * CPU route can read it), as for the erasure-code calls. */

static int crc_tiles(int len, int nstripes, int def);

static hipError_t
ensure_cpart(ctx_t *c, size_t bytes)
{
        hipError_t e;
        if (bytes <= c->cpart_cap)
                return hipSuccess;
        if (c->d_cpart)
                (void) hipFree(c->d_cpart);
        c->d_cpart = NULL;
        c->cpart_cap = 0;
        if ((e = hipMalloc(&c->d_cpart, bytes)) != hipSuccess)
                return e;
        c->cpart_cap = bytes;
        return hipSuccess;
}

/* The device a checksum buffer lives on (-1: host memory, the CPU route). */
static int
crc_device(const void *buf, uint64_t len)
{
        int kind, dev, cur;
        uintptr_t rb;
        size_t rs;
        if (!buf || !len || !gpu_present())
                return -1;
        (void) classify(buf, (size_t) len, &kind, &dev, &rb, &rs);
        if (kind == CL_DEVICE)
                return dev;
        if (kind == CL_MANAGED && hipGetDevice(&cur) == hipSuccess)
                return cur;
        (void) hipGetLastError();
        return -1;
}

#define CRC_GPU_TRY(fn, what, call)                                                                \
        do {                                                                                       \
                hipError_t e_ = (call);                                                            \
                if (e_ != hipSuccess) {                                                            \
                        fprintf(stderr, "isal_hip: %s: ", fn);                                     \
                        die(what, e_);                                                             \
                }                                                                                  \
        } while (0)

/* crc64_<variant>(init, buf, len) of a buffer on device dev, len <= INT_MAX. */
static uint64_t
gpu_crc64_piece(const char *fn, int dev, int variant, uint64_t init, const unsigned char *buf, int len)
{
        const int tt = crc_tiles(len, 1, 64);
        isal_hip_crc64_geom g;
        struct crcc *cc;
        hipError_t err = hipSuccess;
        const char *what = NULL;
        ctx_t *c;
        uint64_t *h;
        c = ctx_get(dev, &err, &what);
        if (!c) {
                fprintf(stderr, "isal_hip: %s: ", fn);
                die(what, err);
        }
        cc = &c->c64[variant];
        isal_hip_crc64_geometry(len, tt, &g);
        if (!cc->d_tabs || cc->len != len || cc->tt != tt) {
                /* the flavour's tables once, then per length only the maps that
                 * depend on it (OP_BLOCK, OP_LAST, OP_TAIL: ~0.3 ms, not ~4) */
                const size_t tb = (size_t) ISAL_HIP_CRC64_TAB_ENTRIES * 8,
                             op = (size_t) ISAL_HIP_CRC64_OP_ENTRIES * 8;
                const int full = !cc->d_tabs || cc->len < 0;
                uint64_t *t = (uint64_t *) malloc(tb);
                if (!t) {
                        fprintf(stderr, "isal_hip: out of host memory\n");
                        abort();
                }
                if (full)
                        isal_hip_crc64_tables(variant, len, tt, t);
                else
                        isal_hip_crc64_len_tables(variant, len, tt, t);
                cc->len = -1;
                if (!cc->d_tabs)
                        CRC_GPU_TRY(fn, "hipMalloc (checksum tables)", hipMalloc(&cc->d_tabs, tb));
                /* the thread's earlier checksum calls have completed (each one
                 * synchronises), so the tables may be overwritten */
                if (full) {
                        CRC_GPU_TRY(fn, "hipMemcpy (checksum tables)",
                                    hipMemcpy(cc->d_tabs, t, tb, hipMemcpyHostToDevice));
                } else {
                        CRC_GPU_TRY(fn, "hipMemcpy (checksum tables)",
                                    hipMemcpy((uint64_t *) cc->d_tabs + ISAL_HIP_CRC64_OP_BLOCK,
                                              t + ISAL_HIP_CRC64_OP_BLOCK, 2 * op, hipMemcpyHostToDevice));
                        CRC_GPU_TRY(fn, "hipMemcpy (checksum tables)",
                                    hipMemcpy((uint64_t *) cc->d_tabs + ISAL_HIP_CRC64_OP_TAIL,
                                              t + ISAL_HIP_CRC64_OP_TAIL, op, hipMemcpyHostToDevice));
                }
                free(t);
                cc->len = len;
                cc->tt = tt;
        }
        CRC_GPU_TRY(fn, "hipMalloc (checksum partials)", ensure_cpart(c, (size_t) (g.nblk ? g.nblk : 1) * 256 * 8));
        CRC_GPU_TRY(fn, "argument buffer", ensure_args(c, 64));
        h = (uint64_t *) c->h_args;
        h[0] = (uint64_t) (uintptr_t) buf;
        h[2] = 0;
        CRC_GPU_TRY(fn, "crc64 launch",
                    (hipError_t) isal_hip_launch_crc64((const uint64_t *) c->h_args_dev, 1, 1, 1, len,
                                                       ((uintptr_t) buf & 15) == 0, isal_hip_crc64_is_refl(variant),
                                                       tt, (const uint64_t *) cc->d_tabs, (uint64_t *) c->d_cpart,
                                                       isal_hip_crc64_init_term(variant, len, init),
                                                       (uint64_t *) c->h_args_dev + 2,
                                                       c->stream));
        CRC_GPU_TRY(fn, "hipStreamSynchronize (checksum)", hipStreamSynchronize(c->stream));
        return h[2];
}

/* ISAL_HIP_BACKEND=gpu: a host buffer is copied into the thread's staging
 * buffer on its current device, piece by piece, and checksummed there (the
 * kernels for every call, as for the erasure-code calls; tests). Returns the
 * staging address of [buf, buf + n) and the device in *dev. */
static const unsigned char *
crc_stage(const char *fn, const unsigned char *buf, size_t n, int *dev)
{
        hipError_t err = hipSuccess;
        const char *what = NULL;
        ctx_t *c;
        if (hipGetDevice(dev) != hipSuccess || !(c = ctx_get(*dev, &err, &what))) {
                fprintf(stderr, "isal_hip: %s: ", fn);
                die(what ? what : "hipGetDevice", err != hipSuccess ? err : hipErrorNoDevice);
        }
        CRC_GPU_TRY(fn, "hipMalloc (staging)", ensure_stage(c, n));
        CRC_GPU_TRY(fn, "hipMemcpyAsync (staging)", hipMemcpyAsync(c->d_stage, buf, n, hipMemcpyHostToDevice, c->stream));
        return c->d_stage;
}

static int
crc_staged(const unsigned char *buf, uint64_t len)
{
        return len && buf && backend() == BACKEND_GPU && gpu_present();
}

static uint64_t
crc64_route(const char *fn, int variant, uint64_t init, const unsigned char *buf, uint64_t len)
{
        const int dev = crc_device(buf, len);
        int prev;
        if (dev < 0 && crc_staged(buf, len)) {
                const uint64_t piece = stage_limit();
                int sdev;
                while (len) {
                        const uint64_t n = len < piece ? len : piece;
                        const unsigned char *d = crc_stage(fn, buf, (size_t) n, &sdev);
                        uint64_t left = n;
                        while (left) { /* the kernels take an int length */
                                const int m = left > ((uint64_t) 1 << 30) ? 1 << 30 : (int) left;
                                init = gpu_crc64_piece(fn, sdev, variant, init, d, m);
                                d += m;
                                left -= (uint64_t) m;
                        }
                        buf += n;
                        len -= n;
                }
                return init;
        }
        if (dev < 0)
                return isal_cpu_crc64(variant, init, buf, len);
        if ((prev = isal_hip_dev_enter(dev)) == -2) {
                fprintf(stderr, "isal_hip: %s: ", fn);
                die("hipSetDevice (to the device holding the buffer)", hipErrorInvalidDevice);
        }
        /* the kernels take an int length: pieces of 1 GiB, chained through the
         * register (crc64(crc64(init, A), B) = crc64(init, A || B)) */
        while (len) {
                const int n = len > ((uint64_t) 1 << 30) ? 1 << 30 : (int) len;
                init = gpu_crc64_piece(fn, dev, variant, init, buf, n);
                buf += n;
                len -= (uint64_t) n;
        }
        isal_hip_dev_leave(prev);
        return init;
}

static uint32_t
gpu_crc32c(const char *fn, int dev, uint32_t init, const unsigned char *buf, int len)
{
        const int tt = crc_tiles(len, 1, 64);
        isal_hip_crc_geom g;
        struct crcc *cc;
        hipError_t err = hipSuccess;
        const char *what = NULL;
        const size_t tab = ISAL_HIP_CRC_TAB_DWORDS,
                     plan = ISAL_HIP_CRC_PLAN_DWORDS + ISAL_HIP_CRC_EXT_DWORDS + ISAL_HIP_CRC_B16_DWORDS +
                            ISAL_HIP_CRC_FPRE_DWORDS;
        size_t part;
        ctx_t *c;
        uint32_t *h;
        c = ctx_get(dev, &err, &what);
        if (!c) {
                fprintf(stderr, "isal_hip: %s: ", fn);
                die(what, err);
        }
        cc = &c->c32;
        isal_hip_crc_geometry(len, tt, &g);
        if (!cc->d_tabs || cc->len != len || cc->tt != tt) {
                /* all tables once, then per length only the combine plan */
                const int full = !cc->d_tabs || cc->len < 0;
                uint32_t *t = (uint32_t *) malloc((tab + plan) * 4);
                if (!t) {
                        fprintf(stderr, "isal_hip: out of host memory\n");
                        abort();
                }
                isal_hip_crc32c_plan(len, tt, t + tab);
                if (full) {
                        isal_hip_crc32c_tables(t);
                        isal_hip_crc32c_ext_tables(t, t + ISAL_HIP_CRC_EXT_TAB);
                        isal_hip_crc32c_byte_tables(t + ISAL_HIP_CRC_B16_TAB);
                        isal_hip_crc32c_pre_tables(t, t + ISAL_HIP_CRC_FPRE_TAB);
                }
                cc->len = -1;
                if (!cc->d_tabs)
                        CRC_GPU_TRY(fn, "hipMalloc (checksum tables)", hipMalloc(&cc->d_tabs, (tab + plan) * 4));
                if (full)
                        CRC_GPU_TRY(fn, "hipMemcpy (checksum tables)",
                                    hipMemcpy(cc->d_tabs, t, (tab + plan) * 4, hipMemcpyHostToDevice));
                else
                        CRC_GPU_TRY(fn, "hipMemcpy (checksum tables)",
                                    hipMemcpy((uint32_t *) cc->d_tabs + tab, t + tab, ISAL_HIP_CRC_PLAN_DWORDS * 4,
                                              hipMemcpyHostToDevice));
                free(t);
                cc->len = len;
                cc->tt = tt;
        }
        part = (size_t) g.nblk * 256;
        CRC_GPU_TRY(fn, "hipMalloc (checksum partials)", ensure_cpart(c, (part + 256) * 4));
        CRC_GPU_TRY(fn, "argument buffer", ensure_args(c, 64));
        ((uint64_t *) c->h_args)[0] = (uint64_t) (uintptr_t) buf;
        h = (uint32_t *) c->h_args + 4;
        *h = 0;
        CRC_GPU_TRY(fn, "crc32c launch",
                    (hipError_t) isal_hip_launch_crc((const uint64_t *) c->h_args_dev, 1, 0, 1, 1, len,
                                                     ((uintptr_t) buf & 15) == 0, tt, (const uint32_t *) cc->d_tabs,
                                                     (uint32_t *) c->d_cpart, (uint32_t *) c->d_cpart + part, 1, 0,
                                                     c->stream));
        CRC_GPU_TRY(fn, "crc32c combine launch",
                    (hipError_t) isal_hip_launch_crc_combine((const uint32_t *) c->d_cpart,
                                                             (const uint32_t *) c->d_cpart + part,
                                                             (const uint32_t *) cc->d_tabs + tab, g.nblk, g.tail != 0,
                                                             init, (uint32_t *) c->h_args_dev + 4, 1, c->stream));
        CRC_GPU_TRY(fn, "hipStreamSynchronize (checksum)", hipStreamSynchronize(c->stream));
        return *h;
}

static unsigned int
crc32c_route(const char *fn, const unsigned char *buf, int len, unsigned int init)
{
        int dev, prev;
        unsigned int r;
        if (len <= 0)
                return init; /* the reference's loop runs no byte */
        dev = crc_device(buf, (uint64_t) len);
        if (dev < 0 && crc_staged(buf, (uint64_t) len)) {
                const int piece = stage_limit() < ((size_t) 1 << 30) ? (int) stage_limit() : 1 << 30;
                int sdev;
                /* crc32_iscsi chains through its register: crc(crc(init, A), B) = crc(init, A || B) */
                while (len) {
                        const int n = len < piece ? len : piece;
                        const unsigned char *d = crc_stage(fn, buf, (size_t) n, &sdev);
                        init = gpu_crc32c(fn, sdev, init, d, n);
                        buf += n;
                        len -= n;
                }
                return init;
        }
        if (dev < 0)
                return isal_cpu_crc32c(init, buf, (uint64_t) len);
        if ((prev = isal_hip_dev_enter(dev)) == -2) {
                fprintf(stderr, "isal_hip: %s: ", fn);
                die("hipSetDevice (to the device holding the buffer)", hipErrorInvalidDevice);
        }
        r = gpu_crc32c(fn, dev, init, buf, len);
        isal_hip_dev_leave(prev);
        return r;
}

unsigned int
crc32_iscsi(unsigned char *buffer, int len, unsigned int init_crc)
{
        return crc32c_route("crc32_iscsi", buffer, len, init_crc);
}

unsigned int
crc32_iscsi_base(unsigned char *buffer, int len, unsigned int crc_init)
{
        return crc32c_route("crc32_iscsi_base", buffer, len, crc_init);
}

#define CRC64_ENTRY(name, variant)                                                                 \
        uint64_t name(uint64_t init_crc, const unsigned char *buf, uint64_t len)                   \
        {                                                                                          \
                return crc64_route(#name, variant, init_crc, buf, len);                            \
        }                                                                                          \
        uint64_t name##_base(uint64_t init_crc, const unsigned char *buf, uint64_t len)            \
        {                                                                                          \
                return crc64_route(#name "_base", variant, init_crc, buf, len);                    \
        }
CRC64_ENTRY(crc64_ecma_refl, ISAL_HIP_CRC64_ECMA_REFL)
CRC64_ENTRY(crc64_ecma_norm, ISAL_HIP_CRC64_ECMA_NORM)
CRC64_ENTRY(crc64_iso_refl, ISAL_HIP_CRC64_ISO_REFL)
CRC64_ENTRY(crc64_iso_norm, ISAL_HIP_CRC64_ISO_NORM)
CRC64_ENTRY(crc64_jones_refl, ISAL_HIP_CRC64_JONES_REFL)
CRC64_ENTRY(crc64_jones_norm, ISAL_HIP_CRC64_JONES_NORM)
CRC64_ENTRY(crc64_rocksoft_refl, ISAL_HIP_CRC64_ROCKSOFT_REFL)
CRC64_ENTRY(crc64_rocksoft_norm, ISAL_HIP_CRC64_ROCKSOFT_NORM)
#undef CRC64_ENTRY

/* ---- the batch entry points run on the batch's device -------------------- */

int
isal_hip_batch_set_tables(isal_hip_batch *b, const unsigned char *gftbls)
{
        int prev, r;
        if (!b)
                return ISAL_HIP_EINVAL;
        if ((prev = isal_hip_dev_enter(b->device)) == -2)
                return ISAL_HIP_EHIP;
        r = batch_set_tables_impl(b, gftbls);
        isal_hip_dev_leave(prev);
        return r;
}

int
isal_hip_batch_encode(isal_hip_batch *b, void *stream)
{
        int prev, r;
        if (!b)
                return ISAL_HIP_EINVAL;
        if ((prev = isal_hip_dev_enter(b->device)) == -2)
                return ISAL_HIP_EHIP;
        r = batch_encode_impl(b, stream);
        isal_hip_dev_leave(prev);
        return r;
}

int
isal_hip_batch_update(isal_hip_batch *b, int vec_i, void *stream)
{
        int prev, r;
        if (!b)
                return ISAL_HIP_EINVAL;
        if ((prev = isal_hip_dev_enter(b->device)) == -2)
                return ISAL_HIP_EHIP;
        r = batch_update_impl(b, vec_i, stream);
        isal_hip_dev_leave(prev);
        return r;
}

int
isal_hip_batch_check(isal_hip_batch *b, unsigned long long *bad, void *stream)
{
        int prev, r;
        if (!b)
                return ISAL_HIP_EINVAL;
        if ((prev = isal_hip_dev_enter(b->device)) == -2)
                return ISAL_HIP_EHIP;
        r = batch_check_impl(b, bad, stream);
        isal_hip_dev_leave(prev);
        return r;
}

int
isal_hip_batch_crc(isal_hip_batch *b, unsigned int init, unsigned int *crc, void *stream)
{
        int prev, r;
        if (!b)
                return ISAL_HIP_EINVAL;
        if ((prev = isal_hip_dev_enter(b->device)) == -2)
                return ISAL_HIP_EHIP;
        r = batch_crc_impl(b, init, crc, stream);
        isal_hip_dev_leave(prev);
        return r;
}

int
isal_hip_batch_crc64(isal_hip_batch *b, int variant, unsigned long long init,
                     unsigned long long *crc, void *stream)
{
        int prev, r;
        if (!b)
                return ISAL_HIP_EINVAL;
        if ((prev = isal_hip_dev_enter(b->device)) == -2)
                return ISAL_HIP_EHIP;
        r = batch_crc64_impl(b, variant, init, crc, stream);
        isal_hip_dev_leave(prev);
        return r;
}

int
isal_hip_batch_encode_crc64(isal_hip_batch *b, int variant, unsigned long long init,
                            unsigned long long *crc, void *stream)
{
        int prev, r;
        if (!b)
                return ISAL_HIP_EINVAL;
        if ((prev = isal_hip_dev_enter(b->device)) == -2)
                return ISAL_HIP_EHIP;
        r = batch_encode_crc64_impl(b, variant, init, crc, stream);
        isal_hip_dev_leave(prev);
        return r;
}

int
isal_hip_batch_encode_crc(isal_hip_batch *b, unsigned int init, unsigned int *crc, void *stream)
{
        int prev, r;
        if (!b)
                return ISAL_HIP_EINVAL;
        if ((prev = isal_hip_dev_enter(b->device)) == -2)
                return ISAL_HIP_EHIP;
        r = batch_encode_crc_impl(b, init, crc, stream);
        isal_hip_dev_leave(prev);
        return r;
}
