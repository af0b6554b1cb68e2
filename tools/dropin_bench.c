/*
 * dropin_bench.c — throughput of the synchronous drop-in ec_encode_data on
 * device-resident shards (the way the reference's API is driven: one call
 * per stripe, erasure_code/erasure_code_perf.c:126-132), from T threads.
 *
 * usage: dropin_bench K P LEN STRIPES THREADS SECONDS [CALLS_PER_THREAD [OP]]
 *
 * OP (default encode): the synchronous call per stripe — encode
 * (ec_encode_data), or a raid.h call over K sources: pq_gen / pq_check (P = 2
 * rows: P, Q) or xor_gen / xor_check (P = 1), e.g. the reference harness
 * raid/pq_gen_perf.c drives pq_gen the same way (one call per stripe). The
 * check ops run on consistent stripes (every call must return 0) and finish
 * with one corrupted byte that must be reported.
 *
 * STRIPES stripes of K + P shards live in HBM (one hipMalloc, shard s*(K+P)+i
 * at offset ((s*(K+P)+i) * LEN)); thread t encodes stripes t, t+T, ... in a
 * loop, one ec_encode_data(LEN, K, P, gftbls, data, coding) per stripe, for
 * SECONDS (or exactly CALLS_PER_THREAD calls each when given, for traces).
 * Prints one JSON object: calls, wall seconds, us per call (one thread's view:
 * wall / calls per thread), calls/s and GiB/s of (K+P)*LEN per call (the
 * reference's perf_print convention, erasure_code_perf.c:304).
 *
 * DROPIN_MEM=host|pinned puts the stripes in pageable malloc memory or
 * hipHostMalloc memory instead of HBM (with ISAL_HIP_BACKEND=gpu: the per-call
 * cost of the reference's own tests forced onto the kernels, e.g.
 * raid/xor_check_test.c's 1 KiB calls over 17 host buffers).
 *
 * Self-check (no oracle): for the first and last stripe, 8192 sampled columns
 * of every parity row are recomputed on the host from the library's host GF
 * math (gf_mul of the generator matrix, itself pinned by the reference's
 * golden fixtures) and compared.
 *
 * Build: make -C isa-l_amd tools  (gcc, links libisal_hip.so + libamdhip64).
 */
#include <hip/hip_runtime_api.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "erasure_code.h"
#include "raid.h"

enum { OP_ENCODE, OP_PQ_GEN, OP_XOR_GEN, OP_PQ_CHECK, OP_XOR_CHECK };
static const char *const op_names[] = {"encode", "pq_gen", "xor_gen", "pq_check", "xor_check", NULL};
static int g_op = OP_ENCODE;
enum { MEM_DEVICE, MEM_HOST, MEM_PINNED };
static int g_mem = MEM_DEVICE;

/* stripes in host memory are copied by the CPU; in HBM through
 * hipMemcpyDefault (the runtime infers the direction from the pointers) */
static void
copy(void *dst, const void *src, size_t n)
{
        if (g_mem != MEM_DEVICE)
                memcpy(dst, src, n);
        else
                (void) hipMemcpy(dst, src, n, hipMemcpyDefault);
}
static long long g_check_fail;

static double
now(void)
{
        struct timespec t;
        clock_gettime(CLOCK_MONOTONIC, &t);
        return (double) t.tv_sec + (double) t.tv_nsec * 1e-9;
}

typedef struct {
        int t, nthreads, k, p, len, stripes;
        long long fixed_calls;
        unsigned char *base, *tbls;
        long long calls;
        double first_call_us;
} worker_t;

/* Warm-up and timed calls run on the SAME threads: the library's per-thread
 * context (stream, pinned argument buffer, cached tables) lives as long as its
 * thread, so a thread created for the timed run would pay its context
 * creation inside the timed window. */
static pthread_barrier_t warm_done, go;
static double g_deadline;
#define WARM_CALLS 2

static unsigned char *
shard(const worker_t *w, int s, int i)
{
        return w->base + ((size_t) s * (size_t) (w->k + w->p) + (size_t) i) * (size_t) w->len;
}

/* one call of the selected op on stripe s; returns its return value (0 for
 * ec_encode_data) */
static int
call_op(const worker_t *w, int s)
{
        unsigned char *data[256], *coding[256];
        void *arr[257];
        int i;
        if (g_op == OP_ENCODE) {
                for (i = 0; i < w->k; i++)
                        data[i] = shard(w, s, i);
                for (i = 0; i < w->p; i++)
                        coding[i] = shard(w, s, w->k + i);
                ec_encode_data(w->len, w->k, w->p, w->tbls, data, coding);
                return 0;
        }
        for (i = 0; i < w->k + w->p; i++)
                arr[i] = shard(w, s, i);
        switch (g_op) {
        case OP_PQ_GEN: return pq_gen(w->k + 2, w->len, arr);
        case OP_XOR_GEN: return xor_gen(w->k + 1, w->len, arr);
        case OP_PQ_CHECK: return pq_check(w->k + 2, w->len, arr);
        default: return xor_check(w->k + 1, w->len, arr);
        }
}

static void
encode_one(worker_t *w, int *s)
{
        if (call_op(w, *s) != 0)
                __atomic_add_fetch(&g_check_fail, 1, __ATOMIC_RELAXED);
        *s += w->nthreads;
        if (*s >= w->stripes)
                *s = w->t % w->stripes;
}

static void *
run(void *arg)
{
        worker_t *w = (worker_t *) arg;
        int s = w->t, i;
        (void) hipSetDevice(0);
        for (i = 0; i < WARM_CALLS; i++)
                encode_one(w, &s);
        pthread_barrier_wait(&warm_done);
        pthread_barrier_wait(&go); /* main has set g_deadline */
        w->calls = 0;
        for (;;) {
                double t0;
                if (w->fixed_calls ? w->calls >= w->fixed_calls : now() >= g_deadline)
                        break;
                t0 = w->calls ? 0 : now();
                encode_one(w, &s);
                if (!w->calls)
                        w->first_call_us = (now() - t0) * 1e6;
                w->calls++;
        }
        return NULL;
}

/* parity columns of stripe s recomputed on the host from gf_mul and the
 * generator rows; 0 on match */
static int
check_stripe(const worker_t *w, const unsigned char *a, int s)
{
        const int k = w->k, p = w->p, len = w->len, ncol = len < 8192 ? len : 8192;
        unsigned char *src = malloc((size_t) k * len), *par = malloc((size_t) p * len);
        int i, l, c, bad = 0;
        uint64_t x = 88172645463325252ull + (uint64_t) s;
        if (!src || !par)
                return 1;
        for (i = 0; i < k; i++)
                copy(src + (size_t) i * len, shard(w, s, i), (size_t) len);
        for (l = 0; l < p; l++)
                copy(par + (size_t) l * len, shard(w, s, k + l), (size_t) len);
        for (c = 0; c < ncol && !bad; c++) {
                int col;
                x ^= x << 13;
                x ^= x >> 7;
                x ^= x << 17;
                col = c < 64 ? c : c >= ncol - 64 ? len - (ncol - c) : (int) (x % (uint64_t) len);
                for (l = 0; l < p; l++) {
                        unsigned char acc = 0;
                        for (i = 0; i < k; i++)
                                acc ^= gf_mul(a[(k + l) * k + i], src[(size_t) i * len + col]);
                        if (acc != par[(size_t) l * len + col]) {
                                fprintf(stderr, "dropin_bench: stripe %d row %d col %d: got %u want %u\n", s, l,
                                        col, par[(size_t) l * len + col], acc);
                                bad = 1;
                        }
                }
        }
        free(src);
        free(par);
        return bad;
}

int
main(int argc, char **argv)
{
        int k, p, len, stripes, nthreads, i, ok;
        double seconds, t0, wall;
        long long calls = 0, fixed = 0;
        size_t total, nsrc_bytes;
        unsigned char *a, *tbls, *base, *h;
        uint64_t x = 0x9E3779B97F4A7C15ull;
        worker_t *w;
        pthread_t *th;
        hipError_t e;

        if (argc < 7) {
                fprintf(stderr, "usage: %s K P LEN STRIPES THREADS SECONDS [CALLS_PER_THREAD [OP]]\n", argv[0]);
                return 2;
        }
        k = atoi(argv[1]);
        p = atoi(argv[2]);
        len = atoi(argv[3]);
        stripes = atoi(argv[4]);
        nthreads = atoi(argv[5]);
        seconds = atof(argv[6]);
        if (argc > 7)
                fixed = atoll(argv[7]);
        if (argc > 8) {
                for (i = 0; op_names[i] && strcmp(op_names[i], argv[8]); i++)
                        ;
                if (!op_names[i]) {
                        fprintf(stderr, "dropin_bench: unknown op %s\n", argv[8]);
                        return 2;
                }
                g_op = i;
                if (g_op != OP_ENCODE)
                        p = g_op == OP_PQ_GEN || g_op == OP_PQ_CHECK ? 2 : 1;
        }
        if (k < 1 || p < 1 || k + p > 255 || len < 1 || stripes < 1 || nthreads < 1 || nthreads > 256) {
                fprintf(stderr, "dropin_bench: bad arguments\n");
                return 2;
        }
        if (stripes < nthreads)
                stripes = nthreads;
        total = (size_t) stripes * (size_t) (k + p) * (size_t) len;
        if (getenv("DROPIN_MEM"))
                g_mem = !strcmp(getenv("DROPIN_MEM"), "host") ? MEM_HOST
                        : !strcmp(getenv("DROPIN_MEM"), "pinned") ? MEM_PINNED : MEM_DEVICE;
        e = g_mem == MEM_DEVICE ? hipMalloc((void **) &base, total)
            : g_mem == MEM_PINNED ? hipHostMalloc((void **) &base, total, 0)
            : (base = aligned_alloc(64, (total + 63) / 64 * 64)) ? hipSuccess : hipErrorOutOfMemory;
        if (e != hipSuccess) {
                fprintf(stderr, "dropin_bench: allocation of %zu bytes: %s\n", total, hipGetErrorString(e));
                return 1;
        }
        /* sources random, parity zero; one host stripe of random bytes copied
         * into every stripe with a per-stripe byte rotation */
        nsrc_bytes = (size_t) k * (size_t) len;
        h = malloc(nsrc_bytes);
        if (!h)
                return 1;
        for (size_t b = 0; b < nsrc_bytes; b++) {
                x ^= x << 13;
                x ^= x >> 7;
                x ^= x << 17;
                h[b] = (unsigned char) (x >> 32);
        }
        if (g_mem == MEM_DEVICE)
                (void) hipMemset(base, 0, total);
        else
                memset(base, 0, total);
        for (i = 0; i < stripes; i++) {
                const size_t rot = ((size_t) i * 977) % nsrc_bytes;
                unsigned char *dst = base + (size_t) i * (size_t) (k + p) * (size_t) len;
                copy(dst, h + rot, nsrc_bytes - rot);
                if (rot)
                        copy(dst + nsrc_bytes - rot, h, rot);
        }
        free(h);
        if (g_mem == MEM_DEVICE)
                (void) hipDeviceSynchronize();

        a = malloc((size_t) (k + p) * (size_t) k);
        tbls = malloc((size_t) 32 * (size_t) k * (size_t) p);
        w = calloc((size_t) nthreads, sizeof(*w));
        th = calloc((size_t) nthreads, sizeof(*th));
        if (!a || !tbls || !w || !th)
                return 1;
        gf_gen_rs_matrix(a, k + p, k);
        if (g_op != OP_ENCODE) {
                /* the RAID rows: P = all ones, Q = 2^j (raid_base.c:44-68) */
                unsigned char q = 1;
                for (i = 0; i < k; i++) {
                        a[(size_t) k * k + i] = 1;
                        if (p == 2) {
                                a[(size_t) (k + 1) * k + i] = q;
                                q = gf_mul(q, 2);
                        }
                }
        }
        ec_init_tables(k, p, a + (size_t) k * k, tbls);
        if (g_op == OP_PQ_CHECK || g_op == OP_XOR_CHECK) {
                /* consistent parity first: the timed checks must all pass */
                const int gen = g_op;
                worker_t g0 = {.t = 0, .nthreads = 1, .k = k, .p = p, .len = len, .stripes = stripes,
                               .base = base, .tbls = tbls};
                g_op = gen == OP_PQ_CHECK ? OP_PQ_GEN : OP_XOR_GEN;
                for (i = 0; i < stripes; i++)
                        if (call_op(&g0, i) != 0) {
                                fprintf(stderr, "dropin_bench: parity generation failed\n");
                                return 1;
                        }
                g_op = gen;
        }

        for (i = 0; i < nthreads; i++) {
                w[i] = (worker_t){.t = i, .nthreads = nthreads, .k = k, .p = p, .len = len,
                                  .stripes = stripes, .fixed_calls = fixed, .base = base, .tbls = tbls};
        }
        pthread_barrier_init(&warm_done, NULL, (unsigned) nthreads + 1);
        pthread_barrier_init(&go, NULL, (unsigned) nthreads + 1);
        for (i = 0; i < nthreads; i++)
                pthread_create(&th[i], NULL, run, &w[i]);
        pthread_barrier_wait(&warm_done); /* every thread's context is warm */
        t0 = now();
        g_deadline = t0 + seconds;
        pthread_barrier_wait(&go);
        for (i = 0; i < nthreads; i++) {
                pthread_join(th[i], NULL);
                calls += w[i].calls;
        }
        wall = now() - t0;
        ok = check_stripe(&w[0], a, 0) == 0 && check_stripe(&w[0], a, stripes - 1) == 0 && g_check_fail == 0;
        if (g_check_fail)
                fprintf(stderr, "dropin_bench: %lld calls returned non-zero\n", g_check_fail);
        if (ok && (g_op == OP_PQ_CHECK || g_op == OP_XOR_CHECK)) {
                /* one corrupted byte in the middle of source 1 of stripe 0 must be reported */
                unsigned char *b = shard(&w[0], 0, 1) + len / 2, v;
                copy(&v, b, 1);
                v ^= 0x08;
                copy(b, &v, 1);
                if (call_op(&w[0], 0) == 0) {
                        fprintf(stderr, "dropin_bench: corrupted stripe not reported\n");
                        ok = 0;
                }
                v ^= 0x08;
                copy(b, &v, 1);
        }
        printf("{\"op\": \"%s\", \"k\": %d, \"p\": %d, \"len\": %d, \"stripes\": %d, \"threads\": %d, \"mem\": \"%s\", \"calls\": %lld, "
               "\"wall_s\": %.4f, \"us_per_call\": %.2f, \"calls_per_s\": %.1f, \"gib_s\": %.3f, "
               "\"first_timed_call_us_thread0\": %.1f, \"self_check\": %s}\n",
               op_names[g_op], k, p, len, stripes, nthreads, g_mem == MEM_DEVICE ? "device" : g_mem == MEM_HOST ? "host" : "pinned", calls, wall, wall / ((double) calls / nthreads) * 1e6,
               (double) calls / wall, (double) calls * (double) (k + p) * (double) len / wall / (double) (1 << 30),
               w[0].first_call_us, ok ? "true" : "false");
        if (g_mem == MEM_DEVICE)
                (void) hipFree(base);
        else if (g_mem == MEM_PINNED)
                (void) hipHostFree(base);
        else
                free(base);
        return ok ? 0 : 1;
}
