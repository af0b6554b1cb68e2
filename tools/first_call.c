/*
 * first_call.c — what a drop-in caller pays to start using libisal_hip.so:
 * the time from dlopen() of the library to its first kernel-argument
 * ec_encode_data returning on device-resident shards, split into steps.
 *
 *   dlopen       dlopen("libisal_hip.so") (+ libamdhip64 and its
 *                dependencies; no GPU work yet)
 *   hip_init     hipMalloc of the stripe (initialises the HIP runtime and
 *                the device) and its fill
 *   first_call   the first ec_encode_data (per-thread context: stream,
 *                mailbox; the code object holding the encode kernels is
 *                loaded on this first launch)
 *   second_call  the next call (steady state)
 *
 * usage: first_call LIB K P LEN   (prints one JSON line; checks the parity
 * of both calls against the library's own host gf_mul)
 *
 * Build: make -C isa-l_amd tools (gcc, -ldl -lamdhip64; not linked against
 * libisal_hip.so: the point is to time its loading).
 */
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>

typedef void (*encode_fn)(int, int, int, unsigned char *, unsigned char **, unsigned char **);
typedef void (*gen_fn)(unsigned char *, int, int);
typedef void (*init_fn)(int, int, unsigned char *, unsigned char *);
typedef unsigned char (*mul_fn)(unsigned char, unsigned char);

static double
now_ms(void)
{
        struct timespec t;
        clock_gettime(CLOCK_MONOTONIC, &t);
        return (double) t.tv_sec * 1e3 + (double) t.tv_nsec * 1e-6;
}

int
main(int argc, char **argv)
{
        const char *path;
        int k, p, len, i, l, j, ok = 1;
        double t0, t1, t2, t3, t4;
        void *lib;
        encode_fn enc;
        gen_fn gen;
        init_fn init;
        mul_fn mul;
        unsigned char *a, *tbls, *base, *h, *data[256], *coding[256];
        struct stat st;

        if (argc < 5) {
                fprintf(stderr, "usage: %s LIB K P LEN\n", argv[0]);
                return 2;
        }
        path = argv[1];
        k = atoi(argv[2]);
        p = atoi(argv[3]);
        len = atoi(argv[4]);
        if (k < 1 || p < 1 || k + p > 255 || len < 16 || len % 16) {
                fprintf(stderr, "first_call: bad arguments\n");
                return 2;
        }
        t0 = now_ms();
        lib = dlopen(path, RTLD_NOW | RTLD_LOCAL);
        if (!lib) {
                fprintf(stderr, "first_call: %s\n", dlerror());
                return 1;
        }
        enc = (encode_fn) dlsym(lib, "ec_encode_data");
        gen = (gen_fn) dlsym(lib, "gf_gen_rs_matrix");
        init = (init_fn) dlsym(lib, "ec_init_tables");
        mul = (mul_fn) dlsym(lib, "gf_mul");
        if (!enc || !gen || !init || !mul) {
                fprintf(stderr, "first_call: missing symbol\n");
                return 1;
        }
        t1 = now_ms();
        if (hipMalloc((void **) &base, (size_t) (k + p) * len) != hipSuccess) {
                fprintf(stderr, "first_call: hipMalloc failed\n");
                return 1;
        }
        h = malloc((size_t) (k + p) * len);
        a = malloc((size_t) (k + p) * k);
        tbls = malloc((size_t) 32 * k * p);
        if (!h || !a || !tbls)
                return 1;
        for (i = 0; i < k * len; i++)
                h[i] = (unsigned char) (i * 131u + (i >> 9) * 7u + 1u);
        (void) hipMemcpy(base, h, (size_t) k * len, hipMemcpyHostToDevice);
        (void) hipMemset(base + (size_t) k * len, 0, (size_t) p * len);
        (void) hipDeviceSynchronize();
        gen(a, k + p, k);
        init(k, p, a + (size_t) k * k, tbls);
        for (i = 0; i < k; i++)
                data[i] = base + (size_t) i * len;
        for (l = 0; l < p; l++)
                coding[l] = base + (size_t) (k + l) * len;
        t2 = now_ms();
        enc(len, k, p, tbls, data, coding);
        t3 = now_ms();
        enc(len, k, p, tbls, data, coding);
        t4 = now_ms();
        /* parity check of sampled columns (the library's own host gf_mul) */
        (void) hipMemcpy(h + (size_t) k * len, base + (size_t) k * len, (size_t) p * len, hipMemcpyDeviceToHost);
        for (i = 0; i < len && ok; i += len / 97 + 1)
                for (l = 0; l < p; l++) {
                        unsigned char acc = 0;
                        for (j = 0; j < k; j++)
                                acc ^= mul(a[(size_t) (k + l) * k + j], h[(size_t) j * len + i]);
                        if (acc != h[(size_t) (k + l) * len + i])
                                ok = 0;
                }
        printf("{\"lib\": \"%s\", \"lib_bytes\": %lld, \"k\": %d, \"p\": %d, \"len\": %d, \"dlopen_ms\": %.3f, "
               "\"hip_init_and_alloc_ms\": %.3f, \"first_call_ms\": %.3f, \"second_call_us\": %.1f, "
               "\"dlopen_to_first_return_ms\": %.3f, \"self_check\": %s}\n",
               path, stat(path, &st) == 0 ? (long long) st.st_size : -1LL, k, p, len, t1 - t0, t2 - t1, t3 - t2,
               (t4 - t3) * 1e3, t3 - t0, ok ? "true" : "false");
        (void) hipFree(base);
        return ok ? 0 : 1;
}
