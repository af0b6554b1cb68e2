/*
 * stage_probe.c — how fast can a synchronous host-resident drop-in call move
 * its shards? (GPU box diagnostic for the shim's staging path, not shipped.)
 *
 * A storage caller hands ec_encode_data plain pageable buffers: k sources in,
 * p parity out. This times, for one k=10 p=4 call of `len`-byte shards:
 *   async      whether a pageable hipMemcpyAsync returns before the copy is done;
 *   register   hipHostRegister + hipHostUnregister of one shard;
 *   memcpy     one host thread copying a shard into pinned memory (bounce rate);
 *   seq        all k H2D then all p D2H on one stream, one sync (the shim's
 *              current chunked path without the kernel);
 *   2thr       H2D issued by one host thread on one stream while a second
 *              thread issues the D2H on another (do pageable copies overlap?);
 *   reg        register all shards, H2D and D2H on two streams, unregister;
 *   bounce     pinned bounce ring: memcpy chunk i+1 while chunk i DMAs.
 * Build: gcc -O2 tools/stage_probe.c -I/opt/rocm/include -D__HIP_PLATFORM_AMD__
 *        -L/opt/rocm/lib -lamdhip64 -lpthread -o tools/stage_probe
 */
#include <hip/hip_runtime_api.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define CK(x)                                                                                      \
        do {                                                                                       \
                hipError_t e_ = (x);                                                               \
                if (e_ != hipSuccess) {                                                            \
                        fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                    \
                        exit(1);                                                                   \
                }                                                                                  \
        } while (0)

static double
now(void)
{
        struct timespec t;
        clock_gettime(CLOCK_MONOTONIC, &t);
        return t.tv_sec + t.tv_nsec * 1e-9;
}

enum { K = 10, P = 4 };
static size_t len;
static unsigned char *hs[K + P], *ds[K + P];
static hipStream_t s1, s2;

static void *
d2h_thread(void *arg)
{
        (void) arg;
        for (int l = 0; l < P; l++)
                CK(hipMemcpyAsync(hs[K + l], ds[K + l], len, hipMemcpyDeviceToHost, s2));
        CK(hipStreamSynchronize(s2));
        return NULL;
}

static double
best(double (*f)(void), int reps)
{
        double b = 1e9;
        for (int i = 0; i < reps; i++) {
                double t = f();
                if (t < b)
                        b = t;
        }
        return b;
}

static double
t_seq(void)
{
        double t0 = now();
        for (int j = 0; j < K; j++)
                CK(hipMemcpyAsync(ds[j], hs[j], len, hipMemcpyHostToDevice, s1));
        for (int l = 0; l < P; l++)
                CK(hipMemcpyAsync(hs[K + l], ds[K + l], len, hipMemcpyDeviceToHost, s1));
        CK(hipStreamSynchronize(s1));
        return now() - t0;
}

static double
t_h2d_only(void)
{
        double t0 = now();
        for (int j = 0; j < K; j++)
                CK(hipMemcpyAsync(ds[j], hs[j], len, hipMemcpyHostToDevice, s1));
        CK(hipStreamSynchronize(s1));
        return now() - t0;
}

static double
t_2thr(void)
{
        pthread_t th;
        double t0 = now();
        pthread_create(&th, NULL, d2h_thread, NULL);
        for (int j = 0; j < K; j++)
                CK(hipMemcpyAsync(ds[j], hs[j], len, hipMemcpyHostToDevice, s1));
        CK(hipStreamSynchronize(s1));
        pthread_join(th, NULL);
        return now() - t0;
}

/* H2D of the k sources split over two host threads / two streams (even
 * shards on s1 from this thread, odd shards on s2 from a helper): does a
 * second issuing thread hide the per-copy cost? */
static void *
h2d_odd_thread(void *arg)
{
        (void) arg;
        for (int j = 1; j < K; j += 2)
                CK(hipMemcpyAsync(ds[j], hs[j], len, hipMemcpyHostToDevice, s2));
        CK(hipStreamSynchronize(s2));
        return NULL;
}

static double
t_h2d_2thr(void)
{
        pthread_t th;
        double t0 = now();
        pthread_create(&th, NULL, h2d_odd_thread, NULL);
        for (int j = 0; j < K; j += 2)
                CK(hipMemcpyAsync(ds[j], hs[j], len, hipMemcpyHostToDevice, s1));
        CK(hipStreamSynchronize(s1));
        pthread_join(th, NULL);
        return now() - t0;
}

static double
t_reg(void)
{
        double t0 = now();
        for (int i = 0; i < K + P; i++)
                CK(hipHostRegister(hs[i], len, hipHostRegisterDefault));
        for (int j = 0; j < K; j++)
                CK(hipMemcpyAsync(ds[j], hs[j], len, hipMemcpyHostToDevice, s1));
        for (int l = 0; l < P; l++)
                CK(hipMemcpyAsync(hs[K + l], ds[K + l], len, hipMemcpyDeviceToHost, s2));
        CK(hipStreamSynchronize(s1));
        CK(hipStreamSynchronize(s2));
        for (int i = 0; i < K + P; i++)
                CK(hipHostUnregister(hs[i]));
        return now() - t0;
}

static unsigned char *pin;
static size_t chunk = 1 << 20;

/* H2D of the k sources through a 4-slot pinned ring, memcpy overlapped with DMA */
static double
t_bounce(void)
{
        hipEvent_t ev[4];
        int used[4] = {0};
        for (int i = 0; i < 4; i++)
                CK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
        double t0 = now();
        int slot = 0;
        for (int j = 0; j < K; j++)
                for (size_t o = 0; o < len; o += chunk) {
                        size_t n = len - o < chunk ? len - o : chunk;
                        if (used[slot])
                                CK(hipEventSynchronize(ev[slot]));
                        memcpy(pin + slot * chunk, hs[j] + o, n);
                        CK(hipMemcpyAsync(ds[j] + o, pin + slot * chunk, n, hipMemcpyHostToDevice, s1));
                        CK(hipEventRecord(ev[slot], s1));
                        used[slot] = 1;
                        slot = (slot + 1) & 3;
                }
        CK(hipStreamSynchronize(s1));
        double t = now() - t0;
        for (int i = 0; i < 4; i++)
                CK(hipEventDestroy(ev[i]));
        return t;
}

int
main(int argc, char **argv)
{
        size_t lens[] = {1 << 20, 2 << 20, 4 << 20, 8 << 20};
        CK(hipSetDevice(0));
        CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
        CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
        CK(hipHostMalloc((void **) &pin, 4 * (8 << 20), 0));
        (void) argc;
        (void) argv;
        for (unsigned li = 0; li < sizeof(lens) / sizeof(lens[0]); li++) {
                len = lens[li];
                for (int i = 0; i < K + P; i++) {
                        hs[i] = (unsigned char *) aligned_alloc(4096, len);
                        memset(hs[i], i + 1, len);
                        CK(hipMalloc((void **) &ds[i], len));
                }
                /* async? one pageable H2D / D2H: time to return vs to complete */
                double a0 = now();
                CK(hipMemcpyAsync(ds[0], hs[0], len, hipMemcpyHostToDevice, s1));
                double a1 = now();
                CK(hipStreamSynchronize(s1));
                double a2 = now();
                CK(hipMemcpyAsync(hs[K], ds[K], len, hipMemcpyDeviceToHost, s1));
                double a3 = now();
                CK(hipStreamSynchronize(s1));
                double a4 = now();
                /* warm everything once */
                t_seq();
                t_2thr();
                double r0 = now();
                CK(hipHostRegister(hs[0], len, hipHostRegisterDefault));
                double r1 = now();
                CK(hipHostUnregister(hs[0]));
                double r2 = now();
                double m0 = now();
                for (int i = 0; i < K; i++)
                        memcpy(pin + (i & 3) * (8 << 20), hs[i], len);
                double m1 = now();
                double h2d2 = best(t_h2d_2thr, 5);
                double seq = best(t_seq, 5), h2d = best(t_h2d_only, 5), thr = best(t_2thr, 5),
                       reg = best(t_reg, 3);
                double bnc[3];
                size_t chunks[3] = {256 << 10, 1 << 20, 2 << 20};
                for (int c = 0; c < 3; c++) {
                        chunk = chunks[c];
                        bnc[c] = best(t_bounce, 5);
                }
                double mb = (double) len * (K + P) / 1e6, mbin = (double) len * K / 1e6;
                printf("{\"len\": %zu, \"call_MB\": %.1f, "
                       "\"h2d_return_us\": %.1f, \"h2d_complete_us\": %.1f, "
                       "\"d2h_return_us\": %.1f, \"d2h_complete_us\": %.1f, "
                       "\"register_us\": %.1f, \"unregister_us\": %.1f, "
                       "\"memcpy_to_pinned_gb_s\": %.1f, "
                       "\"seq_us\": %.1f, \"seq_gb_s\": %.1f, \"h2d_only_gb_s\": %.1f, "
                       "\"two_threads_us\": %.1f, \"two_threads_gb_s\": %.1f, "
                       "\"register_all_2streams_us\": %.1f, "
                       "\"bounce_h2d_gb_s_256k\": %.1f, \"bounce_h2d_gb_s_1m\": %.1f, "
                       "\"bounce_h2d_gb_s_2m\": %.1f, \"h2d_two_threads_gb_s\": %.1f}\n",
                       len, mb, (a1 - a0) * 1e6, (a2 - a0) * 1e6, (a3 - a2) * 1e6, (a4 - a2) * 1e6,
                       (r1 - r0) * 1e6, (r2 - r1) * 1e6, mbin / (m1 - m0) / 1e3, seq * 1e6,
                       mb / seq / 1e3, mbin / h2d / 1e3, thr * 1e6, mb / thr / 1e3, reg * 1e6,
                       mbin / bnc[0] / 1e3, mbin / bnc[1] / 1e3, mbin / bnc[2] / 1e3, mbin / h2d2 / 1e3);
                fflush(stdout);
                for (int i = 0; i < K + P; i++) {
                        free(hs[i]);
                        CK(hipFree(ds[i]));
                }
        }
        return 0;
}
