/* Per-call latency of the synchronous drop-in path from a plain C process
 * (/opt/rocm HIP runtime, no torch) — GPU box diagnostic. */
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "raid.h"

static double
now(void)
{
        struct timespec t;
        clock_gettime(CLOCK_MONOTONIC, &t);
        return t.tv_sec + t.tv_nsec * 1e-9;
}

int
main(void)
{
        enum { V = 17, N = 1024, REPS = 2000 };
        void *b[V];
        hipPointerAttribute_t a;
        double t;
        int i, r;
        for (i = 0; i < V; i++) {
                b[i] = malloc(N);
                for (r = 0; r < N; r++)
                        ((unsigned char *) b[i])[r] = (unsigned char) rand();
        }
        xor_gen(V, N, b);
        t = now();
        for (r = 0; r < REPS; r++)
                xor_check(V, N, b);
        printf("xor_check host 17x1KiB: %.1f us/call\n", (now() - t) / REPS * 1e6);
        t = now();
        for (r = 0; r < REPS * V; r++)
                (void) hipPointerGetAttributes(&a, b[r % V]);
        printf("hipPointerGetAttributes(host): %.2f us\n", (now() - t) / (REPS * V) * 1e6);
        {
                void *h, *d;
                hipStream_t st;
                (void) hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
                (void) hipHostMalloc(&h, 1 << 20, 0);
                (void) hipMalloc(&d, 1 << 20);
                t = now();
                for (r = 0; r < REPS; r++) {
                        (void) hipMemcpyAsync(d, h, 20 * 1024, hipMemcpyHostToDevice, st);
                        (void) hipStreamSynchronize(st);
                }
                printf("H2D 20 KiB pinned + sync: %.1f us\n", (now() - t) / REPS * 1e6);
                t = now();
                for (r = 0; r < REPS; r++) {
                        (void) hipMemcpyAsync(h, d, 8, hipMemcpyDeviceToHost, st);
                        (void) hipStreamSynchronize(st);
                }
                printf("D2H 8 B pinned + sync: %.1f us\n", (now() - t) / REPS * 1e6);
                t = now();
                for (r = 0; r < REPS; r++) {
                        (void) hipMemsetAsync(d, 0xff, 8, st);
                        (void) hipStreamSynchronize(st);
                }
                printf("memset 8 B + sync: %.1f us\n", (now() - t) / REPS * 1e6);
                t = now();
                for (r = 0; r < REPS; r++) {
                        (void) hipMemcpyAsync(d, h, 20 * 1024, hipMemcpyHostToDevice, st);
                        (void) hipMemcpyAsync(h, d, 8, hipMemcpyDeviceToHost, st);
                        (void) hipStreamSynchronize(st);
                }
                printf("H2D 20 KiB + D2H 8 B + one sync: %.1f us\n", (now() - t) / REPS * 1e6);
                {
                        void *dv[V];
                        for (i = 0; i < V; i++) {
                                (void) hipMalloc(&dv[i], N);
                                (void) hipMemcpy(dv[i], b[i], N, hipMemcpyHostToDevice);
                        }
                        t = now();
                        for (r = 0; r < REPS; r++)
                                xor_check(V, N, dv);
                        printf("xor_check device 17x1KiB: %.1f us/call\n", (now() - t) / REPS * 1e6);
                }
        }
        return 0;
}
