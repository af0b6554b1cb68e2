/*
 * isal_hip_raid.c — RAID-5/6 parity (include/raid.h) on the erasure-code
 * kernels. Replaces the reference raid/ path (raid_base.c:44-140 semantics,
 * multibinary dispatch raid_multibinary.asm) — SURVEY.md §8(f) "next" row 2.
 *
 *   xor_gen  = ec_encode_data with one row of 1s over array[0..vects-2]
 *   pq_gen   = ec_encode_data with rows {1,..,1} and {2^0, 2^1, .., 2^(n-1)}:
 *              the reference's Horner loop q = D_j ^ 2q from the last source
 *              down (raid_base.c:56-62) is exactly sum_j 2^j * D_j
 *   *_check  = the verify kernel (recompute + compare, first mismatch)
 */
#define ISAL_HIP_DEPRECATED /* defining, not using */
#include <stdlib.h>
#include <string.h>

#include "raid.h"
#include "erasure_code.h"
#include "isal_hip_internal.h"

/* gftbls (base format: byte 1 of each 32-B entry is the coefficient) for
 * rows = 1 (P) or 2 (P, Q) over n sources. */
static unsigned char *
raid_build(int n, int rows)
{
        unsigned char *t = (unsigned char *) calloc((size_t) 32 * n * rows, 1);
        unsigned char q = 1;
        int j;
        if (!t)
                return NULL;
        for (j = 0; j < n; j++) {
                t[(size_t) j * 32 + 1] = 1; /* P row */
                if (rows == 2) {
                        t[((size_t) n + j) * 32 + 1] = q; /* Q row: 2^j */
                        q = gf_mul(q, 2);
                }
        }
        return t;
}

/* The tables for up to RAID_CACHE_MAX sources are built once per (n, rows)
 * and shared by every later call and thread (immutable once published), so
 * a RAID call allocates nothing and the shim's per-thread table cache finds
 * the same coefficients call after call. *owned: the caller frees it. */
#define RAID_CACHE_MAX 255
static unsigned char *raid_cache[2][RAID_CACHE_MAX + 1];

static const unsigned char *
raid_tables(int n, int rows, int *owned)
{
        unsigned char *t, *want = NULL;
        *owned = 0;
        if (n < 1 || rows < 1 || rows > 2)
                return NULL;
        if (n > RAID_CACHE_MAX) {
                *owned = 1;
                return raid_build(n, rows);
        }
        t = __atomic_load_n(&raid_cache[rows - 1][n], __ATOMIC_ACQUIRE);
        if (t)
                return t;
        if (!(t = raid_build(n, rows)))
                return NULL;
        if (!__atomic_compare_exchange_n(&raid_cache[rows - 1][n], &want, t, 0, __ATOMIC_ACQ_REL,
                                         __ATOMIC_ACQUIRE)) {
                free(t); /* another thread published the same table first */
                return want;
        }
        return t;
}

static int
raid_run(const char *fn, int op, int len, int nsrc, int rows, void **array)
{
        int owned;
        const unsigned char *t = raid_tables(nsrc, rows, &owned);
        unsigned long long bad;
        if (!t)
                return 1;
        bad = isal_hip_run(fn, op, len, nsrc, rows, 0, t, (unsigned char *const *) array, nsrc,
                           (unsigned char *const *) array + nsrc);
        if (owned)
                free((void *) t);
        if (op != ISAL_HIP_OP_VERIFY || bad == ~0ull)
                return 0;
        /* reference pq_check_base: i | 1 when P differs at byte i, else i | 2 */
        return (int) (bad >> 8) | ((bad & 0xff) == 0 ? 1 : 2);
}

int
xor_gen(int vects, int len, void **array)
{
        if (vects < 3)
                return 1;
        return raid_run("xor_gen", ISAL_HIP_OP_ENCODE, len, vects - 1, 1, array);
}

int
xor_gen_base(int vects, int len, void **array)
{
        return xor_gen(vects, len, array);
}

int
xor_check(int vects, int len, void **array)
{
        if (vects < 2)
                return 1;
        /* XOR of all == 0  <=>  XOR of the first vects-1 equals the last */
        return raid_run("xor_check", ISAL_HIP_OP_VERIFY, len, vects - 1, 1, array) ? 1 : 0;
}

int
xor_check_base(int vects, int len, void **array)
{
        return xor_check(vects, len, array);
}

int
pq_gen(int vects, int len, void **array)
{
        if (vects < 4)
                return 1;
        if (len == 0)
                return 0;
        if (len % 32)
                return 1;
        return raid_run("pq_gen", ISAL_HIP_OP_ENCODE, len, vects - 2, 2, array);
}

int
pq_gen_base(int vects, int len, void **array)
{
        if (vects < 4)
                return 1;
        return raid_run("pq_gen_base", ISAL_HIP_OP_ENCODE, len & ~7, vects - 2, 2, array);
}

int
pq_check(int vects, int len, void **array)
{
        if (vects < 4)
                return 1;
        return raid_run("pq_check", ISAL_HIP_OP_VERIFY, len, vects - 2, 2, array);
}

int
pq_check_base(int vects, int len, void **array)
{
        return pq_check(vects, len, array);
}

int xor_gen_sse(int vects, int len, void **array) { return xor_gen(vects, len, array); }
int xor_gen_avx(int vects, int len, void **array) { return xor_gen(vects, len, array); }
int xor_check_sse(int vects, int len, void **array) { return xor_check(vects, len, array); }
int pq_gen_sse(int vects, int len, void **array) { return pq_gen(vects, len, array); }
int pq_gen_avx(int vects, int len, void **array) { return pq_gen(vects, len, array); }
int pq_gen_avx2(int vects, int len, void **array) { return pq_gen(vects, len, array); }
int pq_check_sse(int vects, int len, void **array) { return pq_check(vects, len, array); }
