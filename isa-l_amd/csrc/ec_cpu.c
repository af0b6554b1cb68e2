/*
 * ec_cpu.c — the engine's host route: GF(2^8) encode / update / verify of
 * HOST-resident shards on the CPU.
 *
 * Why a CPU route in a GPU engine: a drop-in call is one synchronous stripe
 * (reference erasure_code.h:108-147). For host-resident shards of a few KiB a
 * GPU round trip (~30 us: classify, DMA in, launch, DMA out, sync) costs more
 * than the arithmetic, and the reference itself routes short lengths to its
 * portable path (ec_highlevel_func.c:159-194, :347-350). The shim therefore
 * sends small host calls here (ISAL_HIP_CPU_MAX_BYTES), and also uses this
 * route for ISAL_HIP_BACKEND=cpu, on hosts without a usable GPU, and as the
 * fallback when a HIP call fails part-way through a host-resident call (the
 * reference API has no error channel, so a call must not fail where the
 * reference succeeds). Device-resident shards never come here.
 *
 * Semantics are ec_base.c:282-342 (and the verify op of the RAID checks,
 * raid_base.c:70-140): only byte 1 of each 32-byte gftbls entry — the
 * coefficient c — is read, exactly like the reference's base functions, so
 * the answer is the reference's for ANY gftbls. The arithmetic is written
 * fresh for this route, in three widths picked by what the CPU has:
 *   - GFNI + AVX-512: c*x is the GF(2)-linear map x -> A_c x with A_c the 8x8
 *     bit matrix whose column j is c*2^j; vgf2p8affineqb applies it to 64
 *     bytes at once (the reference's fastest kernels do the same,
 *     gf_vect_gfni.inc:34-72); tails use masked loads/stores;
 *   - AVX2: c*x = lo_c[x & 15] ^ hi_c[x >> 4] with 16-entry nibble product
 *     tables, 32 columns per vpshufb pair;
 *   - per byte with the same nibble tables.
 * ISAL_HIP_CPU_SIMD = 2 / 1 / 0 caps the width (tests run all three).
 */
#include <immintrin.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "erasure_code.h"
#include "isal_hip_internal.h"

typedef struct {
        uint8_t lo[16]; /* c * {0x00 .. 0x0f} */
        uint8_t hi[16]; /* c * {0x00, 0x10 .. 0xf0} */
        uint64_t aff;   /* A_c for vgf2p8affineqb: byte 7-i, bit j = bit i of c*2^j */
} nib_t;

#define BLOCK 4096 /* columns per block: a block of every source stays in L1/L2 */
#define GROUP 4    /* outputs per pass over the sources (accumulators in registers) */

/* By linearity from c*2^b (b = 0..7): entry i is entry (i with its lowest set
 * bit cleared) XOR the product of that bit — 30 XORs, no multiplies. */
static void
nib_tables(unsigned char c, nib_t *t)
{
        uint8_t p[8];
        int b, i;
        p[0] = c;
        for (b = 1; b < 8; b++)
                p[b] = (uint8_t) ((p[b - 1] << 1) ^ ((p[b - 1] & 0x80) ? 0x1d : 0));
        t->lo[0] = t->hi[0] = 0;
        for (i = 1; i < 16; i++) {
                b = __builtin_ctz((unsigned) i);
                t->lo[i] = (uint8_t) (t->lo[i & (i - 1)] ^ p[b]);
                t->hi[i] = (uint8_t) (t->hi[i & (i - 1)] ^ p[b + 4]);
        }
        t->aff = 0; /* filled by aff_matrix() when the GFNI path runs */
}

/* A_c from the column images c*2^b already in the nibble tables (lo[1 << b],
 * hi[1 << (b - 4)]): a bit-matrix transpose, only for the GFNI path. */
static void
aff_matrix(nib_t *t)
{
        int b, i;
        t->aff = 0;
        for (b = 0; b < 8; b++) { /* column b: the image c*2^b of input bit b */
                const uint8_t img = b < 4 ? t->lo[1 << b] : t->hi[1 << (b - 4)];
                for (i = 0; i < 8; i++) /* output bit i lives in byte 7 - i */
                        if ((img >> i) & 1)
                                t->aff |= (uint64_t) 1 << (8 * (7 - i) + b);
        }
}

static inline uint8_t
mul_nib(const nib_t *t, uint8_t x)
{
        return (uint8_t) (t->lo[x & 15] ^ t->hi[x >> 4]);
}

static inline unsigned long long
mkey(long long col, int row)
{
        return ((unsigned long long) col << 8) | (unsigned) row;
}

/* ---- per byte ------------------------------------------------------------ */

/* Outputs r0 .. r0+G-1 over columns [a, b). T[n*k + j] = tables of c[r0+n][j].
 * verify: compare instead of store; returns the smallest mismatch key. */
static unsigned long long
group_scalar(long long a, long long b, int k, int r0, int G, const nib_t *T,
             unsigned char *const *src, unsigned char *const *dst, int verify)
{
        long long i;
        int n, j;
        for (i = a; i < b; i++)
                for (n = 0; n < G; n++) {
                        uint8_t s = 0;
                        for (j = 0; j < k; j++)
                                s ^= mul_nib(&T[n * k + j], src[j][i]);
                        if (!verify)
                                dst[r0 + n][i] = s;
                        else if (dst[r0 + n][i] != s)
                                return mkey(i, r0 + n); /* columns ascend, rows ascend */
                }
        return ~0ull;
}

static void
mad_scalar(long long a, long long b, int rows, const nib_t *T, const unsigned char *src,
           unsigned char *const *dst)
{
        long long i;
        int l;
        for (l = 0; l < rows; l++)
                for (i = a; i < b; i++)
                        dst[l][i] ^= mul_nib(&T[l], src[i]);
}

/* ---- AVX2: 32 columns per step ------------------------------------------- */

#define AVX2 __attribute__((target("avx2")))

static inline AVX2 __attribute__((always_inline)) __m256i
tab256(const uint8_t *t16)
{
        return _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *) t16));
}

static inline AVX2 __attribute__((always_inline)) __m256i
mul32(const nib_t *t, __m256i lo, __m256i hi)
{
        return _mm256_xor_si256(_mm256_shuffle_epi8(tab256(t->lo), lo),
                                _mm256_shuffle_epi8(tab256(t->hi), hi));
}

/* G is a compile-time constant at every call site (always_inline), so the
 * accumulators live in registers. */
static inline AVX2 __attribute__((always_inline)) unsigned long long
group_avx2_g(long long a, long long b, int k, int r0, const int G, const nib_t *T,
             unsigned char *const *src, unsigned char *const *dst, int verify)
{
        const __m256i m = _mm256_set1_epi8(0x0f);
        long long i = a;
        int j, n;
        for (; i + 32 <= b; i += 32) {
                __m256i acc[GROUP];
                for (n = 0; n < G; n++)
                        acc[n] = _mm256_setzero_si256();
                for (j = 0; j < k; j++) {
                        const __m256i x = _mm256_loadu_si256((const __m256i *) (src[j] + i));
                        const __m256i lo = _mm256_and_si256(x, m);
                        const __m256i hi = _mm256_and_si256(_mm256_srli_epi64(x, 4), m);
                        for (n = 0; n < G; n++)
                                acc[n] = _mm256_xor_si256(acc[n], mul32(&T[n * k + j], lo, hi));
                }
                if (!verify) {
                        for (n = 0; n < G; n++)
                                _mm256_storeu_si256((__m256i *) (dst[r0 + n] + i), acc[n]);
                } else {
                        unsigned long long best = ~0ull;
                        for (n = 0; n < G; n++) {
                                const __m256i d = _mm256_loadu_si256((const __m256i *) (dst[r0 + n] + i));
                                const unsigned eq = (unsigned) _mm256_movemask_epi8(_mm256_cmpeq_epi8(d, acc[n]));
                                if (eq != 0xffffffffu) {
                                        const unsigned long long key = mkey(i + __builtin_ctz(~eq), r0 + n);
                                        if (key < best)
                                                best = key;
                                }
                        }
                        if (best != ~0ull)
                                return best;
                }
        }
        return i < b ? group_scalar(i, b, k, r0, G, T, src, dst, verify) : ~0ull;
}

static AVX2 unsigned long long
group_avx2(long long a, long long b, int k, int r0, int G, const nib_t *T,
           unsigned char *const *src, unsigned char *const *dst, int verify)
{
        switch (G) {
        case 1:
                return group_avx2_g(a, b, k, r0, 1, T, src, dst, verify);
        case 2:
                return group_avx2_g(a, b, k, r0, 2, T, src, dst, verify);
        case 3:
                return group_avx2_g(a, b, k, r0, 3, T, src, dst, verify);
        default:
                return group_avx2_g(a, b, k, r0, GROUP, T, src, dst, verify);
        }
}

static AVX2 void
mad_avx2(long long a, long long b, int rows, const nib_t *T, const unsigned char *src,
         unsigned char *const *dst)
{
        const __m256i m = _mm256_set1_epi8(0x0f);
        long long i = a;
        int l;
        for (; i + 32 <= b; i += 32) {
                const __m256i x = _mm256_loadu_si256((const __m256i *) (src + i));
                const __m256i lo = _mm256_and_si256(x, m);
                const __m256i hi = _mm256_and_si256(_mm256_srli_epi64(x, 4), m);
                for (l = 0; l < rows; l++) {
                        __m256i *d = (__m256i *) (dst[l] + i);
                        _mm256_storeu_si256(d, _mm256_xor_si256(_mm256_loadu_si256(d), mul32(&T[l], lo, hi)));
                }
        }
        if (i < b)
                mad_scalar(i, b, rows, T, src, dst);
}

/* ---- GFNI + AVX-512: 64 columns per step ---------------------------------- */

#define GFNI __attribute__((target("avx512f,avx512bw,gfni")))
#define GFNI_MIN_COLUMNS 4096 /* shorter calls use the AVX2 path (see isal_cpu_run) */

static inline GFNI __attribute__((always_inline)) __mmask64
cols_mask(long long n)
{
        return n >= 64 ? ~(__mmask64) 0 : (((__mmask64) 1 << n) - 1);
}

static inline GFNI __attribute__((always_inline)) unsigned long long
group_gfni_g(long long a, long long b, int k, int r0, const int G, const nib_t *T,
             unsigned char *const *src, unsigned char *const *dst, int verify)
{
        long long i;
        int j, n;
        for (i = a; i < b; i += 64) {
                const __mmask64 m = cols_mask(b - i); /* masked-off bytes are never touched */
                __m512i acc[GROUP];
                for (n = 0; n < G; n++)
                        acc[n] = _mm512_setzero_si512();
                for (j = 0; j < k; j++) {
                        const __m512i x = _mm512_maskz_loadu_epi8(m, src[j] + i);
                        for (n = 0; n < G; n++)
                                acc[n] = _mm512_xor_si512(
                                        acc[n], _mm512_gf2p8affine_epi64_epi8(
                                                        x, _mm512_set1_epi64((long long) T[n * k + j].aff), 0));
                }
                if (!verify) {
                        for (n = 0; n < G; n++)
                                _mm512_mask_storeu_epi8(dst[r0 + n] + i, m, acc[n]);
                } else {
                        unsigned long long best = ~0ull;
                        for (n = 0; n < G; n++) {
                                const __m512i d = _mm512_maskz_loadu_epi8(m, dst[r0 + n] + i);
                                const __mmask64 ne = _mm512_mask_cmpneq_epi8_mask(m, d, acc[n]);
                                if (ne) {
                                        const unsigned long long key = mkey(i + __builtin_ctzll(ne), r0 + n);
                                        if (key < best)
                                                best = key;
                                }
                        }
                        if (best != ~0ull)
                                return best;
                }
        }
        return ~0ull;
}

static GFNI unsigned long long
group_gfni(long long a, long long b, int k, int r0, int G, const nib_t *T,
           unsigned char *const *src, unsigned char *const *dst, int verify)
{
        switch (G) {
        case 1:
                return group_gfni_g(a, b, k, r0, 1, T, src, dst, verify);
        case 2:
                return group_gfni_g(a, b, k, r0, 2, T, src, dst, verify);
        case 3:
                return group_gfni_g(a, b, k, r0, 3, T, src, dst, verify);
        default:
                return group_gfni_g(a, b, k, r0, GROUP, T, src, dst, verify);
        }
}

static GFNI void
mad_gfni(long long a, long long b, int rows, const nib_t *T, const unsigned char *src,
         unsigned char *const *dst)
{
        long long i;
        int l;
        for (i = a; i < b; i += 64) {
                const __mmask64 m = cols_mask(b - i);
                const __m512i x = _mm512_maskz_loadu_epi8(m, src + i);
                for (l = 0; l < rows; l++) {
                        const __m512i d = _mm512_maskz_loadu_epi8(m, dst[l] + i);
                        _mm512_mask_storeu_epi8(dst[l] + i, m,
                                                _mm512_xor_si512(d, _mm512_gf2p8affine_epi64_epi8(
                                                                            x, _mm512_set1_epi64((long long) T[l].aff), 0)));
                }
        }
}

enum { SIMD_NONE = 0, SIMD_AVX2 = 1, SIMD_GFNI = 2 };

/* Widest path this CPU has, capped by ISAL_HIP_CPU_SIMD (0 / 1 / 2). */
static int
cpu_simd(void)
{
        static int have = -1;
        long long cap;
        if (have < 0)
                have = __builtin_cpu_supports("avx512bw") && __builtin_cpu_supports("gfni")
                               ? SIMD_GFNI
                               : __builtin_cpu_supports("avx2") ? SIMD_AVX2 : SIMD_NONE;
        cap = isal_hip_knob(ISAL_HIP_KNOB_CPU_SIMD);
        return cap >= 0 && cap < have ? (int) cap : have;
}

/* ---- entry ---------------------------------------------------------------- */

unsigned long long
isal_cpu_run(int op, long long c0, int len, int k, int rows, int vec_i, const unsigned char *gftbls,
             unsigned char *const *src, int nsrc, unsigned char *const *dst)
{
        /* short calls stay on 256-bit code: on the container's Xeon the first
         * 512-bit instructions of a burst of tiny calls cost more than they
         * save (xor_check_test: 16 s AVX2, 30 s GFNI) */
        const int simd0 = cpu_simd();
        const int simd = simd0 == SIMD_GFNI && (long long) len - c0 < GFNI_MIN_COLUMNS
                                 && isal_hip_knob(ISAL_HIP_KNOB_CPU_SIMD) != SIMD_GFNI
                         ? SIMD_AVX2
                         : simd0;
        const int ncoef = op == ISAL_HIP_OP_UPDATE ? rows : rows * k;
        nib_t stack_tab[64], *T;
        unsigned long long best = ~0ull;
        long long a;
        int l, j;

        if (len <= c0 || rows <= 0 || k < 0)
                return best;
        T = ncoef <= 64 ? stack_tab : (nib_t *) malloc(sizeof(nib_t) * (size_t) ncoef);
        if (!T)
                abort(); /* out of host memory: the reference would not get this far either */

        if (op == ISAL_HIP_OP_UPDATE) {
                /* dst[l] ^= c[l][vec_i] * src (ec_base.c:327-342) */
                for (l = 0; l < rows; l++) {
                        nib_tables(gftbls[((size_t) l * k + vec_i) * 32 + 1], &T[l]);
                        if (simd == SIMD_GFNI)
                                aff_matrix(&T[l]);
                }
                for (a = c0; a < len; a += BLOCK) {
                        const long long b = len - a < BLOCK ? len : a + BLOCK;
                        if (simd == SIMD_GFNI)
                                mad_gfni(a, b, rows, T, src[0], dst);
                        else if (simd == SIMD_AVX2)
                                mad_avx2(a, b, rows, T, src[0], dst);
                        else
                                mad_scalar(a, b, rows, T, src[0], dst);
                }
        } else {
                /* dst[l] = XOR_j c[l][j] * src[j] (ec_base.c:309-325), or compare */
                const int verify = op == ISAL_HIP_OP_VERIFY;
                (void) nsrc;
                for (l = 0; l < rows; l++)
                        for (j = 0; j < k; j++) {
                                nib_t *tj = &T[(size_t) l * k + j];
                                nib_tables(gftbls[((size_t) l * k + j) * 32 + 1], tj);
                                if (simd == SIMD_GFNI)
                                        aff_matrix(tj);
                        }
                for (a = c0; a < len && best == ~0ull; a += BLOCK) {
                        const long long b = len - a < BLOCK ? len : a + BLOCK;
                        int r0;
                        for (r0 = 0; r0 < rows; r0 += GROUP) {
                                const int G = rows - r0 < GROUP ? rows - r0 : GROUP;
                                const nib_t *Tg = T + (size_t) r0 * k;
                                unsigned long long key;
                                if (k == 0) { /* empty sum: zero parity */
                                        int n;
                                        for (n = 0; n < G && !verify; n++)
                                                memset(dst[r0 + n] + a, 0, (size_t) (b - a));
                                        for (n = 0; n < G && verify; n++) {
                                                long long i;
                                                for (i = a; i < b; i++)
                                                        if (dst[r0 + n][i]) {
                                                                key = mkey(i, r0 + n);
                                                                best = key < best ? key : best;
                                                                break;
                                                        }
                                        }
                                        continue;
                                }
                                key = simd == SIMD_GFNI ? group_gfni(a, b, k, r0, G, Tg, src, dst, verify)
                                      : simd == SIMD_AVX2 ? group_avx2(a, b, k, r0, G, Tg, src, dst, verify)
                                                          : group_scalar(a, b, k, r0, G, Tg, src, dst, verify);
                                if (key < best)
                                        best = key;
                        }
                }
        }
        if (T != stack_tab)
                free(T);
        return best;
}
