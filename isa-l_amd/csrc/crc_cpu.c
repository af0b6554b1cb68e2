/*
 * crc_cpu.c — the CPU route of the reference's checksum entry points
 * (crc32_iscsi: include/crc.h:136-150, semantics crc/crc_base.c:205-219;
 * crc64_*: include/crc64.h:54-163, semantics crc/crc64_base.c:569-670) for
 * buffers in host memory. Device-resident buffers go to the GPU checksum
 * kernels instead (isal_hip_shim.c "checksum entry points").
 *
 *   CRC32C: from 256 bytes on, the CRC64 section's carry-less folding with
 *           the Castagnoli constants; the rest through the SSE4.2 crc32
 *           instruction, which computes exactly the reference's reflected
 *           byte step (no inversions), 8 bytes at a time; without SSE4.2 /
 *           PCLMULQDQ, slicing-by-8 tables of the same polynomial.
 *   CRC64:  from 256 bytes on, carry-less multiplication (PCLMULQDQ): eight
 *           128-bit lanes fold 128 bytes per step, then the lanes fold into
 *           one and its 16 bytes go through the sliced loop below; the
 *           register enters by XOR into the first 8 bytes (raw(s, D) =
 *           raw(0, D ^ s), crc64_host.c). Shorter inputs and CPUs without
 *           PCLMULQDQ: slicing-by-8 in the "u-domain" of crc64_host.c (u = the
 *           register, byte-swapped for the norm flavours), where 8 bytes d
 *           advance the register as u' = XOR_j A_j[byte j of (d ^ u)] for every
 *           flavour; the ragged tail runs the reference's byte loop on its table.
 * Tables are built once per process (pthread_once).
 */
#include <immintrin.h>
#include <pthread.h>
#include <stdint.h>
#include <string.h>

#include "isal_hip.h"
#include "isal_hip_internal.h"

/* ---- CRC32C ---------------------------------------------------------------- */

#define CRC32C_POLY_REFL 0x82F63B78u
#define CRC32C_POLY_NORM 0x1EDC6F41u

static uint32_t c32_slice[8][256];
static int c32_hw;
static uint64_t c32_fk[8][2]; /* folding constants, as c64_fk (the CRC64 section) */
static int c32_clmul;

static uint64_t
c32_rev64(uint64_t x)
{
        uint64_t r = 0;
        int i;
        for (i = 0; i < 64; i++)
                r |= ((x >> i) & 1) << (63 - i);
        return r;
}
static pthread_once_t c32_once = PTHREAD_ONCE_INIT;

static void
c32_init(void)
{
        int i, j;
        for (i = 0; i < 256; i++) {
                uint32_t c = (uint32_t) i;
                for (j = 0; j < 8; j++)
                        c = (c & 1) ? (c >> 1) ^ CRC32C_POLY_REFL : c >> 1;
                c32_slice[0][i] = c;
        }
        for (i = 0; i < 256; i++)
                for (j = 1; j < 8; j++)
                        c32_slice[j][i] = (c32_slice[j - 1][i] >> 8) ^ c32_slice[0][c32_slice[j - 1][i] & 0xff];
        for (i = 0; i < 8; i++) {
                /* K'(n) = rev64(x^(n-1) mod P) of the CRC64 section's folding, P of
                 * degree 32 (normal form 0x1EDC6F41): the same identities hold
                 * for the 32-bit register XORed into the first 4 bytes */
                const int d = 128 * (i + 1);
                uint32_t r = 1;
                for (j = 1; j <= d + 63; j++) {
                        r = (r >> 31) ? (r << 1) ^ CRC32C_POLY_NORM : r << 1;
                        if (j == d - 1)
                                c32_fk[i][1] = c32_rev64(r);
                }
                c32_fk[i][0] = c32_rev64(r);
        }
        __builtin_cpu_init();
        c32_hw = __builtin_cpu_supports("sse4.2");
        c32_clmul = __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("ssse3");
}

__attribute__((target("sse4.2"))) static uint32_t
c32_sse42(uint32_t crc, const unsigned char *p, uint64_t len)
{
        uint64_t c = crc;
        while (len && ((uintptr_t) p & 7)) {
                c = __builtin_ia32_crc32qi((uint32_t) c, *p++);
                len--;
        }
        while (len >= 8) {
                uint64_t w;
                memcpy(&w, p, 8);
                c = __builtin_ia32_crc32di(c, w);
                p += 8;
                len -= 8;
        }
        while (len--)
                c = __builtin_ia32_crc32qi((uint32_t) c, *p++);
        return (uint32_t) c;
}

static uint32_t
c32_sliced(uint32_t crc, const unsigned char *p, uint64_t len)
{
        while (len >= 8) {
                uint64_t w;
                memcpy(&w, p, 8);
                w ^= crc;
                crc = c32_slice[7][w & 0xff] ^ c32_slice[6][(w >> 8) & 0xff] ^ c32_slice[5][(w >> 16) & 0xff] ^
                      c32_slice[4][(w >> 24) & 0xff] ^ c32_slice[3][(w >> 32) & 0xff] ^
                      c32_slice[2][(w >> 40) & 0xff] ^ c32_slice[1][(w >> 48) & 0xff] ^ c32_slice[0][w >> 56];
                p += 8;
                len -= 8;
        }
        while (len--)
                crc = (crc >> 8) ^ c32_slice[0][(crc ^ *p++) & 0xff];
        return crc;
}


/* ---- CRC64 ----------------------------------------------------------------- */

static uint64_t c64_byte[ISAL_HIP_CRC64_NVARIANTS][256];
static uint64_t c64_slice[ISAL_HIP_CRC64_NVARIANTS][8 * 256];
static int c64_clmul;
static pthread_once_t c64_once = PTHREAD_ONCE_INIT;

/*
 * Folding. A 16-byte block read as the polynomial B(x) (first byte highest)
 * and a register s satisfy raw(s, B) = raw(0, B + s x^64), and for blocks
 * V then B', raw(0, V || B') = raw(0, V x^128 + B'): a running 128-bit V
 * absorbs the next block as V' = (V x^128 mod P) + B', and with V = H x^64 + L
 * (H, L 64-bit) V x^d = H (x^(d+64) mod P) + L (x^d mod P), two 64x64
 * carry-less products of at most 127 bits. Eight lanes each advance by
 * d = 1024 bits per 128-byte step and finally by 128 (7 - j) bits into one.
 *   norm flavours: blocks byte-reversed into integers (bit i = x^i), the
 *     constants K(n) = x^n mod P as they are;
 *   refl flavours: blocks as loaded (bit i = x^(127-i)), so H is the low
 *     qword and L the high one, and rev128(a b) = clmul(rev a, rev b) << 1;
 *     with K'(n) = rev64(x^(n-1) mod P) the shift cancels:
 *     rev128(H x^(d+64)) = clmul(rev H, K'(d+64)), likewise for L with K'(d).
 * fk[v][m] holds the (H, L) constant pair for d = 128 (m + 1), m = 0..7.
 */
static uint64_t c64_fk[ISAL_HIP_CRC64_NVARIANTS][8][2];

static uint64_t
xpow_mod(uint64_t p, int n) /* x^n mod (x^64 + p), normal form */
{
        uint64_t r = 1;
        int i;
        for (i = 0; i < n; i++)
                r = (r >> 63) ? (r << 1) ^ p : r << 1;
        return r;
}

static uint64_t
rev64(uint64_t x)
{
        uint64_t r = 0;
        int i;
        for (i = 0; i < 64; i++)
                r |= ((x >> i) & 1) << (63 - i);
        return r;
}

static void
c64_init(void)
{
        int v, m;
        for (v = 0; v < ISAL_HIP_CRC64_NVARIANTS; v++) {
                const uint64_t p = isal_hip_crc64_poly(v);
                const int refl = isal_hip_crc64_is_refl(v);
                isal_hip_crc64_cpu_tables(v, c64_byte[v], c64_slice[v]);
                for (m = 0; m < 8; m++) {
                        const int d = 128 * (m + 1);
                        c64_fk[v][m][0] = refl ? rev64(xpow_mod(p, d + 63)) : xpow_mod(p, d + 64);
                        c64_fk[v][m][1] = refl ? rev64(xpow_mod(p, d - 1)) : xpow_mod(p, d);
                }
        }
        __builtin_cpu_init();
        c64_clmul = __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("ssse3");
}

/* Sliced raw update of the u-domain register over n bytes (n % 8 == 0). */
static uint64_t
c64_sliced(const uint64_t *a, uint64_t u, const unsigned char *buf, uint64_t n)
{
        while (n >= 8) {
                uint64_t x;
                memcpy(&x, buf, 8);
                x ^= u;
                u = a[0 * 256 + (x & 0xff)] ^ a[1 * 256 + ((x >> 8) & 0xff)] ^ a[2 * 256 + ((x >> 16) & 0xff)] ^
                    a[3 * 256 + ((x >> 24) & 0xff)] ^ a[4 * 256 + ((x >> 32) & 0xff)] ^
                    a[5 * 256 + ((x >> 40) & 0xff)] ^ a[6 * 256 + ((x >> 48) & 0xff)] ^ a[7 * 256 + (x >> 56)];
                buf += 8;
                n -= 8;
        }
        return u;
}

typedef __m128i c64_v2di;

__attribute__((target("pclmul,ssse3"), always_inline)) static inline c64_v2di
c64_fold(c64_v2di v, c64_v2di k, const int refl)
{
        /* refl: H = qword 0 times k[0], L = qword 1 times k[1];
         * norm: H = qword 1 times k[0], L = qword 0 times k[1] */
        return refl ? _mm_xor_si128(_mm_clmulepi64_si128(v, k, 0x00), _mm_clmulepi64_si128(v, k, 0x11))
                    : _mm_xor_si128(_mm_clmulepi64_si128(v, k, 0x01), _mm_clmulepi64_si128(v, k, 0x10));
}

/* A block as the folding's 128-bit integer (see above). */
__attribute__((target("pclmul,ssse3"), always_inline)) static inline c64_v2di
c64_load(const unsigned char *p, const int refl)
{
        const __m128i bs = _mm_set_epi8(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
        const __m128i x = _mm_loadu_si128((const __m128i *) p);
        return refl ? x : _mm_shuffle_epi8(x, bs);
}

/* u-domain register after the first n bytes (n a multiple of 128, >= 128);
 * refl is a constant at both call sites, so each gets its own loop. */
__attribute__((target("pclmul,ssse3"), always_inline)) static inline uint64_t
c64_folded(const uint64_t (*fk)[2], const uint64_t *slice, const int refl, uint64_t u,
           const unsigned char *buf, uint64_t n)
{
        const __m128i bs = _mm_set_epi8(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
        c64_v2di l0, l1, l2, l3, l4, l5, l6, l7, k;
        unsigned char last[16];
        uint64_t i;
        l0 = c64_load(buf, refl);
        l1 = c64_load(buf + 16, refl);
        l2 = c64_load(buf + 32, refl);
        l3 = c64_load(buf + 48, refl);
        l4 = c64_load(buf + 64, refl);
        l5 = c64_load(buf + 80, refl);
        l6 = c64_load(buf + 96, refl);
        l7 = c64_load(buf + 112, refl);
        /* the register enters as the first 8 bytes of the stream */
        l0 = _mm_xor_si128(l0, refl ? _mm_set_epi64x(0, (long long) u)
                                    : _mm_set_epi64x((long long) __builtin_bswap64(u), 0));
        k = _mm_set_epi64x((long long) fk[7][1], (long long) fk[7][0]);
        for (i = 128; i < n; i += 128) {
                l0 = _mm_xor_si128(c64_fold(l0, k, refl), c64_load(buf + i, refl));
                l1 = _mm_xor_si128(c64_fold(l1, k, refl), c64_load(buf + i + 16, refl));
                l2 = _mm_xor_si128(c64_fold(l2, k, refl), c64_load(buf + i + 32, refl));
                l3 = _mm_xor_si128(c64_fold(l3, k, refl), c64_load(buf + i + 48, refl));
                l4 = _mm_xor_si128(c64_fold(l4, k, refl), c64_load(buf + i + 64, refl));
                l5 = _mm_xor_si128(c64_fold(l5, k, refl), c64_load(buf + i + 80, refl));
                l6 = _mm_xor_si128(c64_fold(l6, k, refl), c64_load(buf + i + 96, refl));
                l7 = _mm_xor_si128(c64_fold(l7, k, refl), c64_load(buf + i + 112, refl));
        }
#define C64_K(m) _mm_set_epi64x((long long) fk[m][1], (long long) fk[m][0])
        l7 = _mm_xor_si128(l7, _mm_xor_si128(c64_fold(l0, C64_K(6), refl), c64_fold(l1, C64_K(5), refl)));
        l7 = _mm_xor_si128(l7, _mm_xor_si128(c64_fold(l2, C64_K(4), refl), c64_fold(l3, C64_K(3), refl)));
        l7 = _mm_xor_si128(l7, _mm_xor_si128(c64_fold(l4, C64_K(2), refl), c64_fold(l5, C64_K(1), refl)));
        l7 = _mm_xor_si128(l7, c64_fold(l6, C64_K(0), refl));
#undef C64_K
        /* raw(0, the 16 bytes of the last lane) */
        if (!refl)
                l7 = _mm_shuffle_epi8(l7, bs);
        _mm_storeu_si128((__m128i *) last, l7);
        return c64_sliced(slice, 0, last, 16);
}

__attribute__((target("pclmul,ssse3"))) static uint64_t
c64_folded_refl(int variant, uint64_t u, const unsigned char *buf, uint64_t n)
{
        return c64_folded((const uint64_t(*)[2]) c64_fk[variant], c64_slice[variant], 1, u, buf, n);
}

__attribute__((target("pclmul,ssse3"))) static uint64_t
c64_folded_norm(int variant, uint64_t u, const unsigned char *buf, uint64_t n)
{
        return c64_folded((const uint64_t(*)[2]) c64_fk[variant], c64_slice[variant], 0, u, buf, n);
}

uint64_t
isal_cpu_crc64(int variant, uint64_t init, const unsigned char *buf, uint64_t len)
{
        const int refl = isal_hip_crc64_is_refl(variant);
        const uint64_t *t = c64_byte[variant];
        uint64_t s = ~init, u, n;
        pthread_once(&c64_once, c64_init);
        u = refl ? s : __builtin_bswap64(s);
        n = len & ~(uint64_t) 127;
        if (c64_clmul && len >= 256 && isal_hip_knob(ISAL_HIP_KNOB_CPU_SIMD) != 0) {
                u = refl ? c64_folded_refl(variant, u, buf, n) : c64_folded_norm(variant, u, buf, n);
                buf += n;
                len -= n;
        }
        n = len & ~(uint64_t) 7;
        u = c64_sliced(c64_slice[variant], u, buf, n);
        buf += n;
        len -= n;
        s = refl ? u : __builtin_bswap64(u);
        while (len--) {
                const unsigned char b = *buf++;
                s = refl ? t[(s ^ b) & 0xff] ^ (s >> 8) : t[((s >> 56) ^ b) & 0xff] ^ (s << 8);
        }
        return ~s;
}

/* ---- CRC32C through the same folding (reflected, 32-bit register) --------- */

__attribute__((target("pclmul,ssse3"))) static uint32_t
c32_folded(uint32_t crc, const unsigned char *buf, uint64_t n)
{
        c64_v2di l0, l1, l2, l3, l4, l5, l6, l7, k;
        unsigned char last[16];
        uint64_t i;
        l0 = _mm_xor_si128(c64_load(buf, 1), _mm_set_epi64x(0, (long long) crc));
        l1 = c64_load(buf + 16, 1);
        l2 = c64_load(buf + 32, 1);
        l3 = c64_load(buf + 48, 1);
        l4 = c64_load(buf + 64, 1);
        l5 = c64_load(buf + 80, 1);
        l6 = c64_load(buf + 96, 1);
        l7 = c64_load(buf + 112, 1);
        k = _mm_set_epi64x((long long) c32_fk[7][1], (long long) c32_fk[7][0]);
        for (i = 128; i < n; i += 128) {
                l0 = _mm_xor_si128(c64_fold(l0, k, 1), c64_load(buf + i, 1));
                l1 = _mm_xor_si128(c64_fold(l1, k, 1), c64_load(buf + i + 16, 1));
                l2 = _mm_xor_si128(c64_fold(l2, k, 1), c64_load(buf + i + 32, 1));
                l3 = _mm_xor_si128(c64_fold(l3, k, 1), c64_load(buf + i + 48, 1));
                l4 = _mm_xor_si128(c64_fold(l4, k, 1), c64_load(buf + i + 64, 1));
                l5 = _mm_xor_si128(c64_fold(l5, k, 1), c64_load(buf + i + 80, 1));
                l6 = _mm_xor_si128(c64_fold(l6, k, 1), c64_load(buf + i + 96, 1));
                l7 = _mm_xor_si128(c64_fold(l7, k, 1), c64_load(buf + i + 112, 1));
        }
#define C32_K(m) _mm_set_epi64x((long long) c32_fk[m][1], (long long) c32_fk[m][0])
        l7 = _mm_xor_si128(l7, _mm_xor_si128(c64_fold(l0, C32_K(6), 1), c64_fold(l1, C32_K(5), 1)));
        l7 = _mm_xor_si128(l7, _mm_xor_si128(c64_fold(l2, C32_K(4), 1), c64_fold(l3, C32_K(3), 1)));
        l7 = _mm_xor_si128(l7, _mm_xor_si128(c64_fold(l4, C32_K(2), 1), c64_fold(l5, C32_K(1), 1)));
        l7 = _mm_xor_si128(l7, c64_fold(l6, C32_K(0), 1));
#undef C32_K
        _mm_storeu_si128((__m128i *) last, l7);
        return c32_sliced(0, last, 16);
}

uint32_t
isal_cpu_crc32c(uint32_t init, const unsigned char *buf, uint64_t len)
{
        const int simd = isal_hip_knob(ISAL_HIP_KNOB_CPU_SIMD) != 0;
        pthread_once(&c32_once, c32_init);
        if (!len)
                return init;
        if (c32_clmul && simd && len >= 256) {
                const uint64_t n = len & ~(uint64_t) 127;
                init = c32_folded(init, buf, n);
                buf += n;
                len -= n;
                if (!len)
                        return init;
        }
        if (c32_hw && simd)
                return c32_sse42(init, buf, len);
        return c32_sliced(init, buf, len);
}
