/*
 * ec_gfni_port.c — TEST/BASELINE INFRASTRUCTURE ONLY: a C-intrinsics port of the
 * reference's fastest x86 erasure-code path, used as a CPU throughput baseline.
 *
 * The reference's own AVX-512+GFNI kernels are NASM sources
 * (erasure_code/gf_{1..6}vect_dot_prod_avx512_gfni.asm, macro GF_MUL_XOR at
 * gf_vect_gfni.inc:34-72) and the image has no nasm, so they cannot be
 * assembled here. This file restates them:
 *   - per coefficient c, an 8x8 GF(2) affine matrix (the reference's
 *     gf_table_gfni[c], ec_base.h:37-102, derived here from c), broadcast to
 *     a zmm register (ec_init_tables_gfni, ec_highlevel_func.c:453-464);
 *   - rows grouped by <= 6 like ec_encode_data_avx512_gfni
 *     (ec_highlevel_func.c:466-497);
 *   - per 64-byte column: load each source once, vgf2p8affineqb + vpxorq into
 *     up to 6 accumulators, store (gf_4vect_dot_prod_avx512_gfni.asm:207-250);
 *     masked tail for len % 64 (:233-242).
 * Only bench.py's cpu_baseline leg and tests/ use it; bit-exactness against
 * the oracle is checked by tests/test_golden_cpu.py when the host CPU has GFNI.
 */
#include <immintrin.h>
#include <stdint.h>
#include <string.h>

static uint64_t
gfni_matrix(unsigned char c)
{
        /* output bit i = parity(A.byte[7-i] & x); column j of the linear map x -> c*x is c*2^j */
        uint64_t A = 0;
        unsigned char v = c;
        int i, j;
        for (j = 0; j < 8; j++) {
                for (i = 0; i < 8; i++)
                        if ((v >> i) & 1)
                                A |= (uint64_t) 1 << (8 * (7 - i) + j);
                v = (unsigned char) ((v << 1) ^ ((v & 0x80) ? 0x1d : 0));
        }
        return A;
}

int
gfni_port_available(void)
{
        return __builtin_cpu_supports("avx512bw") && __builtin_cpu_supports("gfni");
}

__attribute__((target("avx512f,avx512bw,gfni"))) static void
dot_group(int len, int k, int n, const uint64_t *mat /* [n][k] */, unsigned char *const *src,
          unsigned char *const *dst)
{
        __m512i acc[6];
        int i = 0, j, l;
        for (; i + 64 <= len; i += 64) {
                for (l = 0; l < n; l++)
                        acc[l] = _mm512_setzero_si512();
                for (j = 0; j < k; j++) {
                        const __m512i x = _mm512_loadu_si512((const void *) (src[j] + i));
                        for (l = 0; l < n; l++)
                                acc[l] = _mm512_xor_si512(
                                        acc[l],
                                        _mm512_gf2p8affine_epi64_epi8(
                                                x, _mm512_set1_epi64((long long) mat[l * k + j]), 0));
                }
                for (l = 0; l < n; l++)
                        _mm512_storeu_si512((void *) (dst[l] + i), acc[l]);
        }
        if (i < len) {
                const __mmask64 m = (~(__mmask64) 0) >> (64 - (len - i));
                for (l = 0; l < n; l++)
                        acc[l] = _mm512_setzero_si512();
                for (j = 0; j < k; j++) {
                        const __m512i x = _mm512_maskz_loadu_epi8(m, (const void *) (src[j] + i));
                        for (l = 0; l < n; l++)
                                acc[l] = _mm512_xor_si512(
                                        acc[l],
                                        _mm512_gf2p8affine_epi64_epi8(
                                                x, _mm512_set1_epi64((long long) mat[l * k + j]), 0));
                }
                for (l = 0; l < n; l++)
                        _mm512_mask_storeu_epi8((void *) (dst[l] + i), m, acc[l]);
        }
}

/* ec_encode_data with base-format tables (byte 1 of each 32-B entry = c). */
void
gfni_port_ec_encode_data(int len, int k, int rows, const unsigned char *tbls,
                         unsigned char *const *src, unsigned char *const *dst)
{
        uint64_t mat[6 * 256];
        int r0, l, j;
        for (r0 = 0; r0 < rows; r0 += 6) {
                int n = rows - r0 < 6 ? rows - r0 : 6;
                for (l = 0; l < n; l++)
                        for (j = 0; j < k && j < 256; j++)
                                mat[l * k + j] = gfni_matrix(tbls[((r0 + l) * k + j) * 32 + 1]);
                dot_group(len, k, n, mat, src, dst + r0);
        }
}

/* ---- crc32_iscsi with the SSE4.2 crc32 instruction (baseline only) --------
 * The reference's fast CRC32C (crc/crc32_iscsi_01.asm, crc32_iscsi_by16_10.asm)
 * is NASM too. Restated here the way crc32_iscsi_01 works: three independent
 * crc32q streams over the buffer's thirds (the instruction's 3-cycle latency
 * hides behind the other two streams), joined by shifting the first two
 * streams past the bytes that follow them (the reference uses PCLMUL for that
 * join; a bitwise multiply mod P is equivalent and costs nothing at 1 MiB). */
static uint32_t
crc_mulmod(uint32_t a, uint32_t b)
{
        uint32_t p = 0;
        int i;
        for (i = 0; i < 32; i++) {
                if (a & 0x80000000u)
                        p ^= b;
                a <<= 1;
                b = (b & 1) ? (b >> 1) ^ 0x82F63B78u : b >> 1;
        }
        return p;
}

static uint32_t
crc_shift(uint32_t crc, uint64_t nbytes) /* crc followed by nbytes zero bytes */
{
        uint32_t sq = 0x00800000u; /* x^8 */
        while (nbytes) {
                if (nbytes & 1)
                        crc = crc_mulmod(crc, sq);
                sq = crc_mulmod(sq, sq);
                nbytes >>= 1;
        }
        return crc;
}

__attribute__((target("sse4.2"))) unsigned int
gfni_port_crc32_iscsi(const unsigned char *buf, long long len, unsigned int init)
{
        uint64_t c0 = init, c1 = 0, c2 = 0, w0, w1, w2;
        long long third = (len / 24) * 8, i;
        const unsigned char *p1 = buf + third, *p2 = buf + 2 * third, *end = buf + len;
        for (i = 0; i < third; i += 8) {
                memcpy(&w0, buf + i, 8);
                memcpy(&w1, p1 + i, 8);
                memcpy(&w2, p2 + i, 8);
                c0 = _mm_crc32_u64(c0, w0);
                c1 = _mm_crc32_u64(c1, w1);
                c2 = _mm_crc32_u64(c2, w2);
        }
        {
                const unsigned char *q = p2 + third;
                uint32_t c = (uint32_t) c2;
                for (; q + 8 <= end; q += 8) {
                        memcpy(&w2, q, 8);
                        c = (uint32_t) _mm_crc32_u64(c, w2);
                }
                for (; q < end; q++)
                        c = _mm_crc32_u8(c, *q);
                /* join: stream 0 is followed by 2 thirds + the rest, stream 1 by 1 third + rest */
                return crc_shift((uint32_t) c0, (uint64_t) (len - third)) ^
                       crc_shift((uint32_t) c1, (uint64_t) (len - 2 * third)) ^ c;
        }
}
