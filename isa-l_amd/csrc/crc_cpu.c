/*
 * crc_cpu.c — the CPU route of the reference's checksum entry points
 * (crc32_iscsi: include/crc.h:136-150, semantics crc/crc_base.c:205-219;
 * crc64_*: include/crc64.h:54-163, semantics crc/crc64_base.c:569-670) for
 * buffers in host memory. Device-resident buffers go to the GPU checksum
 * kernels instead (isal_hip_shim.c "checksum entry points").
 *
 *   CRC32C: the SSE4.2 crc32 instruction computes exactly the reference's
 *           reflected Castagnoli byte step (no inversions), 8 bytes at a time;
 *           without SSE4.2, slicing-by-8 tables of the same polynomial.
 *   CRC64:  slicing-by-8 in the "u-domain" of crc64_host.c (u = the register,
 *           byte-swapped for the norm flavours), where 8 bytes d advance the
 *           register as u' = XOR_j A_j[byte j of (d ^ u)] for every flavour;
 *           the ragged tail runs the reference's byte loop on its table.
 * Tables are built once per process (pthread_once).
 */
#include <pthread.h>
#include <stdint.h>
#include <string.h>

#include "isal_hip.h"
#include "isal_hip_internal.h"

/* ---- CRC32C ---------------------------------------------------------------- */

#define CRC32C_POLY_REFL 0x82F63B78u

static uint32_t c32_slice[8][256];
static int c32_hw;
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
        __builtin_cpu_init();
        c32_hw = __builtin_cpu_supports("sse4.2");
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

uint32_t
isal_cpu_crc32c(uint32_t init, const unsigned char *buf, uint64_t len)
{
        pthread_once(&c32_once, c32_init);
        if (!len)
                return init;
        if (c32_hw && isal_hip_knob(ISAL_HIP_KNOB_CPU_SIMD) != 0)
                return c32_sse42(init, buf, len);
        return c32_sliced(init, buf, len);
}

/* ---- CRC64 ----------------------------------------------------------------- */

static uint64_t c64_byte[ISAL_HIP_CRC64_NVARIANTS][256];
static uint64_t c64_slice[ISAL_HIP_CRC64_NVARIANTS][8 * 256];
static pthread_once_t c64_once = PTHREAD_ONCE_INIT;

static void
c64_init(void)
{
        int v;
        for (v = 0; v < ISAL_HIP_CRC64_NVARIANTS; v++)
                isal_hip_crc64_cpu_tables(v, c64_byte[v], c64_slice[v]);
}

uint64_t
isal_cpu_crc64(int variant, uint64_t init, const unsigned char *buf, uint64_t len)
{
        const int refl = isal_hip_crc64_is_refl(variant);
        const uint64_t *a = c64_slice[variant], *t = c64_byte[variant];
        uint64_t s = ~init, u;
        pthread_once(&c64_once, c64_init);
        u = refl ? s : __builtin_bswap64(s);
        while (len >= 8) {
                uint64_t x;
                memcpy(&x, buf, 8);
                x ^= u;
                u = a[0 * 256 + (x & 0xff)] ^ a[1 * 256 + ((x >> 8) & 0xff)] ^ a[2 * 256 + ((x >> 16) & 0xff)] ^
                    a[3 * 256 + ((x >> 24) & 0xff)] ^ a[4 * 256 + ((x >> 32) & 0xff)] ^
                    a[5 * 256 + ((x >> 40) & 0xff)] ^ a[6 * 256 + ((x >> 48) & 0xff)] ^ a[7 * 256 + (x >> 56)];
                buf += 8;
                len -= 8;
        }
        s = refl ? u : __builtin_bswap64(u);
        while (len--) {
                const unsigned char b = *buf++;
                s = refl ? t[(s ^ b) & 0xff] ^ (s >> 8) : t[((s >> 56) ^ b) & 0xff] ^ (s << 8);
        }
        return ~s;
}
