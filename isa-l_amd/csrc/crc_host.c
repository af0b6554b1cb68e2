/*
 * crc_host.c — host-side GF(2)[x] constants for the GPU CRC32C kernels.
 *
 * CRC32C here is the reference's crc32_iscsi (crc/crc_base.c:205-219): the
 * reflected Castagnoli polynomial 0x82F63B78, register initialised to the
 * caller's init_crc, no final inversion. That CRC is GF(2)-linear, so
 *   crc(init, A || B) = Z^|B|( crc(init, A) ) ^ crc(0, B),
 * where Z^d ("d zero bytes") is multiplication by x^(8d) modulo the
 * polynomial. The kernels (crc_kernels.hip) compute crc(0, .) of 16-byte lane
 * chunks with slice tables, chain a lane's chunks across 4 KiB tiles with Z^4096,
 * and a combine kernel joins the per-lane partials with the constants built
 * here. Nothing in this file touches shard data: it only derives tables.
 *
 * Representation: bit 31 of a register is the coefficient of x^0 (the
 * reflected convention of the reference's table-driven loop).
 */
#include <stdint.h>
#include <string.h>
#include <pthread.h>

#include "isal_hip_internal.h"

#define CRC32C_POLY 0x82F63B78u

static uint32_t t0[256];       /* crc of one byte from 0 (= byte * x^8 mod P) */
static uint32_t x2n[64];       /* x^(2^i) mod P */
static pthread_once_t once = PTHREAD_ONCE_INIT;

/* a * b mod P, both reflected. */
uint32_t
isal_hip_crc32c_mulmod(uint32_t a, uint32_t b)
{
        uint32_t p = 0;
        int i;
        for (i = 0; i < 32; i++) {
                if (a & 0x80000000u)
                        p ^= b;
                a <<= 1;
                b = (b & 1) ? (b >> 1) ^ CRC32C_POLY : b >> 1;
        }
        return p;
}

static void
init(void)
{
        int b, i;
        for (b = 0; b < 256; b++) {
                uint32_t c = (uint32_t) b;
                for (i = 0; i < 8; i++)
                        c = (c & 1) ? (c >> 1) ^ CRC32C_POLY : c >> 1;
                t0[b] = c;
        }
        x2n[0] = 0x40000000u; /* x^1 */
        for (i = 1; i < 64; i++)
                x2n[i] = isal_hip_crc32c_mulmod(x2n[i - 1], x2n[i - 1]);
}

/* x^(8n) mod P: the multiplier of "append n zero bytes". */
uint32_t
isal_hip_crc32c_xpow8n(unsigned long long n)
{
        uint32_t p = 0x80000000u; /* x^0 */
        int i = 3;
        pthread_once(&once, init);
        while (n) {
                if (n & 1)
                        p = isal_hip_crc32c_mulmod(x2n[i & 63], p);
                n >>= 1;
                i++;
        }
        return p;
}

/* Byte tables of "multiply by K": out[q*256 + v] = (v << 8q) * K. */
static void
mul_tables(uint32_t k, uint32_t *out)
{
        int q, v;
        for (q = 0; q < 4; q++)
                for (v = 0; v < 256; v++)
                        out[q * 256 + v] = isal_hip_crc32c_mulmod((uint32_t) v << (8 * q), k);
}

/* First bit and width of field f of a dword (ISAL_HIP_CRC_FIELDS fields). */
static int
field_lo(int f)
{
        return 5 * f;
}

static int
field_bits(int f)
{
        return f < ISAL_HIP_CRC_FIELDS - 1 ? 5 : 32 - 5 * (ISAL_HIP_CRC_FIELDS - 1);
}

/* Kernel lookup tables (ISAL_HIP_CRC_TAB_DWORDS, layout in
 * isal_hip_internal.h). The field tables follow from linearity: a field's
 * contribution is the XOR of the contributions of its set bits, and bit j of
 * byte i of a 16-byte chunk contributes slice_{15-i}[1 << j], where slice_s[b]
 * is the crc of byte b followed by s zero bytes. */
void
isal_hip_crc32c_tables(uint32_t *tabs)
{
        uint32_t slice[ISAL_HIP_CRC_SLICES][256];
        const uint32_t zk = isal_hip_crc32c_xpow8n(ISAL_HIP_CRC_TILE);
        int s, b, d, f, v, j;
        pthread_once(&once, init);
        for (b = 0; b < 256; b++)
                slice[0][b] = tabs[b] = t0[b];
        for (s = 1; s < ISAL_HIP_CRC_SLICES; s++)
                for (b = 0; b < 256; b++) {
                        const uint32_t c = slice[s - 1][b];
                        slice[s][b] = (c >> 8) ^ t0[c & 0xff];
                }
        for (f = 0; f < ISAL_HIP_CRC_FIELDS; f++)
                for (v = 0; v < 32; v++) {
                        /* value v in field f, restricted to the field's width */
                        const uint32_t word = (uint32_t) (v & ((1 << field_bits(f)) - 1))
                                              << field_lo(f);
                        for (d = 0; d < 4; d++) {
                                uint32_t c = 0;
                                for (j = 0; j < 32; j++)
                                        if (word >> j & 1)
                                                c ^= slice[15 - (4 * d + j / 8)][1u << (j % 8)];
                                tabs[ISAL_HIP_CRC_CHUNK_TAB + (d * ISAL_HIP_CRC_FIELDS + f) * 32 + v] = c;
                        }
                        tabs[ISAL_HIP_CRC_SHIFT_TAB + f * 32 + v] = isal_hip_crc32c_mulmod(word, zk);
                }
}

/* Byte-position tables (ISAL_HIP_CRC_B16_TAB): out[p * 256 + b] = crc of byte
 * b followed by 15 - p zero bytes, then the same shifted by 4080 more zero
 * bytes (multiplied by x^(8*4080) mod P, as the chain shift tables are). */
void
isal_hip_crc32c_byte_tables(uint32_t *out)
{
        uint32_t slice[ISAL_HIP_CRC_SLICES][256], zk;
        int s, b;
        pthread_once(&once, init);
        for (b = 0; b < 256; b++)
                slice[0][b] = t0[b];
        for (s = 1; s < ISAL_HIP_CRC_SLICES; s++)
                for (b = 0; b < 256; b++) {
                        const uint32_t c = slice[s - 1][b];
                        slice[s][b] = (c >> 8) ^ t0[c & 0xff];
                }
        zk = isal_hip_crc32c_xpow8n(ISAL_HIP_CRC_TILE - ISAL_HIP_CRC_SLICES);
        for (s = 0; s < ISAL_HIP_CRC_SLICES; s++)
                for (b = 0; b < 256; b++) {
                        const uint32_t c = slice[ISAL_HIP_CRC_SLICES - 1 - s][b];
                        out[s * 256 + b] = c;
                        out[ISAL_HIP_CRC_SLICES * 256 + s * 256 + b] = isal_hip_crc32c_mulmod(c, zk);
                }
}

/* F' (ISAL_HIP_CRC_FPRE_TAB): every entry of the chunk field tables shifted by
 * 4080 zero bytes. */
void
isal_hip_crc32c_pre_tables(const uint32_t *tabs, uint32_t *out)
{
        const uint32_t z = isal_hip_crc32c_xpow8n(ISAL_HIP_CRC_TILE - ISAL_HIP_CRC_SLICES);
        int e;
        for (e = 0; e < ISAL_HIP_CRC_CHUNK_DWORDS; e++)
                out[e] = isal_hip_crc32c_mulmod(tabs[ISAL_HIP_CRC_CHUNK_TAB + e], z);
}

/* Tables of the multi-tile chain step from the base tables: every entry of a
 * chunk map shifted by m tiles is entry * x^(8*4096*m) mod P; Z^(4096*4) of a
 * field value is its Z^4096 entry shifted by three more tiles. */
void
isal_hip_crc32c_ext_tables(const uint32_t *tabs, uint32_t *ext)
{
        int m, e;
        const uint32_t z3 = isal_hip_crc32c_xpow8n(3ULL * ISAL_HIP_CRC_TILE);
        for (m = 1; m <= 3; m++) {
                const uint32_t zm = isal_hip_crc32c_xpow8n((unsigned long long) m * ISAL_HIP_CRC_TILE);
                for (e = 0; e < ISAL_HIP_CRC_CHUNK_DWORDS; e++)
                        ext[(m - 1) * ISAL_HIP_CRC_CHUNK_DWORDS + e] =
                                isal_hip_crc32c_mulmod(tabs[ISAL_HIP_CRC_CHUNK_TAB + e], zm);
        }
        for (e = 0; e < ISAL_HIP_CRC_FIELDS * 32; e++)
                ext[3 * ISAL_HIP_CRC_CHUNK_DWORDS + e] =
                        isal_hip_crc32c_mulmod(tabs[ISAL_HIP_CRC_SHIFT_TAB + e], z3);
}

/* Geometry of the per-lane partials for shards of `len` bytes, `tt` tiles per
 * workgroup (see isal_hip_internal.h). */
void
isal_hip_crc_geometry(long long len, int tt, isal_hip_crc_geom *g)
{
        memset(g, 0, sizeof(*g));
        g->tt = tt;
        g->nfull = len / ISAL_HIP_CRC_TILE;
        g->tail = (int) (len % ISAL_HIP_CRC_TILE);
        g->ntiles = g->nfull + (g->tail ? 1 : 0);
        g->nblk = (g->ntiles + tt - 1) / tt;
        g->nfull_last = g->nblk ? g->nfull - (g->nblk - 1) * tt : 0;
        if (g->nfull_last < 0)
                g->nfull_last = 0;
}

/* Combine constants (ISAL_HIP_CRC_PLAN_DWORDS), see crc32c_combine:
 *   [0,1024)      byte tables of x^(8*4096*tt)          (Horner across blocks)
 *   [1024,2048)   byte tables of x^(8*4096*nfull_last)  (the last block)
 *   [2048,2304)   W[L]  = x^(8*(16*(255-L) + tail))    (lane L of a full tile -> shard end)
 *   [2304,2560)   Ct[L] = x^(8*max(0, tail-16L-16))     (lane L of the ragged tile -> shard end)
 *   [2560]        x^(8*len)                             (the caller's init_crc) */
void
isal_hip_crc32c_plan(long long len, int tt, uint32_t *plan)
{
        isal_hip_crc_geom g;
        int l;
        isal_hip_crc_geometry(len, tt, &g);
        mul_tables(isal_hip_crc32c_xpow8n((unsigned long long) ISAL_HIP_CRC_TILE * tt), plan);
        mul_tables(isal_hip_crc32c_xpow8n((unsigned long long) ISAL_HIP_CRC_TILE * g.nfull_last),
                   plan + 1024);
        for (l = 0; l < 256; l++) {
                const long long rest = (long long) g.tail - 16 * l - 16;
                plan[2048 + l] = isal_hip_crc32c_xpow8n((unsigned long long) (16 * (255 - l) + g.tail));
                plan[2304 + l] = isal_hip_crc32c_xpow8n((unsigned long long) (rest > 0 ? rest : 0));
        }
        plan[2560] = isal_hip_crc32c_xpow8n((unsigned long long) len);
        plan[2561] = plan[2562] = plan[2563] = 0;
}
