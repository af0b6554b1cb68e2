/*
 * crc64_host.c — host-side tables for the GPU CRC64 kernels (crc64_kernels.hip).
 *
 * The eight CRC64 flavours of the reference (include/crc64.h:54-163, algorithm
 * crc/crc64_base.c:569-670) are table-driven byte loops over a 64-bit register
 * that starts at ~init and is inverted on return; "refl" shifts right with the
 * bit-reversed polynomial, "norm" shifts left with the polynomial itself:
 *   refl: crc = T[(crc ^ b) & 0xff] ^ (crc >> 8)
 *   norm: crc = T[((crc >> 56) ^ b) & 0xff] ^ (crc << 8)
 * Without the inversions ("raw") both are GF(2)-linear in (register, data):
 *   raw(s, A || B) = raw(raw(s, A), B),  raw(s, D) = Z^|D|(s) ^ raw(0, D)
 * with Z^n = "append n zero bytes", a 64x64 GF(2) matrix. Every constant the
 * kernels need is such a linear map, so it is built here by evaluating the
 * bit-serial raw update on basis vectors — one code path for all eight
 * flavours, no polynomial arithmetic specific to a bit order.
 *
 * Linear maps are stored as columns: m[i] = M(e_i); M(v) = XOR of m[i] over the
 * set bits i of v. On the device a map is applied through "field tables": the
 * 64-bit input splits into its two dwords, each into 7 fields (bits [0,5)
 * [5,10) ... [25,30) [30,32)), and table (h, f) holds M(v << (5f + 32h)) for
 * the 32 values v of the field — 32 entries x 8 B = one 256-byte LDS bank row,
 * so a wave's ds_read_b64 lookups into one table never bank-conflict.
 * Nothing here touches shard data.
 */
#include <pthread.h>
#include <stdint.h>
#include <string.h>

#include "isal_hip_internal.h"

/* Normal-form polynomials (x^64 implicit) of reference crc64_base.c's tables:
 * ECMA-182, ISO 3309, Jones, Rocksoft. The refl tables use the bit reversals. */
static const uint64_t poly_norm[4] = {
        0x42F0E1EBA9EA3693ULL,
        0x000000000000001BULL,
        0xAD93D23594C935A9ULL,
        0xAD93D23594C93659ULL,
};

static uint64_t
bitrev64(uint64_t x)
{
        uint64_t r = 0;
        int i;
        for (i = 0; i < 64; i++)
                r |= ((x >> i) & 1) << (63 - i);
        return r;
}

/* The flavour's polynomial in normal form (x^64 implicit), for crc_cpu.c's
 * carry-less folding constants. */
uint64_t
isal_hip_crc64_poly(int variant)
{
        return poly_norm[variant >> 1];
}

int
isal_hip_crc64_is_refl(int variant)
{
        return (variant & 1) == 0; /* ISAL_HIP_CRC64_*_REFL are even */
}

/* Bit-serial raw update of register s with n bytes (buf NULL: zero bytes). */
static uint64_t
raw_update(int variant, uint64_t s, const uint8_t *buf, long long n)
{
        const int refl = isal_hip_crc64_is_refl(variant);
        const uint64_t p = refl ? bitrev64(poly_norm[variant >> 1]) : poly_norm[variant >> 1];
        long long i;
        int j;
        for (i = 0; i < n; i++) {
                const uint8_t b = buf ? buf[i] : 0;
                if (refl) {
                        s ^= b;
                        for (j = 0; j < 8; j++)
                                s = (s & 1) ? (s >> 1) ^ p : s >> 1;
                } else {
                        s ^= (uint64_t) b << 56;
                        for (j = 0; j < 8; j++)
                                s = (s >> 63) ? (s << 1) ^ p : s << 1;
                }
        }
        return s;
}

static uint64_t
apply(const uint64_t m[64], uint64_t v)
{
        uint64_t r = 0;
        int i;
        for (i = 0; i < 64; i++)
                if (v >> i & 1)
                        r ^= m[i];
        return r;
}

/* c = a ∘ b (apply b first). c may alias neither input. */
static void
compose(const uint64_t a[64], const uint64_t b[64], uint64_t c[64])
{
        int i;
        for (i = 0; i < 64; i++)
                c[i] = apply(a, b[i]);
}

/* Z^(2^i), i < ZP2_BITS, per flavour: built once per process (the drop-in
 * checksum calls rebuild their length-dependent maps per length, which then
 * costs one composition per set bit of the length, not a squaring chain). */
#define ZP2_BITS 48
#define NFLAVOURS 8 /* ISAL_HIP_CRC64_NVARIANTS */
static uint64_t zp2[NFLAVOURS][ZP2_BITS][64];
static int zp2_ready[NFLAVOURS];
static pthread_mutex_t zp2_mu = PTHREAD_MUTEX_INITIALIZER;

static const uint64_t (*zpow2(int variant))[64]
{
        if (!__atomic_load_n(&zp2_ready[variant], __ATOMIC_ACQUIRE)) {
                pthread_mutex_lock(&zp2_mu);
                if (!zp2_ready[variant]) {
                        int i, b;
                        for (i = 0; i < 64; i++)
                                zp2[variant][0][i] = raw_update(variant, 1ULL << i, NULL, 1);
                        for (b = 1; b < ZP2_BITS; b++)
                                compose(zp2[variant][b - 1], zp2[variant][b - 1], zp2[variant][b]);
                        __atomic_store_n(&zp2_ready[variant], 1, __ATOMIC_RELEASE);
                }
                pthread_mutex_unlock(&zp2_mu);
        }
        return (const uint64_t (*)[64]) zp2[variant];
}

/* Z^n as columns (products of the cached Z^(2^i)). */
void
isal_hip_crc64_zpow(int variant, unsigned long long n, uint64_t out[64])
{
        const uint64_t (*p2)[64] = zpow2(variant);
        uint64_t acc[64], t[64];
        int i, b;
        for (i = 0; i < 64; i++)
                acc[i] = 1ULL << i;
        for (b = 0; n; b++, n >>= 1) {
                if (!(n & 1))
                        continue;
                if (b < ZP2_BITS) {
                        compose(p2[b], acc, t);
                } else { /* beyond 2^48 bytes: square on from the last cached power */
                        uint64_t sq[64], u[64];
                        int c;
                        memcpy(sq, p2[ZP2_BITS - 1], sizeof(sq));
                        for (c = ZP2_BITS - 1; c < b; c++) {
                                compose(sq, sq, u);
                                memcpy(sq, u, sizeof(u));
                        }
                        compose(sq, acc, t);
                }
                memcpy(acc, t, sizeof(t));
        }
        memcpy(out, acc, sizeof(acc));
}

/* Z^n applied to one register value: one map per set bit of n. */
static uint64_t
zapply(int variant, unsigned long long n, uint64_t v)
{
        const uint64_t (*p2)[64] = zpow2(variant);
        int b;
        for (b = 0; n && b < ZP2_BITS; b++, n >>= 1)
                if (n & 1)
                        v = apply(p2[b], v);
        if (n) { /* beyond 2^48 bytes */
                uint64_t m[64];
                isal_hip_crc64_zpow(variant, n << ZP2_BITS, m);
                v = apply(m, v);
        }
        return v;
}

static int
field_lo(int f)
{
        return 5 * f;
}

static uint32_t
field_mask(int f)
{
        return f < ISAL_HIP_CRC_FIELDS - 1 ? 31u : (1u << (32 - 5 * (ISAL_HIP_CRC_FIELDS - 1))) - 1;
}

/* 14 field tables (448 entries) of the map m. */
static void
op_tables(const uint64_t m[64], uint64_t *out)
{
        int h, f, v;
        for (h = 0; h < 2; h++)
                for (f = 0; f < ISAL_HIP_CRC_FIELDS; f++)
                        for (v = 0; v < 32; v++)
                                out[(h * ISAL_HIP_CRC_FIELDS + f) * 32 + v] =
                                        apply(m, (uint64_t) ((uint32_t) v & field_mask(f))
                                                         << (field_lo(f) + 32 * h));
}

/* 28 field tables of the map chunk -> XOR of basis[bit] (bit j of dword d of
 * the chunk contributes basis[32 * d + j]; dwords are little-endian). */
static void
chunk_tables(const uint64_t basis[128], uint64_t *out)
{
        int d, f, v, j;
        for (d = 0; d < 4; d++)
                for (f = 0; f < ISAL_HIP_CRC_FIELDS; f++)
                        for (v = 0; v < 32; v++) {
                                const uint32_t w = ((uint32_t) v & field_mask(f)) << field_lo(f);
                                uint64_t c = 0;
                                for (j = 0; j < 32; j++)
                                        if (w >> j & 1)
                                                c ^= basis[32 * d + j];
                                out[(d * ISAL_HIP_CRC_FIELDS + f) * 32 + v] = c;
                        }
}

/* The u-domain of the slicing path: u = pi(s), pi = byte swap for the norm
 * flavours. Processing 8 data bytes d (little-endian word) from register s is
 * raw(s, d) = raw(0, d ^ s) (refl: the register is XORed into the low bytes)
 * or raw(0, d ^ bswap(s)) (norm: into the high bytes, first byte = bits
 * 56..63), i.e. raw(0, d ^ pi(s)) — so in u the update is u' = A(d ^ u) with
 * A = pi o raw(0, .) for every flavour, and a 16-byte chunk is two such steps. */
static uint64_t
pi_of(int variant, uint64_t x)
{
        return isal_hip_crc64_is_refl(variant) ? x : __builtin_bswap64(x);
}

static void
slice_tables(int variant, uint64_t *tabs)
{
        uint64_t z[64];
        uint8_t d[8];
        int j, v;
        uint64_t *a = tabs + ISAL_HIP_CRC64_SLICE_TAB, *b = a + 8 * 256;
        /* A' = Z^4080_u o A: the pre-shifted chain's step (crc64_kernels.hip) */
        isal_hip_crc64_zpow(variant, ISAL_HIP_CRC_TILE - 16, z);
        for (j = 0; j < 8; j++)
                for (v = 0; v < 256; v++) {
                        uint64_t r;
                        memset(d, 0, sizeof(d));
                        d[j] = (uint8_t) v;
                        r = raw_update(variant, 0, d, 8);
                        a[j * 256 + v] = pi_of(variant, r);
                        b[j * 256 + v] = pi_of(variant, apply(z, r));
                }
}

/* The maps that depend on the length and the geometry: OP_BLOCK, OP_LAST and
 * OP_TAIL (the rest of the table set depends on the flavour only). */
void
isal_hip_crc64_len_tables(int variant, long long len, int tt, uint64_t *tabs)
{
        uint64_t m[64];
        isal_hip_crc64_geom g;
        isal_hip_crc64_geometry(len, tt, &g);
        isal_hip_crc64_zpow(variant, (unsigned long long) ISAL_HIP_CRC_TILE * g.tt, m);
        op_tables(m, tabs + ISAL_HIP_CRC64_OP_BLOCK);
        isal_hip_crc64_zpow(variant, (unsigned long long) ISAL_HIP_CRC_TILE * g.nfull_last, m);
        op_tables(m, tabs + ISAL_HIP_CRC64_OP_LAST);
        isal_hip_crc64_zpow(variant, (unsigned long long) (g.tail / 16) * 16, m);
        op_tables(m, tabs + ISAL_HIP_CRC64_OP_TAIL);
}

/* Layout: isal_hip_internal.h (ISAL_HIP_CRC64_*). */
void
isal_hip_crc64_tables(int variant, long long len, int tt, uint64_t *tabs)
{
        uint64_t basis[128], m[64];
        uint8_t chunk[16];
        isal_hip_crc64_geom g;
        int b, j, s;
        isal_hip_crc64_geometry(len, tt, &g);
        /* byte table of the reference's loop */
        for (b = 0; b < 256; b++)
                tabs[ISAL_HIP_CRC64_BYTE_TAB + b] =
                        raw_update(variant, isal_hip_crc64_is_refl(variant) ? (uint64_t) b
                                                                              : (uint64_t) b << 56,
                                   NULL, 1);
        /* raw(0, 16-byte chunk): bit j of byte i contributes basis[8i + j] */
        for (j = 0; j < 128; j++) {
                memset(chunk, 0, sizeof(chunk));
                chunk[j / 8] = (uint8_t) (1u << (j % 8));
                basis[j] = raw_update(variant, 0, chunk, 16);
        }
        chunk_tables(basis, tabs + ISAL_HIP_CRC64_CHUNK_TAB);
        isal_hip_crc64_zpow(variant, ISAL_HIP_CRC_TILE, m);
        op_tables(m, tabs + ISAL_HIP_CRC64_SHIFT_TAB);
        /* multi-tile chain step: chunk maps followed by m tiles, Z^(4096*2), Z^(4096*4) */
        for (s = 1; s <= 3; s++) {
                uint64_t bm[128];
                isal_hip_crc64_zpow(variant, (unsigned long long) ISAL_HIP_CRC_TILE * s, m);
                for (j = 0; j < 128; j++)
                        bm[j] = apply(m, basis[j]);
                chunk_tables(bm, tabs + ISAL_HIP_CRC64_CHUNKX_TAB +
                                         (s - 1) * ISAL_HIP_CRC64_CHUNK_ENTRIES);
        }
        isal_hip_crc64_zpow(variant, 2ULL * ISAL_HIP_CRC_TILE, m);
        op_tables(m, tabs + ISAL_HIP_CRC64_SHIFTX_TAB);
        isal_hip_crc64_zpow(variant, 4ULL * ISAL_HIP_CRC_TILE, m);
        op_tables(m, tabs + ISAL_HIP_CRC64_SHIFTX_TAB + ISAL_HIP_CRC64_OP_ENTRIES);
        /* combine plan */
        isal_hip_crc64_len_tables(variant, len, tt, tabs);
        for (s = 0; s < 8; s++) {
                isal_hip_crc64_zpow(variant, 16ULL << s, m);
                op_tables(m, tabs + ISAL_HIP_CRC64_OP_TREE + s * ISAL_HIP_CRC64_OP_ENTRIES);
        }
        slice_tables(variant, tabs);
        /* pre-shifted field tables (u-domain) of the checksum-only kernel */
        isal_hip_crc64_zpow(variant, ISAL_HIP_CRC_TILE - 16, m);
        {
                uint64_t bu[128], bz[128];
                for (j = 0; j < 128; j++) {
                        bu[j] = pi_of(variant, basis[j]);
                        bz[j] = pi_of(variant, apply(m, basis[j]));
                }
                chunk_tables(bu, tabs + ISAL_HIP_CRC64_PRE_TAB);
                chunk_tables(bz, tabs + ISAL_HIP_CRC64_PRE_TAB + ISAL_HIP_CRC64_CHUNK_ENTRIES);
        }
}

/* Tables of the CPU route (crc_cpu.c): the reference's byte table and the
 * slicing-by-8 tables A_j[v] = pi(raw(0, v at byte j of 8)) (the u-domain step
 * of slice_tables above, without the pre-shifted half). */
void
isal_hip_crc64_cpu_tables(int variant, uint64_t byte[256], uint64_t slice[8 * 256])
{
        uint8_t d[8];
        int j, v;
        for (v = 0; v < 256; v++)
                byte[v] = raw_update(variant, isal_hip_crc64_is_refl(variant) ? (uint64_t) v : (uint64_t) v << 56,
                                     NULL, 1);
        for (j = 0; j < 8; j++)
                for (v = 0; v < 256; v++) {
                        memset(d, 0, sizeof(d));
                        d[j] = (uint8_t) v;
                        slice[j * 256 + v] = pi_of(variant, raw_update(variant, 0, d, 8));
                }
}

void
isal_hip_crc64_geometry(long long len, int tt, isal_hip_crc64_geom *g)
{
        g->nfull = len / ISAL_HIP_CRC_TILE;
        g->tail = (int) (len % ISAL_HIP_CRC_TILE);
        g->tt = tt < 1 ? 1 : tt;
        g->nblk = (g->nfull + g->tt - 1) / g->tt;
        g->nfull_last = g->nblk ? g->nfull - (g->nblk - 1) * g->tt : 0;
}

/* Z^len(~init): the register's contribution to crc64(init, buf, len). */
uint64_t
isal_hip_crc64_init_term(int variant, long long len, uint64_t init)
{
        return zapply(variant, (unsigned long long) len, ~init);
}
