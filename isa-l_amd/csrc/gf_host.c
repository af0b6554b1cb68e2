/*
 * gf_host.c — host-side GF(2^8) arithmetic of the MI355X erasure-code engine.
 *
 * These are the O(k^2)..O(k^3) control-plane functions that the reference also
 * runs on the host (erasure_code/ec_base.c:37-280): field multiply/inverse,
 * generator matrices, matrix inversion for decode, and table expansion. They
 * never touch shard data. The data path (encode/update/dot/mad/mul) is routed
 * by isal_hip_shim.c: GPU kernels (ec_kernels.hip) for device-resident and
 * large host-resident calls, the CPU route (ec_cpu.c) for small host calls
 * and as the fallback of a host call whose GPU attempt failed.
 *
 * Field: GF(2^8) modulo x^8+x^4+x^3+x^2+1 (0x11d). The log/antilog tables are
 * computed once from the polynomial (never copied from ec_base.h).
 */
#include <pthread.h>
#include <string.h>

#include "erasure_code.h"
#include "isal_hip_internal.h"

static unsigned char gf_antilog[512]; /* doubled so log a + log b needs no mod */
static unsigned char gf_logt[256];
static pthread_once_t gf_once = PTHREAD_ONCE_INIT;

static void
gf_tables_init(void)
{
        unsigned x = 1;
        int e;
        for (e = 0; e < 255; e++) {
                gf_antilog[e] = (unsigned char) x;
                gf_antilog[e + 255] = (unsigned char) x;
                gf_logt[x] = (unsigned char) e;
                x = (x << 1) ^ ((x & 0x80) ? 0x11d : 0);
        }
        gf_antilog[510] = gf_antilog[0];
        gf_antilog[511] = gf_antilog[1];
}

static inline void
gf_ready(void)
{
        pthread_once(&gf_once, gf_tables_init);
}

unsigned char
gf_mul(unsigned char a, unsigned char b)
{
        gf_ready();
        if (!a || !b)
                return 0;
        return gf_antilog[gf_logt[a] + gf_logt[b]];
}

unsigned char
isal_hip_gf_mul(unsigned char a, unsigned char b)
{
        return gf_mul(a, b);
}

unsigned char
gf_inv(unsigned char a)
{
        gf_ready();
        if (!a)
                return 0;
        return gf_antilog[255 - gf_logt[a]];
}

/* Reference semantics: ec_base.c:78-96. Row r (r = 0..m-k-1) holds (2^r)^j. */
void
gf_gen_rs_matrix(unsigned char *a, int m, int k)
{
        int r, j;
        unsigned char base = 1;
        memset(a, 0, (size_t) k * m);
        for (j = 0; j < k; j++)
                a[(size_t) k * j + j] = 1;
        for (r = k; r < m; r++) {
                unsigned char v = 1;
                for (j = 0; j < k; j++) {
                        a[(size_t) k * r + j] = v;
                        v = gf_mul(v, base);
                }
                base = gf_mul(base, 2);
        }
}

/* Reference semantics: ec_base.c:98-114. */
void
gf_gen_cauchy1_matrix(unsigned char *a, int m, int k)
{
        int i, j;
        memset(a, 0, (size_t) k * m);
        for (j = 0; j < k; j++)
                a[(size_t) k * j + j] = 1;
        for (i = k; i < m; i++)
                for (j = 0; j < k; j++)
                        a[(size_t) k * i + j] = gf_inv((unsigned char) (i ^ j));
}

/* Reference semantics: ec_base.c:116-170 (pivot search, swap, scale, eliminate
 * in the same order, so decode matrices are byte-identical). */
int
gf_invert_matrix(unsigned char *in, unsigned char *out, const int n)
{
        int col, row, c;
        memset(out, 0, (size_t) n * n);
        for (col = 0; col < n; col++)
                out[col * n + col] = 1;

        for (col = 0; col < n; col++) {
                unsigned char *prow = in + col * n, *orow = out + col * n, s;
                if (prow[col] == 0) {
                        for (row = col + 1; row < n; row++)
                                if (in[row * n + col])
                                        break;
                        if (row == n)
                                return -1;
                        for (c = 0; c < n; c++) {
                                unsigned char t = prow[c];
                                prow[c] = in[row * n + c];
                                in[row * n + c] = t;
                                t = orow[c];
                                orow[c] = out[row * n + c];
                                out[row * n + c] = t;
                        }
                }
                s = gf_inv(prow[col]);
                for (c = 0; c < n; c++) {
                        prow[c] = gf_mul(prow[c], s);
                        orow[c] = gf_mul(orow[c], s);
                }
                for (row = 0; row < n; row++) {
                        unsigned char f;
                        if (row == col)
                                continue;
                        f = in[row * n + col];
                        for (c = 0; c < n; c++) {
                                out[row * n + c] ^= gf_mul(f, orow[c]);
                                in[row * n + c] ^= gf_mul(f, prow[c]);
                        }
                }
        }
        return 0;
}

/* 32-byte expansion (ec_base.c:175-280): low-nibble products then high-nibble
 * products. Built from c*1, c*2, c*4, c*8 (and c*16..c*128) by linearity. */
void
gf_vect_mul_init_base(unsigned char c, unsigned char *tbl)
{
        unsigned char p[8];
        int b, i;
        p[0] = c;
        for (b = 1; b < 8; b++)
                p[b] = (unsigned char) ((p[b - 1] << 1) ^ ((p[b - 1] & 0x80) ? 0x1d : 0));
        for (i = 0; i < 16; i++) {
                unsigned char lo = 0, hi = 0;
                for (b = 0; b < 4; b++)
                        if (i & (1 << b)) {
                                lo ^= p[b];
                                hi ^= p[b + 4];
                        }
                tbl[i] = lo;
                tbl[16 + i] = hi;
        }
}

void
gf_vect_mul_init(unsigned char c, unsigned char *tbl)
{
        gf_vect_mul_init_base(c, tbl);
}

void
ec_init_tables_base(int k, int rows, unsigned char *a, unsigned char *gftbls)
{
        int i;
        for (i = 0; i < k * rows; i++)
                gf_vect_mul_init_base(a[i], gftbls + 32 * (size_t) i);
}

/* The engine's tables ARE the base format (byte 1 of each entry = c), so the
 * dispatched and *_base entry points interoperate (reference contract:
 * erasure_code.h:116,153,175,241). */
void
ec_init_tables(int k, int rows, unsigned char *a, unsigned char *gftbls)
{
        ec_init_tables_base(k, rows, a, gftbls);
}

/* ---- device coefficient tables (isal_hip_internal.h layout) -------------- */

size_t
isal_hip_tables_dwords(int k, int rows)
{
        return (size_t) EC_TBL_DWORDS * (size_t) k * (size_t) rows;
}

static void
perm_tables(unsigned char c, uint32_t *t)
{
        unsigned char lo[8], mid[8], hi[4];
        int i;
        for (i = 0; i < 8; i++) {
                lo[i] = gf_mul(c, (unsigned char) i);
                mid[i] = gf_mul(c, (unsigned char) (i << 3));
        }
        for (i = 0; i < 4; i++)
                hi[i] = gf_mul(c, (unsigned char) (i << 6));
        memcpy(&t[0], lo, 8);  /* [0] = entries 0-3, [1] = entries 4-7 (little-endian) */
        memcpy(&t[2], mid, 8);
        memcpy(&t[4], hi, 4);
}

void
isal_hip_build_tables(int k, int rows, const unsigned char *gftbls, uint32_t *tbl)
{
        int r0, j, l;
        for (r0 = 0; r0 < rows; r0 += EC_MAX_ROWS_PER_PASS) {
                int P = rows - r0 < EC_MAX_ROWS_PER_PASS ? rows - r0 : EC_MAX_ROWS_PER_PASS;
                uint32_t *g = tbl + (size_t) EC_TBL_DWORDS * k * r0;
                for (j = 0; j < k; j++)
                        for (l = 0; l < P; l++) {
                                unsigned char c = gftbls[((size_t) (r0 + l) * k + j) * 32 + 1];
                                perm_tables(c, g + ((size_t) j * P + l) * EC_TBL_DWORDS);
                        }
        }
}

/* LDS product tables of the wide passes (layout: isal_hip_internal.h). */
size_t
isal_hip_ldsx_words(int k, int rows)
{
        const int passes = (rows + EC_MAX_ROWS_PER_PASS - 1) / EC_MAX_ROWS_PER_PASS;
        return (size_t) passes * (size_t) k * ISAL_HIP_LDSX_ENTRIES;
}

/* coefficient (r, j) at c[(r * k + j) * stride + off] */
static void
ldsx_build(int k, int rows, const unsigned char *c, int stride, int off, uint64_t *out)
{
        int r0, j, l, v;
        for (r0 = 0; r0 < rows; r0 += EC_MAX_ROWS_PER_PASS) {
                const int P = rows - r0 < EC_MAX_ROWS_PER_PASS ? rows - r0 : EC_MAX_ROWS_PER_PASS;
                uint64_t *t5 = out + (size_t) (r0 / EC_MAX_ROWS_PER_PASS) * k * ISAL_HIP_LDSX_ENTRIES,
                         *t3 = t5 + (size_t) k * 32;
                memset(t5, 0, (size_t) k * ISAL_HIP_LDSX_ENTRIES * 8);
                for (j = 0; j < k; j++)
                        for (l = 0; l < P; l++) {
                                const unsigned char cf = c[((size_t) (r0 + l) * k + j) * stride + off];
                                for (v = 0; v < 32; v++)
                                        t5[(size_t) j * 32 + v] |= (uint64_t) gf_mul(cf, (unsigned char) v) << (8 * l);
                                for (v = 0; v < 8; v++)
                                        t3[(size_t) j * 8 + v] |= (uint64_t) gf_mul(cf, (unsigned char) (v << 5))
                                                                  << (8 * l);
                        }
        }
}

void
isal_hip_build_ldsx_tables(int k, int rows, const unsigned char *gftbls, uint64_t *out)
{
        ldsx_build(k, rows, gftbls, 32, 1, out);
}

/* The same from the rows x k coefficient bytes themselves. */
void
isal_hip_build_ldsx_tables_coef(int k, int rows, const unsigned char *coef, uint64_t *out)
{
        ldsx_build(k, rows, coef, 1, 0, out);
}

void
isal_hip_xor_rows(int k, int rows, const unsigned char *gftbls, isal_hip_xrows *x)
{
        int l, j;
        memset(x, 0, sizeof(*x));
        if (k < 1 || k > 64 || isal_hip_knob(ISAL_HIP_KNOB_CRC_XROWS) == 0)
                return;
        for (l = 0; l < rows && l < EC_MAX_ROWS_PER_PASS; l++) {
                unsigned long long m = 0;
                for (j = 0; j < k; j++) {
                        const unsigned char c = gftbls[((size_t) l * k + j) * 32 + 1];
                        if (c > 1)
                                break;
                        m |= (unsigned long long) c << j;
                }
                if (j == k) {
                        x->rows |= 1u << l;
                        x->src[l] = m;
                }
        }
}

void
isal_hip_enc_masks(int k, int rows, const unsigned char *gftbls, isal_hip_encmask *m)
{
        int g, l, j;
        memset(m, 0, sizeof(*m));
        /* computed whatever ISAL_HIP_ENC_XOR says: the launch applies the knob
         * (ec_kernels.hip enc_xor_masks), so long-lived batch and pipeline
         * handles follow isal_hip_config_reload() like the drop-in calls */
        if (k < 1 || k > 64 || rows < 1)
                return;
        for (g = 0; g * EC_MAX_ROWS_PER_PASS < rows && g < EC_MAX_PASSES; g++) {
                const int r0 = g * EC_MAX_ROWS_PER_PASS;
                const int P = rows - r0 < EC_MAX_ROWS_PER_PASS ? rows - r0 : EC_MAX_ROWS_PER_PASS;
                unsigned long long rm = 0;
                unsigned cm = 0;
                int good = 1;
                for (j = 0; j < k && good; j++) {
                        const unsigned char c = gftbls[((size_t) r0 * k + j) * 32 + 1];
                        good = c <= 1;
                        rm |= (unsigned long long) (c & 1) << j;
                }
                for (l = 0; l < P && good; l++) {
                        const unsigned char c = gftbls[((size_t) (r0 + l) * k) * 32 + 1];
                        good = c <= 1;
                        cm |= (unsigned) (c & 1) << l;
                }
                if (good) {
                        m->ok |= 1u << g;
                        m->r0[g] = rm;
                        m->c0[g] = cm;
                }
        }
}

/* ---- version (reference isal_api.h:93,104) ------------------------------ */

const char *
isal_get_version_str(void)
{
        return "2.32.1";
}

unsigned
isal_get_version(void)
{
        return ISAL_VERSION;
}
