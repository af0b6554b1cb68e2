/*
 * ec_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's portable erasure-code path
 * (/root/reference/erasure_code/ec_base.c). It is the parity checker for the
 * MI355X engine: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it, and never as the thing measured or shipped.
 * The product library (isa-l_amd/, libisal_hip.so) does not link it.
 *
 * Parity is pinned: tests/test_golden_cpu.py checks every function here
 * against tests/golden/, which oracle/gen_golden.c produced by linking the
 * reference's own ec_base.c (recipe: oracle/Makefile, target `golden`).
 *
 * All symbols carry an `oracle_` prefix so the oracle can never satisfy a
 * link against the engine's ABI by accident.
 */
#include <stdint.h>
#include <string.h>

#define GF_POLY 0x11d /* x^8+x^4+x^3+x^2+1, reference doc/functions.md:21-23 */

static unsigned char g_exp[256]; /* g_exp[i] = 2^i, i < 255 (ec_base.h gff_base) */
static unsigned char g_log[256]; /* g_log[2^i] = i            (ec_base.h gflog_base) */
static int g_ready;

static void
oracle_init(void)
{
        unsigned v = 1;
        int i;
        if (g_ready)
                return;
        for (i = 0; i < 255; i++) {
                g_exp[i] = (unsigned char) v;
                g_log[v] = (unsigned char) i;
                v <<= 1;
                if (v & 0x100)
                        v ^= GF_POLY;
        }
        g_exp[255] = g_exp[0];
        g_log[0] = 0; /* never read: zero is special-cased, as in ec_base.c:56-57 */
        g_ready = 1;
}

/* ec_base.c:50-63 — log/exp multiply with the zero rule. */
unsigned char
oracle_gf_mul(unsigned char a, unsigned char b)
{
        int s;
        oracle_init();
        if (a == 0 || b == 0)
                return 0;
        s = g_log[a] + g_log[b];
        if (s > 254)
                s -= 255;
        return g_exp[s];
}

/* ec_base.c:65-76 — inverse via exp[255 - log a]; inv(0) = 0. */
unsigned char
oracle_gf_inv(unsigned char a)
{
        oracle_init();
        if (a == 0)
                return 0;
        return g_exp[(255 - g_log[a]) % 255];
}

/* ec_base.c:78-96 — identity over the first k rows, then row r = powers of 2^r. */
void
oracle_gf_gen_rs_matrix(unsigned char *a, int m, int k)
{
        int r, j;
        unsigned char gen = 1;
        memset(a, 0, (size_t) k * m);
        for (j = 0; j < k; j++)
                a[k * j + j] = 1;
        for (r = k; r < m; r++) {
                unsigned char p = 1;
                for (j = 0; j < k; j++) {
                        a[k * r + j] = p;
                        p = oracle_gf_mul(p, gen);
                }
                gen = oracle_gf_mul(gen, 2);
        }
}

/* ec_base.c:98-114 — identity, then a[i][j] = 1/(i ^ j) for i >= k. */
void
oracle_gf_gen_cauchy1_matrix(unsigned char *a, int m, int k)
{
        int i, j;
        memset(a, 0, (size_t) k * m);
        for (j = 0; j < k; j++)
                a[k * j + j] = 1;
        for (i = k; i < m; i++)
                for (j = 0; j < k; j++)
                        a[k * i + j] = oracle_gf_inv((unsigned char) (i ^ j));
}

/* ec_base.c:116-170 — Gauss-Jordan; pivot = first non-zero row at or below i;
 * the row swap, scale and eliminate order is kept so outputs match exactly. */
int
oracle_gf_invert_matrix(unsigned char *in, unsigned char *out, const int n)
{
        int i, j, c;
        for (i = 0; i < n * n; i++)
                out[i] = 0;
        for (i = 0; i < n; i++)
                out[i * n + i] = 1;

        for (i = 0; i < n; i++) {
                unsigned char piv;
                if (in[i * n + i] == 0) {
                        for (j = i + 1; j < n && in[j * n + i] == 0; j++)
                                ;
                        if (j == n)
                                return -1;
                        for (c = 0; c < n; c++) {
                                unsigned char t = in[i * n + c];
                                in[i * n + c] = in[j * n + c];
                                in[j * n + c] = t;
                                t = out[i * n + c];
                                out[i * n + c] = out[j * n + c];
                                out[j * n + c] = t;
                        }
                }
                piv = oracle_gf_inv(in[i * n + i]);
                for (c = 0; c < n; c++) {
                        in[i * n + c] = oracle_gf_mul(in[i * n + c], piv);
                        out[i * n + c] = oracle_gf_mul(out[i * n + c], piv);
                }
                for (j = 0; j < n; j++) {
                        unsigned char f;
                        if (j == i)
                                continue;
                        f = in[j * n + i];
                        for (c = 0; c < n; c++) {
                                out[j * n + c] ^= oracle_gf_mul(f, out[i * n + c]);
                                in[j * n + c] ^= oracle_gf_mul(f, in[i * n + c]);
                        }
                }
        }
        return 0;
}

/* ec_base.c:175-280 — 32-byte table: [0..15] = c*{0..15}, [16..31] = c*{0x00,0x10..0xf0}. */
void
oracle_gf_vect_mul_init(unsigned char c, unsigned char *tbl)
{
        int i;
        for (i = 0; i < 16; i++) {
                tbl[i] = oracle_gf_mul(c, (unsigned char) i);
                tbl[16 + i] = oracle_gf_mul(c, (unsigned char) (i << 4));
        }
}

/* ec_base.c:37-48 — one 32-byte table per coefficient, row-major. */
void
oracle_ec_init_tables(int k, int rows, const unsigned char *a, unsigned char *tbls)
{
        int i;
        for (i = 0; i < k * rows; i++)
                oracle_gf_vect_mul_init(a[i], tbls + 32 * i);
}

/* ec_base.c:309-325 — only byte 1 (= c) of each table is read. */
void
oracle_ec_encode_data(int len, int k, int rows, const unsigned char *tbls,
                      unsigned char *const *src, unsigned char *const *dest)
{
        int l, i, j;
        for (l = 0; l < rows; l++)
                for (i = 0; i < len; i++) {
                        unsigned char s = 0;
                        for (j = 0; j < k; j++)
                                s ^= oracle_gf_mul(src[j][i], tbls[(l * k + j) * 32 + 1]);
                        dest[l][i] = s;
                }
}

/* ec_base.c:327-342 */
void
oracle_ec_encode_data_update(int len, int k, int rows, int vec_i, const unsigned char *tbls,
                             const unsigned char *data, unsigned char *const *dest)
{
        int l, i;
        for (l = 0; l < rows; l++) {
                unsigned char c = tbls[(l * k + vec_i) * 32 + 1];
                for (i = 0; i < len; i++)
                        dest[l][i] ^= oracle_gf_mul(data[i], c);
        }
}

/* ec_base.c:282-294 */
void
oracle_gf_vect_dot_prod(int len, int vlen, const unsigned char *tbls, unsigned char *const *src,
                        unsigned char *dest)
{
        int i, j;
        for (i = 0; i < len; i++) {
                unsigned char s = 0;
                for (j = 0; j < vlen; j++)
                        s ^= oracle_gf_mul(src[j][i], tbls[j * 32 + 1]);
                dest[i] = s;
        }
}

/* ec_base.c:296-307 */
void
oracle_gf_vect_mad(int len, int vec, int vec_i, const unsigned char *tbls,
                   const unsigned char *src, unsigned char *dest)
{
        int i;
        unsigned char c = tbls[vec_i * 32 + 1];
        (void) vec;
        for (i = 0; i < len; i++)
                dest[i] ^= oracle_gf_mul(src[i], c);
}

/* ec_base.c:344-358 — returns -1 when len is not a multiple of 32. */
int
oracle_gf_vect_mul(int len, const unsigned char *tbl, const unsigned char *src,
                   unsigned char *dest)
{
        int i;
        if (len % 32)
                return -1;
        for (i = 0; i < len; i++)
                dest[i] = oracle_gf_mul(tbl[1], src[i]);
        return 0;
}

/* ---- test helpers -------------------------------------------------------- */

/* Counter-based splitmix64 byte stream: byte n of stream `seed` is byte (n % 8)
 * (little-endian) of mix(seed + (n/8 + 1) * 0x9E3779B97F4A7C15). The Python
 * helper tests/ecutil.py:fill_bytes computes the same bytes with numpy. */
void
oracle_fill_bytes(unsigned char *buf, long long n, unsigned long long seed)
{
        long long w;
        for (w = 0; w * 8 < n; w++) {
                unsigned long long z = seed + (unsigned long long) (w + 1) * 0x9E3779B97F4A7C15ull;
                int b;
                z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
                z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
                z ^= z >> 31;
                for (b = 0; b < 8 && w * 8 + b < n; b++)
                        buf[w * 8 + b] = (unsigned char) (z >> (8 * b));
        }
}

/* FNV-1a 32-bit, for compact fixture digests. */
unsigned int
oracle_fnv1a32(const unsigned char *buf, long long n)
{
        unsigned int h = 0x811c9dc5u;
        long long i;
        for (i = 0; i < n; i++) {
                h ^= buf[i];
                h *= 0x01000193u;
        }
        return h;
}

/* ---- RAID (reference raid/raid_base.c) ----------------------------------- */

/* raid_base.c:100-118 — last vector = XOR of the others; 1 if vects < 3. */
int
oracle_xor_gen(int vects, int len, unsigned char **a)
{
        int i, j;
        if (vects < 3)
                return 1;
        for (i = 0; i < len; i++) {
                unsigned char x = a[0][i];
                for (j = 1; j < vects - 1; j++)
                        x ^= a[j][i];
                a[vects - 1][i] = x;
        }
        return 0;
}

/* raid_base.c:120-140 — 0 if all vectors XOR to zero, else 1. */
int
oracle_xor_check(int vects, int len, unsigned char **a)
{
        int i, j;
        if (vects < 2)
                return 1;
        for (i = 0; i < len; i++) {
                unsigned char x = 0;
                for (j = 0; j < vects; j++)
                        x ^= a[j][i];
                if (x)
                        return 1;
        }
        return 0;
}

static unsigned char
oracle_mul2(unsigned char q)
{
        return (unsigned char) ((q << 1) ^ ((q & 0x80) ? 0x1d : 0));
}

/* raid_base.c:44-68 — P and Q (Horner from the last source: q = D_j ^ 2q);
 * the reference works on 8-byte words, so only len & ~7 bytes are produced. */
int
oracle_pq_gen(int vects, int len, unsigned char **a)
{
        int i, j, n = len & ~7;
        if (vects < 4)
                return 1;
        for (i = 0; i < n; i++) {
                unsigned char p = a[vects - 3][i], q = p;
                for (j = vects - 4; j >= 0; j--) {
                        p ^= a[j][i];
                        q = (unsigned char) (a[j][i] ^ oracle_mul2(q));
                }
                a[vects - 2][i] = p;
                a[vects - 1][i] = q;
        }
        return 0;
}

/* raid_base.c:71-98 — 0, or i|1 (P wrong at byte i) / i|2 (Q wrong). */
int
oracle_pq_check(int vects, int len, unsigned char **a)
{
        int i, j;
        if (vects < 4)
                return 1;
        for (i = 0; i < len; i++) {
                unsigned char p = a[vects - 3][i], q = p;
                for (j = vects - 4; j >= 0; j--) {
                        p ^= a[j][i];
                        q = (unsigned char) (a[j][i] ^ oracle_mul2(q));
                }
                if (a[vects - 2][i] != p)
                        return i | 1;
                if (a[vects - 1][i] != q)
                        return i | 2;
        }
        return 0;
}

/* ---- CRC32C (reference crc/crc_base.c) ------------------------------------ */

/* crc_base.c:205-219 (crc32_iscsi_base): table-driven reflected CRC32C, the
 * register starts at crc_init, no final inversion. The reference's literal
 * table crc32_table_iscsi_refl (crc_base.c:58-...) is the byte table of the
 * reflected Castagnoli polynomial 0x82F63B78 (crc/crc_ref.h:47-61 computes the
 * same CRC bit by bit); it is regenerated here from the polynomial. */
static unsigned int crc32c_tab[256];
static int crc32c_ready;

unsigned int
oracle_crc32_iscsi(const unsigned char *buf, long long len, unsigned int init)
{
        unsigned int crc = init;
        long long i;
        if (!crc32c_ready) {
                int b, k;
                for (b = 0; b < 256; b++) {
                        unsigned int c = (unsigned int) b;
                        for (k = 0; k < 8; k++)
                                c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
                        crc32c_tab[b] = c;
                }
                crc32c_ready = 1;
        }
        for (i = 0; i < len; i++)
                crc = (crc >> 8) ^ crc32c_tab[(crc ^ buf[i]) & 0xff];
        return crc;
}

/* ---- CRC64 (reference crc/crc64_base.c) ----------------------------------- */

/* crc64_base.c:569-670 (crc64_{ecma,iso,jones,rocksoft}_{refl,norm}_base):
 * crc = ~seed; per byte refl: crc = T[(u8) crc ^ byte] ^ (crc >> 8),
 * norm: crc = T[((crc >> 56) ^ byte) & 0xff] ^ (crc << 8); return ~crc. The
 * reference's literal tables (crc64_base.c:32-566) are the byte tables of the
 * polynomials below (normal form; refl uses the bit reversal); they are
 * regenerated here. variant = 2 * family + (norm ? 1 : 0), families in the
 * order of include/crc64.h: ecma, iso, jones, rocksoft. */
static const unsigned long long crc64_poly[4] = {
        0x42F0E1EBA9EA3693ULL, 0x000000000000001BULL, 0xAD93D23594C935A9ULL, 0xAD93D23594C93659ULL
};
static unsigned long long crc64_tab[8][256];
static int crc64_ready[8];

static unsigned long long
rev64(unsigned long long x)
{
        unsigned long long r = 0;
        int i;
        for (i = 0; i < 64; i++)
                r |= ((x >> i) & 1ULL) << (63 - i);
        return r;
}

unsigned long long
oracle_crc64(int variant, const unsigned char *buf, long long len, unsigned long long seed)
{
        const int norm = variant & 1;
        unsigned long long crc = ~seed, *t = crc64_tab[variant & 7];
        long long i;
        if (!crc64_ready[variant & 7]) {
                const unsigned long long p = crc64_poly[(variant >> 1) & 3];
                const unsigned long long pr = rev64(p);
                int b, k;
                for (b = 0; b < 256; b++) {
                        unsigned long long c;
                        if (norm) {
                                c = (unsigned long long) b << 56;
                                for (k = 0; k < 8; k++)
                                        c = (c >> 63) ? (c << 1) ^ p : c << 1;
                        } else {
                                c = (unsigned long long) b;
                                for (k = 0; k < 8; k++)
                                        c = (c & 1) ? (c >> 1) ^ pr : c >> 1;
                        }
                        t[b] = c;
                }
                crc64_ready[variant & 7] = 1;
        }
        for (i = 0; i < len; i++) {
                if (norm)
                        crc = t[((crc >> 56) ^ buf[i]) & 0xff] ^ (crc << 8);
                else
                        crc = t[(crc ^ buf[i]) & 0xff] ^ (crc >> 8);
        }
        return ~crc;
}
