/*
 * gen_golden.c — TEST INFRASTRUCTURE ONLY: writes tests/golden/ec_base_golden.json.
 *
 * Built by `make -C oracle golden` against oracle/_ref/libisal_ref.so, i.e. the
 * reference's own erasure_code/ec_base.c compiled from /root/reference (this
 * container only). Every expected value in the fixture is produced by the
 * reference functions; the inputs come from a counter-based splitmix64 stream
 * (not libc rand(), whose sequence is libc-specific — reference SURVEY §4).
 *
 * The fixture is data: expected outputs (full bytes for small cases, FNV-1a-32
 * digests + head/tail bytes for large ones) for the inputs described in it.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* Reference ABI (reference include/erasure_code.h, gf_vect_mul.h). */
void ec_init_tables_base(int k, int rows, unsigned char *a, unsigned char *g_tbls);
void ec_encode_data_base(int len, int k, int rows, unsigned char *v, unsigned char **src,
                         unsigned char **dest);
void ec_encode_data_update_base(int len, int k, int rows, int vec_i, unsigned char *v,
                                unsigned char *data, unsigned char **dest);
void gf_vect_dot_prod_base(int len, int vlen, unsigned char *v, unsigned char **src,
                           unsigned char *dest);
void gf_vect_mad_base(int len, int vec, int vec_i, unsigned char *v, unsigned char *src,
                      unsigned char *dest);
int gf_vect_mul_base(int len, unsigned char *a, unsigned char *src, unsigned char *dest);
void gf_vect_mul_init_base(unsigned char c, unsigned char *tbl);
unsigned char gf_mul(unsigned char a, unsigned char b);
unsigned char gf_inv(unsigned char a);
void gf_gen_rs_matrix(unsigned char *a, int m, int k);
void gf_gen_cauchy1_matrix(unsigned char *a, int m, int k);
int gf_invert_matrix(unsigned char *in, unsigned char *out, const int n);
/* Reference raid ABI (reference include/raid.h; raid_base.c via raid_base_aliases.c). */
int xor_gen(int vects, int len, void **array);
int xor_check(int vects, int len, void **array);
int pq_gen(int vects, int len, void **array);
int pq_check(int vects, int len, void **array);
/* Reference crc ABI (reference include/crc.h:137-151; crc/crc_base.c). */
unsigned int crc32_iscsi_base(unsigned char *buffer, int len, unsigned int crc_init);
/* Reference crc64 ABI (include/crc64.h:190-330; crc/crc64_base.c:569-670). */
typedef unsigned long long (*crc64_fn)(unsigned long long, const unsigned char *, unsigned long long);
unsigned long long crc64_ecma_refl_base(unsigned long long, const unsigned char *, unsigned long long);
unsigned long long crc64_ecma_norm_base(unsigned long long, const unsigned char *, unsigned long long);
unsigned long long crc64_iso_refl_base(unsigned long long, const unsigned char *, unsigned long long);
unsigned long long crc64_iso_norm_base(unsigned long long, const unsigned char *, unsigned long long);
unsigned long long crc64_jones_refl_base(unsigned long long, const unsigned char *, unsigned long long);
unsigned long long crc64_jones_norm_base(unsigned long long, const unsigned char *, unsigned long long);
unsigned long long crc64_rocksoft_refl_base(unsigned long long, const unsigned char *,
                                            unsigned long long);
unsigned long long crc64_rocksoft_norm_base(unsigned long long, const unsigned char *,
                                            unsigned long long);

static FILE *out;
static int first_item;

static void
fill_bytes(unsigned char *buf, long long n, unsigned long long seed)
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

static unsigned int
fnv1a32(const unsigned char *buf, long long n)
{
        unsigned int h = 0x811c9dc5u;
        long long i;
        for (i = 0; i < n; i++) {
                h ^= buf[i];
                h *= 0x01000193u;
        }
        return h;
}

static void
put_hex(const unsigned char *b, long long n)
{
        long long i;
        fputc('"', out);
        for (i = 0; i < n; i++)
                fprintf(out, "%02x", b[i]);
        fputc('"', out);
}

static void
item_sep(void)
{
        fprintf(out, first_item ? "\n    " : ",\n    ");
        first_item = 0;
}

/* Coefficient generators used by the encode cases. */
enum { GEN_RS = 0, GEN_CAUCHY = 1, GEN_RANDOM = 2 };
static const char *gen_name[] = { "rs", "cauchy", "random" };

static void
make_coeffs(int gen, int k, int rows, unsigned long long seed, unsigned char *coef)
{
        int m = k + rows;
        unsigned char *a = malloc((size_t) m * k);
        if (gen == GEN_RS) {
                gf_gen_rs_matrix(a, m, k);
                memcpy(coef, a + k * k, (size_t) k * rows);
        } else if (gen == GEN_CAUCHY) {
                gf_gen_cauchy1_matrix(a, m, k);
                memcpy(coef, a + k * k, (size_t) k * rows);
        } else {
                fill_bytes(coef, (long long) k * rows, seed ^ 0xC0EFF1C1E47ull);
        }
        free(a);
}

/* Write one encode case: data[j] = fill_bytes(len, seed + j). */
static void
encode_case(int k, int rows, int len, int gen, unsigned long long seed)
{
        unsigned char *coef = malloc((size_t) k * rows + 1);
        unsigned char *tbl = malloc((size_t) 32 * k * rows + 1);
        unsigned char **src = malloc(sizeof(*src) * k + 1);
        unsigned char **dst = malloc(sizeof(*dst) * rows + 1);
        int j, l;

        make_coeffs(gen, k, rows, seed, coef);
        ec_init_tables_base(k, rows, coef, tbl);
        for (j = 0; j < k; j++) {
                src[j] = malloc((size_t) len + 1);
                fill_bytes(src[j], len, seed + (unsigned long long) j);
        }
        for (l = 0; l < rows; l++)
                dst[l] = malloc((size_t) len + 1);
        ec_encode_data_base(len, k, rows, tbl, src, dst);

        item_sep();
        fprintf(out, "{\"k\": %d, \"rows\": %d, \"len\": %d, \"gen\": \"%s\", \"seed\": %llu, ", k,
                rows, len, gen_name[gen], seed);
        fprintf(out, "\"coef\": ");
        put_hex(coef, (long long) k * rows);
        fprintf(out, ", \"fnv\": [");
        for (l = 0; l < rows; l++)
                fprintf(out, "%s%u", l ? ", " : "", fnv1a32(dst[l], len));
        fprintf(out, "]");
        if ((long long) len * rows <= 2048) {
                fprintf(out, ", \"parity\": [");
                for (l = 0; l < rows; l++) {
                        if (l)
                                fprintf(out, ", ");
                        put_hex(dst[l], len);
                }
                fprintf(out, "]");
        } else {
                fprintf(out, ", \"head\": [");
                for (l = 0; l < rows; l++) {
                        if (l)
                                fprintf(out, ", ");
                        put_hex(dst[l], 16);
                }
                fprintf(out, "], \"tail\": [");
                for (l = 0; l < rows; l++) {
                        if (l)
                                fprintf(out, ", ");
                        put_hex(dst[l] + len - 16, 16);
                }
                fprintf(out, "]");
        }
        fprintf(out, "}");

        for (j = 0; j < k; j++)
                free(src[j]);
        for (l = 0; l < rows; l++)
                free(dst[l]);
        free(src);
        free(dst);
        free(coef);
        free(tbl);
}

/* Streaming update: parity zeroed, then ec_encode_data_update for vec_i in `order`. */
static void
update_case(int k, int rows, int len, int gen, unsigned long long seed, int reverse)
{
        unsigned char *coef = malloc((size_t) k * rows);
        unsigned char *tbl = malloc((size_t) 32 * k * rows);
        unsigned char **src = malloc(sizeof(*src) * k);
        unsigned char **dst = malloc(sizeof(*dst) * rows);
        int j, l;

        make_coeffs(gen, k, rows, seed, coef);
        ec_init_tables_base(k, rows, coef, tbl);
        for (j = 0; j < k; j++) {
                src[j] = malloc((size_t) len + 1);
                fill_bytes(src[j], len, seed + (unsigned long long) j);
        }
        for (l = 0; l < rows; l++) {
                dst[l] = malloc((size_t) len + 1);
                memset(dst[l], 0, (size_t) len);
        }
        for (j = 0; j < k; j++) {
                int v = reverse ? k - 1 - j : j;
                ec_encode_data_update_base(len, k, rows, v, tbl, src[v], dst);
        }
        item_sep();
        fprintf(out,
                "{\"k\": %d, \"rows\": %d, \"len\": %d, \"gen\": \"%s\", \"seed\": %llu, "
                "\"reverse\": %d, \"fnv\": [",
                k, rows, len, gen_name[gen], seed, reverse);
        for (l = 0; l < rows; l++)
                fprintf(out, "%s%u", l ? ", " : "", fnv1a32(dst[l], len));
        fprintf(out, "]}");
        for (j = 0; j < k; j++)
                free(src[j]);
        for (l = 0; l < rows; l++)
                free(dst[l]);
        free(src);
        free(dst);
        free(coef);
        free(tbl);
}

/* Decode as in erasure_code_perf.c:134-168: drop erased rows, invert, and for
 * each erased fragment build its recovery row; recover from the survivors. */
static void
decode_case(int k, int p, int len, int gen, const int *errs, int nerrs, unsigned long long seed)
{
        int m = k + p, i, j, r;
        unsigned char *a = malloc((size_t) m * k), *b = malloc((size_t) k * k),
                      *d = malloc((size_t) k * k), *c = calloc((size_t) k * nerrs, 1);
        unsigned char *tbl = malloc((size_t) 32 * k * m);
        unsigned char **frag = malloc(sizeof(*frag) * m), **rec = malloc(sizeof(*rec) * nerrs);
        unsigned char **surv = malloc(sizeof(*surv) * k);
        char in_err[256] = { 0 };
        int ret, ok = 1;

        if (gen == GEN_RS)
                gf_gen_rs_matrix(a, m, k);
        else
                gf_gen_cauchy1_matrix(a, m, k);
        for (i = 0; i < m; i++)
                frag[i] = malloc((size_t) len + 1);
        for (j = 0; j < k; j++)
                fill_bytes(frag[j], len, seed + (unsigned long long) j);
        ec_init_tables_base(k, p, a + k * k, tbl);
        ec_encode_data_base(len, k, p, tbl, frag, frag + k);
        for (i = 0; i < nerrs; i++)
                in_err[errs[i]] = 1;
        for (i = 0, r = 0; i < k; i++, r++) {
                while (in_err[r])
                        r++;
                surv[i] = frag[r];
                for (j = 0; j < k; j++)
                        b[k * i + j] = a[k * r + j];
        }
        ret = gf_invert_matrix(b, d, k);
        if (ret == 0) {
                for (i = 0; i < nerrs; i++) {
                        int s = errs[i];
                        for (j = 0; j < k; j++)
                                for (r = 0; r < k; r++)
                                        c[k * i + j] ^= gf_mul(d[k * r + j], a[k * s + r]);
                }
                for (i = 0; i < nerrs; i++)
                        rec[i] = malloc((size_t) len + 1);
                ec_init_tables_base(k, nerrs, c, tbl);
                ec_encode_data_base(len, k, nerrs, tbl, surv, rec);
                for (i = 0; i < nerrs; i++)
                        ok &= memcmp(rec[i], frag[errs[i]], (size_t) len) == 0;
        }
        item_sep();
        fprintf(out, "{\"k\": %d, \"p\": %d, \"len\": %d, \"gen\": \"%s\", \"seed\": %llu, \"errs\": [",
                k, p, len, gen_name[gen], seed);
        for (i = 0; i < nerrs; i++)
                fprintf(out, "%s%d", i ? ", " : "", errs[i]);
        fprintf(out, "], \"invert_ret\": %d, \"decode_matrix\": ", ret);
        put_hex(c, (long long) k * nerrs);
        fprintf(out, ", \"recovered_ok\": %d, \"fnv\": [", ok);
        for (i = 0; i < nerrs; i++)
                fprintf(out, "%s%u", i ? ", " : "", fnv1a32(frag[errs[i]], len));
        fprintf(out, "]}");
        if (ret == 0)
                for (i = 0; i < nerrs; i++)
                        free(rec[i]);
        for (i = 0; i < m; i++)
                free(frag[i]);
        free(a), free(b), free(d), free(c), free(tbl), free(frag), free(rec), free(surv);
}

static void
invert_case(int n, unsigned long long seed, int density_shift)
{
        unsigned char *in = malloc((size_t) n * n), *cp = malloc((size_t) n * n),
                      *o = malloc((size_t) n * n);
        int i, ret;
        fill_bytes(in, (long long) n * n, seed);
        /* density_shift > 0 zeroes many entries, forcing pivot swaps and singular cases */
        for (i = 0; i < n * n; i++)
                if (density_shift && (in[i] >> density_shift) != 0)
                        in[i] = 0;
        memcpy(cp, in, (size_t) n * n);
        ret = gf_invert_matrix(cp, o, n);
        item_sep();
        fprintf(out, "{\"n\": %d, \"in\": ", n);
        put_hex(in, (long long) n * n);
        fprintf(out, ", \"ret\": %d, \"out\": ", ret);
        put_hex(o, (long long) n * n);
        fprintf(out, ", \"in_after\": ");
        put_hex(cp, (long long) n * n);
        fprintf(out, "}");
        free(in), free(cp), free(o);
}

int
main(int argc, char **argv)
{
        static unsigned char mul[65536], tbl[256 * 32];
        unsigned char inv[256], mat[64 * 64];
        int a, b, i;
        const char *path = argc > 1 ? argv[1] : "tests/golden/ec_base_golden.json";

        out = fopen(path, "w");
        if (!out) {
                perror(path);
                return 1;
        }
        for (a = 0; a < 256; a++)
                for (b = 0; b < 256; b++)
                        mul[a * 256 + b] = gf_mul((unsigned char) a, (unsigned char) b);
        for (a = 0; a < 256; a++)
                inv[a] = gf_inv((unsigned char) a);
        for (a = 0; a < 256; a++)
                gf_vect_mul_init_base((unsigned char) a, tbl + 32 * a);

        fprintf(out, "{\n  \"generator\": \"oracle/gen_golden.c linked against "
                     "/root/reference/erasure_code/ec_base.c (make -C oracle golden)\",\n");
        fprintf(out, "  \"prng\": \"splitmix64 counter stream, see oracle/ec_oracle.c:oracle_fill_bytes\",\n");
        fprintf(out, "  \"gf_mul_table\": ");
        put_hex(mul, sizeof(mul));
        fprintf(out, ",\n  \"gf_inv_table\": ");
        put_hex(inv, sizeof(inv));
        fprintf(out, ",\n  \"mul_init_tables\": ");
        put_hex(tbl, sizeof(tbl));

        /* generator matrices */
        {
                static const int mk[][2] = { { 6, 4 },   { 14, 10 }, { 26, 20 }, { 32, 16 },
                                             { 3, 1 },   { 9, 8 },   { 40, 32 }, { 64, 48 },
                                             { 127, 100 } };
                fprintf(out, ",\n  \"rs_matrices\": [");
                first_item = 1;
                for (i = 0; i < (int) (sizeof(mk) / sizeof(mk[0])); i++) {
                        unsigned char *m = malloc((size_t) mk[i][0] * mk[i][1]);
                        gf_gen_rs_matrix(m, mk[i][0], mk[i][1]);
                        item_sep();
                        fprintf(out, "{\"m\": %d, \"k\": %d, \"a\": ", mk[i][0], mk[i][1]);
                        put_hex(m, (long long) mk[i][0] * mk[i][1]);
                        fprintf(out, "}");
                        free(m);
                }
                fprintf(out, "],\n  \"cauchy_matrices\": [");
                first_item = 1;
                for (i = 0; i < (int) (sizeof(mk) / sizeof(mk[0])); i++) {
                        unsigned char *m = malloc((size_t) mk[i][0] * mk[i][1]);
                        gf_gen_cauchy1_matrix(m, mk[i][0], mk[i][1]);
                        item_sep();
                        fprintf(out, "{\"m\": %d, \"k\": %d, \"a\": ", mk[i][0], mk[i][1]);
                        put_hex(m, (long long) mk[i][0] * mk[i][1]);
                        fprintf(out, "}");
                        free(m);
                }
                fprintf(out, "]");
        }

        /* gf_invert_matrix: the fixed matrices of gf_inverse_test.c:132-174 are
         * covered by the tests directly; here random dense/sparse matrices. */
        fprintf(out, ",\n  \"invert\": [");
        first_item = 1;
        for (i = 0; i < 24; i++)
                invert_case(1 + (i % 12), 1000 + i, 0);
        for (i = 0; i < 24; i++)
                invert_case(2 + (i % 10), 2000 + i, 6);
        for (i = 0; i < 4; i++)
                invert_case(32 + 16 * i, 3000 + i, 0);
        fprintf(out, "]");
        (void) mat;

        /* encode cases */
        fprintf(out, ",\n  \"encode\": [");
        first_item = 1;
        encode_case(4, 2, 65536, GEN_CAUCHY, 1);           /* config C1 */
        encode_case(10, 4, 1 << 20, GEN_RS, 2);            /* config C2, one stripe */
        encode_case(20, 6, 1 << 20, GEN_RS, 3);            /* config C4 shape, shorter shard */
        encode_case(10, 4, 4096, GEN_RS, 4);
        for (i = 0; i <= 64; i++)                          /* every tail length 0..64 */
                encode_case(1 + i % 7, 1 + i % 6, i, i % 3, 100 + i);
        for (i = 0; i < 40; i++) {                         /* ragged lengths, wide shapes */
                int len = 16 + (i * 997) % 5000;
                encode_case(1 + (i * 5) % 32, 1 + (i * 3) % 16, len, i % 3, 200 + i);
        }
        encode_case(64, 16, 1000, GEN_RANDOM, 300);
        encode_case(100, 27, 333, GEN_CAUCHY, 301);        /* m = 127, the max fragment count of erasure_code_test.c */
        encode_case(255, 1, 257, GEN_RANDOM, 302);
        encode_case(1, 32, 777, GEN_RANDOM, 303);
        fprintf(out, "]");

        /* update (ec_encode_data_update accumulated over all sources) */
        fprintf(out, ",\n  \"update\": [");
        first_item = 1;
        update_case(20, 6, 1 << 18, GEN_RS, 400, 0);
        update_case(10, 4, 4096, GEN_RS, 401, 1);
        for (i = 0; i < 20; i++)
                update_case(1 + (i * 3) % 17, 1 + i % 9, i * 13, i % 3, 410 + i, i & 1);
        fprintf(out, "]");

        /* decode */
        fprintf(out, ",\n  \"decode\": [");
        first_item = 1;
        {
                static const int e1[] = { 4, 6, 7 }, e2[] = { 0, 11, 13 }, e3[] = { 1, 2 },
                                 e4[] = { 19, 21, 22, 23, 25, 0 };
                decode_case(10, 4, 1 << 20, GEN_RS, e1, 3, 500); /* config C3, one stripe */
                decode_case(10, 4, 4096, GEN_RS, e2, 3, 501);
                decode_case(4, 2, 65536, GEN_CAUCHY, e3, 2, 502);
                decode_case(20, 6, 8192, GEN_RS, e4, 6, 503);
        }
        fprintf(out, "]");

        /* single-output primitives */
        fprintf(out, ",\n  \"dot_prod\": [");
        first_item = 1;
        for (i = 0; i < 8; i++) {
                int vlen = 1 + i * 3, len = 31 + i * 211, j;
                unsigned char *coef = malloc((size_t) vlen), *t = malloc((size_t) 32 * vlen);
                unsigned char **src = malloc(sizeof(*src) * vlen), *d = malloc((size_t) len);
                fill_bytes(coef, vlen, 600 + i);
                for (j = 0; j < vlen; j++) {
                        gf_vect_mul_init_base(coef[j], t + 32 * j);
                        src[j] = malloc((size_t) len);
                        fill_bytes(src[j], len, 610 + i * 64 + j);
                }
                gf_vect_dot_prod_base(len, vlen, t, src, d);
                item_sep();
                fprintf(out, "{\"vlen\": %d, \"len\": %d, \"coef_seed\": %d, \"src_seed\": %d, \"dest\": ",
                        vlen, len, 600 + i, 610 + i * 64);
                put_hex(d, len);
                fprintf(out, "}");
                for (j = 0; j < vlen; j++)
                        free(src[j]);
                free(coef), free(t), free(src), free(d);
        }
        fprintf(out, "],\n  \"mad\": [");
        first_item = 1;
        for (i = 0; i < 8; i++) {
                int vec = 1 + i * 2, vec_i = (i * 7) % vec, len = 64 + i * 129;
                unsigned char *coef = malloc((size_t) vec), *t = malloc((size_t) 32 * vec);
                unsigned char *s = malloc((size_t) len), *d = malloc((size_t) len);
                fill_bytes(coef, vec, 700 + i);
                for (a = 0; a < vec; a++)
                        gf_vect_mul_init_base(coef[a], t + 32 * a);
                fill_bytes(s, len, 710 + i);
                fill_bytes(d, len, 720 + i);
                gf_vect_mad_base(len, vec, vec_i, t, s, d);
                item_sep();
                fprintf(out,
                        "{\"vec\": %d, \"vec_i\": %d, \"len\": %d, \"coef_seed\": %d, \"src_seed\": "
                        "%d, \"dest_seed\": %d, \"dest\": ",
                        vec, vec_i, len, 700 + i, 710 + i, 720 + i);
                put_hex(d, len);
                fprintf(out, "}");
                free(coef), free(t), free(s), free(d);
        }
        fprintf(out, "],\n  \"vect_mul\": [");
        first_item = 1;
        for (i = 0; i < 6; i++) {
                int len = 32 * (1 + i * 5) + ((i == 5) ? 3 : 0);
                unsigned char c = (unsigned char) (0x53 + 37 * i), t[32];
                unsigned char *s = malloc((size_t) len), *d = calloc((size_t) len, 1);
                int ret;
                gf_vect_mul_init_base(c, t);
                fill_bytes(s, len, 800 + i);
                ret = gf_vect_mul_base(len, t, s, d);
                item_sep();
                fprintf(out, "{\"c\": %d, \"len\": %d, \"src_seed\": %d, \"ret\": %d, \"dest\": ", c,
                        len, 800 + i, ret);
                put_hex(d, len);
                fprintf(out, "}");
                free(s), free(d);
        }
        fprintf(out, "]");

        /* RAID (reference raid_base.c): xor_gen / pq_gen outputs, and the
         * check functions' return values on clean and corrupted arrays. */
        fprintf(out, ",\n  \"raid\": [");
        first_item = 1;
        {
                static const int lens[] = { 0, 1, 13, 31, 32, 101, 1024, 4096 + 7 };
                int v, li;
                for (v = 3; v <= 20; v += (v < 6 ? 1 : 5)) {
                        for (li = 0; li < (int) (sizeof(lens) / sizeof(lens[0])); li++) {
                                int len = lens[li], jj, rx, rp, cx, cp, cx2 = -1, cp2 = -1;
                                unsigned long long seed = 900 + v * 31 + li;
                                unsigned char *bx[24], *bp[24];
                                for (jj = 0; jj < v; jj++) {
                                        bx[jj] = malloc((size_t) len + 1);
                                        bp[jj] = malloc((size_t) len + 1);
                                        fill_bytes(bx[jj], len, seed + jj);
                                        fill_bytes(bp[jj], len, seed + jj);
                                }
                                rx = xor_gen(v, len, (void **) bx);
                                rp = pq_gen(v, len, (void **) bp);
                                cx = xor_check(v, len, (void **) bx);
                                cp = pq_check(v, len & ~7, (void **) bp);
                                if (len >= 8) {
                                        /* corrupt one byte of a source, check, restore */
                                        int at = (len & ~7) - 2 - (li % 3), vi = (li + v) % (v > 3 ? v - 2 : 1);
                                        bx[vi][at] ^= 0x20;
                                        cx2 = xor_check(v, len, (void **) bx);
                                        bx[vi][at] ^= 0x20;
                                        if (v >= 4) {
                                                bp[vi][at] ^= 0x20;
                                                cp2 = pq_check(v, len & ~7, (void **) bp);
                                                bp[vi][at] ^= 0x20;
                                        }
                                }
                                item_sep();
                                fprintf(out,
                                        "{\"vects\": %d, \"len\": %d, \"seed\": %llu, \"xor_ret\": %d, "
                                        "\"pq_ret\": %d, \"xor_check\": %d, \"pq_check\": %d, "
                                        "\"xor_check_corrupt\": %d, \"pq_check_corrupt\": %d, "
                                        "\"xor_fnv\": %u, \"p_fnv\": %u, \"q_fnv\": %u}",
                                        v, len, seed, rx, rp, cx, cp, cx2, cp2,
                                        fnv1a32(bx[v - 1], len), v >= 4 ? fnv1a32(bp[v - 2], len) : 0,
                                        v >= 4 ? fnv1a32(bp[v - 1], len) : 0);
                                for (jj = 0; jj < v; jj++) {
                                        free(bx[jj]);
                                        free(bp[jj]);
                                }
                        }
                }
        }
        fprintf(out, "]");

        /* CRC32C (reference crc_base.c crc32_iscsi_base): the fused fragment
         * checksum of the engine must equal it. The shapes follow
         * crc32_funcs_test.c (zero buffer, 0x8a buffer, random sizes) plus
         * the tile boundaries of the GPU kernels (4 KiB tiles, 16 B lanes). */
        fprintf(out, ",\n  \"crc32_iscsi\": [");
        first_item = 1;
        {
                static const int lens[] = { 0, 1, 3, 15, 16, 17, 255, 256, 1000, 4080, 4095, 4096,
                                            4097, 4112, 8192, 65536, 65536 + 16, 65536 * 3 + 4000,
                                            1 << 20 };
                static const unsigned int inits[] = { 0u, 0xffffffffu, 0x12345678u };
                int li, ii;
                for (li = 0; li < (int) (sizeof(lens) / sizeof(lens[0])); li++)
                        for (ii = 0; ii < 3; ii++) {
                                const int len = lens[li];
                                const unsigned long long seed = 1000 + li * 7 + ii;
                                unsigned char *b = malloc((size_t) len + 1);
                                int kind = (li + ii) % 5 == 0 ? 1 : ((li + ii) % 7 == 0 ? 2 : 0);
                                if (kind == 1)
                                        memset(b, 0, len);
                                else if (kind == 2)
                                        memset(b, 0x8a, len);
                                else
                                        fill_bytes(b, len, seed);
                                item_sep();
                                fprintf(out,
                                        "{\"len\": %d, \"init\": %u, \"fill\": \"%s\", "
                                        "\"seed\": %llu, \"crc\": %u}",
                                        len, inits[ii],
                                        kind == 1 ? "zero" : (kind == 2 ? "8a" : "splitmix"), seed,
                                        crc32_iscsi_base(b, len, inits[ii]));
                                free(b);
                        }
        }
        fprintf(out, "]");

        /* CRC64, all eight flavours of crc64.h (variant = index below). Same
         * buffer shapes as crc32_iscsi plus the 16-byte tail boundaries of
         * the GPU combine. CRC values as decimal strings (64-bit). */
        fprintf(out, ",\n  \"crc64\": [");
        first_item = 1;
        {
                static const crc64_fn fns[8] = { crc64_ecma_refl_base,    crc64_ecma_norm_base,
                                                 crc64_iso_refl_base,     crc64_iso_norm_base,
                                                 crc64_jones_refl_base,   crc64_jones_norm_base,
                                                 crc64_rocksoft_refl_base, crc64_rocksoft_norm_base };
                static const int lens[] = { 0, 1, 7, 16, 31, 4095, 4096, 4097, 4112, 4100,
                                            8192 + 48, 65536 + 4095, 1 << 20 };
                static const unsigned long long inits[] = { 0ULL, ~0ULL, 0x0123456789abcdefULL };
                int vi, li, ii;
                for (vi = 0; vi < 8; vi++)
                        for (li = 0; li < (int) (sizeof(lens) / sizeof(lens[0])); li++) {
                                const int len = lens[li];
                                const unsigned long long seed = 5000 + vi * 97 + li;
                                unsigned char *b = malloc((size_t) len + 1);
                                const int kind = (vi + li) % 6 == 0 ? 1 : ((vi + li) % 9 == 0 ? 2 : 0);
                                ii = (vi + li) % 3;
                                if (kind == 1)
                                        memset(b, 0, len);
                                else if (kind == 2)
                                        memset(b, 0x8a, len);
                                else
                                        fill_bytes(b, len, seed);
                                item_sep();
                                fprintf(out,
                                        "{\"variant\": %d, \"len\": %d, \"init\": \"%llu\", "
                                        "\"fill\": \"%s\", \"seed\": %llu, \"crc\": \"%llu\"}",
                                        vi, len, inits[ii],
                                        kind == 1 ? "zero" : (kind == 2 ? "8a" : "splitmix"), seed,
                                        fns[vi](inits[ii], b, (unsigned long long) len));
                                free(b);
                        }
        }
        fprintf(out, "]\n}\n");
        fclose(out);
        return 0;
}
