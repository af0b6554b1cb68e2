/*
 * ec_diff_fuzz.c — TEST INFRASTRUCTURE: differential libFuzzer target.
 *
 * Every input becomes one call of the engine's C ABI (libisal_hip: GPU
 * kernels or CPU route, whichever the shim picks) and the same call of the
 * oracle restatement of the reference (oracle/ec_oracle.c, the checker); the
 * outputs, return codes and the canary bytes around every output buffer must
 * agree or the target aborts. It covers what the reference's own fuzz harness
 * (tests/fuzz/ec_fuzz_test.c:80-138,184-217,322-348, raid_fuzz_test.c) drives —
 * table expansion, encode, dot product, multiply-accumulate and RAID with
 * len in [0, 16384], k and rows up to 16, arbitrary gftbls bytes — and adds
 * what that harness never checks: the results themselves, update sequences,
 * gf_vect_mul's len % 32 contract, byte-misaligned shards and the check
 * functions' mismatch positions.
 *
 * Input: byte 0 op, 1-2 len, 3 k, 4 rows, 5 misalignment, 6 vec_i / corrupt
 * position, then payload bytes (coefficients, tables, data) — cycled when the
 * input is shorter than the call needs, so every input runs a call.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "erasure_code.h"
#include "raid.h"

void oracle_ec_init_tables(int k, int rows, const unsigned char *a, unsigned char *tbls);
void oracle_ec_encode_data(int len, int k, int rows, const unsigned char *tbls,
                           unsigned char *const *src, unsigned char *const *dst);
void oracle_ec_encode_data_update(int len, int k, int rows, int vec_i, const unsigned char *tbls,
                                  const unsigned char *data, unsigned char *const *dst);
void oracle_gf_vect_dot_prod(int len, int vlen, const unsigned char *tbls, unsigned char *const *src,
                             unsigned char *dest);
void oracle_gf_vect_mad(int len, int vec, int vec_i, const unsigned char *tbls,
                        const unsigned char *src, unsigned char *dest);
int oracle_gf_vect_mul(int len, const unsigned char *tbl, const unsigned char *src,
                       unsigned char *dest);
int oracle_xor_gen(int vects, int len, unsigned char **a);
int oracle_pq_gen(int vects, int len, unsigned char **a);
int oracle_xor_check(int vects, int len, unsigned char **a);
int oracle_pq_check(int vects, int len, unsigned char **a);

int LLVMFuzzerTestOneInput(const uint8_t *data, size_t size);

#define MAX_K 16
#define MAX_ROWS 16
#define MAX_LEN 16384
#define PAD 16
#define CANARY 0xA5

enum { OP_ENCODE, OP_ENCODE_BASE, OP_UPDATE, OP_DOT, OP_MAD, OP_MUL, OP_XOR_GEN, OP_PQ_GEN,
       OP_XOR_CHECK, OP_PQ_CHECK, OP_INIT, NOPS };

static const char *const op_name[NOPS] = {"ec_encode_data", "ec_encode_data_base",
                                          "ec_encode_data_update", "gf_vect_dot_prod",
                                          "gf_vect_mad", "gf_vect_mul", "xor_gen", "pq_gen",
                                          "xor_check", "pq_check", "ec_init_tables"};

static void
fail(int op, int len, int k, int rows, const char *what, long long at)
{
        fprintf(stderr, "ec_diff_fuzz: %s len=%d k=%d rows=%d: %s (at %lld)\n", op_name[op], len, k,
                rows, what, at);
        abort();
}

/* payload stream: the input's bytes after the header, cycled */
typedef struct {
        const uint8_t *p;
        size_t n, i;
} feed_t;

static void
fill(feed_t *f, unsigned char *dst, size_t n)
{
        for (size_t j = 0; j < n; j++) {
                dst[j] = f->n ? f->p[f->i % f->n] : (unsigned char) (j * 131 + 7);
                f->i++;
        }
}

/* A buffer of len bytes at byte offset `off`, with CANARY padding both sides. */
static unsigned char *
buf_new(int len, int off)
{
        unsigned char *b = (unsigned char *) malloc((size_t) len + 2 * PAD + 16);
        if (!b)
                abort();
        memset(b, CANARY, (size_t) len + 2 * PAD + 16);
        return b + PAD + off;
}

static void
buf_free(unsigned char *p, int off)
{
        free(p - PAD - off);
}

static void
canaries(int op, int len, int k, int rows, unsigned char *p, int off)
{
        for (int j = 1; j <= PAD; j++)
                if (p[-j] != CANARY)
                        fail(op, len, k, rows, "wrote before the buffer", -j);
        for (int j = 0; j < PAD; j++)
                if (p[len + j] != CANARY)
                        fail(op, len, k, rows, "wrote past the buffer", len + j);
        (void) off;
}

static void
same(int op, int len, int k, int rows, const unsigned char *got, const unsigned char *want, int n,
     const char *what)
{
        for (int j = 0; j < n; j++)
                if (got[j] != want[j])
                        fail(op, len, k, rows, what, j);
}

int
LLVMFuzzerTestOneInput(const uint8_t *data, size_t size)
{
        if (size < 7)
                return 0;
        const int op = data[0] % NOPS;
        int len = ((data[1] << 8) | data[2]) % (MAX_LEN + 1);
        const int k = 1 + data[3] % MAX_K, rows = 1 + data[4] % MAX_ROWS;
        const int off = data[5] & 15, sel = data[6];
        feed_t f = {data + 7, size - 7, 0};
        unsigned char *src[MAX_K + 2], *dst[MAX_ROWS + 2], *ref[MAX_ROWS + 2];
        unsigned char a[MAX_K * MAX_ROWS], tb[32 * MAX_K * MAX_ROWS], ot[32 * MAX_K * MAX_ROWS];
        int i, vects;

        switch (op) {
        case OP_INIT:
                fill(&f, a, (size_t) k * rows);
                ec_init_tables(k, rows, a, tb);
                oracle_ec_init_tables(k, rows, a, ot);
                same(op, 0, k, rows, tb, ot, 32 * k * rows, "tables differ");
                ec_init_tables_base(k, rows, a, tb);
                same(op, 0, k, rows, tb, ot, 32 * k * rows, "base tables differ");
                return 0;
        case OP_ENCODE:
        case OP_ENCODE_BASE:
        case OP_UPDATE:
        case OP_DOT:
        case OP_MAD:
        case OP_MUL: {
                const int nout = op == OP_ENCODE || op == OP_ENCODE_BASE || op == OP_UPDATE ? rows : 1;
                const int nsrc = op == OP_UPDATE || op == OP_MAD || op == OP_MUL ? 1 : k;
                const int vec_i = sel % k;
                if (op == OP_MUL && (sel & 1))
                        len &= ~31; /* half the gf_vect_mul calls take the len % 32 == 0 path */
                if (op == OP_DOT || op == OP_MAD || op == OP_MUL) {
                        fill(&f, tb, (size_t) 32 * k); /* raw table bytes, as the reference harness */
                } else {
                        fill(&f, a, (size_t) k * rows);
                        ec_init_tables(k, rows, a, tb);
                }
                for (i = 0; i < nsrc; i++) {
                        src[i] = buf_new(len, off);
                        fill(&f, src[i], (size_t) len);
                }
                for (i = 0; i < nout; i++) {
                        dst[i] = buf_new(len, (off + i) & 15);
                        ref[i] = (unsigned char *) malloc((size_t) len + 1);
                        if (!ref[i])
                                abort();
                        fill(&f, dst[i], (size_t) len); /* update / mad fold into this */
                        memcpy(ref[i], dst[i], (size_t) len);
                }
                int rc = 0, orc = 0;
                switch (op) {
                case OP_ENCODE:
                        ec_encode_data(len, k, rows, tb, src, dst);
                        oracle_ec_encode_data(len, k, rows, tb, src, ref);
                        break;
                case OP_ENCODE_BASE:
                        ec_encode_data_base(len, k, rows, tb, src, dst);
                        oracle_ec_encode_data(len, k, rows, tb, src, ref);
                        break;
                case OP_UPDATE:
                        ec_encode_data_update(len, k, rows, vec_i, tb, src[0], dst);
                        oracle_ec_encode_data_update(len, k, rows, vec_i, tb, src[0], ref);
                        break;
                case OP_DOT:
                        gf_vect_dot_prod(len, k, tb, src, dst[0]);
                        oracle_gf_vect_dot_prod(len, k, tb, src, ref[0]);
                        break;
                case OP_MAD:
                        gf_vect_mad(len, k, vec_i, tb, src[0], dst[0]);
                        oracle_gf_vect_mad(len, k, vec_i, tb, src[0], ref[0]);
                        break;
                default:
                        rc = gf_vect_mul(len, tb + 32 * vec_i, src[0], dst[0]);
                        orc = oracle_gf_vect_mul(len, tb + 32 * vec_i, src[0], ref[0]);
                        break;
                }
                if (rc != orc)
                        fail(op, len, k, rows, "return code differs", rc);
                for (i = 0; i < nout; i++) {
                        same(op, len, k, rows, dst[i], ref[i], len, "output differs");
                        canaries(op, len, k, rows, dst[i], (off + i) & 15);
                        buf_free(dst[i], (off + i) & 15);
                        free(ref[i]);
                }
                for (i = 0; i < nsrc; i++) {
                        canaries(op, len, k, rows, src[i], off);
                        buf_free(src[i], off);
                }
                return 0;
        }
        default: {
                /* RAID: vects = sources + parity, len a multiple of 32 (the
                 * reference harness's rounding, raid_fuzz_test.c:61-90) */
                const int gen = op == OP_XOR_GEN || op == OP_PQ_GEN;
                const int pq = op == OP_PQ_GEN || op == OP_PQ_CHECK;
                void *arr[MAX_K + 2];
                unsigned char *oarr[MAX_K + 2];
                vects = k + (pq ? 2 : 1);
                len &= ~31;
                for (i = 0; i < vects; i++) {
                        src[i] = buf_new(len, off);
                        fill(&f, src[i], (size_t) len);
                        oarr[i] = (unsigned char *) malloc((size_t) len + 1);
                        if (!oarr[i])
                                abort();
                }
                if (!gen) {
                        /* make the parity right, then corrupt one byte in half the inputs */
                        if (pq)
                                oracle_pq_gen(vects, len, src);
                        else
                                oracle_xor_gen(vects, len, src);
                        if ((sel & 1) && len)
                                src[(sel >> 1) % vects][(data[1] * 257 + data[2]) % len] ^= 1 + (sel >> 4);
                }
                for (i = 0; i < vects; i++) {
                        memcpy(oarr[i], src[i], (size_t) len);
                        arr[i] = src[i];
                }
                int rc, orc;
                if (op == OP_XOR_GEN) {
                        rc = xor_gen(vects, len, arr);
                        orc = oracle_xor_gen(vects, len, oarr);
                } else if (op == OP_PQ_GEN) {
                        rc = pq_gen(vects, len, arr);
                        orc = oracle_pq_gen(vects, len, oarr);
                } else if (op == OP_XOR_CHECK) {
                        rc = xor_check(vects, len, arr);
                        orc = oracle_xor_check(vects, len, oarr);
                } else {
                        rc = pq_check(vects, len, arr);
                        orc = oracle_pq_check(vects, len, oarr);
                }
                if (rc != orc)
                        fail(op, len, vects, 0, "return code differs", rc);
                for (i = 0; i < vects; i++) {
                        same(op, len, vects, 0, src[i], oarr[i], len, "vector differs");
                        canaries(op, len, vects, 0, src[i], off);
                        buf_free(src[i], off);
                        free(oarr[i]);
                }
                return 0;
        }
        }
}
