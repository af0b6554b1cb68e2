/*
 * abi_edges.c — TEST INFRASTRUCTURE: the engine's host code under ASan+UBSan.
 *
 * Built with -fsanitize=address,undefined against lib/asan/libisal_hip.so
 * (make -C isa-l_amd asan) together with the oracle restatement
 * (oracle/ec_oracle.c, the checker), and run by tests/test_sanitizers_cpu.py.
 * It drives every host path of the C ABI with edge-case arguments — lengths
 * 0..300 and ragged, k = 0..64, rows beyond one kernel pass, byte-misaligned
 * shards with canaries, out-of-range vec_i, singular matrices, len % 32
 * vect_mul, RAID vects below the minimum, invalid extension-API arguments,
 * bogus knob values — and compares every data result with the oracle. On a
 * host without a GPU the data path is the CPU route; with one, both routes
 * run (ISAL_HIP_BACKEND=cpu and auto). Exit status 0 = all checks passed.
 * (Reference counterpart: tools/test_checks.sh:47, UBSan over the tests.)
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "erasure_code.h"
#include "isal_hip.h"
#include "raid.h"

/* oracle (ec_oracle.c, compiled into this driver) */
void oracle_gf_gen_rs_matrix(unsigned char *a, int m, int k);
int oracle_gf_invert_matrix(unsigned char *in, unsigned char *out, const int n);
void oracle_ec_init_tables(int k, int rows, const unsigned char *a, unsigned char *tbls);
void oracle_ec_encode_data(int len, int k, int rows, const unsigned char *tbls,
                           unsigned char *const *src, unsigned char *const *dst);
void oracle_ec_encode_data_update(int len, int k, int rows, int vec_i, const unsigned char *tbls,
                                  const unsigned char *data, unsigned char *const *dst);
void oracle_fill_bytes(unsigned char *buf, long long n, unsigned long long seed);
int oracle_xor_gen(int vects, int len, unsigned char **a);
int oracle_pq_gen(int vects, int len, unsigned char **a);
int oracle_pq_check(int vects, int len, unsigned char **a);
int oracle_xor_check(int vects, int len, unsigned char **a);

static int failures;

#define CHECK(cond, ...)                                                                           \
        do {                                                                                       \
                if (!(cond)) {                                                                     \
                        fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);                       \
                        fprintf(stderr, __VA_ARGS__);                                              \
                        fprintf(stderr, "\n");                                                     \
                        failures++;                                                                \
                }                                                                                  \
        } while (0)

#define PAD 32
#define CANARY 0x5c

static unsigned long long rng_state = 0x1234;

static unsigned
rnd(unsigned n)
{
        rng_state = rng_state * 6364136223846793005ull + 1442695040888963407ull;
        return n ? (unsigned) (rng_state >> 33) % n : 0;
}

/* a shard with PAD canary bytes on both sides, at a byte offset 0..31 */
static unsigned char *
shard(unsigned char **base, int len, int off)
{
        *base = (unsigned char *) malloc((size_t) len + 2 * PAD + 32);
        memset(*base, CANARY, (size_t) len + 2 * PAD + 32);
        return *base + PAD + off;
}

static int
canaries_ok(const unsigned char *base, int len, int off)
{
        int i;
        for (i = 0; i < PAD + off; i++)
                if (base[i] != CANARY)
                        return 0;
        for (i = PAD + off + len; i < len + 2 * PAD + 32; i++)
                if (base[i] != CANARY)
                        return 0;
        return 1;
}

static void
encode_case(int len, int k, int rows, int update)
{
        unsigned char *coef = (unsigned char *) malloc((size_t) (k * rows) + 1);
        unsigned char *tb = (unsigned char *) malloc((size_t) 32 * k * rows + 1);
        unsigned char **sb = calloc((size_t) k + 1, sizeof(*sb)), **src = calloc((size_t) k + 1, sizeof(*src));
        unsigned char **db = calloc((size_t) rows, sizeof(*db)), **dst = calloc((size_t) rows, sizeof(*dst));
        unsigned char **want = calloc((size_t) rows, sizeof(*want));
        int *off = calloc((size_t) (k + rows), sizeof(int)), j, l;
        for (j = 0; j < k * rows; j++)
                coef[j] = (unsigned char) rnd(256);
        oracle_ec_init_tables(k, rows, coef, tb);
        for (j = 0; j < k; j++) {
                off[j] = (int) rnd(32);
                src[j] = shard(&sb[j], len, off[j]);
                oracle_fill_bytes(src[j], len, rng_state + (unsigned) j);
        }
        for (l = 0; l < rows; l++) {
                off[k + l] = (int) rnd(32);
                dst[l] = shard(&db[l], len, off[k + l]);
                memset(dst[l], 0, (size_t) len);
                want[l] = (unsigned char *) calloc((size_t) len + 1, 1);
        }
        oracle_ec_encode_data(len, k, rows, tb, src, want);
        if (update) {
                for (j = k - 1; j >= 0; j--)
                        ec_encode_data_update(len, k, rows, j, tb, src[j], dst);
        } else {
                ec_encode_data(len, k, rows, tb, src, dst);
        }
        for (l = 0; l < rows; l++) {
                CHECK(memcmp(dst[l], want[l], (size_t) len) == 0, "%s len=%d k=%d rows=%d row %d",
                      update ? "update" : "encode", len, k, rows, l);
                CHECK(canaries_ok(db[l], len, off[k + l]), "canary len=%d k=%d rows=%d", len, k, rows);
        }
        for (j = 0; j < k; j++)
                CHECK(canaries_ok(sb[j], len, off[j]), "source canary");
        for (j = 0; j < k; j++)
                free(sb[j]);
        for (l = 0; l < rows; l++) {
                free(db[l]);
                free(want[l]);
        }
        free(coef);
        free(tb);
        free(sb);
        free(src);
        free(db);
        free(dst);
        free(want);
        free(off);
}

static void
data_paths(void)
{
        static const int lens[] = {0, 1, 2, 15, 16, 17, 31, 32, 33, 63, 64, 65, 255, 300, 4095, 4097, 12345};
        int i, it;
        for (i = 0; i < (int) (sizeof(lens) / sizeof(lens[0])); i++)
                for (it = 0; it < 4; it++) {
                        const int k = it == 0 ? 1 : (int) rnd(40) + 1, rows = (int) rnd(20) + 1;
                        encode_case(lens[i], k, rows, 0);
                        encode_case(lens[i], k, rows, 1);
                }
        /* k = 0: the empty sum (no sources) must give zero parity without touching src */
        {
                unsigned char z[64], *d[2] = {z, z + 32}, t[32] = {0};
                memset(z, 0xEE, sizeof(z));
                ec_encode_data(32, 0, 2, t, NULL, d);
                for (i = 0; i < 64; i++)
                        CHECK(z[i] == 0, "k=0 parity byte %d", i);
        }
        /* vec_i outside [0, k): ignored (undefined in the reference), never an out-of-bounds access */
        {
                unsigned char a[14 * 10], tb[32 * 10 * 4], s[100], p0[100], p1[100], p2[100], p3[100];
                unsigned char *p[4] = {p0, p1, p2, p3};
                oracle_gf_gen_rs_matrix(a, 14, 10);
                ec_init_tables(10, 4, a + 10 * 10, tb);
                memset(p0, 7, 100);
                ec_encode_data_update(100, 10, 4, 10, tb, s, p);
                ec_encode_data_update(100, 10, 4, -1, tb, s, p);
                CHECK(p0[0] == 7 && p0[99] == 7, "out-of-range vec_i wrote parity");
        }
        /* gf_vect_mul: len % 32 != 0 -> -1 and nothing written (ec_base.c:350-353) */
        {
                unsigned char tbl[32], s[96], d[96];
                gf_vect_mul_init(0x53, tbl);
                memset(d, 1, sizeof(d));
                CHECK(gf_vect_mul(95, tbl, s, d) != 0 && d[0] == 1, "gf_vect_mul(95)");
                oracle_fill_bytes(s, 96, 3);
                CHECK(gf_vect_mul(96, tbl, s, d) == 0, "gf_vect_mul(96)");
                for (i = 0; i < 96; i++)
                        CHECK(d[i] == gf_mul(0x53, s[i]), "gf_vect_mul byte %d", i);
                CHECK(gf_vect_mul(0, tbl, s, d) == 0, "gf_vect_mul(0)");
        }
}

static void
matrices(void)
{
        int n, it, i;
        for (n = 1; n <= 32; n++)
                for (it = 0; it < 4; it++) {
                        unsigned char in[32 * 32], in2[32 * 32], out[32 * 32], want[32 * 32];
                        int r1, r2;
                        for (i = 0; i < n * n; i++)
                                in[i] = (unsigned char) (it == 3 && i % n == 0 ? 0 : rnd(256));
                        memcpy(in2, in, (size_t) n * n);
                        r1 = gf_invert_matrix(in, out, n);
                        r2 = oracle_gf_invert_matrix(in2, want, n);
                        CHECK(r1 == r2, "invert ret n=%d", n);
                        if (r1 == 0)
                                CHECK(memcmp(out, want, (size_t) n * n) == 0, "invert n=%d", n);
                }
}

static void
raid(void)
{
        static const int lens[] = {0, 8, 16, 32, 40, 64, 1024, 4096 + 32};
        int li, v, j;
        unsigned char *b[20], *o[20];
        for (li = 0; li < (int) (sizeof(lens) / sizeof(lens[0])); li++)
                for (v = 1; v <= 20; v += (v < 6 ? 1 : 7)) {
                        const int len = lens[li];
                        int r1, r2;
                        for (j = 0; j < v; j++) {
                                b[j] = (unsigned char *) malloc((size_t) len + 1);
                                o[j] = (unsigned char *) malloc((size_t) len + 1);
                                oracle_fill_bytes(b[j], len, (unsigned long long) (17 * li + j));
                                memcpy(o[j], b[j], (size_t) len);
                        }
                        r1 = xor_gen(v, len, (void **) b);
                        r2 = oracle_xor_gen(v, len, o);
                        CHECK(r1 == r2, "xor_gen ret v=%d len=%d", v, len);
                        CHECK(xor_check(v, len, (void **) b) == oracle_xor_check(v, len, o),
                              "xor_check v=%d len=%d", v, len);
                        r1 = pq_gen_base(v, len, (void **) b); /* raid_base.c semantics */
                        r2 = oracle_pq_gen(v, len, o);
                        CHECK(r1 == r2, "pq_gen ret v=%d len=%d", v, len);
                        if (r1 == 0 && v >= 4 && len) {
                                CHECK(memcmp(b[v - 1], o[v - 1], (size_t) len) == 0, "pq_gen Q v=%d", v);
                                b[v / 2][len - 1] ^= 0x10;
                                o[v / 2][len - 1] ^= 0x10;
                        }
                        CHECK(pq_check(v, len, (void **) b) == oracle_pq_check(v, len, o),
                              "pq_check v=%d len=%d", v, len);
                        for (j = 0; j < v; j++) {
                                free(b[j]);
                                free(o[j]);
                        }
                }
}

static void
extension_api(void)
{
        isal_hip_batch *b = NULL;
        isal_hip_pipe *p = NULL;
        isal_hip_multi *m = NULL;
        unsigned char tb[32 * 4], *ptrs[4] = {0};
        long long first, count;
        int rc;
        CHECK(isal_hip_batch_create(NULL, 16, 2, 2, tb, 1, ptrs, ptrs) == ISAL_HIP_EINVAL, "batch NULL out");
        CHECK(isal_hip_batch_create(&b, -1, 2, 2, tb, 1, ptrs, ptrs) == ISAL_HIP_EINVAL, "batch len<0");
        CHECK(isal_hip_batch_create(&b, 16, 2, 0, tb, 1, ptrs, ptrs) == ISAL_HIP_EINVAL, "batch rows=0");
        CHECK(isal_hip_batch_create(&b, 16, 2, 2, NULL, 1, ptrs, ptrs) == ISAL_HIP_EINVAL, "batch tbls");
        CHECK(isal_hip_batch_encode(NULL, NULL) == ISAL_HIP_EINVAL, "batch_encode NULL");
        CHECK(isal_hip_batch_update(NULL, 0, NULL) == ISAL_HIP_EINVAL, "batch_update NULL");
        CHECK(isal_hip_batch_crc(NULL, 0, NULL, NULL) == ISAL_HIP_EINVAL, "batch_crc NULL");
        CHECK(isal_hip_batch_crc64(NULL, 0, 0, NULL, NULL) == ISAL_HIP_EINVAL, "batch_crc64 NULL");
        CHECK(isal_hip_batch_destroy(NULL) == ISAL_HIP_OK, "batch_destroy NULL");
        CHECK(isal_hip_pipe_create(&p, 0, 2, 2, tb, 2, ISAL_HIP_PIPE_ENCODE) == ISAL_HIP_EINVAL, "pipe len 0");
        CHECK(isal_hip_pipe_create(&p, 16, 2, 2, tb, 2, 7) == ISAL_HIP_EINVAL, "pipe mode");
        CHECK(isal_hip_pipe_submit(NULL, ptrs, ptrs) == ISAL_HIP_EINVAL, "pipe submit NULL");
        CHECK(isal_hip_pipe_destroy(NULL) == ISAL_HIP_OK, "pipe destroy NULL");
        CHECK(isal_hip_multi_create(&m, -1, 16, 2, 2, tb, 2) == ISAL_HIP_EINVAL, "multi ndev<0");
        CHECK(isal_hip_multi_encode(NULL, 1, ptrs, ptrs) == ISAL_HIP_EINVAL, "multi encode NULL");
        CHECK(isal_hip_multi_destroy(NULL) == ISAL_HIP_OK, "multi destroy NULL");
        isal_hip_multi_partition(1000003, 8, 7, &first, &count);
        CHECK(first == 875002 && count == 125001, "partition %lld %lld", first, count);
        isal_hip_multi_partition(5, 8, 0, &first, &count);
        CHECK(first == 0 && count == 0, "partition small");
        isal_hip_multi_partition(5, 0, 0, &first, &count);
        CHECK(first == 0 && count == 0, "partition ndev 0");
        /* with no usable GPU the device-side extension reports EHIP, never crashes */
        rc = isal_hip_batch_create(&b, 4096, 2, 2, tb, 1, ptrs, ptrs);
        if (rc == ISAL_HIP_OK)
                isal_hip_batch_destroy(b);
        else
                CHECK(rc == ISAL_HIP_EHIP, "batch_create without GPU rc=%d", rc);
}

int
main(void)
{
        const char *backends[] = {"cpu", "auto", "bogus"};
        int i;
        for (i = 0; i < 3; i++) {
                setenv("ISAL_HIP_BACKEND", backends[i], 1);
                setenv("ISAL_HIP_CPU_SIMD", i == 1 ? "0" : "1", 1);
                isal_hip_config_reload();
                data_paths();
                raid();
        }
        matrices();
        extension_api();
        printf("abi_edges: %s (%d failures; cpu-route calls %llu, kernel launches %llu)\n",
               failures ? "FAIL" : "Pass", failures, isal_hip_cpu_calls(), isal_hip_kernel_launches());
        return failures != 0;
}
