/*
 * erasure_code.h — Reed-Solomon erasure-code API of the MI355X engine.
 *
 * Drop-in replacement for the reference include/erasure_code.h: the same
 * extern "C" signatures (reference erasure_code.h:74-246, 1064-1133), served
 * by libisal_hip.so. Semantics kept from the reference:
 *   - GF(2^8) with polynomial x^8+x^4+x^3+x^2+1 (0x11d);
 *   - gftbls holds 32 bytes per coefficient, row-major (row l, source j at
 *     (l*k + j)*32), in the portable format of ec_init_tables_base;
 *   - every call is synchronous; buffers are owned by the caller; any len >= 0
 *     and any byte alignment is accepted; bytes outside [ptr, ptr+len) are
 *     never touched;
 *   - data-path calls return void and add no failure mode (the reference API
 *     has no error channel; erasure_code.h:108-110 of the reference).
 * Differences: shard buffers may live in host memory OR in device memory
 * (hipMalloc / hipMallocManaged); the engine classifies each pointer
 * (hipPointerGetAttributes) and routes the call (isal_hip.h, "routing"):
 *   - any shard in device memory: GPU kernels;
 *   - all shards in host memory and (k + rows) * len at most a size limit:
 *     the engine's CPU route (ec_cpu.c: AVX-512 GFNI affine, else AVX2 nibble
 *     shuffles, else per byte) — below it the GPU round trip costs more. The
 *     limit is 8 MiB, or 2 MiB when every shard is page-locked and the
 *     kernels can use it in place (the numbers and knobs: isal_hip.h,
 *     "routing");
 *   - larger host calls: GPU kernels, page-locked shards in place, pageable
 *     ones through HBM staging.
 * A GPU runtime error during a host-resident call is reported once on stderr
 * and the columns not yet final finish on the CPU route, so results are
 * unchanged. A call with any device-resident shard (which no CPU route can
 * read), or any call under ISAL_HIP_BACKEND=gpu, aborts on a GPU error instead.
 * The *_base data-path entry points are routed the same way (their outputs
 * are identical by construction).
 */
#ifndef ISAL_HIP_ERASURE_CODE_H
#define ISAL_HIP_ERASURE_CODE_H

#include "isal_api.h"
#include "gf_vect_mul.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- table expansion (host) ------------------------------------------- */

/* Expand rows*k coefficients in a[] into 32*k*rows bytes of gftbls.
 * Replaces ec_init_tables (reference erasure_code.h:74-75). */
void ec_init_tables(int k, int rows, unsigned char *a, unsigned char *gftbls);

/* Replaces ec_init_tables_base (reference erasure_code.h:83-84, ec_base.c:37-48). */
void ec_init_tables_base(int k, int rows, unsigned char *a, unsigned char *gftbls);

/* ---- encode / decode (GPU data path) ------------------------------------ */

/* coding[l][i] = XOR_j c[l][j] * data[j][i], l < rows, i < len.
 * Replaces ec_encode_data (reference erasure_code.h:108-110; semantics of
 * ec_base.c:309-325). */
void ec_encode_data(int len, int k, int rows, unsigned char *gftbls, unsigned char **data,
                    unsigned char **coding);

/* Replaces ec_encode_data_base (reference erasure_code.h:118-120). */
void ec_encode_data_base(int len, int k, int rows, unsigned char *gftbls, unsigned char **data,
                         unsigned char **coding);

/* coding[l][i] ^= c[l][vec_i] * data[i]: fold one source into the parity.
 * Replaces ec_encode_data_update (reference erasure_code.h:145-147;
 * semantics of ec_base.c:327-342). */
void ec_encode_data_update(int len, int k, int rows, int vec_i, unsigned char *gftbls,
                           unsigned char *data, unsigned char **coding);

/* Replaces ec_encode_data_update_base (reference erasure_code.h:156-158). */
void ec_encode_data_update_base(int len, int k, int rows, int vec_i, unsigned char *gftbls,
                                unsigned char *data, unsigned char **coding);

/* dest[i] = XOR_j c[j] * src[j][i] (one output).
 * Replaces gf_vect_dot_prod (reference erasure_code.h:206-208, ec_base.c:282-294). */
void gf_vect_dot_prod(int len, int vlen, unsigned char *gftbls, unsigned char **src,
                      unsigned char *dest);

/* Replaces gf_vect_dot_prod_base (reference erasure_code.h:181-183). */
void gf_vect_dot_prod_base(int len, int vlen, unsigned char *gftbls, unsigned char **src,
                           unsigned char *dest);

/* dest[i] ^= c[vec_i] * src[i] (one output).
 * Replaces gf_vect_mad (reference erasure_code.h:233-235, ec_base.c:296-307). */
void gf_vect_mad(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src,
                 unsigned char *dest);

/* Replaces gf_vect_mad_base (reference erasure_code.h:244-246). */
void gf_vect_mad_base(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src,
                      unsigned char *dest);

/* ---- deprecated per-ISA names (binary compatibility) -------------------- */
/*
 * The reference exports x86 per-ISA variants of every data-path function
 * (erasure_code.h:249-1050, isa-l.def:5-48) for callers built against older
 * releases. Here each is an alias of the corresponding engine entry point
 * (same GPU path, same results): gf_Nvect_dot_prod_* == ec_encode_data with
 * rows = N, gf_Nvect_mad_* == ec_encode_data_update with rows = N. Unlike the
 * reference SIMD kernels, which return without work for len below their
 * vector width (e.g. gf_vect_dot_prod_avx512.asm:226-229), these compute for
 * every len >= 0.
 */
#ifndef ISAL_HIP_DEPRECATED
#define ISAL_HIP_DEPRECATED __attribute__((deprecated))
#endif
ISAL_HIP_DEPRECATED void ec_encode_data_sse(int len, int k, int rows, unsigned char *gftbls, unsigned char **data, unsigned char **coding);
ISAL_HIP_DEPRECATED void ec_encode_data_update_sse(int len, int k, int rows, int vec_i, unsigned char *gftbls, unsigned char *data, unsigned char **coding);
ISAL_HIP_DEPRECATED void gf_vect_dot_prod_sse(int len, int vlen, unsigned char *gftbls, unsigned char **src, unsigned char *dest);
ISAL_HIP_DEPRECATED void gf_vect_mad_sse(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src, unsigned char *dest);
ISAL_HIP_DEPRECATED void gf_2vect_dot_prod_sse(int len, int vlen, unsigned char *gftbls, unsigned char **src, unsigned char **dest);
ISAL_HIP_DEPRECATED void gf_2vect_mad_sse(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src, unsigned char **dest);
ISAL_HIP_DEPRECATED void gf_3vect_dot_prod_sse(int len, int vlen, unsigned char *gftbls, unsigned char **src, unsigned char **dest);
ISAL_HIP_DEPRECATED void gf_3vect_mad_sse(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src, unsigned char **dest);
ISAL_HIP_DEPRECATED void gf_4vect_dot_prod_sse(int len, int vlen, unsigned char *gftbls, unsigned char **src, unsigned char **dest);
ISAL_HIP_DEPRECATED void gf_4vect_mad_sse(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src, unsigned char **dest);
ISAL_HIP_DEPRECATED void gf_5vect_dot_prod_sse(int len, int vlen, unsigned char *gftbls, unsigned char **src, unsigned char **dest);
ISAL_HIP_DEPRECATED void gf_5vect_mad_sse(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src, unsigned char **dest);
ISAL_HIP_DEPRECATED void gf_6vect_dot_prod_sse(int len, int vlen, unsigned char *gftbls, unsigned char **src, unsigned char **dest);
ISAL_HIP_DEPRECATED void gf_6vect_mad_sse(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src, unsigned char **dest);
ISAL_HIP_DEPRECATED void ec_encode_data_avx(int len, int k, int rows, unsigned char *gftbls, unsigned char **data, unsigned char **coding);
ISAL_HIP_DEPRECATED void ec_encode_data_update_avx(int len, int k, int rows, int vec_i, unsigned char *gftbls, unsigned char *data, unsigned char **coding);
ISAL_HIP_DEPRECATED void gf_vect_dot_prod_avx(int len, int vlen, unsigned char *gftbls, unsigned char **src, unsigned char *dest);
ISAL_HIP_DEPRECATED void gf_vect_mad_avx(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src, unsigned char *dest);
ISAL_HIP_DEPRECATED void gf_2vect_dot_prod_avx(int len, int vlen, unsigned char *gftbls, unsigned char **src, unsigned char **dest);
ISAL_HIP_DEPRECATED void gf_2vect_mad_avx(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src, unsigned char **dest);
ISAL_HIP_DEPRECATED void gf_3vect_dot_prod_avx(int len, int vlen, unsigned char *gftbls, unsigned char **src, unsigned char **dest);
ISAL_HIP_DEPRECATED void gf_3vect_mad_avx(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src, unsigned char **dest);
ISAL_HIP_DEPRECATED void gf_4vect_dot_prod_avx(int len, int vlen, unsigned char *gftbls, unsigned char **src, unsigned char **dest);
ISAL_HIP_DEPRECATED void gf_4vect_mad_avx(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src, unsigned char **dest);
ISAL_HIP_DEPRECATED void gf_5vect_dot_prod_avx(int len, int vlen, unsigned char *gftbls, unsigned char **src, unsigned char **dest);
ISAL_HIP_DEPRECATED void gf_5vect_mad_avx(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src, unsigned char **dest);
ISAL_HIP_DEPRECATED void gf_6vect_dot_prod_avx(int len, int vlen, unsigned char *gftbls, unsigned char **src, unsigned char **dest);
ISAL_HIP_DEPRECATED void gf_6vect_mad_avx(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src, unsigned char **dest);
ISAL_HIP_DEPRECATED void ec_encode_data_avx2(int len, int k, int rows, unsigned char *gftbls, unsigned char **data, unsigned char **coding);
ISAL_HIP_DEPRECATED void ec_encode_data_update_avx2(int len, int k, int rows, int vec_i, unsigned char *gftbls, unsigned char *data, unsigned char **coding);
ISAL_HIP_DEPRECATED void gf_vect_dot_prod_avx2(int len, int vlen, unsigned char *gftbls, unsigned char **src, unsigned char *dest);
ISAL_HIP_DEPRECATED void gf_vect_mad_avx2(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src, unsigned char *dest);
ISAL_HIP_DEPRECATED void gf_2vect_dot_prod_avx2(int len, int vlen, unsigned char *gftbls, unsigned char **src, unsigned char **dest);
ISAL_HIP_DEPRECATED void gf_2vect_mad_avx2(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src, unsigned char **dest);
ISAL_HIP_DEPRECATED void gf_3vect_dot_prod_avx2(int len, int vlen, unsigned char *gftbls, unsigned char **src, unsigned char **dest);
ISAL_HIP_DEPRECATED void gf_3vect_mad_avx2(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src, unsigned char **dest);
ISAL_HIP_DEPRECATED void gf_4vect_dot_prod_avx2(int len, int vlen, unsigned char *gftbls, unsigned char **src, unsigned char **dest);
ISAL_HIP_DEPRECATED void gf_4vect_mad_avx2(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src, unsigned char **dest);
ISAL_HIP_DEPRECATED void gf_5vect_dot_prod_avx2(int len, int vlen, unsigned char *gftbls, unsigned char **src, unsigned char **dest);
ISAL_HIP_DEPRECATED void gf_5vect_mad_avx2(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src, unsigned char **dest);
ISAL_HIP_DEPRECATED void gf_6vect_dot_prod_avx2(int len, int vlen, unsigned char *gftbls, unsigned char **src, unsigned char **dest);
ISAL_HIP_DEPRECATED void gf_6vect_mad_avx2(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src, unsigned char **dest);

/* ---- GF(2^8) helpers and matrices (host) -------------------------------- */

/* Replaces gf_mul (reference erasure_code.h:1064-1065, ec_base.c:50-63). */
unsigned char gf_mul(unsigned char a, unsigned char b);

/* Replaces gf_inv (reference erasure_code.h:1074-1075, ec_base.c:65-76); gf_inv(0) = 0. */
unsigned char gf_inv(unsigned char a);

/* m x k Vandermonde-style generator: identity on top, a[k+r][j] = (2^r)^j below.
 * Replaces gf_gen_rs_matrix (reference erasure_code.h:1101-1102, ec_base.c:78-96). */
void gf_gen_rs_matrix(unsigned char *a, int m, int k);

/* m x k Cauchy generator: identity on top, a[i][j] = 1/(i ^ j) below.
 * Replaces gf_gen_cauchy1_matrix (reference erasure_code.h:1117-1118, ec_base.c:98-114). */
void gf_gen_cauchy1_matrix(unsigned char *a, int m, int k);

/* Gauss-Jordan inverse of an n x n matrix; destroys in; returns 0, or -1 if
 * singular. Same pivot order as the reference so decode matrices match byte
 * for byte. Replaces gf_invert_matrix (reference erasure_code.h:1132-1133,
 * ec_base.c:116-170). */
int gf_invert_matrix(unsigned char *in, unsigned char *out, const int n);

#ifdef __cplusplus
}
#endif

#endif /* ISAL_HIP_ERASURE_CODE_H */
