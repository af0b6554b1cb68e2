/*
 * isal_hip_compat.c — deprecated per-ISA entry points of the reference ABI
 * (declared in include/erasure_code.h and include/gf_vect_mul.h, reference
 * erasure_code.h:249-1050, gf_vect_mul.h:46-97, exported by isa-l.def:5-48).
 * Each forwards to the engine's GPU entry point. Generated list; keep in sync
 * with exports.map.
 */
#define ISAL_HIP_DEPRECATED /* defining, not using */
#include "erasure_code.h"

void
ec_encode_data_sse(int len, int k, int rows, unsigned char *gftbls, unsigned char **data,
                  unsigned char **coding)
{
        ec_encode_data(len, k, rows, gftbls, data, coding);
}

void
ec_encode_data_update_sse(int len, int k, int rows, int vec_i, unsigned char *gftbls,
                         unsigned char *data, unsigned char **coding)
{
        ec_encode_data_update(len, k, rows, vec_i, gftbls, data, coding);
}

void
gf_vect_dot_prod_sse(int len, int vlen, unsigned char *gftbls, unsigned char **src,
                    unsigned char *dest)
{
        gf_vect_dot_prod(len, vlen, gftbls, src, dest);
}

void
gf_vect_mad_sse(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src,
               unsigned char *dest)
{
        gf_vect_mad(len, vec, vec_i, gftbls, src, dest);
}

void
gf_2vect_dot_prod_sse(int len, int vlen, unsigned char *gftbls, unsigned char **src,
                     unsigned char **dest)
{
        ec_encode_data(len, vlen, 2, gftbls, src, dest);
}

void
gf_2vect_mad_sse(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src,
                unsigned char **dest)
{
        ec_encode_data_update(len, vec, 2, vec_i, gftbls, src, dest);
}

void
gf_3vect_dot_prod_sse(int len, int vlen, unsigned char *gftbls, unsigned char **src,
                     unsigned char **dest)
{
        ec_encode_data(len, vlen, 3, gftbls, src, dest);
}

void
gf_3vect_mad_sse(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src,
                unsigned char **dest)
{
        ec_encode_data_update(len, vec, 3, vec_i, gftbls, src, dest);
}

void
gf_4vect_dot_prod_sse(int len, int vlen, unsigned char *gftbls, unsigned char **src,
                     unsigned char **dest)
{
        ec_encode_data(len, vlen, 4, gftbls, src, dest);
}

void
gf_4vect_mad_sse(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src,
                unsigned char **dest)
{
        ec_encode_data_update(len, vec, 4, vec_i, gftbls, src, dest);
}

void
gf_5vect_dot_prod_sse(int len, int vlen, unsigned char *gftbls, unsigned char **src,
                     unsigned char **dest)
{
        ec_encode_data(len, vlen, 5, gftbls, src, dest);
}

void
gf_5vect_mad_sse(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src,
                unsigned char **dest)
{
        ec_encode_data_update(len, vec, 5, vec_i, gftbls, src, dest);
}

void
gf_6vect_dot_prod_sse(int len, int vlen, unsigned char *gftbls, unsigned char **src,
                     unsigned char **dest)
{
        ec_encode_data(len, vlen, 6, gftbls, src, dest);
}

void
gf_6vect_mad_sse(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src,
                unsigned char **dest)
{
        ec_encode_data_update(len, vec, 6, vec_i, gftbls, src, dest);
}

void
ec_encode_data_avx(int len, int k, int rows, unsigned char *gftbls, unsigned char **data,
                  unsigned char **coding)
{
        ec_encode_data(len, k, rows, gftbls, data, coding);
}

void
ec_encode_data_update_avx(int len, int k, int rows, int vec_i, unsigned char *gftbls,
                         unsigned char *data, unsigned char **coding)
{
        ec_encode_data_update(len, k, rows, vec_i, gftbls, data, coding);
}

void
gf_vect_dot_prod_avx(int len, int vlen, unsigned char *gftbls, unsigned char **src,
                    unsigned char *dest)
{
        gf_vect_dot_prod(len, vlen, gftbls, src, dest);
}

void
gf_vect_mad_avx(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src,
               unsigned char *dest)
{
        gf_vect_mad(len, vec, vec_i, gftbls, src, dest);
}

void
gf_2vect_dot_prod_avx(int len, int vlen, unsigned char *gftbls, unsigned char **src,
                     unsigned char **dest)
{
        ec_encode_data(len, vlen, 2, gftbls, src, dest);
}

void
gf_2vect_mad_avx(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src,
                unsigned char **dest)
{
        ec_encode_data_update(len, vec, 2, vec_i, gftbls, src, dest);
}

void
gf_3vect_dot_prod_avx(int len, int vlen, unsigned char *gftbls, unsigned char **src,
                     unsigned char **dest)
{
        ec_encode_data(len, vlen, 3, gftbls, src, dest);
}

void
gf_3vect_mad_avx(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src,
                unsigned char **dest)
{
        ec_encode_data_update(len, vec, 3, vec_i, gftbls, src, dest);
}

void
gf_4vect_dot_prod_avx(int len, int vlen, unsigned char *gftbls, unsigned char **src,
                     unsigned char **dest)
{
        ec_encode_data(len, vlen, 4, gftbls, src, dest);
}

void
gf_4vect_mad_avx(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src,
                unsigned char **dest)
{
        ec_encode_data_update(len, vec, 4, vec_i, gftbls, src, dest);
}

void
gf_5vect_dot_prod_avx(int len, int vlen, unsigned char *gftbls, unsigned char **src,
                     unsigned char **dest)
{
        ec_encode_data(len, vlen, 5, gftbls, src, dest);
}

void
gf_5vect_mad_avx(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src,
                unsigned char **dest)
{
        ec_encode_data_update(len, vec, 5, vec_i, gftbls, src, dest);
}

void
gf_6vect_dot_prod_avx(int len, int vlen, unsigned char *gftbls, unsigned char **src,
                     unsigned char **dest)
{
        ec_encode_data(len, vlen, 6, gftbls, src, dest);
}

void
gf_6vect_mad_avx(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src,
                unsigned char **dest)
{
        ec_encode_data_update(len, vec, 6, vec_i, gftbls, src, dest);
}

void
ec_encode_data_avx2(int len, int k, int rows, unsigned char *gftbls, unsigned char **data,
                   unsigned char **coding)
{
        ec_encode_data(len, k, rows, gftbls, data, coding);
}

void
ec_encode_data_update_avx2(int len, int k, int rows, int vec_i, unsigned char *gftbls,
                          unsigned char *data, unsigned char **coding)
{
        ec_encode_data_update(len, k, rows, vec_i, gftbls, data, coding);
}

void
gf_vect_dot_prod_avx2(int len, int vlen, unsigned char *gftbls, unsigned char **src,
                     unsigned char *dest)
{
        gf_vect_dot_prod(len, vlen, gftbls, src, dest);
}

void
gf_vect_mad_avx2(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src,
                unsigned char *dest)
{
        gf_vect_mad(len, vec, vec_i, gftbls, src, dest);
}

void
gf_2vect_dot_prod_avx2(int len, int vlen, unsigned char *gftbls, unsigned char **src,
                      unsigned char **dest)
{
        ec_encode_data(len, vlen, 2, gftbls, src, dest);
}

void
gf_2vect_mad_avx2(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src,
                 unsigned char **dest)
{
        ec_encode_data_update(len, vec, 2, vec_i, gftbls, src, dest);
}

void
gf_3vect_dot_prod_avx2(int len, int vlen, unsigned char *gftbls, unsigned char **src,
                      unsigned char **dest)
{
        ec_encode_data(len, vlen, 3, gftbls, src, dest);
}

void
gf_3vect_mad_avx2(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src,
                 unsigned char **dest)
{
        ec_encode_data_update(len, vec, 3, vec_i, gftbls, src, dest);
}

void
gf_4vect_dot_prod_avx2(int len, int vlen, unsigned char *gftbls, unsigned char **src,
                      unsigned char **dest)
{
        ec_encode_data(len, vlen, 4, gftbls, src, dest);
}

void
gf_4vect_mad_avx2(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src,
                 unsigned char **dest)
{
        ec_encode_data_update(len, vec, 4, vec_i, gftbls, src, dest);
}

void
gf_5vect_dot_prod_avx2(int len, int vlen, unsigned char *gftbls, unsigned char **src,
                      unsigned char **dest)
{
        ec_encode_data(len, vlen, 5, gftbls, src, dest);
}

void
gf_5vect_mad_avx2(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src,
                 unsigned char **dest)
{
        ec_encode_data_update(len, vec, 5, vec_i, gftbls, src, dest);
}

void
gf_6vect_dot_prod_avx2(int len, int vlen, unsigned char *gftbls, unsigned char **src,
                      unsigned char **dest)
{
        ec_encode_data(len, vlen, 6, gftbls, src, dest);
}

void
gf_6vect_mad_avx2(int len, int vec, int vec_i, unsigned char *gftbls, unsigned char *src,
                 unsigned char **dest)
{
        ec_encode_data_update(len, vec, 6, vec_i, gftbls, src, dest);
}

int
gf_vect_mul_sse(int len, unsigned char *gftbl, void *src, void *dest)
{
        return gf_vect_mul(len, gftbl, src, dest);
}

int
gf_vect_mul_avx(int len, unsigned char *gftbl, void *src, void *dest)
{
        return gf_vect_mul(len, gftbl, src, dest);
}
