/*
 * gf_vect_mul.h — GF(2^8) vector-times-constant API of the MI355X engine.
 *
 * Same C signatures as the reference include/gf_vect_mul.h. Every data-path
 * function runs on the GPU (libisal_hip.so); pointers may be host or device
 * memory, and every call is synchronous, exactly like the reference.
 */
#ifndef ISAL_HIP_GF_VECT_MUL_H
#define ISAL_HIP_GF_VECT_MUL_H

#include "isal_api.h"

#ifdef __cplusplus
extern "C" {
#endif

/*
 * Expand constant c into the 32-byte table {c*0x00..c*0x0f, c*0x00,c*0x10..c*0xf0}.
 * Replaces gf_vect_mul_init (reference gf_vect_mul.h:112-113). The engine always
 * emits the portable ("base") table format, so tables interoperate with every
 * *_base entry point.
 */
void gf_vect_mul_init(unsigned char c, unsigned char *gftbl);

/* Replaces gf_vect_mul_init_base (reference gf_vect_mul.h:125-126, ec_base.c:175-280). */
void gf_vect_mul_init_base(unsigned char c, unsigned char *gftbl);

/*
 * dest[i] = c * src[i] for i < len, with c = gftbl[1].
 * Returns 0 on success, non-zero (and touches nothing) if len is not a
 * multiple of 32 — the reference's only error contract for this function.
 * Replaces gf_vect_mul (reference gf_vect_mul.h:148-149).
 */
int gf_vect_mul(int len, unsigned char *gftbl, void *src, void *dest);

/* Deprecated per-ISA names (reference gf_vect_mul.h:46-97, isa-l.def:11-12):
 * aliases of gf_vect_mul. */
#ifndef ISAL_HIP_DEPRECATED
#define ISAL_HIP_DEPRECATED __attribute__((deprecated))
#endif
ISAL_HIP_DEPRECATED int gf_vect_mul_sse(int len, unsigned char *gftbl, void *src, void *dest);
ISAL_HIP_DEPRECATED int gf_vect_mul_avx(int len, unsigned char *gftbl, void *src, void *dest);

/* Replaces gf_vect_mul_base (reference gf_vect_mul.h:170-171, ec_base.c:344-358). */
int gf_vect_mul_base(int len, unsigned char *gftbl, unsigned char *src, unsigned char *dest);

#ifdef __cplusplus
}
#endif

#endif /* ISAL_HIP_GF_VECT_MUL_H */
