/*
 * raid.h — RAID-5 XOR and RAID-6 P+Q parity of the MI355X engine.
 *
 * Same C signatures as the reference include/raid.h (xor_gen :65, xor_check
 * :82, pq_gen :102, pq_check :121, per-ISA names :144-262, *_base :280-324).
 * These are Reed-Solomon special cases and run on the same GPU kernels as
 * ec_encode_data: P = XOR of the sources (one all-ones coefficient row),
 * Q = sum_j 2^j * D_j over GF(2^8)/0x11d (the reference's Horner loop,
 * raid_base.c:44-68). array[] holds the sources followed by the parity
 * vector(s); pointers may be host or device memory.
 *
 * Return values (0 = pass) follow the reference:
 *   xor_gen / xor_gen_base    1 if vects < 3
 *   pq_gen                    1 if vects < 4 or len % 32 (the dispatched x86
 *                             kernels' contract, pq_gen_avx512.asm:127-132)
 *   pq_gen_base               1 if vects < 4; only the first len & ~7 bytes
 *                             are produced (raid_base.c:44-48)
 *   xor_check(_base)          1 if vects < 2 or the XOR of all vectors != 0
 *   pq_check(_base)           1 if vects < 4; on mismatch at byte i:
 *                             i | 1 (P wrong) or i | 2 (Q wrong),
 *                             raid_base.c:96-99
 */
#ifndef ISAL_HIP_RAID_H
#define ISAL_HIP_RAID_H

#ifdef __cplusplus
extern "C" {
#endif

#ifndef ISAL_HIP_DEPRECATED
#define ISAL_HIP_DEPRECATED __attribute__((deprecated))
#endif

/* XOR parity of array[0..vects-2] into array[vects-1]. Replaces xor_gen (reference raid.h:65). */
int xor_gen(int vects, int len, void **array);

/* 0 if array[0..vects-1] XOR to zero. Replaces xor_check (reference raid.h:82). */
int xor_check(int vects, int len, void **array);

/* P, Q of array[0..vects-3] into array[vects-2], array[vects-1]. Replaces pq_gen (reference raid.h:102). */
int pq_gen(int vects, int len, void **array);

/* 0 if P and Q match the sources. Replaces pq_check (reference raid.h:121). */
int pq_check(int vects, int len, void **array);

/* Baseline twins (reference raid.h:280-324, raid_base.c). */
int pq_gen_base(int vects, int len, void **array);
int xor_gen_base(int vects, int len, void **array);
int xor_check_base(int vects, int len, void **array);
int pq_check_base(int vects, int len, void **array);

/* Deprecated per-ISA names (reference raid.h:144-262, isa-l.def:58-64). */
ISAL_HIP_DEPRECATED int xor_gen_sse(int vects, int len, void **array);
ISAL_HIP_DEPRECATED int xor_gen_avx(int vects, int len, void **array);
ISAL_HIP_DEPRECATED int xor_check_sse(int vects, int len, void **array);
ISAL_HIP_DEPRECATED int pq_gen_sse(int vects, int len, void **array);
ISAL_HIP_DEPRECATED int pq_gen_avx(int vects, int len, void **array);
ISAL_HIP_DEPRECATED int pq_gen_avx2(int vects, int len, void **array);
ISAL_HIP_DEPRECATED int pq_check_sse(int vects, int len, void **array);

#ifdef __cplusplus
}
#endif

#endif /* ISAL_HIP_RAID_H */
