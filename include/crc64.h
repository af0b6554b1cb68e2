/*
 * crc64.h — the CRC64 entry points of the MI355X engine.
 *
 * Same C signatures and semantics as the reference include/crc64.h:54-163
 * and its *_base twins (:190-339; isa-l.def:90-122): ECMA-182, ISO 3309,
 * Jones and Rocksoft polynomials, reflected (refl) or normal (norm) bit
 * order; the register starts at ~init_crc and is inverted on return
 * (crc/crc64_base.c:569-670), so crc64_x(crc64_x(init, A), B) ==
 * crc64_x(init, A || B) and crc64_x(init, buf, 0) == init.
 *
 * Routing: a buffer in device memory (hipMalloc / managed) is checksummed by
 * the GPU CRC64 kernels on the device that holds it (in pieces of at most
 * 1 GiB); a host buffer by the engine's CPU route (slicing-by-8). The
 * checksums of whole stripes, fused with the encode, are isal_hip.h's
 * isal_hip_batch_crc64 / isal_hip_batch_encode_crc64.
 */
#ifndef ISAL_HIP_CRC64_H
#define ISAL_HIP_CRC64_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

uint64_t crc64_ecma_refl(uint64_t init_crc, const unsigned char *buf, uint64_t len);
uint64_t crc64_ecma_norm(uint64_t init_crc, const unsigned char *buf, uint64_t len);
uint64_t crc64_iso_refl(uint64_t init_crc, const unsigned char *buf, uint64_t len);
uint64_t crc64_iso_norm(uint64_t init_crc, const unsigned char *buf, uint64_t len);
uint64_t crc64_jones_refl(uint64_t init_crc, const unsigned char *buf, uint64_t len);
uint64_t crc64_jones_norm(uint64_t init_crc, const unsigned char *buf, uint64_t len);
uint64_t crc64_rocksoft_refl(uint64_t init_crc, const unsigned char *buf, uint64_t len);
uint64_t crc64_rocksoft_norm(uint64_t init_crc, const unsigned char *buf, uint64_t len);

uint64_t crc64_ecma_refl_base(uint64_t init_crc, const unsigned char *buf, uint64_t len);
uint64_t crc64_ecma_norm_base(uint64_t init_crc, const unsigned char *buf, uint64_t len);
uint64_t crc64_iso_refl_base(uint64_t init_crc, const unsigned char *buf, uint64_t len);
uint64_t crc64_iso_norm_base(uint64_t init_crc, const unsigned char *buf, uint64_t len);
uint64_t crc64_jones_refl_base(uint64_t init_crc, const unsigned char *buf, uint64_t len);
uint64_t crc64_jones_norm_base(uint64_t init_crc, const unsigned char *buf, uint64_t len);
uint64_t crc64_rocksoft_refl_base(uint64_t init_crc, const unsigned char *buf, uint64_t len);
uint64_t crc64_rocksoft_norm_base(uint64_t init_crc, const unsigned char *buf, uint64_t len);

#ifdef __cplusplus
}
#endif

#endif /* ISAL_HIP_CRC64_H */
