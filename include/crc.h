/*
 * crc.h — the iSCSI CRC (CRC32C) entry points of the MI355X engine.
 *
 * Same C signatures and semantics as the reference include/crc.h:136-150
 * (crc32_iscsi, crc32_iscsi_base; isa-l.def:75,78): reflected Castagnoli
 * polynomial 0x1EDC6F41, the register starts at init_crc, no final inversion
 * (crc/crc_base.c:205-219); len <= 0 returns init_crc. The reference's other
 * CRC32/CRC16 functions are outside this engine's scope.
 *
 * Routing: a buffer in device memory (hipMalloc / managed) is checksummed by
 * the GPU kernels on the device that holds it; a host buffer by the engine's
 * CPU route (SSE4.2 crc32, else slicing-by-8). The same checksums of whole
 * stripes, fused with the encode, are isal_hip.h's isal_hip_batch_*crc*.
 */
#ifndef ISAL_HIP_CRC_H
#define ISAL_HIP_CRC_H

#ifdef __cplusplus
extern "C" {
#endif

unsigned int crc32_iscsi(unsigned char *buffer, int len, unsigned int init_crc);
unsigned int crc32_iscsi_base(unsigned char *buffer, int len, unsigned int crc_init);

#ifdef __cplusplus
}
#endif

#endif /* ISAL_HIP_CRC_H */
