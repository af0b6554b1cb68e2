/*
 * CPU check of the CRC32C kernels' pre-shifted chain algebra
 * (crc_kernels.hip): byte-position tables P / P' of the fused kernel and
 * field tables F / F' of the checksum-only kernel (crc_host.c, included so
 * its byte table is the reference), every lane of one block chained
 *   b' = P'(w0 ^ b, w1, w2, w3)  (last tile: P)   and   b' = F'(...)  (last: F),
 * lanes joined with x^(8 * 16 * (255 - L)) and compared with the bytewise CRC
 * of the whole block. Test infrastructure only.
 */
#include <stdio.h>
#include <stdlib.h>

#include "../../isa-l_amd/csrc/crc_host.c"

static uint32_t
bytes_tab(const uint32_t *t, const uint32_t w[4])
{
        uint32_t r = 0;
        int p;
        for (p = 0; p < 16; p++)
                r ^= t[p * 256 + ((w[p / 4] >> (8 * (p % 4))) & 0xff)];
        return r;
}

static uint32_t
fields32(const uint32_t *t, const uint32_t w[4])
{
        uint32_t r = 0;
        int d, f;
        for (d = 0; d < 4; d++)
                for (f = 0; f < ISAL_HIP_CRC_FIELDS; f++)
                        r ^= t[(d * ISAL_HIP_CRC_FIELDS + f) * 32 +
                               ((w[d] >> field_lo(f)) & ((1u << field_bits(f)) - 1))];
        return r;
}

int
main(void)
{
        const int nt = 5, len = nt * ISAL_HIP_CRC_TILE;
        uint8_t *buf = malloc(len);
        uint32_t *tabs = malloc(4 * ISAL_HIP_CRC_TAB_DWORDS), *pos = malloc(4 * ISAL_HIP_CRC_B16_DWORDS),
                 *fpre = malloc(4 * ISAL_HIP_CRC_FPRE_DWORDS);
        uint32_t x_b = 0, x_f = 0, want = 0;
        int i, L, t;
        srand(11);
        for (i = 0; i < len; i++)
                buf[i] = (uint8_t) rand();
        isal_hip_crc32c_tables(tabs);
        isal_hip_crc32c_byte_tables(pos);
        isal_hip_crc32c_pre_tables(tabs, fpre);
        for (L = 0; L < 256; L++) {
                uint32_t b = 0, c = 0;
                for (t = 0; t < nt; t++) {
                        uint32_t w[4], v[4];
                        memcpy(w, buf + (size_t) t * ISAL_HIP_CRC_TILE + 16 * L, 16);
                        memcpy(v, w, 16);
                        w[0] ^= b;
                        b = bytes_tab(t + 1 == nt ? pos : pos + 16 * 256, w);
                        v[0] ^= c;
                        c = fields32(t + 1 == nt ? tabs + ISAL_HIP_CRC_CHUNK_TAB : fpre, v);
                }
                {
                        const uint32_t z = isal_hip_crc32c_xpow8n(16ULL * (255 - L));
                        x_b ^= isal_hip_crc32c_mulmod(b, z);
                        x_f ^= isal_hip_crc32c_mulmod(c, z);
                }
        }
        for (i = 0; i < len; i++)
                want = (want >> 8) ^ tabs[(want ^ buf[i]) & 0xff];
        if (x_b != want || x_f != want) {
                printf("byte path %08x field path %08x want %08x\nFAIL\n", x_b, x_f, want);
                return 1;
        }
        printf("crc32c chain algebra ok (byte-position and field paths)\n");
        free(buf);
        free(tabs);
        free(pos);
        free(fpre);
        return 0;
}
