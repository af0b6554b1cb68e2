/*
 * CPU check of the fused / checksum-only CRC64 kernels' chain algebra
 * (crc64_kernels.hip): builds the engine's table set (crc64_host.c, included
 * so its bit-serial raw update is the reference), emulates every lane of one
 * workgroup block both ways the kernels chain —
 *   slicing path:  u1 = A(lo8 ^ b), b' = A'(hi8 ^ u1)   (last tile: A)
 *   field path:    b' = F'_u(chunk ^ b)                 (last tile: F_u)
 * — joins the lanes with Z^(16 * (255 - L)) and compares with the bit-serial
 * CRC of the whole block, for all eight flavours. Test infrastructure only.
 */
#include <stdio.h>
#include <stdlib.h>

#include "../../isa-l_amd/csrc/crc64_host.c"

static uint64_t
slice(const uint64_t *t, uint64_t x)
{
        uint64_t r = 0;
        int j;
        for (j = 0; j < 8; j++)
                r ^= t[j * 256 + ((x >> (8 * j)) & 0xff)];
        return r;
}

static uint64_t
fields(const uint64_t *t, const uint32_t w[4])
{
        uint64_t r = 0;
        int d, f;
        for (d = 0; d < 4; d++)
                for (f = 0; f < ISAL_HIP_CRC_FIELDS; f++)
                        r ^= t[(d * ISAL_HIP_CRC_FIELDS + f) * 32 +
                               ((w[d] >> field_lo(f)) & field_mask(f))];
        return r;
}

int
main(void)
{
        const int nt = 5, len = nt * ISAL_HIP_CRC_TILE;
        uint8_t *buf = malloc(len);
        uint64_t *tabs = malloc(sizeof(uint64_t) * ISAL_HIP_CRC64_TAB_ENTRIES);
        int variant, i, bad = 0;
        srand(7);
        for (i = 0; i < len; i++)
                buf[i] = (uint8_t) rand();
        for (variant = 0; variant < 8; variant++) {
                const uint64_t *A = tabs + ISAL_HIP_CRC64_SLICE_TAB, *A2 = A + 8 * 256;
                const uint64_t *F = tabs + ISAL_HIP_CRC64_PRE_TAB, *F2 = F + ISAL_HIP_CRC64_CHUNK_ENTRIES;
                uint64_t x_sl = 0, x_fd = 0, m[64];
                int L, t;
                isal_hip_crc64_tables(variant, len, nt, tabs);
                for (L = 0; L < 256; L++) {
                        uint64_t b = 0, c = 0;
                        for (t = 0; t < nt; t++) {
                                const uint8_t *p = buf + (size_t) t * ISAL_HIP_CRC_TILE + 16 * L;
                                uint32_t w[4];
                                uint64_t lo, hi, u1;
                                memcpy(w, p, 16);
                                lo = (uint64_t) w[0] | (uint64_t) w[1] << 32;
                                hi = (uint64_t) w[2] | (uint64_t) w[3] << 32;
                                u1 = slice(A, lo ^ b);
                                b = slice(t + 1 == nt ? A : A2, hi ^ u1);
                                w[0] ^= (uint32_t) c;
                                w[1] ^= (uint32_t) (c >> 32);
                                c = fields(t + 1 == nt ? F : F2, w);
                        }
                        isal_hip_crc64_zpow(variant, 16ULL * (255 - L), m);
                        x_sl ^= apply(m, pi_of(variant, b));
                        x_fd ^= apply(m, pi_of(variant, c));
                }
                {
                        const uint64_t want = raw_update(variant, 0, buf, len);
                        if (x_sl != want || x_fd != want) {
                                printf("variant %d: slicing %016llx fields %016llx want %016llx\n",
                                       variant, (unsigned long long) x_sl,
                                       (unsigned long long) x_fd, (unsigned long long) want);
                                bad = 1;
                        }
                }
        }
        printf(bad ? "FAIL\n" : "crc64 chain algebra ok (8 flavours, slicing and field paths)\n");
        free(buf);
        free(tabs);
        return bad;
}
