/*
 * isal_hip_pipe.c — streaming erasure coding of HOST-resident stripes.
 *
 * The reference path starts and ends in host memory (shards arriving from a NIC
 * or a disk buffer). This pipeline overlaps the three legs on separate HIP
 * streams, stripe after stripe:
 *
 *   h2d stream : copy source j of stripe i into HBM slot (i % depth)
 *   compute    : as each source lands (event), fold it into the slot's
 *                device-resident parity with ec_encode_data_update semantics
 *                (mode UPDATE, reference ec_base.c:327-342), or encode the
 *                stripe once all k sources landed (mode ENCODE, ec_base.c:309-325)
 *   d2h stream : copy the finished parity rows back to the caller's buffers
 *
 * so the copy engines (one per direction) and the CUs work concurrently.
 * Host buffers should be pinned (hipHostMalloc / hipHostRegister / torch
 * pin_memory) for the copies to be asynchronous; pageable buffers still give
 * correct results, without overlap.
 */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "isal_hip.h"
#include "isal_hip_internal.h"

struct isal_hip_pipe {
        int len, k, rows, depth, mode, device;
        hipStream_t h2d, comp, d2h;
        unsigned char *d_buf; /* depth x (k + rows) x len */
        uint64_t *d_ptrs;     /* depth x (k + rows) */
        uint32_t *d_tbl;
        uint64_t *d_ldsx;      /* LDS product tables of the wide passes (NULL: not used) */
        isal_hip_encmask em;   /* 0/1 rows and columns of the coefficients */
        hipEvent_t *src_ready; /* depth x k */
        hipEvent_t *parity_done, *slot_free;
        int *slot_used;
        long long submitted;
};

#define PIPE_CK(call)                                                                              \
        do {                                                                                       \
                if ((call) != hipSuccess)                                                          \
                        return ISAL_HIP_EHIP;                                                      \
        } while (0)

int
isal_hip_pipe_create(isal_hip_pipe **out, int len, int k, int rows, const unsigned char *gftbls,
                     int depth, int mode)
{
        isal_hip_pipe *p;
        size_t nptr, i, ntbl;
        uint64_t *h_ptrs;
        uint32_t *h_tbl;
        int rc = ISAL_HIP_OK;

        if (!out || len <= 0 || k <= 0 || rows <= 0 || depth <= 0 || !gftbls ||
            (mode != ISAL_HIP_PIPE_UPDATE && mode != ISAL_HIP_PIPE_ENCODE))
                return ISAL_HIP_EINVAL;
        *out = NULL;
        /* More than 4 stripes in flight only slows the copies: with H2D and D2H
         * both streaming, 6-8 queued stripes drop H2D from ~49 to 31-35 GB/s
         * (plain torch copies show the same, tools/pcie_probe.py,
         * profiles/r02/r02_pcie_probe.txt), so extra slots are not allocated. */
        if (depth > ISAL_HIP_PIPE_MAX_DEPTH)
                depth = ISAL_HIP_PIPE_MAX_DEPTH;
        p = (isal_hip_pipe *) calloc(1, sizeof(*p));
        if (!p)
                return ISAL_HIP_ENOMEM;
        p->len = len;
        p->k = k;
        p->rows = rows;
        p->depth = depth;
        p->mode = mode;
        nptr = (size_t) depth * (size_t) (k + rows);
        p->src_ready = (hipEvent_t *) calloc((size_t) depth * k, sizeof(hipEvent_t));
        p->parity_done = (hipEvent_t *) calloc((size_t) depth, sizeof(hipEvent_t));
        p->slot_free = (hipEvent_t *) calloc((size_t) depth, sizeof(hipEvent_t));
        p->slot_used = (int *) calloc((size_t) depth, sizeof(int));
        h_ptrs = (uint64_t *) malloc(nptr * 8);
        ntbl = isal_hip_tables_dwords(k, rows);
        h_tbl = (uint32_t *) malloc(ntbl * 4 + 4);
        if (!p->src_ready || !p->parity_done || !p->slot_free || !p->slot_used || !h_ptrs || !h_tbl) {
                free(h_ptrs);
                free(h_tbl);
                isal_hip_pipe_destroy(p);
                return ISAL_HIP_ENOMEM;
        }
        if (hipGetDevice(&p->device) != hipSuccess ||
            hipStreamCreateWithFlags(&p->h2d, hipStreamNonBlocking) != hipSuccess ||
            hipStreamCreateWithFlags(&p->comp, hipStreamNonBlocking) != hipSuccess ||
            hipStreamCreateWithFlags(&p->d2h, hipStreamNonBlocking) != hipSuccess ||
            hipMalloc((void **) &p->d_buf, nptr * (size_t) len) != hipSuccess ||
            hipMalloc((void **) &p->d_ptrs, nptr * 8) != hipSuccess ||
            hipMalloc((void **) &p->d_tbl, ntbl * 4 + 4) != hipSuccess)
                rc = ISAL_HIP_EHIP;
        for (i = 0; rc == ISAL_HIP_OK && i < (size_t) depth * k; i++)
                if (hipEventCreateWithFlags(&p->src_ready[i], hipEventDisableTiming) != hipSuccess)
                        rc = ISAL_HIP_EHIP;
        for (i = 0; rc == ISAL_HIP_OK && i < (size_t) depth; i++)
                if (hipEventCreateWithFlags(&p->parity_done[i], hipEventDisableTiming) != hipSuccess ||
                    hipEventCreateWithFlags(&p->slot_free[i], hipEventDisableTiming) != hipSuccess)
                        rc = ISAL_HIP_EHIP;
        if (rc == ISAL_HIP_OK) {
                /* slot s holds sources then parity, each `len` bytes (256-B multiple
                 * offsets keep every shard 16-byte aligned when len % 16 == 0) */
                for (i = 0; i < nptr; i++)
                        h_ptrs[i] = (uint64_t) (uintptr_t) (p->d_buf + i * (size_t) len);
                isal_hip_build_tables(k, rows, gftbls, h_tbl);
                isal_hip_enc_masks(k, rows, gftbls, &p->em);
                if (hipMemcpy(p->d_ptrs, h_ptrs, nptr * 8, hipMemcpyHostToDevice) != hipSuccess ||
                    hipMemcpy(p->d_tbl, h_tbl, ntbl * 4, hipMemcpyHostToDevice) != hipSuccess)
                        rc = ISAL_HIP_EHIP;
        }
        if (rc == ISAL_HIP_OK && mode == ISAL_HIP_PIPE_ENCODE && k <= 64 && rows >= 4) {
                /* the wide passes' LDS product tables (ec_encode_ldsx) */
                const size_t nw = isal_hip_ldsx_words(k, rows);
                uint64_t *hx = (uint64_t *) malloc(nw * 8);
                if (!hx || hipMalloc((void **) &p->d_ldsx, nw * 8) != hipSuccess)
                        rc = hx ? ISAL_HIP_EHIP : ISAL_HIP_ENOMEM;
                if (rc == ISAL_HIP_OK) {
                        isal_hip_build_ldsx_tables(k, rows, gftbls, hx);
                        if (hipMemcpy(p->d_ldsx, hx, nw * 8, hipMemcpyHostToDevice) != hipSuccess)
                                rc = ISAL_HIP_EHIP;
                        p->em.ldsx = p->d_ldsx;
                }
                free(hx);
        }
        free(h_ptrs);
        free(h_tbl);
        if (rc != ISAL_HIP_OK) {
                isal_hip_pipe_destroy(p);
                return rc;
        }
        *out = p;
        return ISAL_HIP_OK;
}

static int
pipe_submit_impl(isal_hip_pipe *p, unsigned char *const *data, unsigned char *const *coding)
{
        int slot, j, l, stride, vec16;
        unsigned char *base;
        const uint64_t *ptrs;
        if (!p || !data || !coding)
                return ISAL_HIP_EINVAL;
        slot = (int) (p->submitted % p->depth);
        stride = p->k + p->rows;
        base = p->d_buf + (size_t) slot * stride * (size_t) p->len;
        ptrs = p->d_ptrs + (size_t) slot * stride;
        vec16 = (p->len % 16) == 0;
        /* back-pressure: the slot is reusable once its previous parity left HBM */
        if (p->slot_used[slot])
                PIPE_CK(hipEventSynchronize(p->slot_free[slot]));
        if (p->mode == ISAL_HIP_PIPE_UPDATE)
                PIPE_CK(hipMemsetAsync(base + (size_t) p->k * p->len, 0, (size_t) p->rows * p->len,
                                       p->comp));
        /* Host shards that are adjacent in memory (a stripe laid out as one
         * k x len block, the common NIC/disk-buffer case) move as ONE copy:
         * fewer, larger DMA transfers reach a higher PCIe rate. */
        for (j = 0; j < p->k;) {
                int run = 1, v;
                hipEvent_t e;
                while (j + run < p->k && data[j + run] == data[j] + (size_t) run * p->len)
                        run++;
                e = p->src_ready[(size_t) slot * p->k + j];
                PIPE_CK(hipMemcpyAsync(base + (size_t) j * p->len, data[j], (size_t) run * p->len,
                                       hipMemcpyHostToDevice, p->h2d));
                PIPE_CK(hipEventRecord(e, p->h2d));
                if (p->mode == ISAL_HIP_PIPE_UPDATE) {
                        PIPE_CK(hipStreamWaitEvent(p->comp, e, 0));
                        for (v = j; v < j + run; v++)
                                if (isal_hip_launch_update(ptrs, stride, v, p->k, p->d_tbl, p->len,
                                                           p->k, p->rows, v, 1, vec16, p->comp))
                                        return ISAL_HIP_EHIP;
                } else {
                        PIPE_CK(hipStreamWaitEvent(p->comp, e, 0));
                }
                j += run;
        }
        if (p->mode == ISAL_HIP_PIPE_ENCODE) {
                if (isal_hip_launch_encode(ptrs, stride, 0, p->k, p->d_tbl, p->len, p->k, p->rows, 1,
                                           vec16, &p->em, p->comp))
                        return ISAL_HIP_EHIP;
        }
        PIPE_CK(hipEventRecord(p->parity_done[slot], p->comp));
        PIPE_CK(hipStreamWaitEvent(p->d2h, p->parity_done[slot], 0));
        for (l = 0; l < p->rows;) {
                int run = 1;
                while (l + run < p->rows && coding[l + run] == coding[l] + (size_t) run * p->len)
                        run++;
                PIPE_CK(hipMemcpyAsync(coding[l], base + (size_t) (p->k + l) * p->len,
                                       (size_t) run * p->len, hipMemcpyDeviceToHost, p->d2h));
                l += run;
        }
        PIPE_CK(hipEventRecord(p->slot_free[slot], p->d2h));
        p->slot_used[slot] = 1;
        p->submitted++;
        return ISAL_HIP_OK;
}

static int
pipe_flush_impl(isal_hip_pipe *p)
{
        if (!p)
                return ISAL_HIP_EINVAL;
        PIPE_CK(hipStreamSynchronize(p->h2d));
        PIPE_CK(hipStreamSynchronize(p->comp));
        PIPE_CK(hipStreamSynchronize(p->d2h));
        return ISAL_HIP_OK;
}

int
isal_hip_pipe_destroy(isal_hip_pipe *p)
{
        size_t i;
        if (!p)
                return ISAL_HIP_OK;
        if (p->h2d)
                (void) isal_hip_pipe_flush(p);
        if (p->src_ready)
                for (i = 0; i < (size_t) p->depth * p->k; i++)
                        if (p->src_ready[i])
                                (void) hipEventDestroy(p->src_ready[i]);
        for (i = 0; p->parity_done && i < (size_t) p->depth; i++) {
                if (p->parity_done[i])
                        (void) hipEventDestroy(p->parity_done[i]);
                if (p->slot_free && p->slot_free[i])
                        (void) hipEventDestroy(p->slot_free[i]);
        }
        if (p->h2d)
                (void) hipStreamDestroy(p->h2d);
        if (p->comp)
                (void) hipStreamDestroy(p->comp);
        if (p->d2h)
                (void) hipStreamDestroy(p->d2h);
        if (p->d_buf)
                (void) hipFree(p->d_buf);
        if (p->d_ptrs)
                (void) hipFree(p->d_ptrs);
        if (p->d_tbl)
                (void) hipFree(p->d_tbl);
        if (p->d_ldsx)
                (void) hipFree(p->d_ldsx);
        free(p->src_ready);
        free(p->parity_done);
        free(p->slot_free);
        free(p->slot_used);
        free(p);
        return ISAL_HIP_OK;
}

/* the pipeline's calls run on its device (its streams and buffers are there) */
int
isal_hip_pipe_submit(isal_hip_pipe *p, unsigned char *const *data, unsigned char *const *coding)
{
        int prev, r;
        if (!p)
                return ISAL_HIP_EINVAL;
        if ((prev = isal_hip_dev_enter(p->device)) == -2)
                return ISAL_HIP_EHIP;
        r = pipe_submit_impl(p, data, coding);
        isal_hip_dev_leave(prev);
        return r;
}

/* the pipeline's calls run on its device (its streams and buffers are there) */
int
isal_hip_pipe_flush(isal_hip_pipe *p)
{
        int prev, r;
        if (!p)
                return ISAL_HIP_EINVAL;
        if ((prev = isal_hip_dev_enter(p->device)) == -2)
                return ISAL_HIP_EHIP;
        r = pipe_flush_impl(p);
        isal_hip_dev_leave(prev);
        return r;
}
