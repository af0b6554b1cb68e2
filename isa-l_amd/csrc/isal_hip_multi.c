/*
 * isal_hip_multi.c — one process driving several GPUs (include/isal_hip.h
 * "multi-device").
 *
 * Stripes are independent: a call's nstripes are split into
 * contiguous ranges [d*S/G, (d+1)*S/G) (isal_hip_multi_partition), and GPU d
 * encodes its range from host memory through its own streaming pipeline
 * (isal_hip_pipe.c: H2D / encode / D2H overlapped on three streams), driven by
 * its own host thread. Nothing crosses between GPUs — no collective is needed
 * on the data path, and each GPU uses its own PCIe link, so the host-memory
 * rate adds up across devices. This is the C caller's multi-GPU entry (the
 * reference's callers are C storage stacks, e.g. examples/ec/ec_simple_example.c);
 * the benchmark's torchrun path partitions stripes with the same function.
 */
#include <hip/hip_runtime_api.h>
#include <pthread.h>
#include <stdlib.h>

#include "isal_hip.h"
#include "isal_hip_internal.h"

struct isal_hip_multi {
        int ndev, len, k, rows;
        isal_hip_pipe **pipe; /* one per device, created on that device */
};

void
isal_hip_multi_partition(long long nstripes, int ndev, int dev, long long *first, long long *count)
{
        long long lo, hi;
        if (nstripes < 0 || ndev <= 0 || dev < 0 || dev >= ndev) {
                *first = *count = 0;
                return;
        }
        /* balanced and contiguous: sizes differ by at most one stripe */
        lo = (long long) ((__int128) nstripes * dev / ndev);
        hi = (long long) ((__int128) nstripes * (dev + 1) / ndev);
        *first = lo;
        *count = hi - lo;
}

int
isal_hip_multi_create(isal_hip_multi **out, int ndev, int len, int k, int rows,
                      const unsigned char *gftbls, int depth)
{
        isal_hip_multi *m;
        int n = 0, cur = 0, d, rc = ISAL_HIP_OK;
        if (!out || len <= 0 || k <= 0 || rows <= 0 || !gftbls || depth <= 0 || ndev < 0)
                return ISAL_HIP_EINVAL;
        *out = NULL;
        if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
                (void) hipGetLastError();
                return ISAL_HIP_EHIP;
        }
        if (ndev == 0)
                ndev = n;
        if (ndev > n)
                return ISAL_HIP_EINVAL;
        m = (isal_hip_multi *) calloc(1, sizeof(*m));
        if (!m || !(m->pipe = (isal_hip_pipe **) calloc((size_t) ndev, sizeof(*m->pipe)))) {
                free(m);
                return ISAL_HIP_ENOMEM;
        }
        m->ndev = ndev;
        m->len = len;
        m->k = k;
        m->rows = rows;
        if (hipGetDevice(&cur) != hipSuccess)
                cur = 0;
        for (d = 0; d < ndev && rc == ISAL_HIP_OK; d++) {
                if (hipSetDevice(d) != hipSuccess)
                        rc = ISAL_HIP_EHIP;
                else
                        rc = isal_hip_pipe_create(&m->pipe[d], len, k, rows, gftbls, depth,
                                                  ISAL_HIP_PIPE_ENCODE);
        }
        (void) hipSetDevice(cur);
        if (rc != ISAL_HIP_OK) {
                isal_hip_multi_destroy(m);
                return rc;
        }
        *out = m;
        return ISAL_HIP_OK;
}

int
isal_hip_multi_ndev(const isal_hip_multi *m)
{
        return m ? m->ndev : 0;
}

typedef struct {
        isal_hip_multi *m;
        int dev;
        long long first, count;
        unsigned char *const *data, *const *coding;
        int rc, started;
} job_t;

static void *
worker(void *arg)
{
        job_t *j = (job_t *) arg;
        const isal_hip_multi *m = j->m;
        long long s;
        int rc = ISAL_HIP_OK, frc;
        if (hipSetDevice(j->dev) != hipSuccess) {
                j->rc = ISAL_HIP_EHIP;
                return NULL;
        }
        for (s = j->first; s < j->first + j->count && rc == ISAL_HIP_OK; s++)
                rc = isal_hip_pipe_submit(m->pipe[j->dev], j->data + s * m->k,
                                          j->coding + s * m->rows);
        frc = isal_hip_pipe_flush(m->pipe[j->dev]); /* always drain what was queued */
        j->rc = rc != ISAL_HIP_OK ? rc : frc;
        return NULL;
}

int
isal_hip_multi_encode(isal_hip_multi *m, long long nstripes, unsigned char *const *data,
                      unsigned char *const *coding)
{
        job_t *jobs;
        pthread_t *th;
        int d, rc = ISAL_HIP_OK;
        if (!m || nstripes < 0 || (nstripes && (!data || !coding)))
                return ISAL_HIP_EINVAL;
        if (nstripes == 0)
                return ISAL_HIP_OK;
        jobs = (job_t *) calloc((size_t) m->ndev, sizeof(*jobs));
        th = (pthread_t *) calloc((size_t) m->ndev, sizeof(*th));
        if (!jobs || !th) {
                free(jobs);
                free(th);
                return ISAL_HIP_ENOMEM;
        }
        for (d = 0; d < m->ndev; d++) {
                jobs[d].m = m;
                jobs[d].dev = d;
                jobs[d].data = data;
                jobs[d].coding = coding;
                isal_hip_multi_partition(nstripes, m->ndev, d, &jobs[d].first, &jobs[d].count);
                jobs[d].started = pthread_create(&th[d], NULL, worker, &jobs[d]) == 0;
                if (!jobs[d].started)
                        jobs[d].rc = ISAL_HIP_ENOMEM;
        }
        for (d = 0; d < m->ndev; d++) {
                if (jobs[d].started)
                        pthread_join(th[d], NULL);
                if (jobs[d].rc != ISAL_HIP_OK && rc == ISAL_HIP_OK)
                        rc = jobs[d].rc;
        }
        free(jobs);
        free(th);
        return rc;
}

int
isal_hip_multi_destroy(isal_hip_multi *m)
{
        int d, cur = 0;
        if (!m)
                return ISAL_HIP_OK;
        if (hipGetDevice(&cur) != hipSuccess)
                cur = 0;
        for (d = 0; m->pipe && d < m->ndev; d++)
                if (m->pipe[d]) {
                        (void) hipSetDevice(d);
                        (void) isal_hip_pipe_destroy(m->pipe[d]);
                }
        (void) hipSetDevice(cur);
        free(m->pipe);
        free(m);
        return ISAL_HIP_OK;
}
