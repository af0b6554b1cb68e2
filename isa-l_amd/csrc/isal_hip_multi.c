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
 *
 * NUMA: on a two-socket host half of the GPUs hang off each socket. Each
 * device's worker thread is pinned to the CPUs of the NUMA node its PCIe
 * root sits on (sysfs: bus/pci/devices/<bus id>/numa_node and
 * devices/system/node/node<N>/cpulist, intersected with the process's own
 * affinity), so the thread that drives a GPU's copies runs next to it.
 * ISAL_HIP_SYSFS_ROOT points the lookup at another tree (tests).
 *
 * Threading: one handle serves one isal_hip_multi_encode at a time; a second
 * thread calling it on the same handle waits (handle mutex).
 */
#define _GNU_SOURCE
#include <ctype.h>
#include <hip/hip_runtime_api.h>
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "isal_hip.h"
#include "isal_hip_internal.h"

struct isal_hip_multi {
        int ndev, len, k, rows;
        isal_hip_pipe **pipe; /* one per device, created on that device */
        int *node;            /* NUMA node of each device, -1 unknown */
        cpu_set_t *cpus;      /* CPUs its worker runs on (empty: not pinned) */
        pthread_mutex_t lock; /* one encode per handle at a time */
};

/* ---- NUMA placement (pure host code: sysfs files only) ------------------- */

static const char *
sysfs_root(void)
{
        const char *r = getenv("ISAL_HIP_SYSFS_ROOT");
        return r && *r ? r : "/sys";
}

int
isal_hip_pci_numa_node(const char *root, const char *pci_bus_id)
{
        char path[512], id[64];
        size_t i;
        int node = -1;
        FILE *f;
        if (!pci_bus_id || strlen(pci_bus_id) >= sizeof(id))
                return -1;
        for (i = 0; pci_bus_id[i]; i++)
                id[i] = (char) tolower((unsigned char) pci_bus_id[i]);
        id[i] = 0;
        snprintf(path, sizeof(path), "%s/bus/pci/devices/%s/numa_node", root ? root : sysfs_root(), id);
        if (!(f = fopen(path, "r")))
                return -1;
        if (fscanf(f, "%d", &node) != 1)
                node = -1;
        fclose(f);
        return node < 0 ? -1 : node;
}

int
isal_hip_numa_node_cpus(const char *root, int node, int *cpus, int max)
{
        char path[512], buf[8192], *p;
        int n = 0;
        FILE *f;
        if (node < 0 || !cpus || max < 0)
                return -1;
        snprintf(path, sizeof(path), "%s/devices/system/node/node%d/cpulist", root ? root : sysfs_root(),
                 node);
        if (!(f = fopen(path, "r")))
                return -1;
        p = fgets(buf, sizeof(buf), f);
        fclose(f);
        if (!p)
                return -1;
        /* "0-63,128-191"; CPU numbers at or above CPU_SETSIZE (or a total
         * beyond it) mark the file malformed: every range is bounded, so a
         * hostile tree (ISAL_HIP_SYSFS_ROOT) cannot make this loop run away */
        while (*p && *p != '\n') {
                char *end;
                long lo = strtol(p, &end, 10), hi;
                if (end == p || lo < 0 || lo >= CPU_SETSIZE)
                        return -1;
                hi = lo;
                p = end;
                if (*p == '-') {
                        hi = strtol(p + 1, &end, 10);
                        if (end == p + 1 || hi < lo || hi >= CPU_SETSIZE)
                                return -1;
                        p = end;
                }
                if (n > CPU_SETSIZE - (int) (hi - lo + 1))
                        return -1;
                for (; lo <= hi; lo++) {
                        if (n < max)
                                cpus[n] = (int) lo;
                        n++;
                }
                if (*p == ',')
                        p++;
                else if (*p && *p != '\n')
                        return -1;
        }
        return n;
}

/* The CPUs a worker for `node` may use: the node's CPUs this process is
 * allowed to run on. Empty when unknown or when the intersection is empty. */
static void
node_cpuset(int node, cpu_set_t *out)
{
        cpu_set_t allowed;
        int *cpus, n, i;
        CPU_ZERO(out);
        if (node < 0 || sched_getaffinity(0, sizeof(allowed), &allowed) != 0)
                return;
        cpus = (int *) malloc(sizeof(int) * CPU_SETSIZE);
        if (!cpus)
                return;
        n = isal_hip_numa_node_cpus(NULL, node, cpus, CPU_SETSIZE);
        for (i = 0; i < n && i < CPU_SETSIZE; i++)
                if (cpus[i] < CPU_SETSIZE && CPU_ISSET(cpus[i], &allowed))
                        CPU_SET(cpus[i], out);
        free(cpus);
}

int
isal_hip_multi_numa_node(const isal_hip_multi *m, int dev)
{
        return m && dev >= 0 && dev < m->ndev ? m->node[dev] : -1;
}

int
isal_hip_multi_worker_cpus(const isal_hip_multi *m, int dev)
{
        return m && dev >= 0 && dev < m->ndev ? CPU_COUNT(&m->cpus[dev]) : -1;
}

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
        if (!m || !(m->pipe = (isal_hip_pipe **) calloc((size_t) ndev, sizeof(*m->pipe))) ||
            !(m->node = (int *) calloc((size_t) ndev, sizeof(int))) ||
            !(m->cpus = (cpu_set_t *) calloc((size_t) ndev, sizeof(cpu_set_t)))) {
                if (m) {
                        free(m->pipe);
                        free(m->node);
                }
                free(m);
                return ISAL_HIP_ENOMEM;
        }
        pthread_mutex_init(&m->lock, NULL);
        m->ndev = ndev;
        m->len = len;
        m->k = k;
        m->rows = rows;
        if (hipGetDevice(&cur) != hipSuccess)
                cur = 0;
        for (d = 0; d < ndev; d++) {
                char bus[64];
                m->node[d] = hipDeviceGetPCIBusId(bus, (int) sizeof(bus), d) == hipSuccess
                                     ? isal_hip_pci_numa_node(NULL, bus)
                                     : -1;
                node_cpuset(m->node[d], &m->cpus[d]);
        }
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
        /* run next to the device's PCIe root (best effort) */
        if (CPU_COUNT(&m->cpus[j->dev]) > 0)
                (void) pthread_setaffinity_np(pthread_self(), sizeof(cpu_set_t), &m->cpus[j->dev]);
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
        pthread_mutex_lock(&m->lock); /* the pipelines are per handle */
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
        pthread_mutex_unlock(&m->lock);
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
        pthread_mutex_destroy(&m->lock);
        free(m->pipe);
        free(m->node);
        free(m->cpus);
        free(m);
        return ISAL_HIP_OK;
}
