/*
 * isal_hip.h — MI355X-native extensions of the erasure-code engine.
 *
 * The reference API (erasure_code.h) is one synchronous call per stripe. On a
 * GPU that shape is launch- and sync-bound, so the engine adds a batched,
 * stream-ordered "stripe batch": nstripes independent stripes that share one
 * coefficient matrix are encoded by ONE kernel launch over device-resident
 * shards. This is additive: nothing in erasure_code.h depends on it, and the
 * results of a batch are byte-identical to calling ec_encode_data /
 * ec_encode_data_update once per stripe.
 *
 * All functions return 0 on success and a negative ISAL_HIP_E* code on error
 * (they never abort). Streams are hipStream_t passed as void* so that this
 * header needs no HIP include; NULL means the legacy default stream.
 */
#ifndef ISAL_HIP_ISAL_HIP_H
#define ISAL_HIP_ISAL_HIP_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ISAL_HIP_OK 0
#define ISAL_HIP_EINVAL (-1)   /* bad argument (size, count, NULL, unaligned pointer) */
#define ISAL_HIP_EHIP (-2)     /* a HIP runtime call failed */
#define ISAL_HIP_ENOMEM (-3)   /* host or device allocation failed */
#define ISAL_HIP_EDEVICE (-4)  /* a shard pointer is on another GPU than the object's device */

typedef struct isal_hip_batch isal_hip_batch;

/*
 * Describe a batch of stripes. len bytes per shard, k sources, rows outputs.
 * gftbls: 32*k*rows bytes from ec_init_tables (host memory; copied).
 * data:   host array of nstripes*k DEVICE pointers, stripe-major
 *         (data[s*k + j] = shard j of stripe s).
 * coding: host array of nstripes*rows DEVICE pointers (coding[s*rows + l]).
 * Pointer tables and derived coefficient tables are uploaded once here; the
 * launch functions below only enqueue kernels.
 * The batch belongs to the caller's current device at creation: every shard
 * must be hipMalloc memory of that device, managed memory, or page-locked host
 * memory (ISAL_HIP_EDEVICE for memory of another GPU, ISAL_HIP_EINVAL for
 * pageable memory, which no kernel can reach). The batch's kernels run on its
 * device whatever the calling thread's current device is; a stream passed to
 * them must belong to that device (NULL: its legacy default stream).
 */
int isal_hip_batch_create(isal_hip_batch **out, int len, int k, int rows,
                          const unsigned char *gftbls, int nstripes, unsigned char *const *data,
                          unsigned char *const *coding);

/* Replace the coefficient tables (e.g. a decode matrix) of an existing batch.
 * Synchronises the device first: launches already queued on any stream keep
 * the coefficients they were enqueued with. */
int isal_hip_batch_set_tables(isal_hip_batch *b, const unsigned char *gftbls);

/* Enqueue ec_encode_data for every stripe of the batch on stream. */
int isal_hip_batch_encode(isal_hip_batch *b, void *stream);

/* Enqueue ec_encode_data_update(vec_i) for every stripe: source shard
 * data[s*k + vec_i] is folded into coding[s*rows + l] for all l. */
int isal_hip_batch_update(isal_hip_batch *b, int vec_i, void *stream);

/* Enqueue a verify of every stripe (the xor_check / pq_check question for a
 * whole batch, e.g. a scrub): each stripe's coding rows are recomputed from
 * its sources and compared with the stored bytes; nothing is written to the
 * shards. bad: DEVICE array of nstripes words, bad[s] = ~0 when stripe s is
 * consistent, else its first mismatch as column << 8 | row (smallest column,
 * then row). Needs every shard 16-byte aligned (ISAL_HIP_EINVAL otherwise). */
int isal_hip_batch_check(isal_hip_batch *b, unsigned long long *bad, void *stream);

int isal_hip_batch_destroy(isal_hip_batch *b);

/*
 * Fragment checksums (the step storage callers run right after
 * encoding). crc receives nstripes*(k+rows) values in DEVICE memory:
 *   crc[s*(k+rows) + j]     = crc32_iscsi(data[s*k + j],   len, init)  (j < k)
 *   crc[s*(k+rows) + k + l] = crc32_iscsi(coding[s*rows + l], len, init)
 * with the reference's crc32_iscsi semantics (include/crc.h:137-141,
 * crc/crc_base.c:205-219: reflected CRC32C, register starts at init, no final
 * inversion).
 *
 * isal_hip_batch_encode_crc: ec_encode_data for every stripe AND the checksums
 *   of the sources and the fresh parity, in one pass over HBM when the shards
 *   are 16-byte aligned, len % 16 == 0 and k <= 64 (otherwise encode, then a
 *   checksum pass).
 * isal_hip_batch_crc: checksums only (e.g. to verify fragments read back).
 * The first call allocates the per-lane partials: nstripes*(k+rows) *
 * ceil(len/65536) KiB of device memory (~1/64 of the shard bytes).
 */
int isal_hip_batch_encode_crc(isal_hip_batch *b, unsigned int init, unsigned int *crc,
                              void *stream);
int isal_hip_batch_crc(isal_hip_batch *b, unsigned int init, unsigned int *crc, void *stream);

/*
 * CRC64 of every shard: crc[s*(k+rows) + j] as isal_hip_batch_crc, in DEVICE
 * memory, = crc64_<variant>(init, shard, len) with the reference's semantics
 * (include/crc64.h:54-163, crc/crc64_base.c:569-670: register starts at ~init,
 * inverted on return; refl / norm bit order). Variants in the order of
 * crc64.h. The first call per variant uploads its own tables (~80 KiB, kept
 * for the batch's lifetime; no device synchronisation); partials take
 * nstripes*(k+rows) * ceil(len/65536) * 2 KiB of device memory.
 */
#define ISAL_HIP_CRC64_ECMA_REFL 0
#define ISAL_HIP_CRC64_ECMA_NORM 1
#define ISAL_HIP_CRC64_ISO_REFL 2
#define ISAL_HIP_CRC64_ISO_NORM 3
#define ISAL_HIP_CRC64_JONES_REFL 4
#define ISAL_HIP_CRC64_JONES_NORM 5
#define ISAL_HIP_CRC64_ROCKSOFT_REFL 6
#define ISAL_HIP_CRC64_ROCKSOFT_NORM 7
#define ISAL_HIP_CRC64_NVARIANTS 8
int isal_hip_batch_crc64(isal_hip_batch *b, int variant, unsigned long long init,
                         unsigned long long *crc, void *stream);
/* ec_encode_data for every stripe AND crc64_<variant> of the sources and the
 * fresh parity (layout as isal_hip_batch_crc64), in one pass over HBM when the
 * shards are 16-byte aligned, len % 16 == 0, len >= 4096, rows <= 8 and
 * k <= 32 (otherwise encode, then isal_hip_batch_crc64). */
int isal_hip_batch_encode_crc64(isal_hip_batch *b, int variant, unsigned long long init,
                                unsigned long long *crc, void *stream);

/* ---- streaming pipeline for HOST-resident stripes ----------------------- */

/*
 * Stripes whose shards live in host memory (NIC / disk buffers) flow through
 * `depth` HBM slots on three HIP streams: host->device copies of the sources,
 * GF arithmetic, device->host copies of the parity, overlapped across stripes.
 *   ISAL_HIP_PIPE_UPDATE: each source is folded into the parity as soon as it
 *                         lands (ec_encode_data_update semantics, parity
 *                         starts zeroed);
 *   ISAL_HIP_PIPE_ENCODE: one ec_encode_data launch once all k sources landed.
 * Pinned host buffers give full copy/compute overlap; pageable ones work but
 * serialise the copies.
 */
#define ISAL_HIP_PIPE_UPDATE 0
#define ISAL_HIP_PIPE_ENCODE 1
/* depth is capped at this many stripes in flight (more only slows the copies) */
#define ISAL_HIP_PIPE_MAX_DEPTH 4

typedef struct isal_hip_pipe isal_hip_pipe;

int isal_hip_pipe_create(isal_hip_pipe **out, int len, int k, int rows,
                         const unsigned char *gftbls, int depth, int mode);

/* Enqueue one stripe: data = k host source pointers, coding = rows host parity
 * pointers (written when the stripe completes). Blocks only while all `depth`
 * slots are busy. Buffers must stay valid until isal_hip_pipe_flush returns. */
int isal_hip_pipe_submit(isal_hip_pipe *p, unsigned char *const *data, unsigned char *const *coding);

/* Wait until every submitted stripe's parity is in host memory. */
int isal_hip_pipe_flush(isal_hip_pipe *p);

int isal_hip_pipe_destroy(isal_hip_pipe *p);

/* ---- several GPUs from one process ---------------------------------------- */

/*
 * Host-resident stripes encoded on ndev GPUs at once (0 = every visible GPU).
 * A call's stripes are split into contiguous, balanced ranges
 * (isal_hip_multi_partition); GPU d streams its range through its own
 * pipeline (as isal_hip_pipe, mode ENCODE) on its own host thread, so the
 * GPUs never exchange data. isal_hip_multi_encode blocks until every parity
 * shard is in host memory; data[s*k + j] / coding[s*rows + l] are host
 * pointers (pinned for full copy/compute overlap). Callers whose shards are
 * already in each GPU's HBM use one isal_hip_batch per device instead.
 * Each device's worker thread runs on the CPUs of the device's NUMA node
 * (sysfs; ISAL_HIP_SYSFS_ROOT overrides "/sys"), within the process's own
 * affinity. One handle runs one isal_hip_multi_encode at a time: a second
 * thread calling it on the same handle blocks until the first returns.
 */
typedef struct isal_hip_multi isal_hip_multi;

int isal_hip_multi_create(isal_hip_multi **out, int ndev, int len, int k, int rows,
                          const unsigned char *gftbls, int depth);
int isal_hip_multi_ndev(const isal_hip_multi *m);
int isal_hip_multi_encode(isal_hip_multi *m, long long nstripes, unsigned char *const *data,
                          unsigned char *const *coding);
int isal_hip_multi_destroy(isal_hip_multi *m);

/* NUMA node of device dev's PCIe root (-1 unknown), and how many CPUs its
 * worker thread is pinned to (0 = not pinned). */
int isal_hip_multi_numa_node(const isal_hip_multi *m, int dev);
int isal_hip_multi_worker_cpus(const isal_hip_multi *m, int dev);

/* sysfs lookups behind the pinning (root NULL = ISAL_HIP_SYSFS_ROOT or /sys):
 * the NUMA node of a PCI device ("0000:05:00.0"; -1 unknown), and the CPUs of
 * a node's cpulist into cpus[0..max) (returns how many it lists, -1 on error). */
int isal_hip_pci_numa_node(const char *root, const char *pci_bus_id);
int isal_hip_numa_node_cpus(const char *root, int node, int *cpus, int max);

/* Stripes [*first, *first + *count) of nstripes belong to device (or rank)
 * dev of ndev: contiguous, covering, sizes differ by at most one. Pure
 * arithmetic, no GPU needed. */
void isal_hip_multi_partition(long long nstripes, int ndev, int dev, long long *first,
                              long long *count);

/* ---- routing of the drop-in calls and configuration --------------------- */

/*
 * The synchronous drop-in calls (erasure_code.h, gf_vect_mul.h, raid.h) route
 * each call by where its shards live and how large it is:
 *   - any device-resident shard: the GPU kernels. An encode whose shards are
 *     all device-resident and 16-byte aligned, with k + rows <= 32, rows <= 8
 *     and k * rows <= 89, passes its shard pointers and coefficient tables as
 *     kernel arguments: one launch and one stream synchronisation per call
 *     (ISAL_HIP_KARG=0 uploads them with a copy instead);
 *   - host-resident shards, (k + rows) * len > ISAL_HIP_CPU_MAX_BYTES: the GPU
 *     kernels. Page-locked host shards (hipHostMalloc / hipHostRegister) are
 *     read and written in place through their device mapping when the whole
 *     shard lies in one registration (an update's parity excepted: staged);
 *     pageable ones, and page-locked shards that run past their
 *     registration, are staged through HBM, in pipelined 4 MiB column chunks
 *     when longer (ISAL_HIP_CHUNK_KB, ISAL_HIP_PIPE_CHUNKS=0 for one chunk,
 *     ISAL_HIP_PINNED_DIRECT=0 to stage page-locked shards too);
 *   - host-resident shards up to ISAL_HIP_CPU_MAX_BYTES (default 8 MiB; when
 *     every shard is page-locked, ISAL_HIP_CPU_MAX_BYTES_PINNED, default
 *     2 MiB), or a host without a usable GPU: the engine's CPU route.
 * Per calling thread the library keeps a blocking HIP stream, a pinned
 * argument buffer and the last call's coefficient tables. A thread that makes
 * a large staged host call also gets a copy-out helper thread, two more
 * streams and nine events, kept until the thread exits: at most
 * ISAL_HIP_MAX_HELPERS (default 8) helpers live in a process — a thread
 * beyond that issues its copies alone (slower, same result). Streams share
 * the process's GPU_MAX_HW_QUEUES hardware queues.
 * ISAL_HIP_BACKEND=gpu forces the kernels for every call (and aborts when no
 * GPU is usable), =cpu sends every host-resident call to the CPU route,
 * =auto (default) is the rule above. Routing classifies each shard pointer
 * with hipPointerGetAttributes, so the HIP runtime is initialised on a host
 * with a GPU even under =cpu (device-resident shards still go to the GPU).
 * If a HIP call fails during a host-resident call, the call completes on the
 * CPU route and the failure is reported once on stderr; ISAL_HIP_LOG=1 logs
 * every call's route.
 * Several GPUs: the reference API has no device argument, so a call runs on
 * the GPU that holds its device-resident (hipMalloc) shards — the thread's
 * current device is switched to it for the call and restored before the call
 * returns — else, with no such shard, on the thread's current device. All of
 * one call's device-resident shards must be on ONE GPU (a call that mixes GPUs
 * aborts, naming the entry point: no kernel and no CPU route can reach both).
 * Managed memory runs on either; page-locked host memory is used in place
 * only on the GPU it was registered with, and staged elsewhere. A thread keeps
 * one context (stream, buffers, mailbox) per GPU it has called on.
 * Environment knobs are read once; isal_hip_config_reload() re-reads them
 * (call it only while no other thread is inside the library).
 */
void isal_hip_config_reload(void);

/* The device choice above as a pure function (test hook; the drop-in calls use
 * it): n shards with kind[i] (ISAL_HIP_MEM_*) and dev[i] (the device their
 * pointer attributes name; read for DEVICE and PINNED only), the caller's
 * current device cur. Returns the device the call runs on (-1: none, cur < 0
 * and no device shard), -2 when device shards are on two GPUs (*bad = the
 * first shard on a second one; -1 otherwise), -3 for bad arguments.
 * in_place[i] (optional): 1 where a kernel on that device uses shard i where it
 * lies, 0 where it must be staged through HBM. */
#define ISAL_HIP_MEM_PAGEABLE 0
#define ISAL_HIP_MEM_DEVICE 1
#define ISAL_HIP_MEM_MANAGED 2
#define ISAL_HIP_MEM_PINNED 3
int isal_hip_route_device(int n, const int *kind, const int *dev, int cur, int *bad, int *in_place);

/* Per-thread, per-device contexts the drop-in calls have created since the
 * process started (a thread's first call on each GPU makes one). */
unsigned long long isal_hip_contexts_created(void);

/* Kernel-argument drop-in calls whose completion word had not arrived after
 * the 20 ms spin, so that hipStreamSynchronize completed them (the kernel
 * waited behind other work, or ran long). */
unsigned long long isal_hip_slow_waits(void);

/* Drop-in calls served by the CPU route, and of those the HIP-failure
 * fallbacks, since the process started. */
unsigned long long isal_hip_cpu_calls(void);
unsigned long long isal_hip_fallbacks(void);

/* ---- introspection (tests, benchmarks) --------------------------------- */

/* Number of erasure-code kernels this process has launched through the engine. */
unsigned long long isal_hip_kernel_launches(void);

/* Maximum parity rows one kernel pass produces (larger rows are split into passes). */
int isal_hip_max_rows_per_pass(void);

/* Name of the compiled GPU target ("gfx950"). */
const char *isal_hip_target(void);

/* Ask the HIP runtime for the attributes of every kernel the library's
 * launchers can launch (each registers itself when the library loads):
 * returns how many have no usable device code (0: all present; each one is
 * named on stderr), ISAL_HIP_EHIP without a usable GPU. *nkernels (optional)
 * receives how many were checked. */
int isal_hip_selftest_kernels(int *nkernels);

#ifdef __cplusplus
}
#endif

#endif /* ISAL_HIP_ISAL_HIP_H */
