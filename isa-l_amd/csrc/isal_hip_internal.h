/*
 * isal_hip_internal.h — contract between the C host shim (isal_hip_shim.c,
 * gf_host.c) and the HIP kernel launchers (ec_kernels.hip). Not installed.
 *
 * Device argument layout (one contiguous device allocation per call or batch):
 *
 *   ptrs : uint64_t[nstripes][ptr_stride]   shard device addresses; for a
 *          stripe s, sources at [s][src_idx0 + j], outputs at [s][dst_idx0 + l]
 *   tbl  : uint32_t coefficient tables, grouped by row pass g (rows r0..r0+P-1,
 *          P <= EC_MAX_ROWS_PER_PASS): group g starts at dword 5*k*r0 and is
 *          laid out [j < k][l < P][5], so one source's tables for every output
 *          of the pass are contiguous (one scalar-load burst per source).
 *
 * The 5 dwords of one coefficient c are three v_perm_b32 byte-lookup tables
 * (GF(2^8) multiplication is GF(2)-linear, so c*x = c*(x&7) ^ c*(x&0x38) ^ c*(x&0xc0)):
 *   [0],[1]  c*{0,1,..,7}             (entries 0-3 in [0], 4-7 in [1])
 *   [2],[3]  c*{0,8,16,..,56}
 *   [4]      c*{0,64,128,192}
 */
#ifndef ISAL_HIP_INTERNAL_H
#define ISAL_HIP_INTERNAL_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EC_MAX_ROWS_PER_PASS 8
#define EC_TBL_DWORDS 5

/* Host GF math (gf_host.c). */
unsigned char isal_hip_gf_mul(unsigned char a, unsigned char b);
/* Fill the grouped perm tables above from 32-byte-per-coefficient gftbls
 * (only byte 1 of each 32 B entry, the coefficient itself, is read — exactly
 * what ec_base.c reads, so any gftbls gives the reference's answer). */
void isal_hip_build_tables(int k, int rows, const unsigned char *gftbls, uint32_t *tbl);
size_t isal_hip_tables_dwords(int k, int rows);

/* 0/1 structure of an encode's coefficient passes. Every gf_gen_rs_matrix
 * parity block has row 0 = all ones and column 0 = all ones (ec_base.c
 * gf_gen_rs_matrix: p = 1 for j = 0, gen = 1 for the first parity row); so
 * does RAID pq_gen's. A product with a 0/1 coefficient is x & mask (one VALU
 * op per dword, or none when it starts the sum) instead of three v_perm
 * lookups and their folds. Pass g (rows 8g..8g+P-1) qualifies — bit g of
 * `ok` — when its first row and its column of source 0 hold only 0 and 1 and
 * k <= 64; then r0[g] has bit j set where row 8g's coefficient of source j is
 * 1, and c0[g] bit l where row 8g + l's coefficient of source 0 is 1.
 * The masks are computed whatever the knobs say; ISAL_HIP_ENC_XOR=0 makes the
 * launch ignore them (every pass takes the lookup path). */
#define EC_MAX_PASSES 32
typedef struct {
        unsigned ok;
        unsigned c0[EC_MAX_PASSES];
        unsigned long long r0[EC_MAX_PASSES];
        /* device copy of isal_hip_build_ldsx_tables' output, or NULL: the
         * wide passes may then look their products up in LDS (ec_kernels.hip
         * ec_encode_ldsx). isal_hip_enc_masks leaves it NULL; a caller that
         * uploads the tables sets it. */
        const uint64_t *ldsx;
} isal_hip_encmask;
void isal_hip_enc_masks(int k, int rows, const unsigned char *gftbls, isal_hip_encmask *m);

/* LDS product tables of a pass of P <= 8 rows: for each source j, a 32-entry
 * table T5_j[v] (8 bytes, byte l = c[r0 + l][j] * v: bits 0-4 of a source
 * byte) and an 8-entry table T3_j[v] (byte l = c[r0 + l][j] * (v << 5): bits
 * 5-7); pass g occupies k * ISAL_HIP_LDSX_ENTRIES words: [k][32] T5, then
 * [k][8] T3. A source byte's products with all P coefficients are two
 * lookups (T5 ^ T3). */
#define ISAL_HIP_LDSX_ENTRIES 40
size_t isal_hip_ldsx_words(int k, int rows);
void isal_hip_build_ldsx_tables(int k, int rows, const unsigned char *gftbls, uint64_t *out);
void isal_hip_build_ldsx_tables_coef(int k, int rows, const unsigned char *coef, uint64_t *out);

/* Kernel launchers (ec_kernels.hip). Return 0 or a hipError_t value.
 * `stream` is a hipStream_t. `vec16` = every shard address is 16-byte aligned. */
int isal_hip_launch_encode(const uint64_t *d_ptrs, int ptr_stride, int src_idx0, int dst_idx0,
                           const uint32_t *d_tbl, int len, int k, int rows, long long nstripes,
                           int vec16, const isal_hip_encmask *em, void *stream);
/* One stripe of device-resident, 16-byte aligned shards whose pointer table
 * (k sources then rows outputs) and coefficient tables (one pass: rows <=
 * EC_MAX_ROWS_PER_PASS, the layout above) travel as 2 KiB of kernel
 * arguments — no argument upload before the launch. Needs k + rows <=
 * ISAL_HIP_KARG_PTRS and 5 * k * rows <= ISAL_HIP_KARG_TBL. */
#define ISAL_HIP_KARG_PTRS 32
#define ISAL_HIP_KARG_TBL 448
typedef struct {
        uint64_t ptrs[ISAL_HIP_KARG_PTRS];
        uint32_t tbl[ISAL_HIP_KARG_TBL];
} isal_hip_karg;
/* Completion of a kernel-argument call without the runtime's wake-up: every
 * workgroup waits for its (write-through) stores and counts itself in *cnt;
 * the last one resets *cnt (and *res) for the next call and writes mail[1] =
 * the verify result (*res, ~0 for encode / update), then mail[0] = seq
 * (system-scope stores) into page-locked host memory that the calling thread
 * spins on (isal_hip_shim.c wait_done; ec_kernels.hip karg_done). cnt = NULL:
 * no protocol (the caller synchronises the stream). res: device word a
 * verify's mismatching lanes atomically lower (~0 between calls); NULL for
 * encode / update. */
typedef struct {
        unsigned *cnt;
        unsigned long long *res;
        unsigned long long *mail; /* device view of the host mailbox */
        unsigned long long seq;
} isal_hip_kdone;
/* cnt: ISAL_HIP_KDONE_GROUPS group counters ISAL_HIP_KDONE_STRIDE words apart
 * (one 64-byte line each), then the top counter: workgroups count in groups
 * of max(32, ceil(n / GROUPS)) and each group's last one counts in the top
 * counter — at most 256 atomics on any one word instead of one per workgroup
 * (a single word serialised 1024 workgroups' atomics: +10 us per call). */
#define ISAL_HIP_KDONE_GROUPS 256
#define ISAL_HIP_KDONE_STRIDE 16
#define ISAL_HIP_KDONE_WORDS ((ISAL_HIP_KDONE_GROUPS + 1) * ISAL_HIP_KDONE_STRIDE)
/* busy: kernel-argument calls of this process in flight, this one included
 * (chooses the lane width, ec_kernels.hip karg_narrow). */
int isal_hip_launch_encode_karg(const isal_hip_karg *a, const isal_hip_kdone *d, int len, int k, int rows,
                                const isal_hip_encmask *em, int busy, const uint64_t *ldsx, void *stream);
/* whether a drop-in encode of this shape runs on LDS product tables (then the
 * caller passes them to isal_hip_launch_encode_karg; NULL keeps v_perm) */
int isal_hip_karg_ldsx(int k, int rows);
/* ec_encode_data_update of one stripe the same way: ptrs = {source, rows
 * parity}, tbl = the source's tables for rows <= EC_MAX_ROWS_PER_PASS outputs. */
int isal_hip_launch_update_karg(const isal_hip_karg *a, const isal_hip_kdone *d, int len, int rows,
                                void *stream);
/* Verify of one stripe the same way (ptrs = k sources then rows stored
 * outputs, tables as for the encode): the first mismatch, key (column << 8 |
 * row), arrives in mail[1] (~0: none). Needs d->cnt, d->res and d->mail. */
int isal_hip_launch_verify_karg(const isal_hip_karg *a, const isal_hip_kdone *d, int len, int k, int rows,
                                const isal_hip_encmask *em, void *stream);
int isal_hip_launch_update(const uint64_t *d_ptrs, int ptr_stride, int src_idx, int dst_idx0,
                           const uint32_t *d_tbl, int len, int k, int rows, int vec_i,
                           long long nstripes, int vec16, void *stream);

/* Verify one stripe (nstripes = 1): recompute rows outputs from the sources and
 * compare with the bytes at the output pointers. Each workgroup writes the
 * minimum key (col0 + column) << 8 | row of its mismatches (~0 if none) to
 * its own slot; *nslots receives the number of slots written (at most
 * EC_VERIFY_SLOTS(rows)); the caller takes the minimum. */
#define EC_VERIFY_MAX_GRID 2048
#define EC_VERIFY_SLOTS(rows) \
        ((((rows) + EC_MAX_ROWS_PER_PASS - 1) / EC_MAX_ROWS_PER_PASS) * EC_VERIFY_MAX_GRID)
int isal_hip_launch_verify(const uint64_t *d_ptrs, int ptr_stride, int src_idx0, int dst_idx0,
                           const uint32_t *d_tbl, int len, int k, int rows, long long col0,
                           unsigned long long *slots, int *nslots, int vec16, const isal_hip_encmask *em,
                           void *stream);

/* Verify every stripe of a batch (16-byte aligned shards): bad[s] = ~0 when
 * stripe s's stored rows equal its recomputed parity, else its first
 * mismatch as column << 8 | row (bad: device memory, nstripes words, set on
 * the stream before the kernels). */
int isal_hip_launch_verify_batch(const uint64_t *d_ptrs, int ptr_stride, int src_idx0, int dst_idx0,
                                 const uint32_t *d_tbl, int len, int k, int rows, long long nstripes,
                                 const isal_hip_encmask *em, unsigned long long *bad, void *stream);

/* The shim's generic synchronous call (host or device shard pointers); fn
 * names the entry point in abort messages. op: ISAL_HIP_OP_ENCODE (dst = coded sources, nsrc = k), ISAL_HIP_OP_UPDATE
 * (dst ^= c[.][vec_i] * src[0], nsrc = 1), ISAL_HIP_OP_VERIFY (compare dst
 * with the coded sources). Returns ~0, or for VERIFY the first mismatch as
 * column << 8 | row. */
#define ISAL_HIP_OP_ENCODE 0
#define ISAL_HIP_OP_UPDATE 1
#define ISAL_HIP_OP_VERIFY 2
unsigned long long isal_hip_run(const char *fn, int op, int len, int k, int rows, int vec_i,
                                const unsigned char *gftbls, unsigned char *const *src, int nsrc,
                                unsigned char *const *dst);

/* Parity rows of a pass whose coefficients are all 0 or 1 (RS Vandermonde row
 * 0, RAID P): such a row is the XOR of some sources, so — CRC being
 * GF(2)-linear in the data — its raw CRC chains are the XOR of those sources'
 * chains. The fused encode+CRC kernels do not checksum row 0 when it is such
 * a row (bit 0 of rows; a compile-time kernel variant): they form its chains
 * from the source chains once per block. rows: bit l set for such a row l <
 * EC_MAX_ROWS_PER_PASS (k <= 64); src[l]: bit j set where c[l][j] == 1. */
typedef struct {
        unsigned rows;
        unsigned long long src[EC_MAX_ROWS_PER_PASS];
} isal_hip_xrows;
void isal_hip_xor_rows(int k, int rows, const unsigned char *gftbls, isal_hip_xrows *x);

/* Make dev the calling thread's current device for a call on an object that
 * belongs to it; returns what isal_hip_dev_leave restores (-1: nothing, -2:
 * the switch failed). */
int isal_hip_dev_enter(int dev);
void isal_hip_dev_leave(int prev);

/* Kernel registry (isal_hip_selftest_kernels): every kernel a launcher can
 * launch registers its host handle and a name when the library loads
 * (ec_device.h ISAL_LAUNCH). */
void isal_hip_kreg_add(const void *fn, const char *name);

/* Launch counter shared by the shim and the launchers. */
void isal_hip_count_launch(void);

/* ---- environment knobs (isal_hip_knobs.c): read once, -1 when unset ------- */
enum {
        ISAL_HIP_KNOB_BACKEND,       /* auto(0) | gpu(1) | cpu(2); -2 = unknown word */
        ISAL_HIP_KNOB_CPU_MAX_BYTES, /* auto route: host calls up to this many bytes run on the CPU */
        ISAL_HIP_KNOB_LOG,           /* 1: log every drop-in call's route to stderr, 2: + vector encode kernels */
        ISAL_HIP_KNOB_CPU_SIMD,      /* CPU route width cap: 0 per byte, 1 AVX2, 2 GFNI (tests) */
        ISAL_HIP_KNOB_STAGE_MB,      /* HBM staging per host call (MiB) */
        ISAL_HIP_KNOB_ENC_GLDS,      /* 0: wide encode passes (5-8 rows) load through registers, not the LDS-DMA ring */
        ISAL_HIP_KNOB_CRC_TILES,     /* 4 KiB tiles per CRC workgroup (tests: block geometry) */
        ISAL_HIP_KNOB_CRC_XROWS,     /* 0: fused checksums compute 0/1 parity rows too (tests: no derivation) */
        ISAL_HIP_KNOB_FAULT,         /* fault-injection site of GPU-routed calls (tests) */
        ISAL_HIP_KNOB_FAULT_CHUNK,   /* ... only in this column chunk of a call (tests; unset: every chunk) */
        ISAL_HIP_KNOB_CHUNK_KB,      /* column-chunk bytes per shard of large host calls (pipelined) */
        ISAL_HIP_KNOB_PIPE_CHUNKS,   /* 0: large host calls one chunk at a time (no copy overlap) */
        ISAL_HIP_KNOB_PINNED_DIRECT, /* 0: stage page-locked host shards like pageable ones */
        ISAL_HIP_KNOB_CPU_MAX_BYTES_PINNED, /* auto route limit when every host shard is page-locked */
        ISAL_HIP_KNOB_PAR_COPY,      /* 0: one thread issues a staged call's copies (no helper) */
        ISAL_HIP_KNOB_ENC_XOR,       /* 0: the encode computes 0/1 rows and columns with lookups too */
        ISAL_HIP_KNOB_ENC_LDS,       /* encode low table halves from LDS: 1 always, 0 never (default: 5-6 looked-up rows) */
        ISAL_HIP_KNOB_KARG,          /* 0: device-resident drop-in encodes upload their arguments */
        ISAL_HIP_KNOB_MAX_HELPERS,   /* copy-out helper threads per process (default 8) */
        ISAL_HIP_KNOB_KARG_DONE,     /* 0: kernel-argument calls wait in hipStreamSynchronize (no host mailbox) */
        ISAL_HIP_KNOB_ENC_GROUP,     /* 12/10/8/6/5/4: encode load group forced (tests: every group path) */
        ISAL_HIP_KNOB_KARG_NARROW,   /* drop-in kernel-argument encode with 4-byte lanes: 1 on, 0 off */
        ISAL_HIP_KNOB_ENC_WIDE5,     /* 0: 6-8 row passes keep the largest load group (no groups of 5) */
        ISAL_HIP_KNOB_ENC_LDSX,      /* 0: wide passes compute products with v_perm, not LDS product tables */
        ISAL_HIP_KNOB_COUNT
};
long long isal_hip_knob(int id);
/* bumped by every isal_hip_config_reload(): caches derived from knobs check it */
unsigned isal_hip_knob_generation(void);

/* ---- the host (CPU) route (ec_cpu.c) ---------------------------------------
 * Same ops and return value as isal_hip_run, over HOST-resident shards only,
 * for columns [c0, len): the drop-in calls' route for small host calls, for
 * ISAL_HIP_BACKEND=cpu, for hosts without a GPU, and the fallback when a HIP
 * call fails mid-way (columns before c0 are already final). */
unsigned long long isal_cpu_run(int op, long long c0, int len, int k, int rows, int vec_i,
                                const unsigned char *gftbls, unsigned char *const *src, int nsrc,
                                unsigned char *const *dst);

/* ---- CRC32C of shards (crc_host.c, crc_kernels.hip) -------------------------
 * crc32_iscsi semantics (reference crc/crc_base.c:205-219). Each workgroup
 * covers `tt` consecutive 4 KiB tiles of one shard; lane L owns bytes
 * [16L, 16L+16) of every tile and chains its chunks with Z^4096, leaving one
 * partial per (shard, block, lane):
 *   part[((shard * nblk) + blk) * 256 + L]   (shard = stripe * nshard_total + i)
 * and, when len % 4096 != 0, the crc of its chunk of the last (ragged) tile:
 *   tail[shard * 256 + L]
 * crc32c_combine joins them with the constants of isal_hip_crc32c_plan. */
#define ISAL_HIP_CRC_TILE 4096
#define ISAL_HIP_CRC_SLICES 16
/* Kernel lookup tables (isal_hip_crc32c_tables), all indexed by 5-bit fields
 * so that one table fills the 32 LDS banks exactly once: a wave's lookups
 * into it never bank-conflict (random byte-indexed tables conflict ~3-way).
 * Each dword of a 16-byte chunk splits into 7 fields, bits [0,5) [5,10)
 * [10,15) [15,20) [20,25) [25,30) [30,32):
 *   [0, 256)                     T0: crc of one byte (bytewise tail loop)
 *   [256 + (d*7 + f)*32 + v]     crc(0, chunk) of field f of dword d = v
 *   [256 + 896 + f*32 + v]       Z^4096 of field f of the chain value = v */
#define ISAL_HIP_CRC_FIELDS 7
#define ISAL_HIP_CRC_CHUNK_TAB 256
#define ISAL_HIP_CRC_SHIFT_TAB (ISAL_HIP_CRC_CHUNK_TAB + 4 * ISAL_HIP_CRC_FIELDS * 32)
#define ISAL_HIP_CRC_TAB_DWORDS (ISAL_HIP_CRC_SHIFT_TAB + ISAL_HIP_CRC_FIELDS * 32)
#define ISAL_HIP_CRC_PLAN_DWORDS (2 * 1024 + 2 * 256 + 4)
/* Multi-tile chain step of crc32c_shards, stored after the plan:
 * Z^(4096*m) o crc(0, chunk) for m = 1..3, then Z^(4096*4). */
#define ISAL_HIP_CRC_CHUNK_DWORDS (4 * ISAL_HIP_CRC_FIELDS * 32)
#define ISAL_HIP_CRC_EXT_TAB (ISAL_HIP_CRC_TAB_DWORDS + ISAL_HIP_CRC_PLAN_DWORDS)
#define ISAL_HIP_CRC_EXT_DWORDS (3 * ISAL_HIP_CRC_CHUNK_DWORDS + ISAL_HIP_CRC_FIELDS * 32)
/* Byte-position tables of the fused kernel's byte path, after EXT:
 *   P:  table p (byte p of a 16-byte chunk) = crc of byte b followed by
 *       15 - p zero bytes, 16 x 256 dwords;
 *   P': the same followed by 4080 more zero bytes (Z^4080 o P: the step of a
 *       pre-shifted chain, crc_kernels.hip). */
#define ISAL_HIP_CRC_B16_TAB (ISAL_HIP_CRC_EXT_TAB + ISAL_HIP_CRC_EXT_DWORDS)
#define ISAL_HIP_CRC_B16_DWORDS (2 * 16 * 256)
void isal_hip_crc32c_byte_tables(uint32_t *out);
/* F' = Z^4080 o crc(0, chunk) as field tables (the layout of CHUNK_TAB), for
 * the checksum-only kernel's pre-shifted chains. */
#define ISAL_HIP_CRC_FPRE_TAB (ISAL_HIP_CRC_B16_TAB + ISAL_HIP_CRC_B16_DWORDS)
#define ISAL_HIP_CRC_FPRE_DWORDS ISAL_HIP_CRC_CHUNK_DWORDS
void isal_hip_crc32c_pre_tables(const uint32_t *tabs, uint32_t *out);
#define ISAL_HIP_CRC_MAX_FUSED_K 64 /* fused encode keeps k source partials in LDS */

typedef struct {
        long long nfull;  /* full 4 KiB tiles */
        int tail;         /* bytes in the ragged last tile (0: none) */
        long long ntiles; /* nfull + (tail != 0) */
        int tt;           /* tiles per workgroup */
        long long nblk;   /* workgroups per shard */
        long long nfull_last; /* full tiles in the last workgroup */
} isal_hip_crc_geom;

/* ---- CRC64 of shards (crc64_host.c, crc64_kernels.hip) ---------------------
 * The eight crc64_* flavours (reference include/crc64.h:54-163). Same lane
 * layout as CRC32C: crc64_shards leaves one 64-bit chain per (shard, block,
 * lane) over the FULL 4 KiB tiles, part[(shard * nblk + blk) * 256 + L];
 * crc64_combine folds them, adds the ragged tail read straight from the shard
 * and the init term. Table buffer (uint64 entries, one per variant and
 * geometry), every map as 14 field tables of 32 entries (crc64_host.c):
 *   BYTE_TAB   reference byte table (tail bytes)
 *   CHUNK_TAB  raw(0, 16-byte chunk), 4 dwords x 7 fields x 32
 *   SHIFT_TAB  Z^4096                      } crc64_shards loads CHUNK..SHIFT
 *   OP_BLOCK   Z^(4096*tt)   OP_LAST Z^(4096*nfull_last)
 *   OP_TREE    Z^(16 * 2^s), s = 0..7 (lane tree)   OP_TAIL Z^(16*(tail/16))
 *   (crc64_combine loads BYTE..OP_TAIL: COMBINE_ENTRIES)
 *   CHUNKX_TAB Z^(4096*m) o raw(0, chunk), m = 1..3 (multi-tile chain step)
 *   SHIFTX_TAB Z^8192, Z^16384
 *   SLICE_TAB  slicing-by-8 tables of the fused kernel's byte-indexed chunk
 *              path, in the "u-domain" u = pi(s) (pi = byte swap for the norm
 *              flavours, identity for refl), where processing 8 bytes d is
 *              u' = A(d ^ u) for every flavour:
 *                A_j[v]  = pi(raw(0, v at byte j of 8)),  8 x 256
 *                A'_j[v] = pi(Z^4080 raw(0, v at byte j of 8)), 8 x 256
 *              (A' advances a lane's chain past the rest of its tile) */
#define ISAL_HIP_CRC64_OP_ENTRIES (2 * ISAL_HIP_CRC_FIELDS * 32)
#define ISAL_HIP_CRC64_BYTE_TAB 0
#define ISAL_HIP_CRC64_CHUNK_TAB 256
#define ISAL_HIP_CRC64_SHIFT_TAB (ISAL_HIP_CRC64_CHUNK_TAB + 4 * ISAL_HIP_CRC_FIELDS * 32)
#define ISAL_HIP_CRC64_OP_BLOCK (ISAL_HIP_CRC64_SHIFT_TAB + ISAL_HIP_CRC64_OP_ENTRIES)
#define ISAL_HIP_CRC64_OP_LAST (ISAL_HIP_CRC64_OP_BLOCK + ISAL_HIP_CRC64_OP_ENTRIES)
#define ISAL_HIP_CRC64_OP_TREE (ISAL_HIP_CRC64_OP_LAST + ISAL_HIP_CRC64_OP_ENTRIES)
#define ISAL_HIP_CRC64_OP_TAIL (ISAL_HIP_CRC64_OP_TREE + 8 * ISAL_HIP_CRC64_OP_ENTRIES)
#define ISAL_HIP_CRC64_COMBINE_ENTRIES (ISAL_HIP_CRC64_OP_TAIL + ISAL_HIP_CRC64_OP_ENTRIES)
#define ISAL_HIP_CRC64_CHUNK_ENTRIES (4 * ISAL_HIP_CRC_FIELDS * 32)
#define ISAL_HIP_CRC64_CHUNKX_TAB ISAL_HIP_CRC64_COMBINE_ENTRIES
#define ISAL_HIP_CRC64_SHIFTX_TAB (ISAL_HIP_CRC64_CHUNKX_TAB + 3 * ISAL_HIP_CRC64_CHUNK_ENTRIES)
#define ISAL_HIP_CRC64_SLICE_TAB (ISAL_HIP_CRC64_SHIFTX_TAB + 2 * ISAL_HIP_CRC64_OP_ENTRIES)
#define ISAL_HIP_CRC64_SLICE_ENTRIES (2 * 8 * 256)
/*   PRE_TAB    field tables of the checksum-only kernel's pre-shifted chains
 *              (u-domain): F_u = pi o raw(0, chunk), F'_u = pi o Z^4080 o raw(0, chunk) */
#define ISAL_HIP_CRC64_PRE_TAB (ISAL_HIP_CRC64_SLICE_TAB + ISAL_HIP_CRC64_SLICE_ENTRIES)
#define ISAL_HIP_CRC64_TAB_ENTRIES (ISAL_HIP_CRC64_PRE_TAB + 2 * ISAL_HIP_CRC64_CHUNK_ENTRIES)

typedef struct {
        long long nfull;      /* full 4 KiB tiles */
        int tail;             /* bytes after them (< 4096) */
        int tt;               /* tiles per workgroup */
        long long nblk;       /* workgroups per shard (0 when nfull == 0) */
        long long nfull_last; /* full tiles in the last workgroup */
} isal_hip_crc64_geom;

int isal_hip_crc64_is_refl(int variant);
void isal_hip_crc64_cpu_tables(int variant, uint64_t byte[256], uint64_t slice[8 * 256]);
uint64_t isal_hip_crc64_poly(int variant);

/* ---- the checksum entry points' CPU route (crc_cpu.c): host buffers --------
 * crc32_iscsi semantics (register starts at init, no inversion) and
 * crc64_<variant> semantics (starts at ~init, inverted on return). */
uint32_t isal_cpu_crc32c(uint32_t init, const unsigned char *buf, uint64_t len);
uint64_t isal_cpu_crc64(int variant, uint64_t init, const unsigned char *buf, uint64_t len);
void isal_hip_crc64_geometry(long long len, int tt, isal_hip_crc64_geom *g);
void isal_hip_crc64_zpow(int variant, unsigned long long n, uint64_t out[64]);
void isal_hip_crc64_tables(int variant, long long len, int tt, uint64_t *tabs);
/* only OP_BLOCK, OP_LAST and OP_TAIL (the length / geometry dependent maps) */
void isal_hip_crc64_len_tables(int variant, long long len, int tt, uint64_t *tabs);
uint64_t isal_hip_crc64_init_term(int variant, long long len, uint64_t init);

/* crc64(init, shard, len) of the nsh shards of each stripe (d_ptrs row
 * stride ptr_stride, shards 0..nsh-1) into out[stripe * nsh + i]; init_term =
 * isal_hip_crc64_init_term(variant, len, init). */
int isal_hip_launch_crc64(const uint64_t *d_ptrs, int ptr_stride, int nsh, long long nstripes,
                          int len, int vec16, int refl, int tt, const uint64_t *d_tabs,
                          uint64_t *d_part, uint64_t init_term, uint64_t *out, void *stream);
/* Encode (one pass, rows <= EC_MAX_ROWS_PER_PASS; d_ptrs rows = k sources then
 * rows parity, stride k + rows) and crc64 of all k + rows shards into
 * out[stripe * (k + rows) + i]. Needs 16-byte aligned shards, len % 16 == 0,
 * len >= ISAL_HIP_CRC_TILE and k <= ISAL_HIP_CRC64_MAX_FUSED_K. */
#define ISAL_HIP_CRC64_MAX_FUSED_K 32 /* source chains: k * 2 KiB of LDS */
int isal_hip_launch_encode_crc64(const uint64_t *d_ptrs, int k, int rows, long long nstripes,
                                 int len, const uint32_t *d_tbl, const isal_hip_xrows *xr, int refl,
                                 int tt, const uint64_t *d_tabs, uint64_t *d_part,
                                 uint64_t init_term, uint64_t *out, void *stream);

uint32_t isal_hip_crc32c_mulmod(uint32_t a, uint32_t b);
uint32_t isal_hip_crc32c_xpow8n(unsigned long long n);
void isal_hip_crc32c_tables(uint32_t *tabs);
void isal_hip_crc32c_ext_tables(const uint32_t *tabs, uint32_t *ext);
void isal_hip_crc_geometry(long long len, int tt, isal_hip_crc_geom *g);
void isal_hip_crc32c_plan(long long len, int tt, uint32_t *plan);

/* CRC partials of shards idx0..idx0+nsh-1 of each stripe (no encoding);
 * shard numbering in part/tail starts at shard0 within nshard_total. */
int isal_hip_launch_crc(const uint64_t *d_ptrs, int ptr_stride, int idx0, int nsh,
                        long long nstripes, int len, int vec16, int tt, const uint32_t *d_tabs,
                        uint32_t *d_part, uint32_t *d_tail, int nshard_total, int shard0,
                        void *stream);
/* Encode (as isal_hip_launch_encode) and leave the CRC partials of the k
 * sources (shards 0..k-1) and the rows outputs (shards k..k+rows-1). Needs
 * 16-byte aligned shards, len % 16 == 0 and k <= ISAL_HIP_CRC_MAX_FUSED_K. */
int isal_hip_launch_encode_crc(const uint64_t *d_ptrs, int ptr_stride, int src_idx0, int dst_idx0,
                               const uint32_t *d_tbl, const isal_hip_xrows *xr, int len, int k,
                               int rows, long long nstripes, int tt, const uint32_t *d_tabs,
                               uint32_t *d_part, uint32_t *d_tail, void *stream);
/* out[sh] = crc32_iscsi of shard sh (sh < nsh) from its partials. */
int isal_hip_launch_crc_combine(const uint32_t *d_part, const uint32_t *d_tail,
                                const uint32_t *d_plan, long long nblk, int has_tail,
                                unsigned int init, uint32_t *out, long long nsh, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* ISAL_HIP_INTERNAL_H */
