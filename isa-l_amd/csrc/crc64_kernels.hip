// crc64_kernels.hip — the reference's eight crc64_* flavours (include/crc64.h:
// 54-163, crc/crc64_base.c:569-670) of erasure-code shards on gfx950.
//
// SURVEY §8(f) rank 4 names CRC32C / CRC64 as the fragment checksum storage
// callers run next to encode. Same decomposition as the CRC32C kernels
// (crc_kernels.hip): lane L owns bytes [16L, 16L+16) of every 4 KiB tile,
// computes raw(0, chunk) and chains its chunks across the workgroup's tiles
// with Z^4096. The register is 64-bit, so every lookup is a ds_read_b64 into a
// 32-entry x 8-byte field table — exactly one 256-byte bank row under
// ds_read_b64's 64-bank mapping, hence conflict-free. All constants are
// variant-independent linear maps built by crc64_host.c; only the byte loop of
// the last < 16 bytes knows the shift direction (REFL).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <type_traits>

#include "ec_device.h"

namespace {

constexpr int kF = ISAL_HIP_CRC_FIELDS;
[[maybe_unused]] constexpr int kOp = ISAL_HIP_CRC64_OP_ENTRIES;
[[maybe_unused]] constexpr int kKernTab = ISAL_HIP_CRC64_OP_BLOCK - ISAL_HIP_CRC64_CHUNK_TAB;  // chunk + shift
[[maybe_unused]] constexpr int kChunk = 0;                                                        // offsets in LDS copy
[[maybe_unused]] constexpr int kShift = ISAL_HIP_CRC64_SHIFT_TAB - ISAL_HIP_CRC64_CHUNK_TAB;

static_assert(ISAL_HIP_CRC_TILE == kTile, "CRC tile = encode tile");
static_assert(kF == 7, "field layout below assumes 7 fields per dword");

template <int OFF, int WIDTH>
__device__ __forceinline__ uint32_t bfe(uint32_t x) {
  uint32_t r;
  asm("v_bfe_u32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "n"(OFF), "n"(WIDTH));
  return r;
}

// Byte offsets (entry index * 8) of the 7 fields of w, bits [0,5) [5,10)
// [10,15) [15,20) [20,25) [25,30) [30,32). w << 3 puts fields 0-4 at their
// entry offsets; the even and odd fields are masked into separate words so
// that one bit-field extract per field lands on zeros below it. Fields 5 and 6
// would leave the dword after the shift and come from w directly.
__device__ __forceinline__ void field_offsets8(uint32_t w, uint32_t (&o)[kF]) {
  const uint32_t s = w << 3;
  const uint32_t ev = s & 0x0F83E0F8u;  // fields 0, 2, 4 at [3,8) [13,18) [23,28)
  const uint32_t od = s & 0x007C1F00u;  // fields 1, 3 at [8,13) [18,23)
  o[0] = ev & 0xF8u;
  o[1] = bfe<5, 8>(od);
  o[2] = bfe<10, 8>(ev);
  o[3] = bfe<15, 8>(od);
  o[4] = bfe<20, 8>(ev);
  o[5] = (w >> 22) & 0xF8u;
  o[6] = (w >> 27) & 0x18u;
}

// 64-bit XOR accumulator kept as two dwords so that every fold is one
// v_bitop3 (3-input XOR) per half: a lookup costs one XOR op instead of two
// (the compiler does not form bitop3 from 64-bit XOR chains by itself).
struct X64 {
  uint32_t lo, hi;
  __device__ __forceinline__ void add2(uint64_t x, uint64_t y) {
    lo = xor3(lo, static_cast<uint32_t>(x), static_cast<uint32_t>(y));
    hi = xor3(hi, static_cast<uint32_t>(x >> 32), static_cast<uint32_t>(y >> 32));
  }
  __device__ __forceinline__ void add(uint64_t x) {
    lo ^= static_cast<uint32_t>(x);
    hi ^= static_cast<uint32_t>(x >> 32);
  }
  __device__ __forceinline__ uint64_t get() const {
    return (static_cast<uint64_t>(hi) << 32) | lo;
  }
};

__device__ __forceinline__ __attribute__((unused)) X64 x64(uint64_t v) {
  return {static_cast<uint32_t>(v), static_cast<uint32_t>(v >> 32)};
}

// Entry of field f of table set t at byte offset o (field tables are 256 B apart).
__device__ __forceinline__ uint64_t tab_at(const uint64_t* t, int f, uint32_t o) {
  return *reinterpret_cast<const uint64_t*>(reinterpret_cast<const char*>(t) + f * 256 + o);
}

// acc ^= the 14 field lookups of the two dwords (w0, w1) in the 14 consecutive
// 32-entry tables at t: seven 3-input XORs per half.
__device__ __forceinline__ void lookup14(X64& acc, const uint64_t* t, uint32_t w0, uint32_t w1) {
  uint32_t o[kF], q[kF];
  field_offsets8(w0, o);
  field_offsets8(w1, q);
  const uint64_t* u = t + kF * 32;
  acc.add2(tab_at(t, 0, o[0]), tab_at(t, 1, o[1]));
  acc.add2(tab_at(t, 2, o[2]), tab_at(t, 3, o[3]));
  acc.add2(tab_at(t, 4, o[4]), tab_at(t, 5, o[5]));
  acc.add2(tab_at(t, 6, o[6]), tab_at(u, 0, q[0]));
  acc.add2(tab_at(u, 1, q[1]), tab_at(u, 2, q[2]));
  acc.add2(tab_at(u, 3, q[3]), tab_at(u, 4, q[4]));
  acc.add2(tab_at(u, 5, q[5]), tab_at(u, 6, q[6]));
}

// acc ^= M(v) for a map stored as 14 field tables.
__device__ __forceinline__ void apply_op_acc(X64& acc, const uint64_t* op, uint64_t v) {
  lookup14(acc, op, static_cast<uint32_t>(v), static_cast<uint32_t>(v >> 32));
}

__device__ __forceinline__ __attribute__((unused)) uint64_t apply_op(const uint64_t* op, uint64_t v) {
  X64 a{0u, 0u};
  apply_op_acc(a, op, v);
  return a.get();
}

// acc ^= raw(0, 16-byte chunk) through the chunk map at t, dwords little-endian.
__device__ __forceinline__ void chunk_acc(X64& acc, const uint64_t* t, uint32_t w0, uint32_t w1,
                                          uint32_t w2, uint32_t w3) {
  constexpr int D = kF * 32;
  lookup14(acc, t, w0, w1);
  lookup14(acc, t + 2 * D, w2, w3);
}

__device__ __forceinline__ uint64_t chunk_crc(const uint64_t* t, uint32_t w0, uint32_t w1,
                                              uint32_t w2, uint32_t w3) {
  X64 a{0u, 0u};
  chunk_acc(a, t, w0, w1, w2, w3);
  return a.get();
}

__device__ __forceinline__ uint32_t le32(const uint8_t* p) {
  return p[0] | (p[1] << 8) | (p[2] << 16) | (static_cast<uint32_t>(p[3]) << 24);
}

// raw(0, 16 bytes at base + off) with byte loads (any alignment).
__device__ __forceinline__ __attribute__((unused)) uint64_t chunk_crc_bytes(const uint64_t* t, uint64_t base,
                                                                           long long off) {
  const uint8_t* p = reinterpret_cast<const uint8_t*>(base) + off;
  return chunk_crc(t, le32(p), le32(p + 4), le32(p + 8), le32(p + 12));
}

template <int N, int NV = 1>
__device__ __forceinline__ void load_lds(uint64_t* dst, const uint64_t* __restrict__ src) {
  const uint4* s = reinterpret_cast<const uint4*>(src);
  uint4* d = reinterpret_cast<uint4*>(dst);
  for (int i = threadIdx.x; i < N / 2; i += kBlock * NV) d[i] = s[i];
}

[[maybe_unused]] constexpr int kCE = ISAL_HIP_CRC64_CHUNK_ENTRIES;

#ifndef ISAL_FUSED64_PART  // standalone kernels: the main object only

// Shards that are not 16-byte aligned: byte loads, one Z^4096 chain step per
// tile. Item = (stripe, shard, block), shard-major within a stripe: part index
// = ((stripe * nsh + i) * nblk + blk) * 256 + L. (Chain steps of 2 and 4
// tiles through shifted chunk maps for aligned shards — ISAL_HIP_CRC64_STEP,
// _BATCH — were superseded by crc64_shards_pre and removed in round 5.)
__global__ __launch_bounds__(kBlock) void crc64_shards_bytes(const uint64_t* __restrict__ ptrs, int ptr_stride,
                                                             int nsh, int len, unsigned nitems, unsigned nblk,
                                                             unsigned tt, unsigned nfull,
                                                             const uint64_t* __restrict__ tabs,
                                                             uint64_t* __restrict__ part) {
  __shared__ uint64_t lt[kKernTab];
  load_lds<kKernTab>(lt, tabs + ISAL_HIP_CRC64_CHUNK_TAB);
  __syncthreads();
  const long long lane = threadIdx.x * kVec;
  for (unsigned w = blockIdx.x; w < nitems; w += gridDim.x) {
    const unsigned si = w / nblk, blk = w - si * nblk;
    const unsigned stripe = si / nsh, i = si - stripe * nsh;
    const uint64_t base = ptrs[static_cast<size_t>(stripe) * ptr_stride + i];
    const unsigned t0 = blk * tt, t1 = t0 + tt < nfull ? t0 + tt : nfull;
    uint64_t a = 0;
    for (unsigned t = t0; t < t1; ++t)
      a = apply_op(lt + kShift, a) ^ chunk_crc_bytes(lt + kChunk, base, static_cast<long long>(t) * kTile + lane);
    part[static_cast<size_t>(w) * kBlock + threadIdx.x] = a;
  }
}

// Pre-shifted chains (the fused kernel's idea) on conflict-free 5-bit field
// tables: a lane keeps b = Z^4080_u(a) in the u-domain, XORs it into the next
// chunk's first 8 bytes like a CRC register and maps the chunk once, b' =
// F'_u(chunk ^ b) — 28 lookups per tile and no chain step — the item's last
// tile applies F_u and leaves the plain chain. (A form with the lookups software-pipelined,
// ISAL_HIP_CRC64_PRE_PIPE=1, ran 2.94-2.95 vs 2.82-2.85 ms on C2 — 56 lookup
// VGPRs in flight cut the occupancy from 7 to 3 waves per SIMD —
// profiles/r03/r03_crc64_prepipe_benches.jsonl; removed in round 5, as was a
// batch of 8 tiles, ISAL_HIP_CRC64_BATCH=8, measured slower.)
// Round 5: each workgroup runs TWO items, their chains interleaved step by
// step, so a lane has two independent lookup chains in flight; B = 4 tiles of
// each item are loaded together (72 VGPRs, 7 waves per SIMD). Same box, two
// interleaved rounds, C2-shaped CRC64 (profiles/r05/r05_crc64_chains_ab.txt):
// one chain with double-buffered loads 0.6542 / 0.6554 of 8 TB/s, two chains
// 0.6671 / 0.6674; 3 or 4 chains, or 2 tiles per batch, measured between or
// below (0.650-0.668).
constexpr int kPreItems = 2, kPreBatch = 4;

__global__ __launch_bounds__(kBlock) void crc64_shards_pre(const uint64_t* __restrict__ ptrs, int ptr_stride,
                                                           int nsh, int len, unsigned nitems, unsigned nblk,
                                                           unsigned tt, unsigned nfull, int uswap,
                                                           const uint64_t* __restrict__ tabs,
                                                           uint64_t* __restrict__ part) {
  constexpr int NI = kPreItems, B = kPreBatch;
  __shared__ uint64_t lt[2 * kCE];  // F_u, F'_u
  load_lds<2 * kCE>(lt, tabs + ISAL_HIP_CRC64_PRE_TAB);
  __syncthreads();
  const long long lane = threadIdx.x * kVec;
  auto step = [&](unsigned t, unsigned t1, X64 b, const uint4& x) __attribute__((always_inline)) {
    X64 c{0u, 0u};
    if (t + 1 == t1)
      chunk_acc(c, lt, x.x ^ b.lo, x.y ^ b.hi, x.z, x.w);
    else
      chunk_acc(c, lt + kCE, x.x ^ b.lo, x.y ^ b.hi, x.z, x.w);
    return c;
  };
  for (unsigned v = blockIdx.x; NI * v < nitems; v += gridDim.x) {
    uint64_t base[NI];
    unsigned t0[NI], t1[NI], n = ~0u;
    X64 bc[NI];
#pragma unroll
    for (int q = 0; q < NI; ++q) {
      const unsigned w = NI * v + q;
      base[q] = 0;
      t0[q] = t1[q] = 0;
      if (w < nitems) {
        const unsigned si = w / nblk, blk = w - si * nblk;
        const unsigned stripe = si / nsh, i = si - stripe * nsh;
        base[q] = ptrs[static_cast<size_t>(stripe) * ptr_stride + i];
        t0[q] = blk * tt;
        t1[q] = t0[q] + tt < nfull ? t0[q] + tt : nfull;
      }
      n = min(n, t1[q] - t0[q]);
      bc[q] = X64{0u, 0u};
    }
    unsigned i = 0;
    for (; i + B <= n; i += B) {
      uint4 x[NI][B];
#pragma unroll
      for (int g = 0; g < B; ++g)
#pragma unroll
        for (int q = 0; q < NI; ++q)
          x[q][g] = load16<kBufNT>(base[q], static_cast<long long>(t0[q] + i + g) * kTile + lane, len);
#pragma unroll
      for (int g = 0; g < B; ++g)
#pragma unroll
        for (int q = 0; q < NI; ++q) bc[q] = step(t0[q] + i + g, t1[q], bc[q], x[q][g]);
    }
#pragma unroll
    for (int q = 0; q < NI; ++q) {
      for (unsigned j = t0[q] + i; j < t1[q]; ++j)
        bc[q] = step(j, t1[q], bc[q], load16<kBufNT>(base[q], static_cast<long long>(j) * kTile + lane, len));
      const unsigned w = NI * v + q;
      if (w < nitems) {
        const uint64_t r = bc[q].get();
        part[static_cast<size_t>(w) * kBlock + threadIdx.x] = uswap ? __builtin_bswap64(r) : r;
      }
    }
  }
}

// Sum over L < 256 of Z^(16 * (255 - L)) v(L), lane l of a wave holding
// v(4l .. 4l + 3): a Horner step with Z^16 inside the lane, then six shuffle
// levels, level s joining lanes l and l + 2^s with Z^(64 * 2^s) (OP_TREE
// s + 2). The result is in lane 0 (lanes the result does not depend on read
// past the wave and compute garbage). No barriers: one wave per shard.
static_assert(kBlock == 256, "wave_fold: 4 lane positions per lane of a 64-lane wave");
__device__ __forceinline__ uint64_t wave_fold(const uint64_t* tree, const uint64_t (&v)[4]) {
  uint64_t h = v[0];
#pragma unroll
  for (int i = 1; i < 4; ++i) h = apply_op(tree, h) ^ v[i];
#pragma unroll
  for (int s = 0; s < 6; ++s) {
    const uint32_t lo = __shfl_down(static_cast<uint32_t>(h), 1u << s, 64);
    const uint32_t hi = __shfl_down(static_cast<uint32_t>(h >> 32), 1u << s, 64);
    h = apply_op(tree + (s + 2) * kOp, h) ^ ((static_cast<uint64_t>(hi) << 32) | lo);
  }
  return h;
}

// One wave per shard (grid-stride, four shards per workgroup at a time, the
// tables loaded once per workgroup):
//  X = raw(0, full tiles): lane l folds the block chains of lanes 4l..4l+3
//      (Horner with Z^(4096*tt), the last block Z^(4096*nfull_last)), then
//      wave_fold;
//  T = raw(0, the tail's whole 16-byte chunks): chunks right-aligned over the
//      256 lane positions, so the last chunk sits at position 255;
//  s = Z^(16q)(X) ^ T, then the last tail % 16 bytes one at a time;
//  crc64 = ~(Z^len(~init) ^ s).
// (Round 5 ran one 256-lane workgroup per shard with an 8-level LDS tree and
// a barrier per level: 0.13 ms per C2 batch, 5 % of the checksum pass.)
template <bool REFL>
__global__ __launch_bounds__(kBlock) void crc64_combine(
    const uint64_t* __restrict__ part, const uint64_t* __restrict__ ptrs, int ptr_stride, int nsh,
    int len, unsigned nblk, unsigned nfull, const uint64_t* __restrict__ tabs, uint64_t init_term,
    uint64_t* __restrict__ out, unsigned nshard_total) {
  constexpr unsigned kWaves = kBlock / 64;
  __shared__ uint64_t lt[ISAL_HIP_CRC64_COMBINE_ENTRIES];
  load_lds<ISAL_HIP_CRC64_COMBINE_ENTRIES>(lt, tabs);
  __syncthreads();
  const int tail = len - static_cast<int>(nfull) * kTile;
  const int q = tail / kVec, rem = tail - q * kVec;
  const unsigned lane = threadIdx.x & 63;
  const uint64_t* tree = lt + ISAL_HIP_CRC64_OP_TREE;
  for (unsigned sh = blockIdx.x * kWaves + (threadIdx.x >> 6); sh < nshard_total; sh += gridDim.x * kWaves) {
    const unsigned stripe = sh / nsh, i = sh - stripe * nsh;
    const uint64_t base = ptrs[static_cast<size_t>(stripe) * ptr_stride + i];
    uint64_t x = 0, tq = 0;
    if (nblk) {
      const uint64_t* pp = part + static_cast<size_t>(sh) * nblk * kBlock + 4 * lane;
      uint64_t v[4] = {0, 0, 0, 0};
      for (unsigned b = 0; b < nblk; ++b) {
        const uint64_t* op = lt + (b + 1 == nblk ? ISAL_HIP_CRC64_OP_LAST : ISAL_HIP_CRC64_OP_BLOCK);
        const uint4* p4 = reinterpret_cast<const uint4*>(pp + static_cast<size_t>(b) * kBlock);
        const uint4 a = p4[0], c = p4[1];
        const uint64_t p[4] = {(static_cast<uint64_t>(a.y) << 32) | a.x, (static_cast<uint64_t>(a.w) << 32) | a.z,
                               (static_cast<uint64_t>(c.y) << 32) | c.x, (static_cast<uint64_t>(c.w) << 32) | c.z};
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = apply_op(op, v[j]) ^ p[j];
      }
      x = wave_fold(tree, v);
    }
    if (q) {
      uint64_t v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = static_cast<int>(4 * lane) + j - (kBlock - q);  // tail chunk at this position
        v[j] = c >= 0 ? chunk_crc_bytes(lt + ISAL_HIP_CRC64_CHUNK_TAB, base,
                                        static_cast<long long>(nfull) * kTile + static_cast<long long>(c) * kVec)
                      : 0;
      }
      tq = wave_fold(tree, v);
    }
    if (lane == 0) {
      uint64_t s = x;
      if (q) s = apply_op(lt + ISAL_HIP_CRC64_OP_TAIL, s) ^ tq;
      const uint8_t* p = reinterpret_cast<const uint8_t*>(base) + (len - rem);
      for (int j = 0; j < rem; ++j) {
        if constexpr (REFL)
          s = lt[ISAL_HIP_CRC64_BYTE_TAB + ((s ^ p[j]) & 0xff)] ^ (s >> 8);
        else
          s = lt[ISAL_HIP_CRC64_BYTE_TAB + (((s >> 56) ^ p[j]) & 0xff)] ^ (s << 8);
      }
      out[sh] = ~(init_term ^ s);
    }
  }
}

constexpr unsigned long long kMaxItems = 1ull << 30;

#else  // ISAL_FUSED64_PART: one object per parity-row count P (parallel build)

// ---------------------------------------------------------------------------
// Fused encode + CRC64 (the fragment checksum in the
// encode pass). The encode half is ec_encode_v16's GF arithmetic on the same
// 16-byte lane chunks; each source chunk already in registers and each parity
// chunk about to be stored also feeds its shard's chain
//   a = Z^4096(a) ^ raw(0, chunk),
// so the stripe is read and written once. Partials land in crc64_shards'
// layout (shards 0..k-1 = sources, k..k+P-1 = parity) and crc64_combine
// finishes them, reading the ragged tail (len % 4096) straight from the
// shards: the kernel's last block encodes that tile without checksumming it.
// Source chains live in LDS (lane-private words).
// ---------------------------------------------------------------------------
template <int P, int U, bool R0 = false, class Feed>
__device__ __forceinline__ void mac_feed(uint32_t (&acc)[P][4], const uint4 (&x)[U], int j,
                                         const uint32_t* __restrict__ tbl, Feed&& feed, unsigned long long x0src = 0) {
  constexpr int PAIR = P <= 4 ? 2 : 1;
#pragma unroll
  for (int u = 0; u + PAIR <= U; u += PAIR) {
    if constexpr (PAIR == 2) {
      mac16x2<P, R0>(acc, x[u], x[u + 1], tbl + (j + u) * P * kTbl, tbl + (j + u + 1) * P * kTbl,
                     r0_mask(x0src, j + u), r0_mask(x0src, j + u + 1));
      feed(j + u, x[u]);
      feed(j + u + 1, x[u + 1]);
    } else {
      mac16<P, R0>(acc, x[u], tbl + (j + u) * P * kTbl, r0_mask(x0src, j + u));
      feed(j + u, x[u]);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  if constexpr (PAIR == 2 && (U & 1)) {
    mac16<P, R0>(acc, x[U - 1], tbl + (j + U - 1) * P * kTbl, r0_mask(x0src, j + U - 1));
    feed(j + U - 1, x[U - 1]);
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int U>
__device__ __forceinline__ void load_grp(uint4 (&x)[U], const uint64_t* __restrict__ sp, int j,
                                         long long off, int len) {
#pragma unroll
  for (int u = 0; u < U; ++u) x[u] = load16<kNT>(sp[j + u], off, len);
}

// ---- the fused kernel's chunk path: pre-shifted chains, byte tables --------
// In the u-domain (crc64_host.c: u = pi(s), one update rule u' = A(d ^ u) for
// every flavour) a lane keeps its chain PRE-SHIFTED: b = Z^4080_u(a), the
// chain advanced by the 4080 bytes of the other lanes' chunks that follow its
// own in the tile. Then the next tile's raw value is raw_u(b, chunk) — b is
// XORed into the chunk's first 8 bytes like a CRC register — and the step
// needs no separate shift map at all:
//   u1 = A(lo8 ^ b),  b' = A'(hi8 ^ u1)   (A' = Z^4080_u o A)
// and the block's last tile ends with A instead of A', leaving the plain
// chain a. 16 byte-indexed lookups per chunk, each offset one SDWA shift
// (byte select + << 3); the 256-entry tables are not bank-conflict-free (8
// entries per bank pair): VALU issue traded for LDS cycles.
//
// Formulations measured and removed (profiles/r05/r05_fused_model.txt):
// 5-bit field tables with a Z^4096 step per tile (ISAL_HIP_CRC64_SLICE=0, C2
// 4.27 ms vs 3.21), hybrid 5+3-bit tables (SLICE=2, +10 %), pre-shifted 5-bit
// field tables (SLICE=4, round 5: conflict-free but VALU-bound, 3.93 vs
// 3.34 ms same box), source chains in registers (SRC_CHAIN=reg, 5 % slower)
// and paired chain steps of the field path (FUSED_PAIR).
constexpr int kSA = 0, kSB = 8 * 256;  // A, A' in LDS
constexpr int kSlLds = 16 * 256;

// Byte b of w times 8 (an 8-byte entry's offset) in one VALU op.
__device__ __forceinline__ void byte_offs8(uint32_t w, uint32_t (&o)[4]) {
  const uint32_t three = 3;
  asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0"
      : "=v"(o[0]) : "v"(three), "v"(w));
  asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1"
      : "=v"(o[1]) : "v"(three), "v"(w));
  asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2"
      : "=v"(o[2]) : "v"(three), "v"(w));
  asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3"
      : "=v"(o[3]) : "v"(three), "v"(w));
}

__device__ __forceinline__ uint64_t tab8_at(const uint64_t* t, int j, uint32_t o) {
  return *reinterpret_cast<const uint64_t*>(reinterpret_cast<const char*>(t) + j * 2048 + o);
}

// acc ^= S(lo | hi << 32) for the slicing table set S at t (8 tables of 256).
__device__ __forceinline__ void slice8_acc(X64& acc, const uint64_t* t, uint32_t lo, uint32_t hi) {
  uint32_t o[4], q[4];
  byte_offs8(lo, o);
  byte_offs8(hi, q);
  acc.add2(tab8_at(t, 0, o[0]), tab8_at(t, 1, o[1]));
  acc.add2(tab8_at(t, 2, o[2]), tab8_at(t, 3, o[3]));
  acc.add2(tab8_at(t, 4, q[0]), tab8_at(t, 5, q[1]));
  acc.add2(tab8_at(t, 6, q[2]), tab8_at(t, 7, q[3]));
}

// One tile of a pre-shifted u-domain chain b (phase 1: the block's last tile,
// which returns the plain chain a instead).
template <int PH>
__device__ __forceinline__ uint64_t chain_step_sl(const uint64_t* lt, uint64_t b, uint32_t w0, uint32_t w1,
                                                  uint32_t w2, uint32_t w3) {
  X64 u{0u, 0u};
  X64 c{0u, 0u};
  slice8_acc(u, lt + kSA, w0 ^ static_cast<uint32_t>(b), w1 ^ static_cast<uint32_t>(b >> 32));
  slice8_acc(c, lt + (PH == 1 ? kSA : kSB), w2 ^ u.lo, w3 ^ u.hi);
  return c.get();
}

// ---- SL 3: the byte-table chain steps software-pipelined with the GF rows --
// In the SL 1 kernel the compiler emits each chain step as pairs of
// ds_read_b64 with an s_waitcnt after every pair (the byte tables conflict, so
// each wait is a full LDS round trip), after the pair's GF work: the wave
// stalls on LDS while it holds VALU work it could issue. Here a source pair's
// region is cut into stages by scheduling barriers, and each stage issues a
// chain's eight lookups of one half-step, then runs one GF row (~38 VALU) of
// independent work before folding them:
//   S   chain states of sources a, b from LDS; selectors; row 0 (masked XOR)
//       (the previous pair's b: fold -> its state); R1a: a's first 8 bytes
//   row r1 | F1a fold, R2a: a's last 8 bytes
//   row r2 | F2a fold -> a's state; R1b
//   row r3 (+ any further rows) | F1b fold, R2b (finished by the next pair)
// Same tables, same arithmetic as chain_step_sl<PH>.
struct Look8 {
  uint64_t v[8];
};

// The lookups are volatile LDS loads: a plain load is placed next to its use
// by instruction selection, before the scheduling barriers are seen, which
// would undo the stages; volatile accesses keep their order against the barriers.
__device__ __forceinline__ uint64_t tab8_issue(const uint64_t* t, int j, uint32_t o) {
  typedef const __attribute__((address_space(3))) char lchar;
  typedef const volatile __attribute__((address_space(3))) uint64_t lu64;
  return *(lu64*)((lchar*)(t) + j * 2048 + o);
}

[[maybe_unused]] __device__ __forceinline__ void issue8(Look8& r, const uint64_t* t, uint32_t lo, uint32_t hi) {
  uint32_t o[4], q[4];
  byte_offs8(lo, o);
  byte_offs8(hi, q);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    r.v[i] = tab8_issue(t, i, o[i]);
    r.v[4 + i] = tab8_issue(t, 4 + i, q[i]);
  }
}

[[maybe_unused]] __device__ __forceinline__ X64 fold8(const Look8& r) {
  X64 a{0u, 0u};
  a.add2(r.v[0], r.v[1]);
  a.add2(r.v[2], r.v[3]);
  a.add2(r.v[4], r.v[5]);
  a.add2(r.v[6], r.v[7]);
  return a;
}

// One source pair; `car` holds the previous pair's second chain, its last
// eight lookups in flight (cp = where its state goes; nullptr: none).
template <int P, bool R0, int PH>
__device__ __forceinline__ void mac_feed_pair_pipe(uint32_t (&acc)[P][4], const uint4& x, const uint4& y,
                                                   const uint32_t* __restrict__ tx,
                                                   const uint32_t* __restrict__ ty, uint32_t mx,
                                                   uint32_t my, uint64_t* pa, uint64_t* pb,
                                                   const uint64_t* lt, Look8& car, uint64_t*& cp) {
  constexpr int R = P - (R0 ? 1 : 0);  // rows through the GF lookups
  constexpr int B1 = R0 ? 1 : 0, B2 = B1 + (R + 2) / 3, B3 = B2 + (R + 1) / 3;
  const uint64_t* t2 = lt + (PH == 1 ? kSA : kSB);
  const uint64_t sa = *pa, sb = *pb;
  const Sel sx[4] = {split(x.x), split(x.y), split(x.z), split(x.w)};
  const Sel sy[4] = {split(y.x), split(y.y), split(y.z), split(y.w)};
  if constexpr (R0) {
    acc[0][0] = xor_and(xor_and(acc[0][0], x.x, mx), y.x, my);
    acc[0][1] = xor_and(xor_and(acc[0][1], x.y, mx), y.y, my);
    acc[0][2] = xor_and(xor_and(acc[0][2], x.z, mx), y.z, my);
    acc[0][3] = xor_and(xor_and(acc[0][3], x.w, mx), y.w, my);
  }
  __builtin_amdgcn_sched_barrier(0);
  if (cp) *cp = fold8(car).get();
  Coef ca[P], cb[P];
  load_coefs<P, B1>(ca, tx);
  load_coefs<P, B1>(cb, ty);
  have_coefs<P, B1>(ca);
  have_coefs<P, B1>(cb);
  __builtin_amdgcn_sched_barrier(0);
  issue8(car, lt + kSA, x.x ^ static_cast<uint32_t>(sa), x.y ^ static_cast<uint32_t>(sa >> 32));
  __builtin_amdgcn_sched_barrier(0);
  mac_rows2<P, B1, B2>(acc, sx, sy, ca, cb);
  __builtin_amdgcn_sched_barrier(0);
  const X64 ua = fold8(car);
  issue8(car, t2, x.z ^ ua.lo, x.w ^ ua.hi);
  __builtin_amdgcn_sched_barrier(0);
  mac_rows2<P, B2, B3>(acc, sx, sy, ca, cb);
  __builtin_amdgcn_sched_barrier(0);
  *pa = fold8(car).get();
  issue8(car, lt + kSA, y.x ^ static_cast<uint32_t>(sb), y.y ^ static_cast<uint32_t>(sb >> 32));
  __builtin_amdgcn_sched_barrier(0);
  mac_rows2<P, B3, P>(acc, sx, sy, ca, cb);
  __builtin_amdgcn_sched_barrier(0);
  const X64 ub = fold8(car);
  issue8(car, t2, y.z ^ ub.lo, y.w ^ ub.hi);
  cp = pb;
  __builtin_amdgcn_sched_barrier(0);
}

// U sources j..j+U-1 (U even, P <= 4) with LDS chain states at la (row stride
// kLa): one chain's eight lookups in flight at a time, the last pair's second
// chain finishing behind the next pair's selectors and row 0.
template <int P, int U, bool R0, int PH>
__device__ __forceinline__ void mac_feed_pipe(uint32_t (&acc)[P][4], const uint4 (&x)[U], int j,
                                              const uint32_t* __restrict__ tbl, uint64_t* la, int kLa,
                                              const uint64_t* lt, unsigned long long x0src) {
  static_assert(U % 2 == 0 && P <= 4, "pairs of sources, tables of both in SGPRs");
  Look8 car;
  uint64_t* cp = nullptr;
#pragma unroll
  for (int u = 0; u < U; u += 2)
    mac_feed_pair_pipe<P, R0, PH>(acc, x[u], x[u + 1], tbl + (j + u) * P * kTbl,
                                  tbl + (j + u + 1) * P * kTbl, r0_mask(x0src, j + u),
                                  r0_mask(x0src, j + u + 1), la + (j + u) * kLa,
                                  la + (j + u + 1) * kLa, lt, car, cp);
  *cp = fold8(car).get();
}

template <int P, int U>
constexpr int fused64_waves() {
  constexpr int est = (4 * U + 6 * P + 88 + 7) / 8 * 8;
  constexpr int w = 512 / est;
  return w > 8 ? 8 : (w < 2 ? 2 : w);
}

// X0: parity row 0 has only 0/1 coefficients (RS Vandermonde row 0, RAID P):
// it is the XOR of the sources in x0src, so (CRC being GF(2)-linear) its
// chain is not computed per tile but formed once per block from those
// sources' chains. A compile-time variant: a runtime row mask in the tile
// loop costs registers.
// SL 3: the chain steps pipelined into the GF rows (load group 10, P <= 4);
// SL 1: the same steps after each source pair's GF work. Chains in the
// u-domain; uswap (norm flavours) turns them back into registers (u =
// bswap(s)) before they are stored.
// NV: independent 256-lane groups per workgroup. They share one LDS copy of the
// tables (each works its own items, no barrier after the table load), so the
// per-lane source chains, not the tables, set how many waves fit a CU.
template <int P, int U, bool X0, int SL, int NV>
__global__ __launch_bounds__(kBlock * NV, (fused64_waves<P, U>())) void ec_encode_crc64_v16(
    const uint64_t* __restrict__ ptrs, int ptr_stride, const uint32_t* __restrict__ tbl, int len,
    int k, unsigned nitems, unsigned nblk, unsigned tt, unsigned nfull, int ragged,
    unsigned long long x0src, int uswap, const uint64_t* __restrict__ tabs, uint64_t* __restrict__ part) {
  static_assert(SL == 1 || SL == 3, "byte-table chunk paths");
  __shared__ uint64_t lt[kSlLds];
  extern __shared__ uint64_t la[];  // [k][kBlock * NV] source chains
  load_lds<kSlLds, NV>(lt, tabs + ISAL_HIP_CRC64_SLICE_TAB);
  constexpr int kLa = kBlock * NV;           // source-chain row stride
  const unsigned tid = threadIdx.x % kBlock;  // lane within its group
  __syncthreads();
  auto to_reg = [&](uint64_t v) __attribute__((always_inline)) { return uswap ? __builtin_bswap64(v) : v; };
  const int nsh = k + P;
  const long long lane = tid * kVec;
  for (unsigned w = blockIdx.x * NV + threadIdx.x / kBlock; w < nitems; w += gridDim.x * NV) {
    const unsigned stripe = w / nblk, blk = w - stripe * nblk;
    const uint64_t* __restrict__ sp = ptrs + static_cast<size_t>(stripe) * ptr_stride;
    const unsigned t0 = blk * tt, t1 = t0 + tt < nfull ? t0 + tt : nfull;
    uint64_t ao[P];
#pragma unroll
    for (int l = 0; l < P; ++l) ao[l] = 0;
    for (int j = 0; j < k; ++j) la[j * kLa + threadIdx.x] = 0;
    // phase 1 marks the block's last tile (it returns the plain chain)
    auto with_phase = [&](bool last, auto&& body) __attribute__((always_inline)) {
      if (last)
        body(std::integral_constant<int, 1>{});
      else
        body(std::integral_constant<int, 0>{});
    };
    for (unsigned t = t0; t < t1; ++t) {
      const long long off = static_cast<long long>(t) * kTile + lane;
      uint32_t acc[P][4] = {};
      int z = 0;  // opaque zero: keeps the coefficient loads inside the loop
      asm volatile("" : "+s"(z));
      with_phase(t + 1 == t1, [&](auto phc) __attribute__((always_inline)) {
        constexpr int PH = decltype(phc)::value;
        auto feed = [&](int j, const uint4& x) __attribute__((always_inline)) {
          uint64_t* a = la + j * kLa + threadIdx.x;
          *a = chain_step_sl<PH>(lt, *a, x.x, x.y, x.z, x.w);
        };
        int j = 0;
        for (; j + U <= k; j += U) {
          uint4 x[U];
          load_grp<U>(x, sp, j, off, len);
          if constexpr (SL == 3)
            mac_feed_pipe<P, U, X0, PH>(acc, x, j, tbl + z, la + threadIdx.x, kLa, lt, x0src);
          else
            mac_feed<P, U, X0>(acc, x, j, tbl + z, feed, x0src);
        }
        for (; j < k; ++j) {
          uint4 x[1];
          load_grp<1>(x, sp, j, off, len);
          mac_feed<P, 1, X0>(acc, x, j, tbl + z, feed, x0src);
        }
#pragma unroll
        for (int l = 0; l < P; ++l) {
          store16<kNT>(sp[k + l], off, make_uint4(acc[l][0], acc[l][1], acc[l][2], acc[l][3]), len);
          if (!(X0 && l == 0)) ao[l] = chain_step_sl<PH>(lt, ao[l], acc[l][0], acc[l][1], acc[l][2], acc[l][3]);
        }
      });
    }
    if (ragged && blk + 1 == nblk) {  // encode the tail tile; combine checksums it
      const long long off = static_cast<long long>(nfull) * kTile + lane;
      if (off + kVec <= len) {
        uint32_t acc[P][4] = {};
        auto none = [](int, const uint4&) {};
        for (int j = 0; j < k; ++j) {
          uint4 x[1];
          load_grp<1>(x, sp, j, off, len);
          mac_feed<P, 1, X0>(acc, x, j, tbl, none, x0src);
        }
#pragma unroll
        for (int l = 0; l < P; ++l)
          store16<kNT>(sp[k + l], off, make_uint4(acc[l][0], acc[l][1], acc[l][2], acc[l][3]), len);
      }
    }
    if constexpr (X0) {  // row 0 = XOR of the sources in x0src: so is its chain
      uint64_t v = 0;
      for (int j = 0; j < k; ++j)
        if ((x0src >> j) & 1ull) v ^= la[j * kLa + threadIdx.x];
      ao[0] = v;
    }
    uint64_t* pp = part + (static_cast<size_t>(stripe) * nsh * nblk + blk) * kBlock + tid;
    const size_t sstep = static_cast<size_t>(nblk) * kBlock;
    for (int j = 0; j < k; ++j) pp[j * sstep] = to_reg(la[j * kLa + threadIdx.x]);
#pragma unroll
    for (int l = 0; l < P; ++l) pp[(k + l) * sstep] = to_reg(ao[l]);
  }
}

// Sources per load group of the fused kernel: the largest candidate dividing k.
int group_u(int k) {
  static const int cand[] = {12, 10, 8, 6, 5, 4};
  for (int u : cand)
    if (k >= u && k % u == 0) return u;
  return 4;
}

// 256-lane groups per workgroup: 2 when that fits more lane groups on a CU
// (160 KiB of LDS; the tables are shared by a workgroup, the source chains are
// per lane). The pipelined path holds 140 VGPRs (3 waves per SIMD): a 512-lane
// workgroup (8 waves) would leave one workgroup, 2 waves per SIMD, per CU.
int fused_nv(int sl, int k) {
  const size_t cap = 160 * 1024, tabs = static_cast<size_t>(kSlLds) * 8,
               la = static_cast<size_t>(k) * kBlock * 8;
  if (tabs + 2 * la >= cap) return 1;  // leave LDS headroom: never the whole 160 KiB
  if (sl == 3) return 1;
  return 2 * (cap / (tabs + 2 * la)) > cap / (tabs + la) ? 2 : 1;
}

// The chain steps pipelined into the GF rows (SL 3) for load group U = 10 and
// P <= 4 — C2 step 3.386 -> 3.305 ms (profiles/r03/r03_pipe64_benches.jsonl);
// elsewhere after each pair's GF work (SL 1).
template <int P, int U>
void launch_fused64(unsigned grid, hipStream_t s, const uint64_t* ptrs, int ptr_stride,
                    const uint32_t* tbl, int len, int k, unsigned nitems,
                    const isal_hip_crc64_geom& g, const isal_hip_xrows& xr, int refl,
                    const uint64_t* tabs, uint64_t* part) {
  const int ragged = g.tail != 0;
  const size_t lds = static_cast<size_t>(k) * kBlock * 8;
#define FUSED64_LAUNCH(X0, SL, NV)                                                                 \
  ISAL_LAUNCH((ec_encode_crc64_v16<P, U, X0, SL, NV>), dim3((grid + NV - 1) / NV),           \
                     dim3(kBlock * NV), lds * NV, s, ptrs, ptr_stride, tbl, len, k, nitems,         \
                     static_cast<unsigned>(g.nblk), static_cast<unsigned>(g.tt),                    \
                     static_cast<unsigned>(g.nfull), ragged, xr.src[0], !refl, tabs, part)
#define FUSED64_X0(SL, NV)                                                                        \
  do {                                                                                            \
    if (xr.rows & 1u) FUSED64_LAUNCH(true, SL, NV); else FUSED64_LAUNCH(false, SL, NV);           \
  } while (0)
  if constexpr (U == 10 && P <= 4) {
    FUSED64_X0(3, 1);
  } else {
    if (fused_nv(1, k) == 2) FUSED64_X0(1, 2); else FUSED64_X0(1, 1);
  }
#undef FUSED64_X0
#undef FUSED64_LAUNCH
}

template <int P>
void fused64_pass(unsigned grid, hipStream_t s, const uint64_t* ptrs, int ptr_stride,
                  const uint32_t* tbl, int len, int k, unsigned nitems,
                  const isal_hip_crc64_geom& g, const isal_hip_xrows& xr, int refl,
                  const uint64_t* tabs, uint64_t* part) {
  switch (group_u(k)) {
#define FUSED64_U(u) \
  case u: launch_fused64<P, u>(grid, s, ptrs, ptr_stride, tbl, len, k, nitems, g, xr, refl, tabs, part); break;
    FUSED64_U(12) FUSED64_U(10) FUSED64_U(8) FUSED64_U(6) FUSED64_U(5)
#undef FUSED64_U
    default: launch_fused64<P, 4>(grid, s, ptrs, ptr_stride, tbl, len, k, nitems, g, xr, refl, tabs, part);
  }
}

// The fused kernels of one P live in their own object (crc64_fused_pP.o, this
// file compiled with -DISAL_FUSED64_PART=P): the (P, U, REG, X0, SL) variants
// of all eight P in one translation unit took the compiler over 20 minutes.
}  // namespace

#define FUSED64_PART_FN2(p) isal_hip_fused64_part_##p
#define FUSED64_PART_FN(p) FUSED64_PART_FN2(p)
extern "C" void FUSED64_PART_FN(ISAL_FUSED64_PART)(
    unsigned nitems, hipStream_t s, const uint64_t* ptrs, int nsh, const uint32_t* tbl, int len,
    int k, const isal_hip_crc64_geom* g, const isal_hip_xrows* xr, int refl, const uint64_t* tabs,
    uint64_t* part) {
  fused64_pass<ISAL_FUSED64_PART>(nitems, s, ptrs, nsh, tbl, len, k, nitems, *g, *xr, refl, tabs,
                                  part);
}

#endif  // ISAL_FUSED64_PART

#ifndef ISAL_FUSED64_PART

int launch_combine64(const uint64_t* part, const uint64_t* ptrs, int ptr_stride, int nsh, int len,
                     const isal_hip_crc64_geom& g, int refl, const uint64_t* tabs,
                     uint64_t init_term, uint64_t* out, unsigned nshard, hipStream_t s) {
  // four shards per workgroup at a time; each workgroup copies the 52 KB
  // table set once, so the grid is capped at what is resident (3 per CU)
  const unsigned want = (nshard + 3) / 4, grid = want < 768 ? want : 768;
  if (refl)
    ISAL_LAUNCH(crc64_combine<true>, dim3(grid), dim3(kBlock), 0, s, part, ptrs, ptr_stride,
                       nsh, len, static_cast<unsigned>(g.nblk), static_cast<unsigned>(g.nfull),
                       tabs, init_term, out, nshard);
  else
    ISAL_LAUNCH(crc64_combine<false>, dim3(grid), dim3(kBlock), 0, s, part, ptrs, ptr_stride,
                       nsh, len, static_cast<unsigned>(g.nblk), static_cast<unsigned>(g.nfull),
                       tabs, init_term, out, nshard);
  isal_hip_count_launch();
  return static_cast<int>(hipGetLastError());
}

}  // namespace

// Fused encode+CRC64 launchers, one object per P (crc64_fused_pP.o).
#define FUSED64_PART_DECL(p)                                                                     \
  extern "C" void isal_hip_fused64_part_##p(unsigned nitems, hipStream_t s, const uint64_t* ptrs, \
                                            int nsh, const uint32_t* tbl, int len, int k,       \
                                            const isal_hip_crc64_geom* g,                       \
                                            const isal_hip_xrows* xr, int refl,                 \
                                            const uint64_t* tabs, uint64_t* part);
FUSED64_PART_DECL(1) FUSED64_PART_DECL(2) FUSED64_PART_DECL(3) FUSED64_PART_DECL(4)
FUSED64_PART_DECL(5) FUSED64_PART_DECL(6) FUSED64_PART_DECL(7) FUSED64_PART_DECL(8)
#undef FUSED64_PART_DECL

extern "C" int isal_hip_launch_crc64(const uint64_t* d_ptrs, int ptr_stride, int nsh,
                                     long long nstripes, int len, int vec16, int refl, int tt,
                                     const uint64_t* d_tabs, uint64_t* d_part, uint64_t init_term,
                                     uint64_t* out, void* stream) {
  if (len < 0 || nsh <= 0 || nstripes <= 0) return 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  isal_hip_crc64_geom g;
  isal_hip_crc64_geometry(len, tt, &g);
  const unsigned long long per_stripe = static_cast<unsigned long long>(nsh) * (g.nblk ? g.nblk : 1);
  const long long per = kMaxItems / per_stripe > 0 ? static_cast<long long>(kMaxItems / per_stripe) : 1;
  for (long long s0 = 0; s0 < nstripes; s0 += per) {
    const long long ns = nstripes - s0 < per ? nstripes - s0 : per;
    const uint64_t* ptrs = d_ptrs + s0 * ptr_stride;
    const unsigned nshard = static_cast<unsigned>(ns * nsh);
    uint64_t* part = d_part + static_cast<size_t>(s0) * nsh * g.nblk * kBlock;
    if (g.nblk) {
      const unsigned nitems = static_cast<unsigned>(ns * nsh * g.nblk);
      if (vec16)
        ISAL_LAUNCH(crc64_shards_pre, dim3((nitems + kPreItems - 1) / kPreItems), dim3(kBlock), 0, s, ptrs,
                           ptr_stride, nsh, len, nitems, static_cast<unsigned>(g.nblk), static_cast<unsigned>(g.tt),
                           static_cast<unsigned>(g.nfull), !refl, d_tabs, part);
      else
        ISAL_LAUNCH(crc64_shards_bytes, dim3(nitems), dim3(kBlock), 0, s, ptrs, ptr_stride, nsh, len, nitems,
                           static_cast<unsigned>(g.nblk), static_cast<unsigned>(g.tt),
                           static_cast<unsigned>(g.nfull), d_tabs, part);
      isal_hip_count_launch();
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) return static_cast<int>(e);
    }
    const int e = launch_combine64(part, ptrs, ptr_stride, nsh, len, g, refl, d_tabs, init_term,
                                   out + s0 * nsh, nshard, s);
    if (e) return e;
  }
  return 0;
}

extern "C" int isal_hip_launch_encode_crc64(const uint64_t* d_ptrs, int k, int rows,
                                            long long nstripes, int len, const uint32_t* d_tbl,
                                            const isal_hip_xrows* xrp, int refl, int tt,
                                            const uint64_t* d_tabs, uint64_t* d_part,
                                            uint64_t init_term, uint64_t* out, void* stream) {
  if (nstripes <= 0) return 0;
  isal_hip_xrows xr{};
  if (xrp) xr = *xrp;
  isal_hip_crc64_geom g;
  isal_hip_crc64_geometry(len, tt, &g);
  if (len % kVec || g.nblk == 0 || rows < 1 || rows > EC_MAX_ROWS_PER_PASS || k < 1 ||
      k > ISAL_HIP_CRC64_MAX_FUSED_K)
    return static_cast<int>(hipErrorInvalidValue);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int nsh = k + rows;
  const long long per = static_cast<long long>(kMaxItems / g.nblk) > 0
                            ? static_cast<long long>(kMaxItems / g.nblk) : 1;
  for (long long s0 = 0; s0 < nstripes; s0 += per) {
    const long long ns = nstripes - s0 < per ? nstripes - s0 : per;
    const unsigned nitems = static_cast<unsigned>(ns * g.nblk);
    const uint64_t* ptrs = d_ptrs + s0 * nsh;
    uint64_t* part = d_part + static_cast<size_t>(s0) * nsh * g.nblk * kBlock;
    switch (rows) {
#define FUSED64_P(p) \
  case p: isal_hip_fused64_part_##p(nitems, s, ptrs, nsh, d_tbl, len, k, &g, &xr, refl, d_tabs, part); break;
      FUSED64_P(1) FUSED64_P(2) FUSED64_P(3) FUSED64_P(4) FUSED64_P(5) FUSED64_P(6) FUSED64_P(7)
      FUSED64_P(8)
#undef FUSED64_P
    }
    isal_hip_count_launch();
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return static_cast<int>(e);
    const int r = launch_combine64(part, ptrs, nsh, nsh, len, g, refl, d_tabs, init_term,
                                   out + s0 * nsh, static_cast<unsigned>(ns * nsh), s);
    if (r) return r;
  }
  return 0;
}

#endif  // !ISAL_FUSED64_PART