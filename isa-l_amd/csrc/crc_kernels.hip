// crc_kernels.hip — CRC32C (the reference's crc32_iscsi, crc/crc_base.c:205-219)
// of erasure-code shards on gfx950, standalone and fused into the encode pass.
//
// storage callers checksum every fragment right after
// encoding (include/crc.h:137). Reading the k sources and writing the parity a
// second time just to checksum them would double the HBM traffic of the stripe,
// so the fused kernel computes the CRCs of all k + rows shards from the same
// registers the encode already holds.
//
// Algorithm (GF(2)-linear CRC, constants from crc_host.c):
//  * lane L of a workgroup owns bytes [16L, 16L+16) of each 4 KiB tile (the
//    encode kernel's layout); crc(0, chunk) = XOR_i T_{15-i}[b_i] with 16 slice
//    tables in LDS (one ds_read_b32 per byte);
//  * across the workgroup's `tt` consecutive tiles the lane chains its chunks:
//    a = Z^4096(a) ^ crc(0, chunk)  (four byte-table lookups);
//  * the lane's chain is a partial (part[], 1 dword per 16*tt bytes: 0.4 % extra
//    writes at tt = 16); crc32c_combine joins the partials of a shard with
//    Horner across workgroups, one multiply per lane to the shard end and a
//    block XOR-reduction, then adds Z^len(init_crc).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <type_traits>

#include "ec_device.h"

namespace {

constexpr uint32_t kCrcPoly = 0x82F63B78u;
constexpr int kCrcTabDw = ISAL_HIP_CRC_TAB_DWORDS;

static_assert(ISAL_HIP_CRC_TILE == kTile, "CRC tile = encode tile");

__device__ __forceinline__ void load_crc_tables(uint32_t* lt, const uint32_t* __restrict__ tabs) {
  const uint4* src = reinterpret_cast<const uint4*>(tabs);
  uint4* dst = reinterpret_cast<uint4*>(lt);
  for (int i = threadIdx.x; i < kCrcTabDw / 4; i += kBlock) dst[i] = src[i];
  __syncthreads();
}

// Byte offsets (entry index * 4) of the 7 fields of w, bits [0,5) [5,10)
// [10,15) [15,20) [20,25) [25,30) [30,32): 11 VALU ops for 7 lookups. Shifting
// w left by 2 puts every field at its entry's byte offset; masking the even
// and the odd fields into separate words leaves two zero bits below each
// field, so one bit-field extract yields the offset.
// One v_bfe_u32. (Through the builtin, LLVM sees that the two low bits are
// zero, narrows the mask to a non-contiguous one and emits shift + and.)
template <int OFF, int WIDTH>
__device__ __forceinline__ uint32_t bfe(uint32_t x) {
  uint32_t r;
  asm("v_bfe_u32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "n"(OFF), "n"(WIDTH));
  return r;
}

__device__ __forceinline__ void field_offsets(uint32_t w, uint32_t (&o)[ISAL_HIP_CRC_FIELDS]) {
  const uint32_t s = w << 2;
  const uint32_t ev = s & 0x07C1F07Cu;  // fields 0, 2, 4 at [2,7) [12,17) [22,27)
  const uint32_t od = s & 0xF83E0F80u;  // fields 1, 3, 5 at [7,12) [17,22) [27,32)
  o[0] = ev & 0x7Cu;
  o[1] = bfe<5, 7>(od);
  o[2] = bfe<10, 7>(ev);
  o[3] = bfe<15, 7>(od);
  o[4] = bfe<20, 7>(ev);
  o[5] = bfe<25, 7>(od);
  o[6] = (w >> 28) & 0xCu;
}

// XOR of the 7 field lookups of w in the 7 consecutive 32-entry tables at t.
__device__ __forceinline__ uint32_t lookup7(const uint32_t* t, uint32_t w) {
  uint32_t o[ISAL_HIP_CRC_FIELDS];
  field_offsets(w, o);
  const char* b = reinterpret_cast<const char*>(t);
  auto at = [&](int f) { return *reinterpret_cast<const uint32_t*>(b + f * 128 + o[f]); };
  return xor3(xor3(at(0), at(1), at(2)), xor3(at(3), at(4), at(5)), at(6));
}

// The chunk map whose 28 field tables start at t, applied to a 16-byte chunk.
__device__ __forceinline__ uint32_t chunk_map(const uint32_t* t, uint32_t w0, uint32_t w1,
                                              uint32_t w2, uint32_t w3) {
  constexpr int D = ISAL_HIP_CRC_FIELDS * 32;  // tables per dword of the chunk
  return xor3(lookup7(t, w0), lookup7(t + D, w1), lookup7(t + 2 * D, w2)) ^ lookup7(t + 3 * D, w3);
}

// crc(0, 16 bytes): 28 conflict-free lookups.
__device__ __forceinline__ __attribute__((unused)) uint32_t chunk_crc(const uint32_t* lt, uint32_t w0, uint32_t w1,
                                              uint32_t w2, uint32_t w3) {
  return chunk_map(lt + ISAL_HIP_CRC_CHUNK_TAB, w0, w1, w2, w3);
}

[[maybe_unused]] __device__ __forceinline__ uint32_t chunk_crc(const uint32_t* lt, const uint4& x) {
  return chunk_crc(lt, x.x, x.y, x.z, x.w);
}

// Z^4096(a): the chain value followed by one tile of zero bytes.
__device__ __forceinline__ uint32_t shift_tile(const uint32_t* lt, uint32_t a) {
  return lookup7(lt + ISAL_HIP_CRC_SHIFT_TAB, a);
}

// ---- byte-indexed path with pre-shifted chains (NB = 4) --------------------
// The fused kernels are VALU-issue-bound: a 5-bit field lookup
// costs ~1.6 VALU for its offset, and every tile also pays a 7-lookup Z^4096
// chain step. Here a lane keeps its chain PRE-SHIFTED, b = Z^4080(a): the
// chain advanced past the 4080 bytes of the other lanes' chunks that follow
// its own in the tile. The next tile's raw CRC is then crc(b, chunk) — b is
// XORed into the chunk's first dword like a CRC register — so a step is one
// map of the 16 chunk bytes, through byte-position tables:
//   b' = P'(w0 ^ b, w1, w2, w3)   P' = Z^4080 o P   (P: crc(0, chunk) per byte)
// and the block's last tile applies P instead, leaving the plain chain a.
// 16 byte lookups per chunk, each offset one SDWA shift (byte select + << 2),
// no chain step; the 256-entry tables are not bank-conflict-free (8 entries
// per bank): VALU issue traded for LDS cycles. LDS: P at 0, P' at 4096 dwords.
[[maybe_unused]] constexpr int kPos = 0, kPosZ = 16 * 256, kPosLds = 32 * 256;

__device__ __forceinline__ void byte_offs4(uint32_t w, uint32_t (&o)[4]) {
  const uint32_t two = 2;
  asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0"
      : "=v"(o[0]) : "v"(two), "v"(w));
  asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1"
      : "=v"(o[1]) : "v"(two), "v"(w));
  asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2"
      : "=v"(o[2]) : "v"(two), "v"(w));
  asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3"
      : "=v"(o[3]) : "v"(two), "v"(w));
}

// r ^= the 4 byte lookups of dword d of a chunk in the position tables at t.
__device__ __forceinline__ __attribute__((unused)) uint32_t lookup4b(uint32_t r, const uint32_t* t,
                                                                    int d, uint32_t w) {
  uint32_t o[4];
  byte_offs4(w, o);
  const char* b = reinterpret_cast<const char*>(t + d * 1024);
  auto at = [&](int j) { return *reinterpret_cast<const uint32_t*>(b + j * 1024 + o[j]); };
  return xor3(xor3(r, at(0), at(1)), at(2), at(3));
}

// One tile of a pre-shifted chain b (LAST: the block's last tile, which
// returns the plain chain; b = 0 gives crc(0, chunk)).
template <bool LAST>
__device__ __forceinline__ __attribute__((unused)) uint32_t pre_step(const uint32_t* lt, uint32_t b,
                                                                    uint32_t w0, uint32_t w1,
                                                                    uint32_t w2, uint32_t w3) {
  const uint32_t* t = lt + (LAST ? kPos : kPosZ);
  uint32_t r = lookup4b(0u, t, 0, w0 ^ b);
  r = lookup4b(r, t, 1, w1);
  r = lookup4b(r, t, 2, w2);
  return lookup4b(r, t, 3, w3);
}

// crc(0, nb bytes) one byte at a time (the lane that straddles len).
__device__ __forceinline__ __attribute__((unused)) uint32_t bytes_crc(const uint32_t* lt, const uint8_t* p, int nb) {
  uint32_t c = 0;
  for (int i = 0; i < nb; ++i) c = (c >> 8) ^ lt[(c ^ p[i]) & 0xff];
  return c;
}

// a * b mod P (reflected; bit 31 = x^0), as isal_hip_crc32c_mulmod.
__device__ __forceinline__ __attribute__((unused)) uint32_t crc_mulmod(uint32_t a, uint32_t b) {
  uint32_t p = 0;
#pragma unroll 8
  for (int i = 0; i < 32; ++i) {
    p ^= (a & 0x80000000u) ? b : 0u;
    a <<= 1;
    b = (b >> 1) ^ ((b & 1u) ? kCrcPoly : 0u);
  }
  return p;
}

#ifndef ISAL_FUSED_PART  // standalone kernels and the combine: the main object only

// ---------------------------------------------------------------------------
// Standalone: partials of nsh shards per stripe. Item = (stripe, shard, block).
// VEC: 16-byte aligned shards (one dwordx4 per lane and tile); otherwise byte loads.
// ---------------------------------------------------------------------------
// Full tiles are read kCrcBatch at a time (all loads issued before any lookup):
// one 16-byte load in flight per lane leaves the kernel latency-bound. Batches
// of 4 (71 VGPRs, 7 waves per SIMD) beat 8 (111, 4) and 6 (93, 5) on the C2
// shape: 0.7529 / 0.7576 -> 0.7620 / 0.7631 of 8 TB/s, two interleaved rounds
// (profiles/r05/r05_crc_batch_ab.txt): the table lookups overlap the VALU
// better with more waves.
constexpr unsigned kCrcBatch = 4;

// Shards that are not 16-byte aligned (byte loads, one Z^4096 chain step per
// tile); aligned shards take crc32c_shards_pre below. (A chain step of four
// tiles through the shifted chunk maps measured 2.90 vs 2.87 ms per C2 step,
// profiles/r01/r01_crc_step_sweep.txt; it and its knob were removed in round 5.)
__global__ __launch_bounds__(kBlock) void crc32c_shards_bytes(
    const uint64_t* __restrict__ ptrs, int ptr_stride, int idx0, int nsh, int len,
    unsigned nitems, unsigned nblk, unsigned tt, unsigned nfull, unsigned ntiles,
    const uint32_t* __restrict__ tabs, uint32_t* __restrict__ part, uint32_t* __restrict__ tail,
    int nshard_total, int shard0) {
  __shared__ uint32_t lt[kCrcTabDw];
  load_crc_tables(lt, tabs);
  for (unsigned w = blockIdx.x; w < nitems; w += gridDim.x) {
    const unsigned si = w / nblk, blk = w - si * nblk;
    const unsigned stripe = si / nsh, i = si - stripe * nsh;
    const uint64_t base = ptrs[static_cast<size_t>(stripe) * ptr_stride + idx0 + i];
    const size_t shard = static_cast<size_t>(stripe) * nshard_total + shard0 + i;
    const unsigned t0 = blk * tt, t1 = t0 + tt < ntiles ? t0 + tt : ntiles;
    uint32_t a = 0;
    for (unsigned t = t0; t < t1; ++t) {
      const long long off = static_cast<long long>(t) * kTile + threadIdx.x * kVec;
      const long long left = len - off;
      const int nb = left >= kVec ? kVec : (left > 0 ? static_cast<int>(left) : 0);
      uint32_t c = 0;
      if (nb == kVec) {
        const uint8_t* p = reinterpret_cast<const uint8_t*>(base) + off;
        uint32_t v[4];
#pragma unroll
        for (int d = 0; d < 4; ++d)
          v[d] = p[4 * d] | (p[4 * d + 1] << 8) | (p[4 * d + 2] << 16) | (static_cast<uint32_t>(p[4 * d + 3]) << 24);
        c = chunk_crc(lt, v[0], v[1], v[2], v[3]);
      } else if (nb > 0) {
        c = bytes_crc(lt, reinterpret_cast<const uint8_t*>(base) + off, nb);
      }
      if (t < nfull)
        a = shift_tile(lt, a) ^ c;
      else
        tail[shard * kBlock + threadIdx.x] = c;
    }
    part[(shard * nblk + blk) * kBlock + threadIdx.x] = a;
  }
}

// Pre-shifted chains on the conflict-free field tables (see pre_step): a lane
// keeps b = Z^4080(a), XORs it into the next chunk's first dword like a CRC
// register and maps the chunk once, b' = F'(w0 ^ b, w1, w2, w3) — 28 lookups
// per tile and no Z^4096 step (35 before) — the block's last full tile applies
// F (crc(0, chunk)) and leaves the plain chain. Double-buffered loads as above.
// LDS: T0 (tail bytes), F (the CHUNK tables), F' (ISAL_HIP_CRC_FPRE_TAB).
constexpr int kPreF = ISAL_HIP_CRC_CHUNK_TAB, kPreFZ = kPreF + ISAL_HIP_CRC_CHUNK_DWORDS;

__global__ __launch_bounds__(kBlock) void crc32c_shards_pre(
    const uint64_t* __restrict__ ptrs, int ptr_stride, int idx0, int nsh, int len,
    unsigned nitems, unsigned nblk, unsigned tt, unsigned nfull, unsigned ntiles,
    const uint32_t* __restrict__ tabs, uint32_t* __restrict__ part, uint32_t* __restrict__ tail,
    int nshard_total, int shard0) {
  __shared__ uint32_t lt[kPreFZ + ISAL_HIP_CRC_CHUNK_DWORDS];
  for (int i = threadIdx.x; i < kPreFZ; i += kBlock) lt[i] = tabs[i];
  for (int i = threadIdx.x; i < ISAL_HIP_CRC_CHUNK_DWORDS; i += kBlock)
    lt[kPreFZ + i] = tabs[ISAL_HIP_CRC_FPRE_TAB + i];
  __syncthreads();
  const long long lane = threadIdx.x * kVec;
  auto step = [&](unsigned t, unsigned tf, uint32_t b, const uint4& x) __attribute__((always_inline)) {
    return t + 1 == tf ? chunk_map(lt + kPreF, x.x ^ b, x.y, x.z, x.w)
                       : chunk_map(lt + kPreFZ, x.x ^ b, x.y, x.z, x.w);
  };
  for (unsigned w = blockIdx.x; w < nitems; w += gridDim.x) {
    const unsigned si = w / nblk, blk = w - si * nblk;
    const unsigned stripe = si / nsh, i = si - stripe * nsh;
    const uint64_t base = ptrs[static_cast<size_t>(stripe) * ptr_stride + idx0 + i];
    const size_t shard = static_cast<size_t>(stripe) * nshard_total + shard0 + i;
    const unsigned t0 = blk * tt, t1 = t0 + tt < ntiles ? t0 + tt : ntiles;
    const unsigned tf = t1 < nfull ? t1 : nfull;  // full tiles of this block
    uint32_t b = 0;
    unsigned t = t0;
    uint4 xn[kCrcBatch];
    if (t + kCrcBatch <= tf) {
#pragma unroll
      for (unsigned g = 0; g < kCrcBatch; ++g)
        xn[g] = load16<kBufNT>(base, static_cast<long long>(t + g) * kTile + lane, len);
    }
    for (; t + kCrcBatch <= tf; t += kCrcBatch) {
      uint4 x[kCrcBatch];
#pragma unroll
      for (unsigned g = 0; g < kCrcBatch; ++g) x[g] = xn[g];
      if (t + 2 * kCrcBatch <= tf) {
#pragma unroll
        for (unsigned g = 0; g < kCrcBatch; ++g)
          xn[g] = load16<kBufNT>(base, static_cast<long long>(t + kCrcBatch + g) * kTile + lane, len);
      }
#pragma unroll
      for (unsigned g = 0; g < kCrcBatch; ++g) b = step(t + g, tf, b, x[g]);
    }
    for (; t < tf; ++t) b = step(t, tf, b, load16<kBufNT>(base, static_cast<long long>(t) * kTile + lane, len));
    if (tf < t1) {  // the ragged tile: its chunk CRCs go to tail[]
      const long long off = static_cast<long long>(tf) * kTile + lane;
      const long long left = len - off;
      const int nb = left >= kVec ? kVec : (left > 0 ? static_cast<int>(left) : 0);
      uint32_t c = 0;
      if (nb == kVec) {
        const uint4 x = load16<kBufNT>(base, off, len);
        c = chunk_map(lt + kPreF, x.x, x.y, x.z, x.w);
      } else if (nb > 0) {
        c = bytes_crc(lt, reinterpret_cast<const uint8_t*>(base) + off, nb);
      }
      tail[shard * kBlock + threadIdx.x] = c;
    }
    part[(shard * nblk + blk) * kBlock + threadIdx.x] = b;
  }
}

// ---------------------------------------------------------------------------
// Combine: one wave per shard (grid-stride, four shards per workgroup at a
// time). Lane l takes lane positions L = 4l .. 4l + 3: it folds their
// partials of every block (Horner with the byte tables of x^(8*4096*tt); the
// last block uses x^(8*4096*nfull_last)), multiplies each by W[L] to move it
// to the shard end, adds the ragged-tile chunk times Ct[L]; the XOR over the
// wave plus x^(8*len) * init is crc32_iscsi(shard, len, init). (Round 5 ran
// one 256-lane workgroup per shard with a barrier per shard.)
// ---------------------------------------------------------------------------
static_assert(kBlock == 256, "crc32c_combine: 4 lane positions per lane of a 64-lane wave");
__global__ __launch_bounds__(kBlock) void crc32c_combine(
    const uint32_t* __restrict__ part, const uint32_t* __restrict__ tail,
    const uint32_t* __restrict__ plan, unsigned nblk, int has_tail, unsigned init,
    uint32_t* __restrict__ out, unsigned nsh) {
  constexpr unsigned kWaves = kBlock / 64;
  __shared__ uint32_t kt[2048];
  for (int i = threadIdx.x; i < 2048; i += kBlock) kt[i] = plan[i];
  __syncthreads();
  const unsigned lane = threadIdx.x & 63;
  const uint4 wl = reinterpret_cast<const uint4*>(plan + 2048)[lane];
  const uint4 cl = reinterpret_cast<const uint4*>(plan + 2304)[lane];
  const uint32_t xlen = plan[2560];
  const uint32_t w4[4] = {wl.x, wl.y, wl.z, wl.w}, c4[4] = {cl.x, cl.y, cl.z, cl.w};
  const uint32_t iterm = crc_mulmod(init, xlen);
  for (unsigned sh = blockIdx.x * kWaves + (threadIdx.x >> 6); sh < nsh; sh += gridDim.x * kWaves) {
    const uint32_t* pp = part + static_cast<size_t>(sh) * nblk * kBlock + 4 * lane;
    uint32_t h[4] = {0, 0, 0, 0};
    for (unsigned b = 0; b < nblk; ++b) {
      const uint32_t* k4 = (b + 1 == nblk) ? kt + 1024 : kt;
      const uint4 p = *reinterpret_cast<const uint4*>(pp + static_cast<size_t>(b) * kBlock);
      const uint32_t pv[4] = {p.x, p.y, p.z, p.w};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        h[j] = xor3(k4[h[j] & 0xff], k4[256 + ((h[j] >> 8) & 0xff)], k4[512 + ((h[j] >> 16) & 0xff)]) ^
               k4[768 + (h[j] >> 24)] ^ pv[j];
    }
    uint32_t v = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) v ^= crc_mulmod(h[j], w4[j]);
    if (has_tail) {
      const uint4 t = reinterpret_cast<const uint4*>(tail + static_cast<size_t>(sh) * kBlock)[lane];
      v ^= crc_mulmod(t.x, c4[0]) ^ crc_mulmod(t.y, c4[1]) ^ crc_mulmod(t.z, c4[2]) ^ crc_mulmod(t.w, c4[3]);
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v ^= __shfl_xor(v, m, 64);
    if (lane == 0) out[sh] = v ^ iterm;
  }
}

constexpr unsigned kMaxCrcItems = 1u << 30;

unsigned crc_grid(unsigned long long nitems) {
  return static_cast<unsigned>(nitems);
}

#else  // ISAL_FUSED_PART: the fused kernels of one P (crc_fused_pP.o)

// ---------------------------------------------------------------------------
// Fused encode + CRC. The encode half is ec_encode_v16's (same loads, same
// GF arithmetic, same stores); the source chunks already in registers and the
// parity chunks about to be stored also feed the CRC chains. Output chains
// live in registers; source chains too when the stripe's k sources form one
// load group (REG: k == U, e.g. C2's k = 10), else in LDS (lane-private words).
// Full tiles run a branch-free loop; the ragged last tile (len % 4096 != 0)
// runs once, after it, with the chunk CRCs going to tail[].
// ---------------------------------------------------------------------------
enum : int {
  kFeedReg = 0,   // full tile, source chain in registers
  kFeedLds = 1,   // full tile, source chain in LDS
  kFeedTail = 2,  // ragged tile: the chunk's crc goes to tail[]
  kFeedNone = 3,  // no source checksums (second pass of rows > 8)
};

// NB = 4: pre-shifted chains (pre_step), LAST marking the block's last tile.
template <int FEED, int NB = 0, bool LAST = false>
struct SrcFeed {
  const uint32_t* lt;
  uint32_t* la;    // [k][kBlock * NV] source chains (LDS)
  uint32_t* ra;    // [U] source chains (registers)
  uint32_t* tail;  // tail row of source shard 0 of this stripe
  unsigned las;    // row stride of la
  unsigned tid;    // lane within its 256-lane group
  __device__ __forceinline__ void operator()(int j, const uint4& x) const {
    if constexpr (FEED != kFeedNone) {
      if constexpr (NB == 4) {
        if constexpr (FEED == kFeedReg) {
          ra[j] = pre_step<LAST>(lt, ra[j], x.x, x.y, x.z, x.w);
        } else if constexpr (FEED == kFeedLds) {
          uint32_t* a = la + j * las + threadIdx.x;
          *a = pre_step<LAST>(lt, *a, x.x, x.y, x.z, x.w);
        } else {
          tail[static_cast<size_t>(j) * kBlock + tid] = pre_step<true>(lt, 0u, x.x, x.y, x.z, x.w);
        }
      } else {
        const uint32_t c = chunk_crc(lt, x);
        if constexpr (FEED == kFeedReg) {
          ra[j] = shift_tile(lt, ra[j]) ^ c;
        } else if constexpr (FEED == kFeedLds) {
          uint32_t* a = la + j * las + threadIdx.x;
          *a = shift_tile(lt, *a) ^ c;
        } else {
          tail[static_cast<size_t>(j) * kBlock + tid] = c;
        }
      }
    }
  }
};

// acc ^= the U sources x[] (sources j..j+U-1) times their coefficients; each
// source also feeds its CRC chain.
template <int P, int U, bool R0 = false, class Feed>
__device__ __forceinline__ void mac_feed16(uint32_t (&acc)[P][4], const uint4 (&x)[U], int j,
                                           const uint32_t* __restrict__ tbl, const Feed& feed, unsigned long long x0src = 0) {
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

template <int U, int MODE>
__device__ __forceinline__ void load_group(uint4 (&x)[U], const uint64_t* __restrict__ sp, int j,
                                           long long off, int len) {
#pragma unroll
  for (int u = 0; u < U; ++u) x[u] = load16<MODE>(sp[j + u], off, len);
}

template <int P, int U, int MODE, bool R0, class Feed>
__device__ __forceinline__ void chunk16_crc(uint32_t (&acc)[P][4], const uint64_t* __restrict__ sp,
                                            int j, long long off, const uint32_t* __restrict__ tbl,
                                            int len, const Feed& feed, unsigned long long x0src) {
  uint4 x[U];
  load_group<U, MODE>(x, sp, j, off, len);
  mac_feed16<P, U, R0>(acc, x, j, tbl, feed, x0src);
}

// REG: k == U, one load group whose chains are indexed at compile time.
// R0: row 0 is the 0/1 row x0src (xor_and instead of GF lookups).
template <int P, class Pol, bool REG, bool R0, class Feed>
__device__ __forceinline__ void accum16_crc(uint32_t (&acc)[P][4], const uint64_t* __restrict__ src,
                                            const uint32_t* __restrict__ tbl, int k, long long off,
                                            int len, const Feed& feed, unsigned long long x0src) {
#pragma unroll
  for (int l = 0; l < P; ++l) acc[l][0] = acc[l][1] = acc[l][2] = acc[l][3] = 0;
  if constexpr (REG) {
    chunk16_crc<P, Pol::U, Pol::LD, R0>(acc, src, 0, off, tbl, len, feed, x0src);
  } else {
    int j = 0;
    for (; j + Pol::U <= k; j += Pol::U)
      chunk16_crc<P, Pol::U, Pol::LD, R0>(acc, src, j, off, tbl, len, feed, x0src);
    if constexpr (Pol::U == 4) {
      if (j + 2 <= k) {
        chunk16_crc<P, 2, Pol::LD, R0>(acc, src, j, off, tbl, len, feed, x0src);
        j += 2;
      }
    }
    for (; j < k; ++j) chunk16_crc<P, 1, Pol::LD, R0>(acc, src, j, off, tbl, len, feed, x0src);
  }
}

template <int P, int U, bool REG>
constexpr int crc_waves() {
  constexpr int est = (4 * U + 8 * P + (REG ? U : 0) + 56 + 7) / 8 * 8;
  constexpr int w = 512 / est;
  return w > 8 ? 8 : (w < 2 ? 2 : w);
}

// SRC: this pass also checksums the k sources (the first pass of a stripe).
// X0 (SRC passes only): parity row 0 has only 0/1 coefficients (RS Vandermonde
// row 0, RAID P), so it is the XOR of the sources in x0src and — CRC being
// GF(2)-linear in the data — so is its chain: it is formed once per block
// from those sources' chains instead of per tile. (A compile-time choice: a
// runtime row mask inside the tile loop costs the register-tight kernel its
// registers.)
// NB = 4: pre-shifted chains through the byte-position tables (pre_step);
// NB = 0: 5-bit field tables and a Z^4096 step per tile.
// NV: independent 256-lane groups per workgroup sharing one LDS copy of the
// tables (no barrier after the table load); the per-lane source chains then
// set how many waves fit a CU.
template <int P, class Pol, bool REG, bool SRC, bool X0 = false, int NB = 0, int NV = 1>
__global__ __launch_bounds__(kBlock * NV, (crc_waves<P, Pol::U, REG>())) void ec_encode_crc_v16(
    const uint64_t* __restrict__ ptrs, int ptr_stride, int src0, int dst0,
    const uint32_t* __restrict__ tbl, int len, int k, unsigned nitems, unsigned nblk, unsigned tt,
    unsigned nfull, unsigned ntiles, unsigned long long x0src, const uint32_t* __restrict__ tabs,
    uint32_t* __restrict__ part, uint32_t* __restrict__ tail, int nshard_total, int out_shard0, int xcd) {
  static_assert(!X0 || SRC, "row 0 is derived from this pass's source chains");
  static_assert(NB == 0 || NB == 4, "byte path: all four dwords");
  constexpr int kFull = SRC ? (REG ? kFeedReg : kFeedLds) : kFeedNone;
  constexpr int kRag = SRC ? kFeedTail : kFeedNone;
  constexpr int NR = REG ? Pol::U : 1;
  constexpr unsigned kLa = kBlock * NV;
  __shared__ uint32_t lt[NB ? kPosLds : kCrcTabDw];
  extern __shared__ uint32_t la[];  // [k][kBlock * NV] when SRC && !REG
  if constexpr (NB) {
    const uint4* src = reinterpret_cast<const uint4*>(tabs + ISAL_HIP_CRC_B16_TAB);
    for (int i = threadIdx.x; i < kPosLds / 4; i += kBlock * NV) reinterpret_cast<uint4*>(lt)[i] = src[i];
    __syncthreads();
  } else {
    load_crc_tables(lt, tabs);
  }
  const unsigned tid = threadIdx.x % kBlock;
  // parity chain step and chunk CRC of the parity's ragged tile
  auto pstep = [&](auto lastc, uint32_t a, const uint32_t (&v)[4]) __attribute__((always_inline)) {
    if constexpr (NB)
      return pre_step<decltype(lastc)::value>(lt, a, v[0], v[1], v[2], v[3]);
    else
      return shift_tile(lt, a) ^ chunk_crc(lt, v[0], v[1], v[2], v[3]);
  };
  auto pchunk = [&](const uint32_t (&v)[4]) __attribute__((always_inline)) {
    if constexpr (NB)
      return pre_step<true>(lt, 0u, v[0], v[1], v[2], v[3]);
    else
      return chunk_crc(lt, v[0], v[1], v[2], v[3]);
  };
  // the last full tile of a block takes the LAST variant (uniform branch)
  auto with_last = [&](bool last, auto&& body) __attribute__((always_inline)) {
    if (last)
      body(std::integral_constant<bool, true>{});
    else
      body(std::integral_constant<bool, false>{});
  };
  for (unsigned ww = blockIdx.x * NV + threadIdx.x / kBlock; ww < nitems; ww += gridDim.x * NV) {
    const unsigned w = xcd_item(ww, nitems, xcd, NV);
    const unsigned stripe = w / nblk, blk = w - stripe * nblk;
    const uint64_t* __restrict__ sp = ptrs + static_cast<size_t>(stripe) * ptr_stride;
    const size_t shard_s = static_cast<size_t>(stripe) * nshard_total;  // source shard 0
    const unsigned t0 = blk * tt, t1 = t0 + tt < ntiles ? t0 + tt : ntiles;
    const unsigned tf = t1 < nfull ? t1 : nfull;  // full tiles of this block end here
    uint32_t ao[P], ra[NR];
#pragma unroll
    for (int l = 0; l < P; ++l) ao[l] = 0;
#pragma unroll
    for (int j = 0; j < NR; ++j) ra[j] = 0;
    if constexpr (SRC && !REG)
      for (int j = 0; j < k; ++j) la[j * kLa + threadIdx.x] = 0;
    auto store_and_chain = [&](auto lastc, uint32_t (&acc)[P][4], long long off)
                               __attribute__((always_inline)) {
#pragma unroll
      for (int l = 0; l < P; ++l) {
        store16<Pol::ST>(sp[dst0 + l], off, make_uint4(acc[l][0], acc[l][1], acc[l][2], acc[l][3]),
                         len);
        if (!(X0 && l == 0)) ao[l] = pstep(lastc, ao[l], acc[l]);
      }
    };
    if constexpr (REG) {
      // Software pipeline: the next tile's sources are in flight while this
      // tile's GF and CRC work runs (the CRC lookups otherwise leave HBM idle).
      uint4 xn[Pol::U];
      if (t0 < tf)
        load_group<Pol::U, Pol::LD>(xn, sp + src0, 0, static_cast<long long>(t0) * kTile + tid * kVec,
                                    len);
      for (unsigned t = t0; t < tf; ++t) {
        const long long off = static_cast<long long>(t) * kTile + tid * kVec;
        uint4 x[Pol::U];
#pragma unroll
        for (int u = 0; u < Pol::U; ++u) x[u] = xn[u];
        if (t + 1 < tf) load_group<Pol::U, Pol::LD>(xn, sp + src0, 0, off + kTile, len);
        uint32_t acc[P][4];
#pragma unroll
        for (int l = 0; l < P; ++l) acc[l][0] = acc[l][1] = acc[l][2] = acc[l][3] = 0;
        int z = 0;  // opaque zero: see below
        asm volatile("" : "+s"(z));
        with_last(t + 1 == tf, [&](auto lastc) __attribute__((always_inline)) {
          mac_feed16<P, Pol::U, X0>(acc, x, 0, tbl + z,
                                    SrcFeed<kFull, NB, decltype(lastc)::value>{
                                        lt, la, ra, tail + shard_s * kBlock, kLa, tid},
                                    x0src);
          store_and_chain(lastc, acc, off);
        });
      }
    } else {
      for (unsigned t = t0; t < tf; ++t) {
        const long long off = static_cast<long long>(t) * kTile + tid * kVec;
        uint32_t acc[P][4];
        // An opaque zero offset per tile keeps the compiler from hoisting all
        // k*P*5 coefficient dwords out of the tile loop (that spills SGPRs).
        int z = 0;
        asm volatile("" : "+s"(z));
        with_last(t + 1 == tf, [&](auto lastc) __attribute__((always_inline)) {
          accum16_crc<P, Pol, REG, X0>(acc, sp + src0, tbl + z, k, off, len,
                                       SrcFeed<kFull, NB, decltype(lastc)::value>{
                                           lt, la, ra, tail + shard_s * kBlock, kLa, tid},
                                       x0src);
          store_and_chain(lastc, acc, off);
        });
      }
    }
    if (tf < t1) {  // the ragged last tile (t == nfull): len % 16 == 0 here
      const long long off = static_cast<long long>(tf) * kTile + tid * kVec;
      uint32_t* trow = tail + shard_s * kBlock;
      if (off + kVec <= len) {
        uint32_t acc[P][4];
        accum16_crc<P, Pol, REG, X0>(acc, sp + src0, tbl, k, off, len,
                                     SrcFeed<kRag, NB>{lt, la, ra, trow, kLa, tid}, x0src);
#pragma unroll
        for (int l = 0; l < P; ++l) {
          store16<Pol::ST>(sp[dst0 + l], off, make_uint4(acc[l][0], acc[l][1], acc[l][2], acc[l][3]),
                           len);
          uint32_t c = 0;
          if (X0 && l == 0) {  // the sources' tail chunks: this lane wrote them above
            for (int j = 0; j < k; ++j)
              if ((x0src >> j) & 1ull) c ^= trow[j * kBlock + tid];
          } else {
            c = pchunk(acc[l]);
          }
          trow[(out_shard0 + l) * kBlock + tid] = c;
        }
      } else {  // lane past len
        if constexpr (SRC)
          for (int j = 0; j < k; ++j) trow[j * kBlock + tid] = 0;
#pragma unroll
        for (int l = 0; l < P; ++l) trow[(out_shard0 + l) * kBlock + tid] = 0;
      }
    }
    if constexpr (X0) {  // row 0's chain = XOR of its sources' chains
      uint32_t v = 0;
      if constexpr (REG) {
#pragma unroll
        for (int j = 0; j < NR; ++j)
          if ((x0src >> j) & 1ull) v ^= ra[j];
      } else {
        for (int j = 0; j < k; ++j)
          if ((x0src >> j) & 1ull) v ^= la[j * kLa + threadIdx.x];
      }
      ao[0] = v;
    }
#pragma unroll
    for (int l = 0; l < P; ++l)
      part[((shard_s + out_shard0 + l) * nblk + blk) * kBlock + tid] = ao[l];
    if constexpr (SRC) {
      if constexpr (REG) {
#pragma unroll
        for (int j = 0; j < NR; ++j) part[((shard_s + j) * nblk + blk) * kBlock + tid] = ra[j];
      } else {
        for (int j = 0; j < k; ++j)
          part[((shard_s + j) * nblk + blk) * kBlock + tid] = la[j * kLa + threadIdx.x];
      }
    }
  }
}

// Memory policy of the fused kernel: non-temporal global loads/stores (a
// 64-bit SGPR base per shard instead of a 4-SGPR buffer descriptor: the CRC
// half needs the scalar registers).
template <int UU>
using FusedPol = EncPol<UU, kNT, kNT>;

int enc_group_crc(int k) {
  static const int cand[] = {12, 10, 8, 6, 5, 4};
  for (int u : cand)
    if (k >= u && k % u == 0) return u;
  return 4;
}

// 256-lane groups per workgroup of the fused kernel: 2 when that fits more
// groups on a CU (160 KiB of LDS: 32 KiB of byte tables per workgroup, 1 KiB
// of chains per source and group), else 1.
//
// Round 5 removed the variants measured slower and their knobs: source chains
// in registers (ISAL_HIP_CRC_SRC_CHAIN=reg: 153 VGPRs, 3 waves per SIMD, 2 %
// behind LDS chains on C2, profiles/r01/r01_crc_tile_sweep.txt) and the 5-bit
// field tables with a Z^4096 step for the sources (ISAL_HIP_CRC_BYTE_DWORDS=0:
// C2 step 3.48 -> 3.74 ms, profiles/r02/r02_fastcrc_*); the byte tables stay
// the fused kernel's chunk path.
int fused_nv32(int k) {
  const size_t cap = 160 * 1024, tabs = kPosLds * 4, la = static_cast<size_t>(k) * kBlock * 4;
  if (tabs + 2 * la >= cap) return 1;  // leave LDS headroom: never the whole 160 KiB
  return 2 * (cap / (tabs + 2 * la)) > cap / (tabs + la) ? 2 : 1;
}

template <int P, int U>
void launch_fused(unsigned grid, size_t lds, hipStream_t s, const uint64_t* ptrs, int ptr_stride,
                  int src0, int dst0, const uint32_t* tbl, int len, int k, unsigned nitems,
                  const isal_hip_crc_geom& g, const isal_hip_xrows& xr, const uint32_t* tabs,
                  uint32_t* part, uint32_t* tail, int nshard_total, int crc_src, int out_shard0) {
#define FUSED_LAUNCH(REG, SRC, X0, LDS, NB, NV)                                                  \
  ISAL_LAUNCH((ec_encode_crc_v16<P, FusedPol<U>, REG, SRC, X0, NB, NV>),                   \
                     dim3((grid + NV - 1) / NV), dim3(kBlock * NV), (LDS) * NV, s, ptrs, ptr_stride, \
                     src0, dst0, tbl, len, k, nitems, static_cast<unsigned>(g.nblk),               \
                     static_cast<unsigned>(g.tt), static_cast<unsigned>(g.nfull),                  \
                     static_cast<unsigned>(g.ntiles), xr.src[0], tabs, part, tail, nshard_total,   \
                     out_shard0, 0)
  const bool x0 = crc_src && (xr.rows & 1u);
  const bool nv2 = crc_src && fused_nv32(k) == 2;
  if (!crc_src)
    FUSED_LAUNCH(false, false, false, 0, 0, 1);
  else if (nv2) {
    if (x0) FUSED_LAUNCH(false, true, true, lds, 4, 2); else FUSED_LAUNCH(false, true, false, lds, 4, 2);
  } else {
    if (x0) FUSED_LAUNCH(false, true, true, lds, 4, 1); else FUSED_LAUNCH(false, true, false, lds, 4, 1);
  }
#undef FUSED_LAUNCH
}

template <int P>
void fused_pass(unsigned grid, size_t lds, hipStream_t s, const uint64_t* ptrs, int ptr_stride,
                int src0, int dst0, const uint32_t* tbl, int len, int k, unsigned nitems,
                const isal_hip_crc_geom& g, const isal_hip_xrows& xr, const uint32_t* tabs,
                uint32_t* part, uint32_t* tail, int nshard_total, int crc_src, int out_shard0) {
#define FUSED_U(u)                                                                               \
  launch_fused<P, u>(grid, lds, s, ptrs, ptr_stride, src0, dst0, tbl, len, k, nitems, g, xr,   \
                     tabs, part, tail, nshard_total, crc_src, out_shard0)
  switch (enc_group_crc(k)) {
    case 12: FUSED_U(12); break;
    case 10: FUSED_U(10); break;
    case 8: FUSED_U(8); break;
    case 6: FUSED_U(6); break;
    case 5: FUSED_U(5); break;
    default: FUSED_U(4); break;
  }
#undef FUSED_U
}

}  // namespace

// The fused kernels of one P live in their own object (this file compiled with
// -DISAL_FUSED_PART=P) so the variants build in parallel.
#define FUSED_PART_FN2(p) isal_hip_fused_crc_part_##p
#define FUSED_PART_FN(p) FUSED_PART_FN2(p)
extern "C" void FUSED_PART_FN(ISAL_FUSED_PART)(
    unsigned grid, size_t lds, hipStream_t s, const uint64_t* ptrs, int ptr_stride, int src0, int dst0,
    const uint32_t* tbl, int len, int k, unsigned nitems, const isal_hip_crc_geom* g,
    const isal_hip_xrows* xr, const uint32_t* tabs, uint32_t* part, uint32_t* tail, int nshard_total,
    int crc_src, int out_shard0) {
  fused_pass<ISAL_FUSED_PART>(grid, lds, s, ptrs, ptr_stride, src0, dst0, tbl, len, k, nitems, *g, *xr,
                              tabs, part, tail, nshard_total, crc_src, out_shard0);
}
#endif  // ISAL_FUSED_PART

#ifndef ISAL_FUSED_PART
}  // namespace

// Fused encode+CRC32C launchers, one object per P (crc_fused_pP.o).
#define FUSED_PART_DECL(p)                                                                          \
  extern "C" void isal_hip_fused_crc_part_##p(                                                      \
      unsigned grid, size_t lds, hipStream_t s, const uint64_t* ptrs, int ptr_stride, int src0,     \
      int dst0, const uint32_t* tbl, int len, int k, unsigned nitems, const isal_hip_crc_geom* g,   \
      const isal_hip_xrows* xr, const uint32_t* tabs, uint32_t* part, uint32_t* tail,               \
      int nshard_total, int crc_src, int out_shard0);
FUSED_PART_DECL(1) FUSED_PART_DECL(2) FUSED_PART_DECL(3) FUSED_PART_DECL(4)
FUSED_PART_DECL(5) FUSED_PART_DECL(6) FUSED_PART_DECL(7) FUSED_PART_DECL(8)
#undef FUSED_PART_DECL

extern "C" int isal_hip_launch_crc(const uint64_t* d_ptrs, int ptr_stride, int idx0, int nsh,
                                   long long nstripes, int len, int vec16, int tt,
                                   const uint32_t* d_tabs, uint32_t* d_part, uint32_t* d_tail,
                                   int nshard_total, int shard0, void* stream) {
  if (len <= 0 || nsh <= 0 || nstripes <= 0) return 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  isal_hip_crc_geom g;
  isal_hip_crc_geometry(len, tt, &g);
  const unsigned long long per_stripe = static_cast<unsigned long long>(nsh) * g.nblk;
  const long long per = static_cast<long long>(kMaxCrcItems / per_stripe) > 0
                            ? static_cast<long long>(kMaxCrcItems / per_stripe) : 1;
  for (long long s0 = 0; s0 < nstripes; s0 += per) {
    const long long ns = nstripes - s0 < per ? nstripes - s0 : per;
    const unsigned nitems = static_cast<unsigned>(ns * per_stripe);
    const uint64_t* ptrs = d_ptrs + s0 * ptr_stride;
    uint32_t* part = d_part + static_cast<size_t>(s0) * nshard_total * g.nblk * kBlock;
    uint32_t* tail = d_tail + static_cast<size_t>(s0) * nshard_total * kBlock;
    if (vec16)
      ISAL_LAUNCH(crc32c_shards_pre, dim3(crc_grid(nitems)), dim3(kBlock), 0, s, ptrs,
                         ptr_stride, idx0, nsh, len, nitems, static_cast<unsigned>(g.nblk),
                         static_cast<unsigned>(tt), static_cast<unsigned>(g.nfull),
                         static_cast<unsigned>(g.ntiles), d_tabs, part, tail, nshard_total, shard0);
    else
      ISAL_LAUNCH(crc32c_shards_bytes, dim3(crc_grid(nitems)), dim3(kBlock), 0, s, ptrs,
                         ptr_stride, idx0, nsh, len, nitems, static_cast<unsigned>(g.nblk),
                         static_cast<unsigned>(tt), static_cast<unsigned>(g.nfull),
                         static_cast<unsigned>(g.ntiles), d_tabs, part, tail, nshard_total, shard0);
    isal_hip_count_launch();
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return static_cast<int>(e);
  }
  return 0;
}

extern "C" int isal_hip_launch_encode_crc(const uint64_t* d_ptrs, int ptr_stride, int src_idx0,
                                          int dst_idx0, const uint32_t* d_tbl,
                                          const isal_hip_xrows* xrp, int len, int k, int rows,
                                          long long nstripes, int tt, const uint32_t* d_tabs,
                                          uint32_t* d_part, uint32_t* d_tail, void* stream) {
  if (len <= 0 || rows <= 0 || nstripes <= 0) return 0;
  if (len % kVec || k > ISAL_HIP_CRC_MAX_FUSED_K) return static_cast<int>(hipErrorInvalidValue);
  hipStream_t s = static_cast<hipStream_t>(stream);
  isal_hip_crc_geom g;
  isal_hip_crc_geometry(len, tt, &g);
  const int nshard_total = k + rows;
  const long long per = static_cast<long long>(kMaxCrcItems / g.nblk) > 0
                            ? static_cast<long long>(kMaxCrcItems / g.nblk) : 1;
  for (long long s0 = 0; s0 < nstripes; s0 += per) {
    const long long ns = nstripes - s0 < per ? nstripes - s0 : per;
    const unsigned nitems = static_cast<unsigned>(ns * g.nblk);
    const uint64_t* ptrs = d_ptrs + s0 * ptr_stride;
    uint32_t* part = d_part + static_cast<size_t>(s0) * nshard_total * g.nblk * kBlock;
    uint32_t* tail = d_tail + static_cast<size_t>(s0) * nshard_total * kBlock;
    for (int r0 = 0; r0 < rows; r0 += EC_MAX_ROWS_PER_PASS) {
      const int P = rows - r0 < EC_MAX_ROWS_PER_PASS ? rows - r0 : EC_MAX_ROWS_PER_PASS;
      const uint32_t* tbl = d_tbl + static_cast<size_t>(kTbl) * k * r0;
      const int crc_src = r0 == 0;
      const size_t lds = crc_src ? static_cast<size_t>(k) * kBlock * 4 : 0;
      isal_hip_xrows xr{};  // a derived row 0 needs this pass's source partials
      if (crc_src && xrp) xr = *xrp;
      switch (P) {
#define FUSED_CASE(n)                                                                          \
  case n:                                                                                      \
    isal_hip_fused_crc_part_##n(crc_grid(nitems), lds, s, ptrs, ptr_stride, src_idx0,          \
                                dst_idx0 + r0, tbl, len, k, nitems, &g, &xr, d_tabs, part,     \
                                tail, nshard_total, crc_src, k + r0);                          \
    break;
        FUSED_CASE(1) FUSED_CASE(2) FUSED_CASE(3) FUSED_CASE(4) FUSED_CASE(5) FUSED_CASE(6)
        FUSED_CASE(7) FUSED_CASE(8)
#undef FUSED_CASE
      }
      isal_hip_count_launch();
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) return static_cast<int>(e);
    }
  }
  return 0;
}

extern "C" int isal_hip_launch_crc_combine(const uint32_t* d_part, const uint32_t* d_tail,
                                           const uint32_t* d_plan, long long nblk, int has_tail,
                                           unsigned int init, uint32_t* out, long long nsh,
                                           void* stream) {
  if (nsh <= 0) return 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const unsigned long long want = (static_cast<unsigned long long>(nsh) + 3) / 4;  // four shards per workgroup
  const unsigned grid = want < 2048 ? static_cast<unsigned>(want) : 2048u;
  ISAL_LAUNCH(crc32c_combine, dim3(grid), dim3(kBlock), 0, s, d_part, d_tail, d_plan,
                     static_cast<unsigned>(nblk), has_tail, init, out, static_cast<unsigned>(nsh));
  isal_hip_count_launch();
  return static_cast<int>(hipGetLastError());
}

#endif  // !ISAL_FUSED_PART