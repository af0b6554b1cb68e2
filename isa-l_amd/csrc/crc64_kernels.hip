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

#include "ec_device.h"

namespace {

constexpr int kF = ISAL_HIP_CRC_FIELDS;
constexpr int kOp = ISAL_HIP_CRC64_OP_ENTRIES;
constexpr int kKernTab = ISAL_HIP_CRC64_OP_BLOCK - ISAL_HIP_CRC64_CHUNK_TAB;  // chunk + shift
constexpr int kChunk = 0;                                                        // offsets in LDS copy
constexpr int kShift = ISAL_HIP_CRC64_SHIFT_TAB - ISAL_HIP_CRC64_CHUNK_TAB;

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

// XOR of the 7 field lookups of w in the 7 consecutive 32-entry tables at t.
__device__ __forceinline__ uint64_t lookup7(const uint64_t* t, uint32_t w) {
  uint32_t o[kF];
  field_offsets8(w, o);
  const char* b = reinterpret_cast<const char*>(t);
  auto at = [&](int f) { return *reinterpret_cast<const uint64_t*>(b + f * 256 + o[f]); };
  return at(0) ^ at(1) ^ at(2) ^ at(3) ^ at(4) ^ at(5) ^ at(6);
}

// M(v) for a map stored as 14 field tables.
__device__ __forceinline__ uint64_t apply_op(const uint64_t* op, uint64_t v) {
  return lookup7(op, static_cast<uint32_t>(v)) ^ lookup7(op + kF * 32, static_cast<uint32_t>(v >> 32));
}

// raw(0, 16-byte chunk), dwords little-endian.
__device__ __forceinline__ uint64_t chunk_crc(const uint64_t* t, uint32_t w0, uint32_t w1,
                                              uint32_t w2, uint32_t w3) {
  constexpr int D = kF * 32;
  return (lookup7(t, w0) ^ lookup7(t + D, w1)) ^ (lookup7(t + 2 * D, w2) ^ lookup7(t + 3 * D, w3));
}

__device__ __forceinline__ uint32_t le32(const uint8_t* p) {
  return p[0] | (p[1] << 8) | (p[2] << 16) | (static_cast<uint32_t>(p[3]) << 24);
}

// raw(0, 16 bytes at base + off) with byte loads (any alignment).
__device__ __forceinline__ uint64_t chunk_crc_bytes(const uint64_t* t, uint64_t base, long long off) {
  const uint8_t* p = reinterpret_cast<const uint8_t*>(base) + off;
  return chunk_crc(t, le32(p), le32(p + 4), le32(p + 8), le32(p + 12));
}

template <int N>
__device__ __forceinline__ void load_lds(uint64_t* dst, const uint64_t* __restrict__ src) {
  const uint4* s = reinterpret_cast<const uint4*>(src);
  uint4* d = reinterpret_cast<uint4*>(dst);
  for (int i = threadIdx.x; i < N / 2; i += kBlock) d[i] = s[i];
}

constexpr unsigned kBatch = 4;  // full tiles whose loads are issued together

// Chains of the full tiles. Item = (stripe, shard, block), shard-major within
// a stripe: part index = ((stripe * nsh + i) * nblk + blk) * 256 + L.
template <bool VEC>
__global__ __launch_bounds__(kBlock) void crc64_shards(const uint64_t* __restrict__ ptrs,
                                                       int ptr_stride, int nsh, int len,
                                                       unsigned nitems, unsigned nblk, unsigned tt,
                                                       unsigned nfull,
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
    unsigned t = t0;
    if constexpr (VEC) {
      for (; t + kBatch <= t1; t += kBatch) {
        uint4 x[kBatch];
#pragma unroll
        for (unsigned g = 0; g < kBatch; ++g)
          x[g] = load16<kBufNT>(base, static_cast<long long>(t + g) * kTile + lane, len);
#pragma unroll
        for (unsigned g = 0; g < kBatch; ++g)
          a = apply_op(lt + kShift, a) ^ chunk_crc(lt + kChunk, x[g].x, x[g].y, x[g].z, x[g].w);
      }
      for (; t < t1; ++t) {
        const uint4 x = load16<kBufNT>(base, static_cast<long long>(t) * kTile + lane, len);
        a = apply_op(lt + kShift, a) ^ chunk_crc(lt + kChunk, x.x, x.y, x.z, x.w);
      }
    } else {
      for (; t < t1; ++t)
        a = apply_op(lt + kShift, a) ^
            chunk_crc_bytes(lt + kChunk, base, static_cast<long long>(t) * kTile + lane);
    }
    part[static_cast<size_t>(w) * kBlock + threadIdx.x] = a;
  }
}

// v(L) <- sum over lanes of Z^(16 * (255 - L)) v(L), result in red[0]:
// 8 levels, level s joins lanes L and L + 2^s with Z^(16 * 2^s).
__device__ __forceinline__ uint64_t lane_tree(uint64_t* red, const uint64_t* tree) {
  for (int s = 0; s < 8; ++s) {
    const int step = 1 << s;
    if ((threadIdx.x & (2 * step - 1)) == 0)
      red[threadIdx.x] = apply_op(tree + s * kOp, red[threadIdx.x]) ^ red[threadIdx.x + step];
    __syncthreads();
  }
  const uint64_t r = red[0];
  __syncthreads();
  return r;
}

// One workgroup per shard (grid-stride):
//  X = raw(0, full tiles): each lane folds its block chains (Horner with
//      Z^(4096*tt), the last block Z^(4096*nfull_last)), then the lane tree;
//  T = raw(0, the tail's whole 16-byte chunks): lane chunks right-aligned in
//      the tree, so lane q-1's chunk is the last one;
//  s = Z^(16q)(X) ^ T, then the last tail % 16 bytes one at a time;
//  crc64 = ~(Z^len(~init) ^ s).
template <bool REFL>
__global__ __launch_bounds__(kBlock) void crc64_combine(
    const uint64_t* __restrict__ part, const uint64_t* __restrict__ ptrs, int ptr_stride, int nsh,
    int len, unsigned nblk, unsigned nfull, const uint64_t* __restrict__ tabs, uint64_t init_term,
    uint64_t* __restrict__ out, unsigned nshard_total) {
  __shared__ uint64_t lt[ISAL_HIP_CRC64_TAB_ENTRIES];
  __shared__ uint64_t red[kBlock];
  load_lds<ISAL_HIP_CRC64_TAB_ENTRIES>(lt, tabs);
  __syncthreads();
  const int tail = len - static_cast<int>(nfull) * kTile;
  const int q = tail / kVec, rem = tail - q * kVec;
  for (unsigned sh = blockIdx.x; sh < nshard_total; sh += gridDim.x) {
    const unsigned stripe = sh / nsh, i = sh - stripe * nsh;
    const uint64_t base = ptrs[static_cast<size_t>(stripe) * ptr_stride + i];
    uint64_t x = 0, tq = 0;
    if (nblk) {
      const uint64_t* pp = part + static_cast<size_t>(sh) * nblk * kBlock + threadIdx.x;
      uint64_t h = 0;
      for (unsigned b = 0; b < nblk; ++b)
        h = apply_op(lt + (b + 1 == nblk ? ISAL_HIP_CRC64_OP_LAST : ISAL_HIP_CRC64_OP_BLOCK), h) ^
            pp[static_cast<size_t>(b) * kBlock];
      red[threadIdx.x] = h;
      __syncthreads();
      x = lane_tree(red, lt + ISAL_HIP_CRC64_OP_TREE);
    }
    if (q) {
      red[threadIdx.x] = 0;
      __syncthreads();
      if (static_cast<int>(threadIdx.x) < q)
        red[threadIdx.x + kBlock - q] = chunk_crc_bytes(
            lt + ISAL_HIP_CRC64_CHUNK_TAB, base, static_cast<long long>(nfull) * kTile + threadIdx.x * kVec);
      __syncthreads();
      tq = lane_tree(red, lt + ISAL_HIP_CRC64_OP_TREE);
    }
    if (threadIdx.x == 0) {
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

}  // namespace

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
        hipLaunchKernelGGL(crc64_shards<true>, dim3(nitems), dim3(kBlock), 0, s, ptrs, ptr_stride,
                           nsh, len, nitems, static_cast<unsigned>(g.nblk), static_cast<unsigned>(g.tt),
                           static_cast<unsigned>(g.nfull), d_tabs, part);
      else
        hipLaunchKernelGGL(crc64_shards<false>, dim3(nitems), dim3(kBlock), 0, s, ptrs, ptr_stride,
                           nsh, len, nitems, static_cast<unsigned>(g.nblk), static_cast<unsigned>(g.tt),
                           static_cast<unsigned>(g.nfull), d_tabs, part);
      isal_hip_count_launch();
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) return static_cast<int>(e);
    }
    // each combine workgroup copies the 52 KB table set once: cap the grid
    const unsigned grid = nshard < 2048 ? nshard : 2048;
    if (refl)
      hipLaunchKernelGGL(crc64_combine<true>, dim3(grid), dim3(kBlock), 0, s, part, ptrs, ptr_stride,
                         nsh, len, static_cast<unsigned>(g.nblk), static_cast<unsigned>(g.nfull),
                         d_tabs, init_term, out + s0 * nsh, nshard);
    else
      hipLaunchKernelGGL(crc64_combine<false>, dim3(grid), dim3(kBlock), 0, s, part, ptrs, ptr_stride,
                         nsh, len, static_cast<unsigned>(g.nblk), static_cast<unsigned>(g.nfull),
                         d_tabs, init_term, out + s0 * nsh, nshard);
    isal_hip_count_launch();
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return static_cast<int>(e);
  }
  return 0;
}
