// ec_kernels.hip — GF(2^8) Reed-Solomon encode / update kernels for gfx950 (MI355X).
//
// Replaces the reference's inner loops gf_{1..6}vect_dot_prod_* (e.g.
// erasure_code/gf_4vect_dot_prod_avx512_gfni.asm:207-250) and gf_{1..6}vect_mad_*
// (e.g. gf_4vect_mad_avx512.asm:161-256), with semantics of ec_base.c:282-342.
//
// Design:
//  * Pure byte arithmetic on the VALU — no MFMA. A GF(2^8) product c*x is GF(2)-
//    linear in x, so it splits into three lookups on bit fields of x:
//    c*(x&7) ^ c*(x&0x38) ^ c*(x&0xc0). Each lookup is ONE v_perm_b32 that
//    indexes an 8-byte table with a 3-bit selector, for 4 packed bytes at once.
//    The selectors depend only on the source byte and are shared by every
//    output row; the tables depend only on the coefficient and are wave-uniform
//    (scalar loads into SGPRs), so one (source, output) pair costs 3 v_perm + 1.5
//    v_xor3 per dword of 4 columns.
//  * One lane owns 16 contiguous bytes of every shard of a stripe (one
//    global_load_dwordx4 per source, one global_store_dwordx4 per output); a
//    256-lane workgroup covers a 4 KiB column tile; a launch covers every tile of
//    every stripe of the batch (many stripes packed into one launch).
//  * Sources are read exactly once per pass of up to EC_MAX_ROWS_PER_PASS outputs;
//    parity is written exactly once.
//  * Tails (len % 16) run a per-byte path in the last lane(s); shards that are
//    not 16-byte aligned run the per-byte kernels (correct for any alignment,
//    never touching bytes outside [ptr, ptr+len)).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "isal_hip_internal.h"

namespace {

constexpr int kBlock = 256;           // 4 waves of 64 lanes
constexpr int kVec = 16;              // bytes per lane per shard
constexpr int kTile = kBlock * kVec;  // 4 KiB column tile per workgroup step
constexpr int kTbl = EC_TBL_DWORDS;

struct Sel {
  uint32_t s0, s1, s2;
};

// Bit-field selectors of 4 packed source bytes: bits 0-2, 3-5, 6-7 of each byte.
__device__ __forceinline__ Sel split(uint32_t x) {
  return {x & 0x07070707u, (x >> 3) & 0x07070707u, (x >> 6) & 0x03030303u};
}

// Wave-uniform tables of one coefficient (held in SGPRs).
struct Coef {
  uint32_t a0, a1, b0, b1, c;
};

__device__ __forceinline__ Coef load_coef(const uint32_t* __restrict__ t) {
  return {t[0], t[1], t[2], t[3], t[4]};
}

// c*x for 4 packed bytes: three v_perm_b32 lookups.
__device__ __forceinline__ uint32_t gf_mul4(const Coef& t, const Sel& s) {
  return __builtin_amdgcn_perm(t.a1, t.a0, s.s0) ^ __builtin_amdgcn_perm(t.b1, t.b0, s.s1) ^
         __builtin_amdgcn_perm(0u, t.c, s.s2);
}

// Shard addresses are device (global, address space 1) pointers: go through an
// addrspace(1) pointer so hipcc emits global_load/store rather than flat_* (a
// flat access also counts on lgkmcnt and would serialise with the SGPR table loads).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef const u32x4 __attribute__((address_space(1)))* gload_t;
typedef u32x4 __attribute__((address_space(1)))* gstore_t;

// Memory access modes: 0 plain global, 1 non-temporal global (nt),
// 2 non-temporal buffer_load/store (wave-uniform descriptor per shard, 32-bit
// lane offset; measured +1.3 % over mode 1 on the 10-read/4-write stream,
// profiles/r01_probe_variants_3.txt). `len` bounds the buffer descriptor.
enum : int { kPlain = 0, kNT = 1, kBufNT = 2 };

template <int MODE = kPlain>
__device__ __forceinline__ uint4 load16(uint64_t base, long long off, int len = 0) {
  u32x4 v;
  if constexpr (MODE == kBufNT) {
    typedef int v4i __attribute__((ext_vector_type(4)));
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(base), 0, len, 0x00020000);
    const v4i r = __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(off), 0, 2 /* nt */);
    v = {static_cast<uint32_t>(r.x), static_cast<uint32_t>(r.y), static_cast<uint32_t>(r.z),
         static_cast<uint32_t>(r.w)};
  } else if constexpr (MODE == kNT) {
    v = __builtin_nontemporal_load((gload_t)(base + off));
  } else {
    v = *(gload_t)(base + off);
  }
  return make_uint4(v.x, v.y, v.z, v.w);
}

template <int MODE = kPlain>
__device__ __forceinline__ void store16(uint64_t base, long long off, uint4 v, int len = 0) {
  if constexpr (MODE == kBufNT) {
    typedef int v4i __attribute__((ext_vector_type(4)));
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(base), 0, len, 0x00020000);
    const v4i w = {static_cast<int>(v.x), static_cast<int>(v.y), static_cast<int>(v.z),
                   static_cast<int>(v.w)};
    __builtin_amdgcn_raw_buffer_store_b128(w, rs, static_cast<int>(off), 0, 2 /* nt */);
  } else {
    u32x4 w = {v.x, v.y, v.z, v.w};
    if constexpr (MODE == kNT)
      __builtin_nontemporal_store(w, (gstore_t)(base + off));
    else
      *(gstore_t)(base + off) = w;
  }
}

// Tuning policy of the vector encode kernel (tools/ec_probe.hip explores others).
//   U      sources whose loads are issued together before any arithmetic
//   LD/ST  memory access modes of source loads / parity stores (above)
//   ORDER  0: work item = (stripe, tile) with tile fastest; 1: stripe fastest;
//          2: XCD-contiguous
// Measured on MI355X (profiles/r01_probe_variants_*.txt): non-temporal loads
// AND stores lift the 10-read/4-write stream from 5.5 to 6.1 TB/s, issuing
// all of a stripe's source loads at once (U = k) adds ~1 %, buffer ops ~1 %;
// the work order and shard padding do not help. The library picks U from k
// at launch (enc_group).
template <int UU, int LDM = kBufNT, int STM = kBufNT, int ORD = 0>
struct EncPol {
  static constexpr int U = UU;
  static constexpr int LD = LDM, ST = STM;
  static constexpr int ORDER = ORD;
};
template <int UU>
using EncNT = EncPol<UU>;
using EncDefault = EncNT<4>;

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // a ^ b ^ c in one VALU op (gfx950)
}

// acc[l] ^= c[l][j] * x for the P outputs of this pass; t = tables of source j.
template <int P>
__device__ __forceinline__ void mac16(uint32_t (&acc)[P][4], const uint4& x,
                                      const uint32_t* __restrict__ t) {
  const Sel s[4] = {split(x.x), split(x.y), split(x.z), split(x.w)};
#pragma unroll
  for (int l = 0; l < P; ++l) {
    const Coef c = load_coef(t + l * kTbl);
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const uint32_t v = xor3(acc[l][d], __builtin_amdgcn_perm(c.a1, c.a0, s[d].s0),
                              __builtin_amdgcn_perm(c.b1, c.b0, s[d].s1));
      acc[l][d] = v ^ __builtin_amdgcn_perm(0u, c.c, s[d].s2);
    }
  }
}

// Two sources at once: the six lookups of a (dword, output) fold into the
// accumulator with three 3-input XORs.
template <int P>
__device__ __forceinline__ void mac16x2(uint32_t (&acc)[P][4], const uint4& x, const uint4& y,
                                        const uint32_t* __restrict__ tx,
                                        const uint32_t* __restrict__ ty) {
  const Sel sx[4] = {split(x.x), split(x.y), split(x.z), split(x.w)};
  const Sel sy[4] = {split(y.x), split(y.y), split(y.z), split(y.w)};
#pragma unroll
  for (int l = 0; l < P; ++l) {
    const Coef a = load_coef(tx + l * kTbl);
    const Coef b = load_coef(ty + l * kTbl);
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      uint32_t v = acc[l][d];
      v = xor3(v, __builtin_amdgcn_perm(a.a1, a.a0, sx[d].s0),
               __builtin_amdgcn_perm(a.b1, a.b0, sx[d].s1));
      v = xor3(v, __builtin_amdgcn_perm(0u, a.c, sx[d].s2),
               __builtin_amdgcn_perm(b.a1, b.a0, sy[d].s0));
      v = xor3(v, __builtin_amdgcn_perm(b.b1, b.b0, sy[d].s1),
               __builtin_amdgcn_perm(0u, b.c, sy[d].s2));
      acc[l][d] = v;
    }
  }
}

// U sources j..j+U-1: issue all U loads before any arithmetic, then fold the
// sources in pairs; the scheduling barriers keep one pair's temporaries live
// at a time (otherwise the scheduler hoists every lookup and spills).
template <int P, int U, int MODE = kPlain>
__device__ __forceinline__ void chunk16(uint32_t (&acc)[P][4], const uint64_t* __restrict__ sp,
                                        int j, long long off, const uint32_t* __restrict__ tbl,
                                        int len) {
  uint4 x[U];
#pragma unroll
  for (int u = 0; u < U; ++u) x[u] = load16<MODE>(sp[j + u], off, len);
  // Pairs share XOR3s but hold two sources' tables (2*P*5 SGPRs): only for P <= 4.
  constexpr int PAIR = P <= 4 ? 2 : 1;
#pragma unroll
  for (int u = 0; u + PAIR <= U; u += PAIR) {
    if constexpr (PAIR == 2)
      mac16x2<P>(acc, x[u], x[u + 1], tbl + (j + u) * P * kTbl, tbl + (j + u + 1) * P * kTbl);
    else
      mac16<P>(acc, x[u], tbl + (j + u) * P * kTbl);
    __builtin_amdgcn_sched_barrier(0);
  }
  if constexpr (PAIR == 2 && (U & 1)) {
    mac16<P>(acc, x[U - 1], tbl + (j + U - 1) * P * kTbl);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// First-mismatch record of the verify kernels: key = column << 8 | row. Each
// workgroup keeps the minimum of its keys in an LDS word (ds_min_u64) and
// writes it to its own slot at the end, so the result needs no device-scope
// atomic and may live in pinned host memory (zero-copy small calls).
__device__ __forceinline__ void note_mismatch(unsigned long long* bad, long long col, int row) {
  atomicMin(bad, (static_cast<unsigned long long>(col) << 8) | static_cast<unsigned>(row));
}

// Per-byte dot product for columns [off, off+nb) of one stripe (tails,
// unaligned shards). VERIFY: compare with the bytes at dst instead of storing.
template <int P, bool VERIFY = false>
__device__ __forceinline__ void dot_bytes(const uint64_t* __restrict__ sp, int src0, int dst0,
                                          const uint32_t* __restrict__ tbl, int k, long long off,
                                          int nb, unsigned long long* bad = nullptr, int row0 = 0,
                                          long long col0 = 0) {
  for (int b = 0; b < nb; ++b) {
    uint32_t acc[P];
#pragma unroll
    for (int l = 0; l < P; ++l) acc[l] = 0;
    for (int j = 0; j < k; ++j) {
      const uint32_t x = reinterpret_cast<const uint8_t*>(sp[src0 + j])[off + b];
      const Sel s = split(x);
#pragma unroll
      for (int l = 0; l < P; ++l) acc[l] ^= gf_mul4(load_coef(tbl + (j * P + l) * kTbl), s);
    }
#pragma unroll
    for (int l = 0; l < P; ++l) {
      uint8_t* d = reinterpret_cast<uint8_t*>(sp[dst0 + l]) + off + b;
      if constexpr (VERIFY) {
        if (static_cast<uint8_t>(acc[l]) != *d) note_mismatch(bad, col0 + off + b, row0 + l);
      } else {
        *d = static_cast<uint8_t>(acc[l]);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Encode: coding[l] = XOR_j c[l][j] * data[j]  (ec_base.c:309-325)
// Work item w = (stripe, 4 KiB tile), tile fastest; grid-stride over items.
// ---------------------------------------------------------------------------
// Waves per SIMD the register allocator must allow (VGPR budget 512/waves).
// Live VGPRs ~ 4U (loads in flight) + 4P (accumulators) + ~32 (selectors,
// table halves, addresses); the 512-entry file gives 512/alloc waves per SIMD.
template <int P, int U>
constexpr int enc_waves() {
  constexpr int est = (4 * U + 4 * P + 32 + 7) / 8 * 8;
  constexpr int w = 512 / est;
  return w > 8 ? 8 : (w < 4 ? 4 : w);
}

// acc[l] = XOR_j c[l][j] * src[j][off..off+16) for one lane.
template <int P, class Pol>
__device__ __forceinline__ void accum16(uint32_t (&acc)[P][4], const uint64_t* __restrict__ src,
                                        const uint32_t* __restrict__ tbl, int k, long long off,
                                        int len) {
#pragma unroll
  for (int l = 0; l < P; ++l) acc[l][0] = acc[l][1] = acc[l][2] = acc[l][3] = 0;
  int j = 0;
  for (; j + Pol::U <= k; j += Pol::U) chunk16<P, Pol::U, Pol::LD>(acc, src, j, off, tbl, len);
  // Remainder. The launcher only picks U > 4 when U divides k, so there the
  // (cheap, correct for any k) single-source loop is dead in practice.
  if constexpr (Pol::U == 4) {
    if (j + 2 <= k) {
      chunk16<P, 2, Pol::LD>(acc, src, j, off, tbl, len);
      j += 2;
    }
  }
  for (; j < k; ++j) chunk16<P, 1, Pol::LD>(acc, src, j, off, tbl, len);
}

template <int P, class Pol = EncDefault>
__global__ __launch_bounds__(kBlock, (enc_waves<P, Pol::U>())) void ec_encode_v16(
    const uint64_t* __restrict__ ptrs, int ptr_stride, int src0, int dst0,
    const uint32_t* __restrict__ tbl, int len, int k, unsigned nitems, unsigned tiles) {
  const unsigned nstripes = nitems / tiles;
  for (unsigned w = blockIdx.x; w < nitems; w += gridDim.x) {
    unsigned stripe, tile;
    if constexpr (Pol::ORDER == 0) {
      stripe = w / tiles;
      tile = w - stripe * tiles;
    } else if constexpr (Pol::ORDER == 2) {
      // XCD-contiguous: blocks b, b+8, b+16.. (one XCD under round-robin
      // dispatch) walk one contiguous eighth of the items. Speed only.
      const unsigned per = nitems >> 3;
      const unsigned v = (nitems & 7) ? w : (w & 7) * per + (w >> 3);
      stripe = v / tiles;
      tile = v - stripe * tiles;
    } else {
      tile = w / nstripes;
      stripe = w - tile * nstripes;
    }
    const uint64_t* __restrict__ sp = ptrs + static_cast<size_t>(stripe) * ptr_stride;
    const long long off = static_cast<long long>(tile) * kTile + threadIdx.x * kVec;
    if (off + kVec <= len) {
      uint32_t acc[P][4];
      accum16<P, Pol>(acc, sp + src0, tbl, k, off, len);
#pragma unroll
      for (int l = 0; l < P; ++l)
        store16<Pol::ST>(sp[dst0 + l], off, make_uint4(acc[l][0], acc[l][1], acc[l][2], acc[l][3]),
                         len);
    } else if (off < len) {
      dot_bytes<P>(sp, src0, dst0, tbl, k, off, static_cast<int>(len - off));
    }
  }
}

// Any alignment: one lane per byte column, 256 columns per work item.
template <int P>
__global__ __launch_bounds__(kBlock) void ec_encode_b1(const uint64_t* __restrict__ ptrs,
                                                       int ptr_stride, int src0, int dst0,
                                                       const uint32_t* __restrict__ tbl, int len,
                                                       int k, unsigned nitems, unsigned tiles) {
  for (unsigned w = blockIdx.x; w < nitems; w += gridDim.x) {
    const unsigned stripe = w / tiles;
    const unsigned tile = w - stripe * tiles;
    const uint64_t* __restrict__ sp = ptrs + static_cast<size_t>(stripe) * ptr_stride;
    const long long off = static_cast<long long>(tile) * kBlock + threadIdx.x;
    if (off < len) dot_bytes<P>(sp, src0, dst0, tbl, k, off, 1);
  }
}

// ---------------------------------------------------------------------------
// Verify (xor_check / pq_check): recompute the parity of each column and
// compare it with the stored rows at dst; the first mismatching (column, row)
// is reduced into *bad with atomicMin. Nothing is written to the shards.
// ---------------------------------------------------------------------------
template <int P>
__global__ __launch_bounds__(kBlock, (enc_waves<P, 4>())) void ec_verify_v16(
    const uint64_t* __restrict__ ptrs, int ptr_stride, int src0, int dst0,
    const uint32_t* __restrict__ tbl, int len, int k, unsigned nitems, unsigned tiles,
    unsigned long long* __restrict__ slots, int row0, long long col0) {
  __shared__ unsigned long long blk_min;
  if (threadIdx.x == 0) blk_min = ~0ull;
  __syncthreads();
  for (unsigned w = blockIdx.x; w < nitems; w += gridDim.x) {
    const unsigned stripe = w / tiles;
    const unsigned tile = w - stripe * tiles;
    const uint64_t* __restrict__ sp = ptrs + static_cast<size_t>(stripe) * ptr_stride;
    const long long off = static_cast<long long>(tile) * kTile + threadIdx.x * kVec;
    if (off + kVec <= len) {
      uint32_t acc[P][4];
      accum16<P, EncNT<4>>(acc, sp + src0, tbl, k, off, len);
#pragma unroll
      for (int l = 0; l < P; ++l) {
        const uint4 e = load16<kBufNT>(sp[dst0 + l], off, len);
        const uint32_t x[4] = {acc[l][0] ^ e.x, acc[l][1] ^ e.y, acc[l][2] ^ e.z, acc[l][3] ^ e.w};
#pragma unroll
        for (int d = 0; d < 4; ++d)
          if (x[d]) {
            note_mismatch(&blk_min, col0 + off + 4 * d + (__builtin_ctz(x[d]) >> 3), row0 + l);
            break;
          }
      }
    } else if (off < len) {
      dot_bytes<P, true>(sp, src0, dst0, tbl, k, off, static_cast<int>(len - off), &blk_min, row0,
                         col0);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) slots[blockIdx.x] = blk_min;
}

template <int P>
__global__ __launch_bounds__(kBlock) void ec_verify_b1(const uint64_t* __restrict__ ptrs,
                                                       int ptr_stride, int src0, int dst0,
                                                       const uint32_t* __restrict__ tbl, int len,
                                                       int k, unsigned nitems, unsigned tiles,
                                                       unsigned long long* __restrict__ slots,
                                                       int row0, long long col0) {
  __shared__ unsigned long long blk_min;
  if (threadIdx.x == 0) blk_min = ~0ull;
  __syncthreads();
  for (unsigned w = blockIdx.x; w < nitems; w += gridDim.x) {
    const unsigned stripe = w / tiles;
    const unsigned tile = w - stripe * tiles;
    const uint64_t* __restrict__ sp = ptrs + static_cast<size_t>(stripe) * ptr_stride;
    const long long off = static_cast<long long>(tile) * kBlock + threadIdx.x;
    if (off < len) dot_bytes<P, true>(sp, src0, dst0, tbl, k, off, 1, &blk_min, row0, col0);
  }
  __syncthreads();
  if (threadIdx.x == 0) slots[blockIdx.x] = blk_min;
}

// ---------------------------------------------------------------------------
// Update: coding[l] ^= c[l][vec_i] * data  (ec_base.c:327-342, gf_vect_mad)
// tbl points at the [P][5] tables of source vec_i for this pass.
// ---------------------------------------------------------------------------
template <int P>
__device__ __forceinline__ void mad_bytes(const uint64_t* __restrict__ sp, int src_idx, int dst0,
                                          const uint32_t* __restrict__ tbl, long long off, int nb) {
  for (int b = 0; b < nb; ++b) {
    const Sel s = split(reinterpret_cast<const uint8_t*>(sp[src_idx])[off + b]);
#pragma unroll
    for (int l = 0; l < P; ++l) {
      uint8_t* d = reinterpret_cast<uint8_t*>(sp[dst0 + l]) + off + b;
      *d = static_cast<uint8_t>(*d ^ gf_mul4(load_coef(tbl + l * kTbl), s));
    }
  }
}

template <int P>
__global__ __launch_bounds__(kBlock) void ec_update_v16(const uint64_t* __restrict__ ptrs,
                                                        int ptr_stride, int src_idx, int dst0,
                                                        const uint32_t* __restrict__ tbl, int len,
                                                        unsigned nitems, unsigned tiles) {
  for (unsigned w = blockIdx.x; w < nitems; w += gridDim.x) {
    const unsigned stripe = w / tiles;
    const unsigned tile = w - stripe * tiles;
    const uint64_t* __restrict__ sp = ptrs + static_cast<size_t>(stripe) * ptr_stride;
    const long long off = static_cast<long long>(tile) * kTile + threadIdx.x * kVec;
    if (off + kVec <= len) {
      const uint4 x = load16<kBufNT>(sp[src_idx], off, len);
      uint4 d[P];
#pragma unroll
      for (int l = 0; l < P; ++l) d[l] = load16<kBufNT>(sp[dst0 + l], off, len);
      const Sel s0 = split(x.x), s1 = split(x.y), s2 = split(x.z), s3 = split(x.w);
#pragma unroll
      for (int l = 0; l < P; ++l) {
        const Coef c = load_coef(tbl + l * kTbl);
        d[l].x ^= gf_mul4(c, s0);
        d[l].y ^= gf_mul4(c, s1);
        d[l].z ^= gf_mul4(c, s2);
        d[l].w ^= gf_mul4(c, s3);
        store16<kBufNT>(sp[dst0 + l], off, d[l], len);
      }
    } else if (off < len) {
      mad_bytes<P>(sp, src_idx, dst0, tbl, off, static_cast<int>(len - off));
    }
  }
}

template <int P>
__global__ __launch_bounds__(kBlock) void ec_update_b1(const uint64_t* __restrict__ ptrs,
                                                       int ptr_stride, int src_idx, int dst0,
                                                       const uint32_t* __restrict__ tbl, int len,
                                                       unsigned nitems, unsigned tiles) {
  for (unsigned w = blockIdx.x; w < nitems; w += gridDim.x) {
    const unsigned stripe = w / tiles;
    const unsigned tile = w - stripe * tiles;
    const uint64_t* __restrict__ sp = ptrs + static_cast<size_t>(stripe) * ptr_stride;
    const long long off = static_cast<long long>(tile) * kBlock + threadIdx.x;
    if (off < len) mad_bytes<P>(sp, src_idx, dst0, tbl, off, 1);
  }
}

// ---------------------------------------------------------------------------
// Host-side launch helpers
// ---------------------------------------------------------------------------
constexpr unsigned kMaxItems = 1u << 30;  // keep w / tiles in 32-bit scalar math

unsigned grid_cap() {
  static unsigned cap = [] {
    const char* e = getenv("ISAL_HIP_GRID_CAP");
    return e ? static_cast<unsigned>(strtoul(e, nullptr, 10)) : 0u;
  }();
  return cap;
}

unsigned grid_for(unsigned nitems) {
  const unsigned cap = grid_cap();
  return (cap && nitems > cap) ? cap : nitems;
}

// Load-group size for k sources: the largest of {12,10,8,6,5,4} dividing k
// (all of a stripe's loads in flight at once for the common k), else 4.
int enc_group(int k) {
  static const int cand[] = {12, 10, 8, 6, 5, 4};
  for (int u : cand)
    if (k >= u && k % u == 0) return u;
  return 4;
}

template <int P, int U>
void launch_v16(unsigned grid, hipStream_t s, const uint64_t* ptrs, int ptr_stride, int src0,
                int dst0, const uint32_t* tbl, int len, int k, unsigned nitems, unsigned tiles) {
  hipLaunchKernelGGL((ec_encode_v16<P, EncNT<U>>), dim3(grid), dim3(kBlock), 0, s, ptrs,
                     ptr_stride, src0, dst0, tbl, len, k, nitems, tiles);
}

template <int P>
hipError_t encode_pass(const uint64_t* ptrs, int ptr_stride, int src0, int dst0, const uint32_t* tbl,
                       int len, int k, unsigned nstripes, bool vec16, hipStream_t s) {
  const unsigned span = vec16 ? kTile : kBlock;
  const unsigned tiles = static_cast<unsigned>((static_cast<long long>(len) + span - 1) / span);
  const unsigned nitems = nstripes * tiles;
  const unsigned grid = grid_for(nitems);
  if (vec16) {
    switch (enc_group(k)) {
      case 12: launch_v16<P, 12>(grid, s, ptrs, ptr_stride, src0, dst0, tbl, len, k, nitems, tiles); break;
      case 10: launch_v16<P, 10>(grid, s, ptrs, ptr_stride, src0, dst0, tbl, len, k, nitems, tiles); break;
      case 8: launch_v16<P, 8>(grid, s, ptrs, ptr_stride, src0, dst0, tbl, len, k, nitems, tiles); break;
      case 6: launch_v16<P, 6>(grid, s, ptrs, ptr_stride, src0, dst0, tbl, len, k, nitems, tiles); break;
      case 5: launch_v16<P, 5>(grid, s, ptrs, ptr_stride, src0, dst0, tbl, len, k, nitems, tiles); break;
      default: launch_v16<P, 4>(grid, s, ptrs, ptr_stride, src0, dst0, tbl, len, k, nitems, tiles); break;
    }
  } else {
    hipLaunchKernelGGL(ec_encode_b1<P>, dim3(grid), dim3(kBlock), 0, s, ptrs, ptr_stride, src0,
                       dst0, tbl, len, k, nitems, tiles);
  }
  isal_hip_count_launch();
  return hipGetLastError();
}

template <int P>
hipError_t update_pass(const uint64_t* ptrs, int ptr_stride, int src_idx, int dst0,
                       const uint32_t* tbl, int len, unsigned nstripes, bool vec16, hipStream_t s) {
  const unsigned span = vec16 ? kTile : kBlock;
  const unsigned tiles = static_cast<unsigned>((static_cast<long long>(len) + span - 1) / span);
  const unsigned nitems = nstripes * tiles;
  if (vec16)
    hipLaunchKernelGGL(ec_update_v16<P>, dim3(grid_for(nitems)), dim3(kBlock), 0, s, ptrs,
                       ptr_stride, src_idx, dst0, tbl, len, nitems, tiles);
  else
    hipLaunchKernelGGL(ec_update_b1<P>, dim3(grid_for(nitems)), dim3(kBlock), 0, s, ptrs,
                       ptr_stride, src_idx, dst0, tbl, len, nitems, tiles);
  isal_hip_count_launch();
  return hipGetLastError();
}

// Largest stripe count per launch so that nitems stays below kMaxItems.
unsigned stripes_per_launch(int len, bool vec16) {
  const long long span = vec16 ? kTile : kBlock;
  const long long tiles = (static_cast<long long>(len) + span - 1) / span;
  const long long n = static_cast<long long>(kMaxItems) / (tiles ? tiles : 1);
  return static_cast<unsigned>(n > 0 ? n : 1);
}

}  // namespace

extern "C" int isal_hip_launch_encode(const uint64_t* d_ptrs, int ptr_stride, int src_idx0,
                                      int dst_idx0, const uint32_t* d_tbl, int len, int k, int rows,
                                      long long nstripes, int vec16, void* stream) {
  if (len <= 0 || rows <= 0 || nstripes <= 0) return 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const unsigned per = stripes_per_launch(len, vec16 != 0);
  for (long long s0 = 0; s0 < nstripes; s0 += per) {
    const unsigned ns = static_cast<unsigned>(nstripes - s0 < per ? nstripes - s0 : per);
    const uint64_t* ptrs = d_ptrs + s0 * ptr_stride;
    for (int r0 = 0; r0 < rows; r0 += EC_MAX_ROWS_PER_PASS) {
      const int P = rows - r0 < EC_MAX_ROWS_PER_PASS ? rows - r0 : EC_MAX_ROWS_PER_PASS;
      const uint32_t* tbl = d_tbl + static_cast<size_t>(kTbl) * k * r0;
      const int dst0 = dst_idx0 + r0;
      hipError_t e = hipSuccess;
      switch (P) {
#define EC_CASE(n)                                                                            \
  case n:                                                                                     \
    e = encode_pass<n>(ptrs, ptr_stride, src_idx0, dst0, tbl, len, k, ns, vec16 != 0, s); \
    break;
        EC_CASE(1) EC_CASE(2) EC_CASE(3) EC_CASE(4) EC_CASE(5) EC_CASE(6) EC_CASE(7) EC_CASE(8)
#undef EC_CASE
      }
      if (e != hipSuccess) return static_cast<int>(e);
    }
  }
  return 0;
}

extern "C" int isal_hip_launch_verify(const uint64_t* d_ptrs, int ptr_stride, int src_idx0,
                                      int dst_idx0, const uint32_t* d_tbl, int len, int k, int rows,
                                      long long col0, unsigned long long* slots, int* nslots,
                                      int vec16, void* stream) {
  *nslots = 0;
  if (len <= 0 || rows <= 0) return 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const unsigned span = vec16 ? kTile : kBlock;
  const unsigned tiles = static_cast<unsigned>((static_cast<long long>(len) + span - 1) / span);
  const unsigned grid = tiles < EC_VERIFY_MAX_GRID ? tiles : EC_VERIFY_MAX_GRID;
  for (int r0 = 0; r0 < rows; r0 += EC_MAX_ROWS_PER_PASS) {
    const int P = rows - r0 < EC_MAX_ROWS_PER_PASS ? rows - r0 : EC_MAX_ROWS_PER_PASS;
    const uint32_t* tbl = d_tbl + static_cast<size_t>(kTbl) * k * r0;
    const int dst0 = dst_idx0 + r0;
    unsigned long long* out = slots + *nslots;
    switch (P) {
#define EC_CASE(n)                                                                            \
  case n:                                                                                     \
    if (vec16)                                                                                \
      hipLaunchKernelGGL(ec_verify_v16<n>, dim3(grid), dim3(kBlock), 0, s, d_ptrs, ptr_stride, \
                         src_idx0, dst0, tbl, len, k, tiles, tiles, out, r0, col0);           \
    else                                                                                      \
      hipLaunchKernelGGL(ec_verify_b1<n>, dim3(grid), dim3(kBlock), 0, s, d_ptrs, ptr_stride,  \
                         src_idx0, dst0, tbl, len, k, tiles, tiles, out, r0, col0);           \
    break;
      EC_CASE(1) EC_CASE(2) EC_CASE(3) EC_CASE(4) EC_CASE(5) EC_CASE(6) EC_CASE(7) EC_CASE(8)
#undef EC_CASE
    }
    *nslots += static_cast<int>(grid);
    isal_hip_count_launch();
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return static_cast<int>(e);
  }
  return 0;
}

extern "C" int isal_hip_launch_update(const uint64_t* d_ptrs, int ptr_stride, int src_idx,
                                      int dst_idx0, const uint32_t* d_tbl, int len, int k, int rows,
                                      int vec_i, long long nstripes, int vec16, void* stream) {
  if (len <= 0 || rows <= 0 || nstripes <= 0) return 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const unsigned per = stripes_per_launch(len, vec16 != 0);
  for (long long s0 = 0; s0 < nstripes; s0 += per) {
    const unsigned ns = static_cast<unsigned>(nstripes - s0 < per ? nstripes - s0 : per);
    const uint64_t* ptrs = d_ptrs + s0 * ptr_stride;
    for (int r0 = 0; r0 < rows; r0 += EC_MAX_ROWS_PER_PASS) {
      const int P = rows - r0 < EC_MAX_ROWS_PER_PASS ? rows - r0 : EC_MAX_ROWS_PER_PASS;
      const uint32_t* tbl =
          d_tbl + static_cast<size_t>(kTbl) * k * r0 + static_cast<size_t>(vec_i) * P * kTbl;
      const int dst0 = dst_idx0 + r0;
      hipError_t e = hipSuccess;
      switch (P) {
#define EC_CASE(n)                                                                          \
  case n:                                                                                   \
    e = update_pass<n>(ptrs, ptr_stride, src_idx, dst0, tbl, len, ns, vec16 != 0, s); \
    break;
        EC_CASE(1) EC_CASE(2) EC_CASE(3) EC_CASE(4) EC_CASE(5) EC_CASE(6) EC_CASE(7) EC_CASE(8)
#undef EC_CASE
      }
      if (e != hipSuccess) return static_cast<int>(e);
    }
  }
  return 0;
}
