// ec_device.h — device-side building blocks shared by the GF(2^8) kernels
// (ec_kernels.hip) and the fused encode+CRC kernels (crc_kernels.hip).
// Included by exactly those translation units; everything lives in an
// anonymous namespace (one private copy per kernel object).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "isal_hip_internal.h"

namespace {

// Every kernel a host launcher names registers itself when the library loads:
// ISAL_LAUNCH odr-uses KernelReg<kernel>::id, so each launcher instantiation
// instantiates the registration with it, and isal_hip_selftest_kernels() asks
// the runtime for every registered kernel's attributes — a kernel with a host
// handle but no device code (the r05e abort, DESIGN.md §3 "Kernel registry")
// is found by a test instead of by a caller's launch.
template <auto K>
struct KernelReg {
  static const int id;
  static int add() {
    isal_hip_kreg_add(reinterpret_cast<const void*>(K), __PRETTY_FUNCTION__);
    return 0;
  }
};
template <auto K>
const int KernelReg<K>::id = KernelReg<K>::add();

#define ISAL_LAUNCH(kernel, ...)              \
  do {                                        \
    (void)KernelReg<kernel>::id;              \
    hipLaunchKernelGGL(kernel, __VA_ARGS__);  \
  } while (0)

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
// profiles/r01/r01_probe_variants_3.txt). `len` bounds the buffer descriptor.
// 3 = buffer ops with sc1 + nt (gfx950 CPol 0x12): in the memory probe the
// 10-read/4-write stream with sc1+nt stores ran +0.5-0.9 % over nt stores
// (profiles/r03/r03_probe_variants.txt); selectable for the encode's stores.
enum : int { kPlain = 0, kNT = 1, kBufNT = 2, kBufSC1NT = 3 };

template <int MODE = kPlain>
__device__ __forceinline__ uint4 load16(uint64_t base, long long off, int len = 0) {
  u32x4 v;
  if constexpr (MODE == kBufNT || MODE == kBufSC1NT) {
    typedef int v4i __attribute__((ext_vector_type(4)));
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(base), 0, len, 0x00020000);
    const v4i r = __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(off), 0,
                                                        MODE == kBufNT ? 2 /* nt */ : 0x12 /* sc1 nt */);
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
  if constexpr (MODE == kBufNT || MODE == kBufSC1NT) {
    typedef int v4i __attribute__((ext_vector_type(4)));
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(base), 0, len, 0x00020000);
    const v4i w = {static_cast<int>(v.x), static_cast<int>(v.y), static_cast<int>(v.z),
                   static_cast<int>(v.w)};
    __builtin_amdgcn_raw_buffer_store_b128(w, rs, static_cast<int>(off), 0,
                                           MODE == kBufNT ? 2 /* nt */ : 0x12 /* sc1 nt */);
  } else {
    u32x4 w = {v.x, v.y, v.z, v.w};
    if constexpr (MODE == kNT)
      __builtin_nontemporal_store(w, (gstore_t)(base + off));
    else
      *(gstore_t)(base + off) = w;
  }
}

// Tuning policy of the vector encode kernel (isa-l_amd/tools/ec_probe.hip explores others).
//   U      sources whose loads are issued together before any arithmetic
//   LD/ST  memory access modes of source loads / parity stores (above)
//   ORDER  work order (EncOrder in ec_kernels.hip): 0 = (stripe, tile) with
//          tile fastest, 2 = XCD-contiguous (the library's); the probe adds others
// Measured on MI355X (profiles/r01/r01_probe_variants_*.txt): non-temporal loads
// AND stores lift the 10-read/4-write stream from 5.5 to 6.1 TB/s, issuing
// all of a stripe's source loads at once (U = k) adds ~1 %, buffer ops ~1 %;
// shard padding does not help. The XCD-contiguous order (2) measured -2.4 %
// on one round-1/2 box and +1.0-1.3 % on every round-3 box (same-box A/B,
// profiles/r03/r03_enc_order_benches.jsonl, r03_probe_variants.txt); the library
// launches order 2 by default (ec_kernels.hip enc_order) and picks U from k
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

// Item of work index w in the XCD-contiguous order: workgroup u runs on XCD
// u % 8 (round-robin dispatch), and with the order on its nv items come from
// the (u % 8)-th contiguous eighth of [0, n), so each XCD streams one region
// (the encode's order 2). A bijection of [0, n); the identity when
// off or when n is not a multiple of 8 * nv.
__device__ __forceinline__ unsigned xcd_item(unsigned w, unsigned n, int on, unsigned nv = 1) {
  if (!on || n % (8 * nv)) return w;
  const unsigned u = w / nv, g = w - u * nv, per = n / (8 * nv);
  return ((u & 7) * per + (u >> 3)) * nv + g;
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // a ^ b ^ c in one VALU op (gfx950)
}

// acc ^ (x & m) in one VALU op: the product of x with a 0/1 coefficient
// (m = ~0 or 0), e.g. row 0 of every RS Vandermonde matrix (all ones).
__device__ __forceinline__ uint32_t xor_and(uint32_t acc, uint32_t x, uint32_t m) {
  return __builtin_amdgcn_bitop3_b32(acc, x, m, 0x78);
}

// Mask of source j for a 0/1 row: bit j of its source set.
__device__ __forceinline__ uint32_t r0_mask(unsigned long long src, int j) {
  return (src >> j) & 1ull ? ~0u : 0u;
}

// acc[l] ^= c[l][j] * x for the P outputs of this pass; t = tables of source j.
// R0: output row 0's coefficient is 0/1 (mask m0), so row 0 is x & m0 — one
// op per dword instead of three v_perm lookups (the fused encode+CRC kernels,
// which are VALU-bound, take it when row 0 is such a row).
// LT: the low table halves (a0, b0) of each coefficient come from an LDS copy
// (lt[l] = {a0, b0}, a broadcast ds_read_b64 into VGPRs) instead of SGPRs —
// a v_perm may read only one SGPR (gfx9 constant bus), so from SGPRs one half
// needs a v_mov into a VGPR per (source, row): 0.5 VALU op per dword of work.
template <bool LT>
__device__ __forceinline__ void low_halves(const Coef& c, const uint2* lt, int l, uint32_t& a0, uint32_t& b0) {
  if constexpr (LT) {
    const uint2 v = lt[l];
    a0 = v.x;
    b0 = v.y;
  } else {
    a0 = c.a0;
    b0 = c.b0;
  }
}

template <int P, bool R0 = false, bool LT = false>
__device__ __forceinline__ void mac16(uint32_t (&acc)[P][4], const uint4& x,
                                      const uint32_t* __restrict__ t, uint32_t m0 = 0,
                                      const uint2* lt = nullptr) {
  const Sel s[4] = {split(x.x), split(x.y), split(x.z), split(x.w)};
  if constexpr (R0) {
    acc[0][0] = xor_and(acc[0][0], x.x, m0);
    acc[0][1] = xor_and(acc[0][1], x.y, m0);
    acc[0][2] = xor_and(acc[0][2], x.z, m0);
    acc[0][3] = xor_and(acc[0][3], x.w, m0);
  }
#pragma unroll
  for (int l = R0 ? 1 : 0; l < P; ++l) {
    const Coef c = load_coef(t + l * kTbl);
    uint32_t a0, b0;
    low_halves<LT>(c, lt, l, a0, b0);
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const uint32_t v = xor3(acc[l][d], __builtin_amdgcn_perm(c.a1, a0, s[d].s0),
                              __builtin_amdgcn_perm(c.b1, b0, s[d].s1));
      acc[l][d] = v ^ __builtin_amdgcn_perm(0u, c.c, s[d].s2);
    }
  }
}

// Two sources at once: the six lookups of a (dword, output) fold into the
// accumulator with three 3-input XORs.
template <int P, bool R0 = false, bool LT = false>
__device__ __forceinline__ void mac16x2(uint32_t (&acc)[P][4], const uint4& x, const uint4& y,
                                        const uint32_t* __restrict__ tx,
                                        const uint32_t* __restrict__ ty, uint32_t mx = 0,
                                        uint32_t my = 0, const uint2* ltx = nullptr,
                                        const uint2* lty = nullptr) {
  const Sel sx[4] = {split(x.x), split(x.y), split(x.z), split(x.w)};
  const Sel sy[4] = {split(y.x), split(y.y), split(y.z), split(y.w)};
  if constexpr (R0) {
    acc[0][0] = xor_and(xor_and(acc[0][0], x.x, mx), y.x, my);
    acc[0][1] = xor_and(xor_and(acc[0][1], x.y, mx), y.y, my);
    acc[0][2] = xor_and(xor_and(acc[0][2], x.z, mx), y.z, my);
    acc[0][3] = xor_and(xor_and(acc[0][3], x.w, mx), y.w, my);
  }
#pragma unroll
  for (int l = R0 ? 1 : 0; l < P; ++l) {
    const Coef a = load_coef(tx + l * kTbl);
    const Coef b = load_coef(ty + l * kTbl);
    uint32_t aa0, ab0, ba0, bb0;
    low_halves<LT>(a, ltx, l, aa0, ab0);
    low_halves<LT>(b, lty, l, ba0, bb0);
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      uint32_t v = acc[l][d];
      v = xor3(v, __builtin_amdgcn_perm(a.a1, aa0, sx[d].s0),
               __builtin_amdgcn_perm(a.b1, ab0, sx[d].s1));
      v = xor3(v, __builtin_amdgcn_perm(0u, a.c, sx[d].s2),
               __builtin_amdgcn_perm(b.a1, ba0, sy[d].s0));
      v = xor3(v, __builtin_amdgcn_perm(b.b1, bb0, sy[d].s1),
               __builtin_amdgcn_perm(0u, b.c, sy[d].s2));
      acc[l][d] = v;
    }
  }
}

// acc[l] ^= c[l][a] * x ^ c[l][b] * y for rows [L0, L1) (selectors and
// coefficient tables already in registers; the fused kernels' pipelined
// paths cut a source pair's rows into stages around their CRC lookups).
template <int P, int L0, int L1>
__device__ __forceinline__ void mac_rows2(uint32_t (&acc)[P][4], const Sel (&sx)[4], const Sel (&sy)[4],
                                          const Coef (&ca)[P], const Coef (&cb)[P]) {
#pragma unroll
  for (int l = L0; l < L1; ++l) {
    const Coef& a = ca[l];
    const Coef& b = cb[l];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      uint32_t v = acc[l][d];
      v = xor3(v, __builtin_amdgcn_perm(a.a1, a.a0, sx[d].s0), __builtin_amdgcn_perm(a.b1, a.b0, sx[d].s1));
      v = xor3(v, __builtin_amdgcn_perm(0u, a.c, sx[d].s2), __builtin_amdgcn_perm(b.a1, b.a0, sy[d].s0));
      v = xor3(v, __builtin_amdgcn_perm(b.b1, b.b0, sy[d].s1), __builtin_amdgcn_perm(0u, b.c, sy[d].s2));
      acc[l][d] = v;
    }
  }
}

// The coefficient tables come in by scalar loads, which share lgkmcnt with
// LDS accesses and may complete out of order: a wait for one of them is a
// wait for every LDS lookup in flight. The pipelined paths load a pair's
// tables and wait for them (have_coefs) in its first stage, behind the fold
// that waits anyway.
template <int P, int L0, int L1 = P>
__device__ __forceinline__ void load_coefs(Coef (&c)[P], const uint32_t* __restrict__ t) {
#pragma unroll
  for (int l = L0; l < L1; ++l) c[l] = load_coef(t + l * kTbl);
}

template <int P, int L0, int L1 = P>
__device__ __forceinline__ void have_coefs(const Coef (&c)[P]) {
#pragma unroll
  for (int l = L0; l < L1; ++l)
    asm volatile("" ::"s"(c[l].a0), "s"(c[l].a1), "s"(c[l].b0), "s"(c[l].b1), "s"(c[l].c));
}

// Encode variants (template FL of chunk16 / accum16 / ec_encode_v16):
//   kEncLUT  every product through the v_perm lookups;
//   kEncXor  the pass's row 0 and its column of source 0 hold only 0/1
//            (isal_hip_encmask; every gf_gen_rs_matrix and RAID P+Q block):
//            row 0 is acc ^= x & m (one VALU op per dword instead of three
//            v_perm, their folds and a table move), and source 0 starts every
//            row's sum as x & m (no lookups, no XOR). Masks arrive as kernel
//            arguments: r0m bit j for row 0's source j, c0m bit l for source
//            0's row l.
//   kEncLds  (a bit, with either) the low table halves from an LDS copy
//            (low_halves), the rest from SGPRs.
enum : int { kEncLUT = 0, kEncXor = 1, kEncLds = 2 };
// Launch-bounds flag of the verify kernels (they also hold the stored parity).
constexpr int kEncVerify = 16;

// Source pairs share XOR3s but hold two sources' tables in SGPRs (5 dwords per
// looked-up row each): pairs while at most 4 rows per source are looked up
// (wider passes paired spilled SGPRs, even with the row tables loaded in
// groups of two rows).
template <int P, int FL>
constexpr int enc_pair() {
  return (P - ((FL & kEncXor) ? 1 : 0)) <= ((FL & kEncLds) ? 8 : 4) ? 2 : 1;
}

// U sources j..j+U-1: issue all U loads before any arithmetic, then fold the
// sources in pairs; the scheduling barriers keep one pair's temporaries live
// at a time (otherwise the scheduler hoists every lookup and spills).
// kEncXor: source j of the group is folded on its own — at j == 0 it starts
// every row's sum as x & m (acc must be zero), in later groups it is an
// ordinary lookup — and the pairs are (j+1, j+2), ...: one loop body for
// both, so the register budget is that of one group.
template <int U, int MODE>
__device__ __forceinline__ void enc_load_group(uint4 (&x)[U], const uint64_t* __restrict__ sp, int j, long long off,
                                           int len) {
#pragma unroll
  for (int u = 0; u < U; ++u) x[u] = load16<MODE>(sp[j + u], off, len);
}

// Fold the already-loaded sources j..j+U-1 into acc (see chunk16).
template <int P, int U, int FL>
__device__ __forceinline__ void enc_fold_group(uint32_t (&acc)[P][4], const uint4 (&x)[U], int j,
                                           const uint32_t* __restrict__ tbl, unsigned long long r0m,
                                           unsigned c0m, const uint2* lt) {
  constexpr bool X = (FL & kEncXor) != 0;
  constexpr bool LT = (FL & kEncLds) != 0;
  constexpr int U0 = X ? 1 : 0;
  if constexpr (X) {
    if (j == 0) {
#pragma unroll
      for (int l = 0; l < P; ++l) {
        const uint32_t m = (c0m >> l) & 1u ? ~0u : 0u;
        acc[l][0] = x[0].x & m;
        acc[l][1] = x[0].y & m;
        acc[l][2] = x[0].z & m;
        acc[l][3] = x[0].w & m;
      }
    } else {
      mac16<P, true, LT>(acc, x[0], tbl + j * P * kTbl, r0_mask(r0m, j), lt + j * P);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  constexpr int PAIR = enc_pair<P, FL>();
#pragma unroll
  for (int u = U0; u + PAIR <= U; u += PAIR) {
    if constexpr (PAIR == 2)
      mac16x2<P, X, LT>(acc, x[u], x[u + 1], tbl + (j + u) * P * kTbl, tbl + (j + u + 1) * P * kTbl,
                        X ? r0_mask(r0m, j + u) : 0u, X ? r0_mask(r0m, j + u + 1) : 0u,
                        lt + (j + u) * P, lt + (j + u + 1) * P);
    else
      mac16<P, X, LT>(acc, x[u], tbl + (j + u) * P * kTbl, X ? r0_mask(r0m, j + u) : 0u, lt + (j + u) * P);
    __builtin_amdgcn_sched_barrier(0);
  }
  if constexpr (PAIR == 2 && ((U - U0) & 1)) {
    mac16<P, X, LT>(acc, x[U - 1], tbl + (j + U - 1) * P * kTbl, X ? r0_mask(r0m, j + U - 1) : 0u,
                    lt + (j + U - 1) * P);
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int P, int U, int MODE = kPlain, int FL = kEncLUT>
__device__ __forceinline__ void chunk16(uint32_t (&acc)[P][4], const uint64_t* __restrict__ sp,
                                        int j, long long off, const uint32_t* __restrict__ tbl,
                                        int len, unsigned long long r0m = 0, unsigned c0m = 0,
                                        const uint2* lt = nullptr) {
  uint4 x[U];
  enc_load_group<U, MODE>(x, sp, j, off, len);
  enc_fold_group<P, U, FL>(acc, x, j, tbl, r0m, c0m, lt);
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
// The kEncXor variant (FL bit 0) keeps a source's raw dwords live beside its
// selectors (row 0 is x & m): 8 more VGPRs; the verify kernel (FL 16) also
// holds the stored parity: 16 more; so do wide passes with small load groups
// (their remainder loops). Without them these spilled to scratch
// (`make -C isa-l_amd isa` reports every kernel's budget; a larger budget
// is not always better: the scheduler then spends it and may spill).
template <int P, int U, int FL = 0>
constexpr int enc_waves() {
  constexpr int est = (4 * U + 4 * P + 32 + 7) / 8 * 8 + ((FL & 1) ? 8 : 0) + ((FL & 16) ? 16 : 0) +
                      (P >= 5 && U <= 6 ? (P == 8 && U == 4 ? 32 : 16) : 0);
  constexpr int w = 512 / (est + ((FL & kEncLds) ? 16 : 0));
  // kEncLds pairs every pass: two sources' low halves of every row in VGPRs;
  // wide passes get 3 waves' worth (VALU-bound: 12 waves per CU still keep
  // ~120 KB of loads in flight, twice what the HBM latency needs)
  if constexpr ((FL & kEncLds) && P >= 5) return 3;
  return w > 8 ? 8 : (w < 4 ? 4 : w);
}

// acc[l] = XOR_j c[l][j] * src[j][off..off+16) for one lane.
template <int P, class Pol, int FL = kEncLUT>
__device__ __forceinline__ void accum16(uint32_t (&acc)[P][4], const uint64_t* __restrict__ src,
                                        const uint32_t* __restrict__ tbl, int k, long long off,
                                        int len, unsigned long long r0m = 0, unsigned c0m = 0,
                                        const uint2* lt = nullptr) {
#pragma unroll
  for (int l = 0; l < P; ++l) acc[l][0] = acc[l][1] = acc[l][2] = acc[l][3] = 0;
  int j = 0;
  for (; j + Pol::U <= k; j += Pol::U) chunk16<P, Pol::U, Pol::LD, FL>(acc, src, j, off, tbl, len, r0m, c0m, lt);
  // Remainder. The launcher only picks U > 4 when U divides k, so there the
  // (cheap, correct for any k) single-source loop is dead in practice.
  if constexpr (Pol::U == 4) {
    if (j + 2 <= k) {
      chunk16<P, 2, Pol::LD, FL>(acc, src, j, off, tbl, len, r0m, c0m, lt);
      j += 2;
    }
  }
  for (; j < k; ++j) chunk16<P, 1, Pol::LD, FL>(acc, src, j, off, tbl, len, r0m, c0m, lt);
}

}  // namespace
