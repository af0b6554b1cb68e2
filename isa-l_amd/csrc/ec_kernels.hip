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
#include <stdio.h>
#include <stdlib.h>

#include <type_traits>
#include <utility>


#include "ec_device.h"

namespace {


// Work order of the vector encode: work item w of nitems -> (stripe, 4 KiB
// column tile). 0: tile fastest. 2 (the library's): XCD-contiguous — blocks
// b, b+8, b+16.. (one XCD under round-robin dispatch) walk one contiguous
// eighth of the items (round 3: -1.0 to -1.3 % per C2 step,
// profiles/r03/r03_enc_order_benches.jsonl); the identity when nitems % 8 != 0.
// The probe (isa-l_amd/tools/ec_probe.hip) specialises further orders.
template <int ORDER>
struct EncOrder;

template <>
struct EncOrder<0> {
  __device__ static void item(unsigned w, unsigned nitems, unsigned tiles, unsigned& stripe, unsigned& tile) {
    stripe = w / tiles;
    tile = w - stripe * tiles;
  }
};

template <>
struct EncOrder<2> {
  __device__ static void item(unsigned w, unsigned nitems, unsigned tiles, unsigned& stripe, unsigned& tile) {
    const unsigned v = xcd_item(w, nitems, 1);
    stripe = v / tiles;
    tile = v - stripe * tiles;
  }
};

// The work items of an encode launch: (stripe, 4 KiB column tile) pairs.
template <int P, class Pol, int FL, int B = kBlock>
__device__ __forceinline__ void encode_items(const uint64_t* __restrict__ ptrs, int ptr_stride, int src0,
                                             int dst0, const uint32_t* __restrict__ tbl, int len, int k,
                                             unsigned nitems, unsigned tiles, unsigned long long r0m,
                                             unsigned c0m) {
  extern __shared__ uint2 enc_lt[];  // kEncLds: {a0, b0} of every coefficient of the pass
  if constexpr ((FL & kEncLds) != 0) {
    for (int i = threadIdx.x; i < k * P; i += B) enc_lt[i] = make_uint2(tbl[i * kTbl], tbl[i * kTbl + 2]);
    __syncthreads();
  }
  for (unsigned w = blockIdx.x; w < nitems; w += gridDim.x) {
    unsigned stripe, tile;
    EncOrder<Pol::ORDER>::item(w, nitems, tiles, stripe, tile);
    const uint64_t* __restrict__ sp = ptrs + static_cast<size_t>(stripe) * ptr_stride;
    const long long off = static_cast<long long>(tile) * (B * kVec) + threadIdx.x * kVec;
    if (off + kVec <= len) {
      uint32_t acc[P][4];
      accum16<P, Pol, FL>(acc, sp + src0, tbl, k, off, len, r0m, c0m, enc_lt);
#pragma unroll
      for (int l = 0; l < P; ++l)
        store16<Pol::ST>(sp[dst0 + l], off, make_uint4(acc[l][0], acc[l][1], acc[l][2], acc[l][3]),
                         len);
    } else if (off < len) {
      dot_bytes<P>(sp, src0, dst0, tbl, k, off, static_cast<int>(len - off));
    }
  }
}

template <int P, class Pol = EncDefault, int FL = kEncLUT, int B = kBlock>
__global__ __launch_bounds__(B, (enc_waves<P, Pol::U, FL>())) void ec_encode_v16(
    const uint64_t* __restrict__ ptrs, int ptr_stride, int src0, int dst0,
    const uint32_t* __restrict__ tbl, int len, int k, unsigned nitems, unsigned tiles,
    unsigned long long r0m, unsigned c0m) {
  encode_items<P, Pol, FL, B>(ptrs, ptr_stride, src0, dst0, tbl, len, k, nitems, tiles, r0m, c0m);
}

// End of a kernel-argument call (isal_hip_kdone): the calling
// thread spins on a page-locked host word instead of waiting for the
// runtime's completion signal and its wake-up (~9 us of the call,
// profiles/r04_dropin_hiptrace_b.txt). The kernel-argument kernels store
// their 16- and 4-byte outputs with sc1 (write-through past the XCD's L2), so
// a workgroup publishes them at agent scope — to every XCD, to copies and to
// later kernels on any stream — by waiting for them (vmcnt) before it counts
// itself; only the workgroup that ran the per-byte tail (plain byte stores,
// `tail`) also issues an agent-scope release (an L2 writeback: once per call,
// not once per workgroup). The last workgroup to count resets the counter
// (and a verify's result word) for the thread's next call — the next launch
// on the same stream cannot start before this one ends — and writes the
// result, then the call's sequence number, to the host mailbox. All plain
// vector memory operations.
// Memory-model note: the scheme rests on gfx9/CDNA semantics that the HIP
// memory model does not spell out — vmcnt counts stores and atomics without
// return, and sc1 stores and agent-scope atomics are performed past the
// per-XCD L2 — so that a workgroup's relaxed count is ordered after its own
// results. The last workgroup adds an agent-scope acquire before it reads the
// verify word the others lowered; on another target this needs a release on
// every count instead.
__device__ __forceinline__ void karg_done(const isal_hip_kdone& d, bool tail) {
  if (d.cnt == nullptr) return;  // wave-uniform: the caller synchronises the stream
  if (tail) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned n = gridDim.x, b = blockIdx.x;
    const unsigned gsz = max(32u, (n + ISAL_HIP_KDONE_GROUPS - 1) / ISAL_HIP_KDONE_GROUPS);
    const unsigned g = b / gsz, gn = min(gsz, n - g * gsz), ng = (n + gsz - 1) / gsz;
    unsigned* gc = d.cnt + g * ISAL_HIP_KDONE_STRIDE;
    unsigned* top = d.cnt + ISAL_HIP_KDONE_GROUPS * ISAL_HIP_KDONE_STRIDE;
    if (__hip_atomic_fetch_add(gc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != gn - 1) return;
    __hip_atomic_store(gc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (__hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ng - 1) {
      __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      unsigned long long r = ~0ull;
      if (d.res != nullptr) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // once per call
        r = __hip_atomic_load(d.res, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(d.res, ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __hip_atomic_store(d.mail + 1, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the result lands before the sequence number
      __hip_atomic_store(d.mail, d.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// One stripe whose shard pointers and coefficient tables travel as kernel
// arguments (isal_hip_karg, 2 KiB): the synchronous drop-in call on
// device-resident shards launches this with no argument upload before it
// (a hipMemcpyAsync + blit kernel per call otherwise).
template <int P, class Pol, int FL>
__global__ __launch_bounds__(kBlock, (enc_waves<P, Pol::U, FL>())) void ec_encode_karg(
    const isal_hip_karg a, const isal_hip_kdone d, int len, int k, unsigned tiles, unsigned long long r0m,
    unsigned c0m) {
  // `a` is the first argument, at offset 0 of the kernarg segment: read it in
  // place (scalar loads) — indexing the by-value copy with runtime indices
  // made the compiler copy all 2 KiB of it to scratch.
  const isal_hip_karg* ka = (const isal_hip_karg*)__builtin_amdgcn_kernarg_segment_ptr();
  encode_items<P, Pol, FL>(ka->ptrs, k + P, 0, k, ka->tbl, len, k, tiles, tiles, r0m, c0m);
  karg_done(d, (len & (kVec - 1)) != 0 && blockIdx.x == gridDim.x - 1);
}

// ---------------------------------------------------------------------------
// Wide passes with the sources staged through LDS by LDS-DMA (ENC_GLDS)
//
// The register-staged encode loads a group of U sources, folds it, loads the
// next: between groups a wave has no load in flight, and with 6-8 rows the
// fold is long (k20p6: four dependent groups of 5 per tile at 3-4 waves per
// SIMD). Here each wave owns a ring of R 1-KiB LDS slots (64 lanes
// x 16 B, the lane-linear layout one global_load_lds_dwordx4 writes) and keeps
// R source loads in flight all the time: it waits for source j's DMA with a
// counted vmcnt (nothing else orders a ds_read behind the issuing wave's own
// LDS-DMA), reads the slot with ds_read_b128, refills the slot with source
// j + R and folds j — the loads cost no VGPRs. The DMA and the slot reads are
// inline asm, so hipcc neither counts nor waits for them: every wait here is
// explicit. Tiles that are not full (a shard's ragged end) take the
// register path.
// ---------------------------------------------------------------------------
typedef __attribute__((address_space(3))) uint8_t lds_u8;

template <class F, int... I>
__device__ __forceinline__ void static_for(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}

__device__ __forceinline__ uint32_t lds_off(const void* p) {
  return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((const lds_u8*)p));
}

// 16 bytes per lane from base + voff into LDS at m0 + 16 * lane (nt)
__device__ __forceinline__ void glds16(uint64_t base_, uint32_t voff, uint32_t m0) {
  // readfirstlane returns a (signed) int: widen each half through uint32_t,
  // or a low half with bit 31 set sign-extends over the high half
  const uint32_t hi = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(base_ >> 32)));
  const uint32_t lo = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(base_)));
  const uint64_t base = (static_cast<uint64_t>(hi) << 32) | lo;
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(base), "s"(m0)
               : "memory");
}

template <int OA, int OB>
__device__ __forceinline__ void lds_read2(uint4& a, uint4& b, uint32_t addr) {
  u32x4 x, y;
  asm volatile("ds_read_b128 %0, %2 offset:%3\n\tds_read_b128 %1, %2 offset:%4\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(x), "=&v"(y)
               : "v"(addr), "i"(OA), "i"(OB)
               : "memory");
  a = make_uint4(x.x, x.y, x.z, x.w);
  b = make_uint4(y.x, y.y, y.z, y.w);
}

template <int OA>
__device__ __forceinline__ void lds_read1(uint4& a, uint32_t addr) {
  u32x4 x;
  asm volatile("ds_read_b128 %0, %1 offset:%2\n\ts_waitcnt lgkmcnt(0)" : "=&v"(x) : "v"(addr), "i"(OA) : "memory");
  a = make_uint4(x.x, x.y, x.z, x.w);
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// vmcnt(n) for a wave-uniform runtime n < 8
__device__ __forceinline__ void vm_wait_rt(int n) {
  switch (n) {
    case 0: vm_wait<0>(); break;
    case 1: vm_wait<1>(); break;
    case 2: vm_wait<2>(); break;
    case 3: vm_wait<3>(); break;
    case 4: vm_wait<4>(); break;
    case 5: vm_wait<5>(); break;
    case 6: vm_wait<6>(); break;
    default: vm_wait<7>(); break;
  }
}

template <int P, int R, int FL>
__global__ __launch_bounds__(kBlock, 4) void ec_encode_glds(const uint64_t* __restrict__ ptrs, int ptr_stride,
                                                           int src0, int dst0, const uint32_t* __restrict__ tbl,
                                                           int len, int k, unsigned nitems, unsigned tiles,
                                                           unsigned long long r0m, unsigned c0m) {
  static_assert(R % 2 == 0 && R >= 4 && R <= 8, "ring of 4..8 slots, folded in pairs");
  constexpr bool X = (FL & kEncXor) != 0;
  constexpr bool LT = (FL & kEncLds) != 0;
  static_assert(LT || P - (X ? 1 : 0) <= 4, "pairs from SGPR tables only up to 4 looked-up rows");
  extern __shared__ uint2 enc_lt[];
  const int ltn = LT ? k * P : 0;
  if constexpr (LT) {
    for (int i = threadIdx.x; i < ltn; i += kBlock) enc_lt[i] = make_uint2(tbl[i * kTbl], tbl[i * kTbl + 2]);
  }
  __syncthreads();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t ring = lds_off(enc_lt) + ((static_cast<uint32_t>(ltn) * 8 + 1023) & ~1023u) + wave * (R * 1024);
  const uint32_t mine = ring + (threadIdx.x & 63) * kVec;
  const uint2* lt = enc_lt;
  for (unsigned w = blockIdx.x; w < nitems; w += gridDim.x) {
    const unsigned v = xcd_item(w, nitems, 1);
    const unsigned stripe = v / tiles;
    const unsigned tile = v - stripe * tiles;
    const uint64_t* __restrict__ sp = ptrs + static_cast<size_t>(stripe) * ptr_stride;
    const long long off = static_cast<long long>(tile) * kTile + threadIdx.x * kVec;
    if (static_cast<long long>(tile + 1) * kTile <= len) {
      vm_wait<0>();  // this wave's stores of an earlier item (one counter for loads and stores)
      const uint32_t voff = static_cast<uint32_t>(off);
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (r < k) glds16(sp[src0 + r], voff, ring + r * 1024);
      uint32_t acc[P][4];
#pragma unroll
      for (int l = 0; l < P; ++l) acc[l][0] = acc[l][1] = acc[l][2] = acc[l][3] = 0;
      for (int j0 = 0; j0 < k; j0 += R) {
        // slots r, r + 1 (compile-time LDS offsets): sources j0 + r, j0 + r + 1
        auto step = [&](auto rc) {
          constexpr int r = decltype(rc)::value * 2;
          const int j = j0 + r;
          if (j >= k) return;
          uint4 x0, x1;
          if (j + 1 < k) {
            // loads issued: sources < min(k, j + R); wait for j + 1
            if (j + R <= k)
              vm_wait<R - 2>();
            else
              vm_wait_rt(k - 2 - j);
            lds_read2<r * 1024, (r + 1) * 1024>(x0, x1, mine);
            if (j + R < k) glds16(sp[src0 + j + R], voff, ring + r * 1024);
            if (j + 1 + R < k) glds16(sp[src0 + j + 1 + R], voff, ring + (r + 1) * 1024);
            __builtin_amdgcn_sched_barrier(0);
            if (X && j == 0) {
#pragma unroll
              for (int l = 0; l < P; ++l) {
                const uint32_t m = (c0m >> l) & 1u ? ~0u : 0u;
                acc[l][0] = x0.x & m;
                acc[l][1] = x0.y & m;
                acc[l][2] = x0.z & m;
                acc[l][3] = x0.w & m;
              }
              mac16<P, X, LT>(acc, x1, tbl + P * kTbl, r0_mask(r0m, 1), lt + P);
            } else {
              mac16x2<P, X, LT>(acc, x0, x1, tbl + j * P * kTbl, tbl + (j + 1) * P * kTbl,
                                X ? r0_mask(r0m, j) : 0u, X ? r0_mask(r0m, j + 1) : 0u, lt + j * P,
                                lt + (j + 1) * P);
            }
          } else {
            vm_wait<0>();
            lds_read1<r * 1024>(x0, mine);
            __builtin_amdgcn_sched_barrier(0);
            if (X && j == 0) {
#pragma unroll
              for (int l = 0; l < P; ++l) {
                const uint32_t m = (c0m >> l) & 1u ? ~0u : 0u;
                acc[l][0] = x0.x & m;
                acc[l][1] = x0.y & m;
                acc[l][2] = x0.z & m;
                acc[l][3] = x0.w & m;
              }
            } else {
              mac16<P, X, LT>(acc, x0, tbl + j * P * kTbl, X ? r0_mask(r0m, j) : 0u, lt + j * P);
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        };
        static_for(step, std::make_integer_sequence<int, R / 2>{});
      }
      // Every DMA of the item has landed already (the last source's wait is
      // vmcnt(0)); the explicit drain makes that visible on every path of the
      // control flow, so the stores and the next item never run inside a
      // counted window (tests/test_kernel_objects_cpu.py checks the ISA).
      vm_wait<0>();
#pragma unroll
      for (int l = 0; l < P; ++l)
        store16<kBufNT>(sp[dst0 + l], off, make_uint4(acc[l][0], acc[l][1], acc[l][2], acc[l][3]), len);
    } else if (off + kVec <= len) {
      uint32_t acc[P][4];
      accum16<P, EncPol<4, kBufNT, kBufNT, 2>, FL>(acc, sp + src0, tbl, k, off, len, r0m, c0m, lt);
#pragma unroll
      for (int l = 0; l < P; ++l)
        store16<kBufNT>(sp[dst0 + l], off, make_uint4(acc[l][0], acc[l][1], acc[l][2], acc[l][3]), len);
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
// Verify (xor_check / pq_check): recompute the parity of each column exactly
// like the encode (same load groups, 0/1 XOR path) and compare it with the
// stored rows at dst; mismatches lower *bad (key = column << 8 | row) with
// atomicMin — an LDS word per workgroup (generic launch: one slot per
// workgroup, so the result may live in page-locked host memory) or the
// call's device result word (kernel-argument launch). Nothing is written to
// the shards.
// ---------------------------------------------------------------------------
// sbad != nullptr (a batch): each stripe's mismatches lower sbad[stripe]
// instead, and items run in the XCD-contiguous order of the encode.
template <int P, class Pol, int FL>
__device__ __forceinline__ void verify_items(const uint64_t* __restrict__ ptrs, int ptr_stride, int src0, int dst0,
                                             const uint32_t* __restrict__ tbl, int len, int k, unsigned nitems,
                                             unsigned tiles, unsigned long long r0m, unsigned c0m,
                                             unsigned long long* bad, int row0, long long col0,
                                             unsigned long long* sbad = nullptr) {
  for (unsigned ww = blockIdx.x; ww < nitems; ww += gridDim.x) {
    const unsigned w = xcd_item(ww, nitems, sbad != nullptr);
    const unsigned stripe = w / tiles;
    if (sbad != nullptr) bad = sbad + stripe;
    const unsigned tile = w - stripe * tiles;
    const uint64_t* __restrict__ sp = ptrs + static_cast<size_t>(stripe) * ptr_stride;
    const long long off = static_cast<long long>(tile) * kTile + threadIdx.x * kVec;
    if (off + kVec <= len) {
      // Up to 3 rows (RAID P / P+Q, the drop-in xor_check / pq_check) the
      // stored rows are loaded before the sources' fold, so their latency
      // overlaps it instead of following it: one HBM round trip less per
      // tile. Wider passes would spill the extra 4 VGPRs per row.
      constexpr bool kEarly = P <= 3;
      uint4 st[kEarly ? P : 1];
      if constexpr (kEarly) {
#pragma unroll
        for (int l = 0; l < P; ++l) st[l] = load16<kBufNT>(sp[dst0 + l], off, len);
      }
      uint32_t acc[P][4];
      accum16<P, Pol, FL>(acc, sp + src0, tbl, k, off, len, r0m, c0m);
#pragma unroll
      for (int l = 0; l < P; ++l) {
        const uint4 e = kEarly ? st[kEarly ? l : 0] : load16<kBufNT>(sp[dst0 + l], off, len);
        const uint32_t x[4] = {acc[l][0] ^ e.x, acc[l][1] ^ e.y, acc[l][2] ^ e.z, acc[l][3] ^ e.w};
#pragma unroll
        for (int d = 0; d < 4; ++d)
          if (x[d]) {
            note_mismatch(bad, col0 + off + 4 * d + (__builtin_ctz(x[d]) >> 3), row0 + l);
            break;
          }
      }
    } else if (off < len) {
      dot_bytes<P, true>(sp, src0, dst0, tbl, k, off, static_cast<int>(len - off), bad, row0, col0);
    }
  }
}

template <int P, class Pol, int FL>
__global__ __launch_bounds__(kBlock, (enc_waves<P, Pol::U, FL | kEncVerify>())) void ec_verify_v16(
    const uint64_t* __restrict__ ptrs, int ptr_stride, int src0, int dst0, const uint32_t* __restrict__ tbl,
    int len, int k, unsigned nitems, unsigned tiles, unsigned long long* __restrict__ slots, int row0,
    long long col0, unsigned long long r0m, unsigned c0m, unsigned long long* sbad) {
  __shared__ unsigned long long blk_min;
  if (threadIdx.x == 0) blk_min = ~0ull;
  __syncthreads();
  verify_items<P, Pol, FL>(ptrs, ptr_stride, src0, dst0, tbl, len, k, nitems, tiles, r0m, c0m, &blk_min, row0,
                           col0, sbad);
  if (slots != nullptr) {
    __syncthreads();
    if (threadIdx.x == 0) slots[blockIdx.x] = blk_min;
  }
}

// One stripe's verify with its arguments in the kernarg segment (as
// ec_encode_karg); the result travels through the completion mailbox.
template <int P, class Pol, int FL>
__global__ __launch_bounds__(kBlock, (enc_waves<P, Pol::U, FL | kEncVerify>())) void ec_verify_karg(
    const isal_hip_karg a, const isal_hip_kdone d, int len, int k, unsigned tiles, unsigned long long r0m,
    unsigned c0m) {
  const isal_hip_karg* ka = (const isal_hip_karg*)__builtin_amdgcn_kernarg_segment_ptr();
  verify_items<P, Pol, FL>(ka->ptrs, k + P, 0, k, ka->tbl, len, k, tiles, tiles, r0m, c0m, d.res, 0, 0);
  karg_done(d, false);
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

template <int P, int ST = kBufNT, int B = kBlock>
__device__ __forceinline__ void update_items(const uint64_t* __restrict__ ptrs, int ptr_stride, int src_idx,
                                             int dst0, const uint32_t* __restrict__ tbl, int len,
                                             unsigned nitems, unsigned tiles) {
  for (unsigned w = blockIdx.x; w < nitems; w += gridDim.x) {
    const unsigned stripe = w / tiles;
    const unsigned tile = w - stripe * tiles;
    const uint64_t* __restrict__ sp = ptrs + static_cast<size_t>(stripe) * ptr_stride;
    const long long off = static_cast<long long>(tile) * (B * kVec) + threadIdx.x * kVec;
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
        store16<ST>(sp[dst0 + l], off, d[l], len);
      }
    } else if (off < len) {
      mad_bytes<P>(sp, src_idx, dst0, tbl, off, static_cast<int>(len - off));
    }
  }
}

// The drop-in call's single stripe, 4 bytes of every shard per lane instead
// of 16 (ISAL_HIP_KARG_NARROW): a C2 stripe is then 1024 workgroups (16 waves
// per CU) instead of 256 (4 per CU), so one call's loads and lookups overlap
// across waves rather than running back to back in one wave per SIMD.
__device__ __forceinline__ uint32_t load4nt(uint64_t base, long long off, int len) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(base), 0, len, 0x00020000);
  return static_cast<uint32_t>(__builtin_amdgcn_raw_buffer_load_b32(rs, static_cast<int>(off), 0, 2 /* nt */));
}

// sc1 + nt (gfx950 CPol 0x12): write-through, see karg_done
__device__ __forceinline__ void store4wt(uint64_t base, long long off, uint32_t v, int len) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(base), 0, len, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b32(static_cast<int>(v), rs, static_cast<int>(off), 0, 0x12);
}

template <int P>
__device__ __forceinline__ void fold4(uint32_t (&acc)[P], uint32_t x, const uint32_t* __restrict__ t) {
  const Sel s = split(x);
#pragma unroll
  for (int l = 0; l < P; ++l) acc[l] ^= gf_mul4(load_coef(t + l * kTbl), s);
}

template <int P>
__global__ __launch_bounds__(kBlock) void ec_encode_karg4(const isal_hip_karg a, const isal_hip_kdone d, int len,
                                                          int k) {
  const isal_hip_karg* ka = (const isal_hip_karg*)__builtin_amdgcn_kernarg_segment_ptr();
  const long long off = (static_cast<long long>(blockIdx.x) * kBlock + threadIdx.x) * 4;
  if (off + 4 <= len) {
    uint32_t acc[P];
#pragma unroll
    for (int l = 0; l < P; ++l) acc[l] = 0;
    int j = 0;
    for (; j + 8 <= k; j += 8) {
      uint32_t x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = load4nt(ka->ptrs[j + u], off, len);
#pragma unroll
      for (int u = 0; u < 8; ++u) fold4<P>(acc, x[u], ka->tbl + (j + u) * P * kTbl);
    }
    for (; j < k; ++j) fold4<P>(acc, load4nt(ka->ptrs[j], off, len), ka->tbl + j * P * kTbl);
#pragma unroll
    for (int l = 0; l < P; ++l) store4wt(ka->ptrs[k + l], off, acc[l], len);
  } else if (off < len) {
    dot_bytes<P>(ka->ptrs, 0, k, ka->tbl, k, off, static_cast<int>(len - off));
  }
  karg_done(d, (len & 3) != 0 && blockIdx.x == gridDim.x - 1);
}

template <int P, int B = kBlock>
__global__ __launch_bounds__(B) void ec_update_v16(const uint64_t* __restrict__ ptrs,
                                                   int ptr_stride, int src_idx, int dst0,
                                                   const uint32_t* __restrict__ tbl, int len,
                                                   unsigned nitems, unsigned tiles) {
  update_items<P, kBufNT, B>(ptrs, ptr_stride, src_idx, dst0, tbl, len, nitems, tiles);
}

// One update call whose pointers (source, then P parity rows) and the source's
// P coefficient tables travel as kernel arguments (as ec_encode_karg).
template <int P>
__global__ __launch_bounds__(kBlock) void ec_update_karg(const isal_hip_karg a, const isal_hip_kdone d, int len,
                                                         unsigned tiles) {
  const isal_hip_karg* ka = (const isal_hip_karg*)__builtin_amdgcn_kernarg_segment_ptr();
  update_items<P, kBufSC1NT>(ka->ptrs, 1 + P, 0, 1, ka->tbl, len, tiles, tiles);
  karg_done(d, (len & (kVec - 1)) != 0 && blockIdx.x == gridDim.x - 1);
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
// Wide passes with the products looked up in LDS (ec_encode_ldsx, round 6)
//
// The v_perm product costs ~4.5 VALU per (source dword, output row), so passes
// of 6-8 rows are VALU-bound ("the memory skeleton"). Here one LDS
// lookup returns the products of one source-byte field with ALL P
// coefficients of the pass: per source j a 32-entry table T5_j (bits 0-4 of
// the byte) and an 8-entry table T3_j (bits 5-7), 8-byte entries whose byte l
// is row l's product (isal_hip_build_ldsx_tables). A lane keeps its 16 byte
// positions as 16 two-dword accumulators (byte l = row l's partial) —
// two lookups and one XOR3 per half per source byte — and transposes them
// into the P rows with v_perm once per tile. Per source dword: 12 offset ops
// (the fields pre-scaled by 8, one SDWA add of the table base each), 8 XOR3
// and 8 ds_read_b64, whatever P. Both tables fill at most one LDS bank row
// (32 x 8 B), so the lookups never bank-conflict.
// ---------------------------------------------------------------------------
struct Acc64 {
  uint32_t lo, hi;
};

template <int B>
__device__ __forceinline__ uint32_t add_byte(uint32_t v, uint32_t base) {
  uint32_t r;
  if constexpr (B == 0)
    asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:DWORD"
        : "=v"(r) : "v"(v), "v"(base));
  else if constexpr (B == 1)
    asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD"
        : "=v"(r) : "v"(v), "v"(base));
  else if constexpr (B == 2)
    asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:DWORD"
        : "=v"(r) : "v"(v), "v"(base));
  else
    asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:DWORD"
        : "=v"(r) : "v"(v), "v"(base));
  return r;
}

__device__ __forceinline__ uint64_t lds_u64(uint32_t addr) {
  return *reinterpret_cast<const __attribute__((address_space(3))) uint64_t*>(static_cast<uintptr_t>(addr));
}

// acc[4d + b] ^= T5[bits 0-4 of byte b of dword d] ^ T3[bits 5-7] for one
// 16-byte source chunk; b5 / b3: LDS byte addresses of the source's tables
__device__ __forceinline__ void ldsx_acc(Acc64 (&acc)[16], const uint4& x, uint32_t b5, uint32_t b3) {
  const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const uint32_t lo8 = (w[d] << 3) & 0xF8F8F8F8u;  // bits 0-4 of each byte, times 8
    const uint32_t hi8 = (w[d] >> 2) & 0x38383838u;  // bits 5-7 of each byte, times 8
    auto one = [&](auto bc) __attribute__((always_inline)) {
      constexpr int b = decltype(bc)::value;
      const uint64_t p = lds_u64(add_byte<b>(lo8, b5));
      const uint64_t q = lds_u64(add_byte<b>(hi8, b3));
      Acc64& a = acc[4 * d + b];
      a.lo = xor3(a.lo, static_cast<uint32_t>(p), static_cast<uint32_t>(q));
      a.hi = xor3(a.hi, static_cast<uint32_t>(p >> 32), static_cast<uint32_t>(q >> 32));
    };
    one(std::integral_constant<int, 0>{});
    one(std::integral_constant<int, 1>{});
    one(std::integral_constant<int, 2>{});
    one(std::integral_constant<int, 3>{});
  }
}

// transpose the 16 accumulators into the P rows' 16 bytes and store them: row
// l, dword d = byte l of acc[4d .. 4d + 3] (rows 0-3 in .lo, 4-7 in .hi)
template <int P, int ST = kBufNT>
__device__ __forceinline__ void ldsx_store(const Acc64 (&acc)[16], const uint64_t* __restrict__ sp, int dst0,
                                           long long off, int len) {
  uint32_t out[P][4];
#pragma unroll
  for (int d = 0; d < 4; ++d) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (4 * h >= P) continue;
      const uint32_t A = h ? acc[4 * d].hi : acc[4 * d].lo, B = h ? acc[4 * d + 1].hi : acc[4 * d + 1].lo;
      const uint32_t C = h ? acc[4 * d + 2].hi : acc[4 * d + 2].lo, D = h ? acc[4 * d + 3].hi : acc[4 * d + 3].lo;
      const uint32_t ab0 = __builtin_amdgcn_perm(B, A, 0x05010400u), ab1 = __builtin_amdgcn_perm(B, A, 0x07030602u);
      const uint32_t cd0 = __builtin_amdgcn_perm(D, C, 0x05010400u), cd1 = __builtin_amdgcn_perm(D, C, 0x07030602u);
      const uint32_t r[4] = {__builtin_amdgcn_perm(cd0, ab0, 0x05040100u), __builtin_amdgcn_perm(cd0, ab0, 0x07060302u),
                             __builtin_amdgcn_perm(cd1, ab1, 0x05040100u), __builtin_amdgcn_perm(cd1, ab1, 0x07060302u)};
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (4 * h + q < P) out[4 * h + q][d] = r[q];
    }
  }
#pragma unroll
  for (int l = 0; l < P; ++l)
    store16<ST>(sp[dst0 + l], off, make_uint4(out[l][0], out[l][1], out[l][2], out[l][3]), len);
}

template <int P, int U, int ST, int B = kBlock>
__device__ __forceinline__ void ldsx_items(const uint64_t* __restrict__ ptrs, int ptr_stride, int src0, int dst0,
                                           const uint32_t* __restrict__ tbl, const uint64_t* __restrict__ ltg,
                                           int len, int k, unsigned nitems, unsigned tiles) {
  extern __shared__ uint64_t ldsx_t[];  // [k][32] T5, then [k][8] T3
  for (int i = threadIdx.x; i < k * ISAL_HIP_LDSX_ENTRIES; i += B) ldsx_t[i] = ltg[i];
  __syncthreads();
  const uint32_t base5 = lds_off(ldsx_t), base3 = base5 + static_cast<uint32_t>(k) * 256u;
  for (unsigned w = blockIdx.x; w < nitems; w += gridDim.x) {
    const unsigned v = xcd_item(w, nitems, 1);
    const unsigned stripe = v / tiles;
    const unsigned tile = v - stripe * tiles;
    const uint64_t* __restrict__ sp = ptrs + static_cast<size_t>(stripe) * ptr_stride;
    const long long off = static_cast<long long>(tile) * (B * kVec) + threadIdx.x * kVec;
    if (off + kVec > len) {
      if (off < len) dot_bytes<P>(sp, src0, dst0, tbl, k, off, static_cast<int>(len - off));
      continue;
    }
    Acc64 acc[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = Acc64{0u, 0u};
    // groups of U sources, double-buffered: group g + 1's loads are issued
    // before group g is folded (2U loads in flight per lane); k is uniform,
    // so the bounds tests are scalar branches
    uint4 a[U];
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = u < k ? load16<kBufNT>(sp[src0 + u], off, len) : make_uint4(0, 0, 0, 0);
    for (int j = 0; j < k; j += U) {
      uint4 b[U];
#pragma unroll
      for (int u = 0; u < U; ++u)
        b[u] = j + U + u < k ? load16<kBufNT>(sp[src0 + j + U + u], off, len) : make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (j + u < k) ldsx_acc(acc, a[u], base5 + (j + u) * 256u, base3 + (j + u) * 64u);
#pragma unroll
      for (int u = 0; u < U; ++u) a[u] = b[u];
    }
    ldsx_store<P, ST>(acc, sp, dst0, off, len);
  }
}

template <int P, int U>
__global__ __launch_bounds__(kBlock) void ec_encode_ldsx(const uint64_t* __restrict__ ptrs, int ptr_stride, int src0,
                                                         int dst0, const uint32_t* __restrict__ tbl,
                                                         const uint64_t* __restrict__ ltg, int len, int k,
                                                         unsigned nitems, unsigned tiles) {
  ldsx_items<P, U, kBufNT>(ptrs, ptr_stride, src0, dst0, tbl, ltg, len, k, nitems, tiles);
}

// The drop-in call's single stripe through the LDS product tables (a wide
// pass of 7-8 rows; the thread's table cache uploads them, isal_hip_shim.c):
// pointers and v_perm tables (for the ragged tail) as kernel arguments, the
// parity stored write-through and completed through the mailbox as
// ec_encode_karg.
template <int P>
__global__ __launch_bounds__(kBlock) void ec_encode_karg_ldsx(const isal_hip_karg a, const isal_hip_kdone d,
                                                              const uint64_t* __restrict__ ltg, int len, int k,
                                                              unsigned tiles) {
  const isal_hip_karg* ka = (const isal_hip_karg*)__builtin_amdgcn_kernarg_segment_ptr();
  ldsx_items<P, 2, kBufSC1NT>(ka->ptrs, k + P, 0, k, ka->tbl, ltg, len, k, tiles, tiles);
  karg_done(d, (len & (kVec - 1)) != 0 && blockIdx.x == gridDim.x - 1);
}

// ---------------------------------------------------------------------------
// Host-side launch helpers
// ---------------------------------------------------------------------------
constexpr unsigned kMaxItems = 1u << 30;  // keep w / tiles in 32-bit scalar math

// One workgroup per item. (A capped grid striding over the items lost 13-20 %
// on C2 at 2048-16384 workgroups, profiles/r04_ldsmin_ab.jsonl; the knob that
// chose it was removed in round 5.)
unsigned grid_for(unsigned nitems) { return nitems; }

// Passes of 5-8 rows stage their sources through the LDS-DMA ring
// (ec_encode_glds, 4 slots per wave; ISAL_HIP_ENC_GLDS=0 off). Same box, two
// interleaved rounds (profiles/r05/r05_glds_ab.jsonl), fraction of 8 TB/s
// registers -> ring of 4: k20p6 0.676/0.673 -> 0.677/0.678, k20p8
// 0.596/0.598 -> 0.603/0.603, k10p8 0.731/0.731 -> 0.736/0.738, k10p6
// 0.765/0.765 -> 0.766/0.769; rings of 6 and 8 (more LDS, fewer
// workgroups per CU) were flat to 3.5 % slower and are not built.
constexpr int kGldsRing = 4;
int enc_glds(int P) {
  return P >= 5 && isal_hip_knob(ISAL_HIP_KNOB_ENC_GLDS) != 0 ? kGldsRing : 0;
}

template <int P, int R, int FL>
void launch_glds(unsigned grid, hipStream_t s, const uint64_t* ptrs, int ptr_stride, int src0, int dst0,
                 const uint32_t* tbl, int len, int k, unsigned nitems, unsigned tiles, unsigned long long r0m,
                 unsigned c0m) {
  if (isal_hip_knob(ISAL_HIP_KNOB_LOG) >= 2)
    fprintf(stderr, "isal_hip: kernel ec_encode_glds<%d, %d, %d>\n", P, R, FL);
  const size_t lds = ((static_cast<size_t>(k) * P * 8 + 1023) & ~static_cast<size_t>(1023)) + 4u * R * 1024u;
  ISAL_LAUNCH((ec_encode_glds<P, R, FL>), dim3(grid), dim3(kBlock), lds, s, ptrs, ptr_stride, src0, dst0, tbl,
                     len, k, nitems, tiles, r0m, c0m);
}

template <int P>
void launch_glds_r(bool x, unsigned grid, hipStream_t s, const uint64_t* ptrs, int ptr_stride, int src0, int dst0,
                   const uint32_t* tbl, int len, int k, unsigned nitems, unsigned tiles, unsigned long long r0m,
                   unsigned c0m) {
  if constexpr (P >= 5) {
    if (x)
      launch_glds<P, kGldsRing, kEncXor | kEncLds>(grid, s, ptrs, ptr_stride, src0, dst0, tbl, len, k, nitems, tiles,
                                                   r0m, c0m);
    else
      launch_glds<P, kGldsRing, kEncLds>(grid, s, ptrs, ptr_stride, src0, dst0, tbl, len, k, nitems, tiles, 0ull, 0u);
  }
}

// Passes of 6-8 rows over k = 10, 15, 20, ... sources load in groups of 5
// (ISAL_HIP_ENC_WIDE5=0 off): the smaller group leaves the registers for a
// wave more per SIMD, and lets 7-8 row passes take the LDS table halves
// without dropping to 3 waves. Same-box A/B, two runs each
// (profiles/r04_wide5_ab.jsonl): k10p6 0.753 -> 0.766 of 8 TB/s, k10p7
// 0.741 -> 0.747, k10p8 0.721 -> 0.732, k20p6 0.663 -> 0.670, k20p8 0.564 ->
// 0.591, k30p6 0.673 -> 0.680, k15p6 (already 5) flat; C2 (4 rows) 0.780 ->
// 0.772 with 5 (profiles/r04_group_ab.jsonl), so narrower passes keep the
// large group.
bool enc_wide5(int k, int P) {
  return P >= 6 && k >= 10 && k % 5 == 0 && isal_hip_knob(ISAL_HIP_KNOB_ENC_WIDE5) != 0;
}

// Load-group size for k sources: the largest of {12,10,8,6,5,4} dividing k
// (all of a stripe's loads in flight at once for the common k), else 4;
// P = the pass's rows (0: not known, the drop-in kernel-argument launch).
int enc_group(int k, int P = 0) {
  static const int cand[] = {12, 10, 8, 6, 5, 4};
  const long long force = isal_hip_knob(ISAL_HIP_KNOB_ENC_GROUP);  // tuning A/B: one of cand
  for (int u : cand)
    if (force == u) return u;
  if (enc_wide5(k, P)) return 5;
  for (int u : cand)
    if (k >= u && k % u == 0) return u;
  return 4;
}

// Low table halves from LDS (kEncLds). Same-box A/B, two runs each
// (profiles/r04_lds_ab.jsonl, with the XOR path): k20p6 0.635 -> 0.663 of
// 8 TB/s, k10p6 0.752 -> 0.754, C2 0.7705 -> 0.7695, k10p8 0.715 -> 0.702,
// decode (p = 3) 0.742 -> 0.744. It pays where pairing from SGPRs is not
// possible (more than 4 looked-up rows) and the pass is not so wide that 3
// waves per SIMD starve it: 5-6 rows, and 7-8 rows loading in groups of 5
// (enc_wide5). ISAL_HIP_ENC_LDS=1 forces it for every width, =0 turns it off.
bool enc_lds(int P, bool x, int U) {
  const long long v = isal_hip_knob(ISAL_HIP_KNOB_ENC_LDS);
  if (v == 0 || v == 1) return v == 1;
  return P - (x ? 1 : 0) > 4 && (P <= 6 || (U == 5 && isal_hip_knob(ISAL_HIP_KNOB_ENC_WIDE5) != 0));
}

template <int P>
size_t lds_bytes(int k) {
  return static_cast<size_t>(k) * P * sizeof(uint2);
}

// XOR fast path (isal_hip_encmask) and LDS table halves only in the default
// policy: XCD-contiguous order, nt buffer loads and stores.

// Dynamic LDS each vector-encode workgroup of a pass of at most 4 rows
// allocates: what it uses, at least 32 KiB — an occupancy cap of 5 workgroups
// (5 waves per SIMD) per CU, whose 160 KiB of LDS the workgroups share. The
// narrow passes' kernels fit 6-8 waves per SIMD by their registers and run
// faster capped, same box, two runs each (profiles/r04_occupancy_ab.jsonl,
// r04_ldsmin_ab.jsonl): C3 decode 0.742-0.746 -> 0.754-0.756 of 8 TB/s,
// k10p1 0.728 -> 0.748, k10p2 0.731 -> 0.757, k4p2 0.780 -> 0.798, C2 flat;
// wider passes (4-5 waves by their registers) measured flat to 2 % slower
// with it (k20p6 0.679 -> 0.664), so they allocate only what they use.
// (The ISAL_HIP_ENC_LDS_MIN knob that varied it was removed in round 5.)
size_t enc_lds_alloc(size_t used, int P) {
  const size_t min = P <= 4 ? 32768 : 0;
  return used > min ? used : min;
}

// ISAL_HIP_LOG=2: name each vector encode launch the way rocprofv3 prints it
// (bench.py's roofline.kernel must name the same instantiation;
// test_bench_kernel_label_matches_launch).
template <int P, class Pol, int FL, int B>
void log_launch() {
  if (isal_hip_knob(ISAL_HIP_KNOB_LOG) >= 2)
    fprintf(stderr, "isal_hip: kernel ec_encode_v16<%d, EncPol<%d, %d, %d, %d>, %d, %d>\n", P, Pol::U, Pol::LD,
            Pol::ST, Pol::ORDER, FL, B);
}

// Lanes per vector-encode workgroup: 128 (2 KiB tiles) for passes of 1-2
// rows, 256 otherwise. Same box, three interleaved rounds, ms per launch
// (profiles/r06/r06_v16_block_ab.jsonl), both with the 32 KiB occupancy cap:
// xor_gen 1.955 / 1.951 / 1.950 at 128 against 1.979 / 1.978 / 1.972 at 256,
// pq_gen 2.110 / 2.112 / 2.116 against 2.137 / 2.134 / 2.129. For 3-4 rows
// 128 lanes lose 1-2 % under that cap (C2 2.449-2.456 vs 2.393-2.401) and
// tie under a 16 KiB one (the same 20 waves per CU as 256 lanes: C2 2.388 /
// 2.396 / 2.388, decode 2.300 / 2.302 / 2.314 vs 2.306 / 2.306 / 2.316).
template <int P>
constexpr int enc_block() {
  return P <= 2 ? 128 : kBlock;
}
constexpr long long kEncMinSpan = 128 * kVec;  // the smallest tile any encode pass uses

template <int P, int U, int FL>
void launch_fl(hipStream_t s, const uint64_t* ptrs, int ptr_stride, int src0, int dst0, const uint32_t* tbl,
               int len, int k, unsigned nstripes, unsigned long long r0m, unsigned c0m) {
  constexpr int B = enc_block<P>();
  log_launch<P, EncPol<U, kBufNT, kBufNT, 2>, FL, B>();
  const unsigned tiles = static_cast<unsigned>((static_cast<long long>(len) + B * kVec - 1) / (B * kVec));
  const unsigned nitems = nstripes * tiles;
  const size_t lds = enc_lds_alloc((FL & kEncLds) ? lds_bytes<P>(k) : 0, P);
  ISAL_LAUNCH((ec_encode_v16<P, EncPol<U, kBufNT, kBufNT, 2>, FL, B>), dim3(grid_for(nitems)), dim3(B), lds, s,
              ptrs, ptr_stride, src0, dst0, tbl, len, k, nitems, tiles, r0m, c0m);
}

template <int P, int U>
void launch_v16(hipStream_t s, const uint64_t* ptrs, int ptr_stride, int src0, int dst0, const uint32_t* tbl,
                int len, int k, unsigned nstripes, bool x, unsigned long long r0m, unsigned c0m) {
  if (enc_lds(P, x, U) && x)
    launch_fl<P, U, kEncXor | kEncLds>(s, ptrs, ptr_stride, src0, dst0, tbl, len, k, nstripes, r0m, c0m);
  else if (enc_lds(P, x, U))
    launch_fl<P, U, kEncLds>(s, ptrs, ptr_stride, src0, dst0, tbl, len, k, nstripes, 0ull, 0u);
  else if (x)
    launch_fl<P, U, kEncXor>(s, ptrs, ptr_stride, src0, dst0, tbl, len, k, nstripes, r0m, c0m);
  else
    launch_fl<P, U, kEncLUT>(s, ptrs, ptr_stride, src0, dst0, tbl, len, k, nstripes, 0ull, 0u);
}

// Passes of 7-8 rows over at most kLdsxMaxK sources take the LDS product
// tables (ec_encode_ldsx) when the caller uploaded them (isal_hip_encmask.ldsx;
// ISAL_HIP_ENC_LDSX=1: every pass of 4-8 rows, =0 off). Against
// ec_encode_glds, ms per launch: bench.py batch encode k20 p8 1.38 vs 1.57,
// k16 p8 2.23 vs 2.46, k10 p8 3.08 vs 3.26, k10 p7 3.01 vs 3.05, same box
// (profiles/r06/r06_wide_ldsx_bench_ab_b.jsonl). Below 7 rows it does not pay
// in the library with loads in plain pairs: k20 p6 1.30 vs 1.29 there (the
// standalone sweep, r06_wide_ldsx_probe_b.jsonl, had it 5 % ahead on another
// layout), k10 p6 and k10 p4 within 1 %, k20 p4 3 % behind. With the pairs
// double-buffered, two interleaved rounds on one box
// (r06_wide_ldsx_pf_bench_ab.jsonl): 5-6 rows over k >= 16 sources gain
// 0-2 % (k16 p6 1.97/1.98 vs 2.01/2.00 ms, k20 p6 1.27/1.29 vs 1.29/1.29,
// k20 p5 1.25/1.25 vs 1.26/1.25), narrower stripes lose up to 2 % (k12 p5
// 1.55 vs 1.52/1.54, k13 p6 1.74 vs 1.73) or are even (k10 p5, k10 p6).
constexpr int kLdsxRows = 4, kLdsxAutoRows = 7, kLdsxWideRows = 5, kLdsxWideK = 16, kLdsxMaxK = 64;
bool enc_ldsx(int P, int k, const uint64_t* ldsx) {
  if (!ldsx || P < kLdsxRows || k > kLdsxMaxK) return false;
  const long long v = isal_hip_knob(ISAL_HIP_KNOB_ENC_LDSX);
  if (v == 0 || v == 1) return v == 1;
  return P >= kLdsxAutoRows || (P >= kLdsxWideRows && k >= kLdsxWideK);
}

// Sources per load group of ec_encode_ldsx: 2, double-buffered (the next
// pair's loads issued before the current pair is folded). The standalone
// sweep (r06_wide_ldsx_probe_c.jsonl, variant ldsx_pf2 against ldsx_u2 =
// plain pairs): k20 p8 1.34/1.36 vs 1.37/1.38 ms, k16 p8 2.10/2.11 vs
// 2.16/2.16, k20 p6 1.26/1.27 vs 1.32/1.31, k10 p7-p8 even. Plain groups of
// 2-4 were within 1 % of each other, 1 and 5 up to 5 % slower, and sources
// staged through a per-wave LDS-DMA ring (2-8 slots) 1-8 % slower than the
// double-buffered pairs.
constexpr int kLdsxGroup = 2;

template <int P, int U>
void launch_ldsx(unsigned grid, hipStream_t s, const uint64_t* ptrs, int ptr_stride, int src0, int dst0,
                 const uint32_t* tbl, const uint64_t* ldsx, int len, int k, unsigned nitems, unsigned tiles) {
  if (isal_hip_knob(ISAL_HIP_KNOB_LOG) >= 2) fprintf(stderr, "isal_hip: kernel ec_encode_ldsx<%d, %d>\n", P, U);
  ISAL_LAUNCH((ec_encode_ldsx<P, U>), dim3(grid), dim3(kBlock), static_cast<size_t>(k) * ISAL_HIP_LDSX_ENTRIES * 8, s,
              ptrs, ptr_stride, src0, dst0, tbl, ldsx, len, k, nitems, tiles);
}

template <int P>
hipError_t encode_pass(const uint64_t* ptrs, int ptr_stride, int src0, int dst0, const uint32_t* tbl,
                       const uint64_t* ldsx, int len, int k, unsigned nstripes, bool vec16, bool x,
                       unsigned long long r0m, unsigned c0m, hipStream_t s) {
  const unsigned span = vec16 ? kTile : kBlock;
  const unsigned tiles = static_cast<unsigned>((static_cast<long long>(len) + span - 1) / span);
  const unsigned nitems = nstripes * tiles;
  const unsigned grid = grid_for(nitems);
  if (vec16 && enc_ldsx(P, k, ldsx)) {
    if constexpr (P >= kLdsxRows) {
      launch_ldsx<P, kLdsxGroup>(grid, s, ptrs, ptr_stride, src0, dst0, tbl, ldsx, len, k, nitems, tiles);
    }
  } else if (vec16 && enc_glds(P)) {
    launch_glds_r<P>(x, grid, s, ptrs, ptr_stride, src0, dst0, tbl, len, k, nitems, tiles, r0m, c0m);
  } else if (vec16) {
    switch (enc_group(k, P)) {
#define EC_GROUP(u)                                                                          \
  case u:                                                                                    \
    launch_v16<P, u>(s, ptrs, ptr_stride, src0, dst0, tbl, len, k, nstripes, x, r0m, c0m);  \
    break;
      EC_GROUP(12) EC_GROUP(10) EC_GROUP(8) EC_GROUP(6) EC_GROUP(5)
#undef EC_GROUP
      default: launch_v16<P, 4>(s, ptrs, ptr_stride, src0, dst0, tbl, len, k, nstripes, x, r0m, c0m); break;
    }
  } else {
    ISAL_LAUNCH(ec_encode_b1<P>, dim3(grid), dim3(kBlock), 0, s, ptrs, ptr_stride, src0,
                       dst0, tbl, len, k, nitems, tiles);
  }
  isal_hip_count_launch();
  return hipGetLastError();
}

// The device update runs 128-lane workgroups (2 KiB tiles): C4 shape (k20 p6,
// 4 MiB x 64), same box, three interleaved rounds
// (profiles/r06/r06_update_block_ab.jsonl): 0.600 / 0.599 / 0.598 ms against
// 0.608 / 0.603 / 0.603 at 256 lanes. The 32 KiB LDS occupancy cap, which
// lifts the update's memory skeleton by 4-8 % (r06_skel_blocks_c2_c3_c4_pq.jsonl),
// costs the kernel 8-10 % at either size (0.650-0.665 ms).
constexpr int kUpdBlock = 128, kUpdTile = kUpdBlock * kVec;

template <int P>
hipError_t update_pass(const uint64_t* ptrs, int ptr_stride, int src_idx, int dst0,
                       const uint32_t* tbl, int len, unsigned nstripes, bool vec16, hipStream_t s) {
  const unsigned span = vec16 ? kTile : kBlock;
  const unsigned tiles = static_cast<unsigned>((static_cast<long long>(len) + span - 1) / span);
  const unsigned nitems = nstripes * tiles;
  // (An occupancy cap through dynamic LDS measured flat at 8 workgroups per
  // CU and 2-9 % slower at 4-6, profiles/r04_update_occupancy_ab.jsonl.)
  if (vec16) {
    // 128-lane workgroups, 2 KiB column tiles (kUpdBlock); the caller splits
    // launches with stripes_per_launch(len, true, kUpdTile)
    const unsigned t2 = static_cast<unsigned>((static_cast<long long>(len) + kUpdTile - 1) / kUpdTile);
    ISAL_LAUNCH((ec_update_v16<P, kUpdBlock>), dim3(grid_for(nstripes * t2)), dim3(kUpdBlock), 0, s, ptrs,
                ptr_stride, src_idx, dst0, tbl, len, nstripes * t2, t2);
  } else
    ISAL_LAUNCH(ec_update_b1<P>, dim3(grid_for(nitems)), dim3(kBlock), 0, s, ptrs,
                       ptr_stride, src_idx, dst0, tbl, len, nitems, tiles);
  isal_hip_count_launch();
  return hipGetLastError();
}

// Largest stripe count per launch so that nitems stays below kMaxItems.
unsigned stripes_per_launch(int len, bool vec16, long long vspan = kTile) {
  const long long span = vec16 ? vspan : kBlock;
  const long long tiles = (static_cast<long long>(len) + span - 1) / span;
  const long long n = static_cast<long long>(kMaxItems) / (tiles ? tiles : 1);
  return static_cast<unsigned>(n > 0 ? n : 1);
}

}  // namespace

// The 0/1 masks of a call, or none under ISAL_HIP_ENC_XOR=0 (read at launch,
// so handles created before isal_hip_config_reload() follow it too).
static const isal_hip_encmask* enc_xor_masks(const isal_hip_encmask* em) {
  return isal_hip_knob(ISAL_HIP_KNOB_ENC_XOR) == 0 ? nullptr : em;
}

extern "C" int isal_hip_launch_encode(const uint64_t* d_ptrs, int ptr_stride, int src_idx0,
                                      int dst_idx0, const uint32_t* d_tbl, int len, int k, int rows,
                                      long long nstripes, int vec16, const isal_hip_encmask* em,
                                      void* stream) {
  if (len <= 0 || rows <= 0 || nstripes <= 0) return 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const uint64_t* ldsx_all = em ? em->ldsx : nullptr;
  em = enc_xor_masks(em);
  const unsigned per = stripes_per_launch(len, vec16 != 0, kEncMinSpan);
  for (long long s0 = 0; s0 < nstripes; s0 += per) {
    const unsigned ns = static_cast<unsigned>(nstripes - s0 < per ? nstripes - s0 : per);
    const uint64_t* ptrs = d_ptrs + s0 * ptr_stride;
    for (int r0 = 0; r0 < rows; r0 += EC_MAX_ROWS_PER_PASS) {
      const int P = rows - r0 < EC_MAX_ROWS_PER_PASS ? rows - r0 : EC_MAX_ROWS_PER_PASS;
      const uint32_t* tbl = d_tbl + static_cast<size_t>(kTbl) * k * r0;
      const uint64_t* ldsx =
          ldsx_all ? ldsx_all + static_cast<size_t>(r0 / EC_MAX_ROWS_PER_PASS) * k * ISAL_HIP_LDSX_ENTRIES : nullptr;
      const int dst0 = dst_idx0 + r0;
      const int g = r0 / EC_MAX_ROWS_PER_PASS;
      const bool x = em && g < EC_MAX_PASSES && ((em->ok >> g) & 1u);
      const unsigned long long r0m = x ? em->r0[g] : 0ull;
      const unsigned c0m = x ? em->c0[g] : 0u;
      hipError_t e = hipSuccess;
      switch (P) {
#define EC_CASE(n)                                                                                      \
  case n:                                                                                               \
    e = encode_pass<n>(ptrs, ptr_stride, src_idx0, dst0, tbl, ldsx, len, k, ns, vec16 != 0, x, r0m, c0m, s); \
    break;
        EC_CASE(1) EC_CASE(2) EC_CASE(3) EC_CASE(4) EC_CASE(5) EC_CASE(6) EC_CASE(7) EC_CASE(8)
#undef EC_CASE
      }
      if (e != hipSuccess) return static_cast<int>(e);
    }
  }
  return 0;
}

// ISAL_HIP_KARG_NARROW: 1 = always the 4-byte-lane kernel, 0 = never;
// default = shards up to 1 MiB while at least kNarrowBusy kernel-argument
// calls are in flight. Round 4, C2 stripes, synchronised calls, same box
// (profiles/r04_karg_narrow_ab.jsonl): 16 threads 3098-3121 -> 3312-3326 GiB/s
// with 4-byte lanes, 1 thread 18.2 -> 17.9 us, 4 MiB shards 24.4 -> 27.0 us
// (4x the load instructions once one call fills the GPU). Round 5, mailbox
// completion, two interleaved rounds (profiles/r05/r05_dropin_done_ab.txt):
// 16-byte lanes are ahead at 1 thread (13.91-14.05 vs 14.50-14.68 us) and 4
// threads (2867-2895 vs 2730-2849 GiB/s), 4-byte lanes at 16 threads
// (4077-4098 vs 4019-4035 GiB/s). Choosing by calls in flight, two rounds
// (profiles/r05/r05_dropin_width_ab.txt): 1 thread 13.74-13.80 us, 16 threads
// 4079-4101 GiB/s; at 8 threads 16-byte lanes led (3884-3931 vs 3790-3830
// GiB/s), so 4-byte lanes start at 12 calls in flight (16 threads keep
// 14-16 in flight).
constexpr int kNarrowBusy = 12;
static bool karg_narrow(int len, int busy) {
  const long long v = isal_hip_knob(ISAL_HIP_KNOB_KARG_NARROW);
  if (v >= 0) return v != 0;
  return len <= (1 << 20) && busy >= kNarrowBusy;
}

static const isal_hip_kdone kNoDone = {nullptr, nullptr, nullptr, 0ull};

// Drop-in encodes of 7-8 rows over at most 12 sources take the LDS product
// tables too, unless ISAL_HIP_ENC_LDSX=0 (with 4-byte lanes, under 12+ calls
// in flight, they keep v_perm). One synchronous call per 1 MiB stripe, two
// interleaved rounds, same box (profiles/r06/r06_dropin_ldsx_ab.txt): k10 p8
// 17.6 / 19.8 us against 19.6 / 21.0 with v_perm, k10 p7 17.9 / 18.5 against
// 19.3 / 19.0; k20 p8 30.1 / 29.7 against 29.7 / 28.5 — each workgroup loads
// its k x 320 B of tables before the first source, which a single stripe's
// latency feels as k grows.
constexpr int kKargLdsxMaxK = 12;
extern "C" int isal_hip_karg_ldsx(int k, int rows) {
  return rows >= kLdsxAutoRows && rows <= EC_MAX_ROWS_PER_PASS && k >= 1 && k <= kKargLdsxMaxK &&
         isal_hip_knob(ISAL_HIP_KNOB_ENC_LDSX) != 0;
}

extern "C" int isal_hip_launch_encode_karg(const isal_hip_karg* a, const isal_hip_kdone* d, int len, int k,
                                           int rows, const isal_hip_encmask* em, int busy, const uint64_t* ldsx,
                                           void* stream) {
  if (!d) d = &kNoDone;
  if (len <= 0 || rows <= 0) return 0;
  if (rows > EC_MAX_ROWS_PER_PASS || k + rows > ISAL_HIP_KARG_PTRS ||
      static_cast<size_t>(kTbl) * k * rows > ISAL_HIP_KARG_TBL)
    return static_cast<int>(hipErrorInvalidValue);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool narrow = karg_narrow(len, busy);
  if (!narrow && isal_hip_karg_ldsx(k, rows) && ldsx) {  // 16-byte lanes on the product tables
    const unsigned tiles = static_cast<unsigned>((static_cast<long long>(len) + kTile - 1) / kTile);
    const size_t lds = static_cast<size_t>(k) * ISAL_HIP_LDSX_ENTRIES * 8;
    if (isal_hip_knob(ISAL_HIP_KNOB_LOG) >= 2) fprintf(stderr, "isal_hip: kernel ec_encode_karg_ldsx<%d>\n", rows);
    switch (rows) {
      case 7: ISAL_LAUNCH(ec_encode_karg_ldsx<7>, dim3(tiles), dim3(kBlock), lds, s, *a, *d, ldsx, len, k, tiles); break;
      case 8: ISAL_LAUNCH(ec_encode_karg_ldsx<8>, dim3(tiles), dim3(kBlock), lds, s, *a, *d, ldsx, len, k, tiles); break;
      default: return static_cast<int>(hipErrorInvalidValue);
    }
    isal_hip_count_launch();
    return static_cast<int>(hipGetLastError());
  }

  if (isal_hip_knob(ISAL_HIP_KNOB_LOG) >= 2)
    fprintf(stderr, "isal_hip: kernel %s<%d>\n", narrow ? "ec_encode_karg4" : "ec_encode_karg", rows);
  if (narrow) {
    const unsigned blocks = static_cast<unsigned>((static_cast<long long>(len) + 4 * kBlock - 1) / (4 * kBlock));
    switch (rows) {
#define EC_KARG4(n)                                                                                           \
  case n:                                                                                                     \
    ISAL_LAUNCH((ec_encode_karg4<n>), dim3(blocks), dim3(kBlock), 0, s, *a, *d, len, k);              \
    break;
      EC_KARG4(1) EC_KARG4(2) EC_KARG4(3) EC_KARG4(4) EC_KARG4(5) EC_KARG4(6) EC_KARG4(7) EC_KARG4(8)
#undef EC_KARG4
      default: return static_cast<int>(hipErrorInvalidValue);
    }
    isal_hip_count_launch();
    return static_cast<int>(hipGetLastError());
  }
  const unsigned tiles = static_cast<unsigned>((static_cast<long long>(len) + kTile - 1) / kTile);
  em = enc_xor_masks(em);
  const bool x = em && (em->ok & 1u);
  const unsigned long long r0m = x ? em->r0[0] : 0ull;
  const unsigned c0m = x ? em->c0[0] : 0u;
  switch (rows * 16 + enc_group(k)) {
#define EC_KARG(n, u)                                                                                   \
  case n * 16 + u:                                                                                      \
    if (x)                                                                                              \
      ISAL_LAUNCH((ec_encode_karg<n, EncPol<u, kBufNT, kBufSC1NT, 2>, kEncXor>), dim3(tiles),      \
                         dim3(kBlock), 0, s, *a, *d, len, k, tiles, r0m, c0m);                          \
    else                                                                                                \
      ISAL_LAUNCH((ec_encode_karg<n, EncPol<u, kBufNT, kBufSC1NT, 2>, kEncLUT>), dim3(tiles),      \
                         dim3(kBlock), 0, s, *a, *d, len, k, tiles, 0ull, 0u);                          \
    break;
#define EC_KARG_U(n) EC_KARG(n, 12) EC_KARG(n, 10) EC_KARG(n, 8) EC_KARG(n, 6) EC_KARG(n, 5) EC_KARG(n, 4)
    EC_KARG_U(1) EC_KARG_U(2) EC_KARG_U(3) EC_KARG_U(4) EC_KARG_U(5) EC_KARG_U(6) EC_KARG_U(7) EC_KARG_U(8)
#undef EC_KARG_U
#undef EC_KARG
    default: return static_cast<int>(hipErrorInvalidValue);
  }
  isal_hip_count_launch();
  return static_cast<int>(hipGetLastError());
}

extern "C" int isal_hip_launch_update_karg(const isal_hip_karg* a, const isal_hip_kdone* d, int len, int rows,
                                           void* stream) {
  if (len <= 0 || rows <= 0) return 0;
  if (!d) d = &kNoDone;
  if (rows > EC_MAX_ROWS_PER_PASS) return static_cast<int>(hipErrorInvalidValue);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const unsigned tiles = static_cast<unsigned>((static_cast<long long>(len) + kTile - 1) / kTile);
  switch (rows) {
#define EC_UKARG(n)                                                                                   \
  case n:                                                                                             \
    ISAL_LAUNCH(ec_update_karg<n>, dim3(tiles), dim3(kBlock), 0, s, *a, *d, len, tiles);       \
    break;
    EC_UKARG(1) EC_UKARG(2) EC_UKARG(3) EC_UKARG(4) EC_UKARG(5) EC_UKARG(6) EC_UKARG(7) EC_UKARG(8)
#undef EC_UKARG
  }
  isal_hip_count_launch();
  return static_cast<int>(hipGetLastError());
}

// Load group of the verify kernels: the largest of {10, 8, 6, 4} dividing k,
// else 4 with the remainder path (fewer instantiations than the encode's
// enc_group; xor_check / pq_check's usual source counts are covered).
static int verify_group(int k) {
  static const int cand[] = {10, 8, 6, 4};
  for (int u : cand)
    if (k >= u && k % u == 0) return u;
  return 4;
}

template <int P, int U, int FL>
void launch_verify_v16(unsigned grid, hipStream_t s, const uint64_t* d_ptrs, int ptr_stride, int src_idx0, int dst0,
                       const uint32_t* tbl, int len, int k, unsigned nitems, unsigned tiles, unsigned long long* out,
                       int r0, long long col0, unsigned long long r0m, unsigned c0m, unsigned long long* sbad) {
  ISAL_LAUNCH((ec_verify_v16<P, EncPol<U, kBufNT, kBufNT, 0>, FL>), dim3(grid), dim3(kBlock), 0, s, d_ptrs,
                     ptr_stride, src_idx0, dst0, tbl, len, k, nitems, tiles, out, r0, col0, r0m, c0m, sbad);
}

// One pass of the 16-byte verify (P rows from r0) over nstripes stripes.
static void verify_pass_v16(int P, int U, bool x, unsigned grid, hipStream_t s, const uint64_t* d_ptrs,
                            int ptr_stride, int src_idx0, int dst0, const uint32_t* tbl, int len, int k,
                            unsigned nitems, unsigned tiles, unsigned long long* out, int r0, long long col0,
                            unsigned long long r0m, unsigned c0m, unsigned long long* sbad) {
  switch (P * 64 + U * 2 + (x ? 1 : 0)) {
#define EC_VCASE(n, u)                                                                                          \
  case n * 64 + u * 2:                                                                                          \
    launch_verify_v16<n, u, kEncLUT>(grid, s, d_ptrs, ptr_stride, src_idx0, dst0, tbl, len, k, nitems, tiles, out, \
                                     r0, col0, 0ull, 0u, sbad);                                                 \
    break;                                                                                                      \
  case n * 64 + u * 2 + 1:                                                                                      \
    launch_verify_v16<n, u, kEncXor>(grid, s, d_ptrs, ptr_stride, src_idx0, dst0, tbl, len, k, nitems, tiles, out, \
                                     r0, col0, r0m, c0m, sbad);                                                 \
    break;
#define EC_VCASE_U(n) EC_VCASE(n, 10) EC_VCASE(n, 8) EC_VCASE(n, 6) EC_VCASE(n, 4)
    EC_VCASE_U(1) EC_VCASE_U(2) EC_VCASE_U(3) EC_VCASE_U(4) EC_VCASE_U(5) EC_VCASE_U(6) EC_VCASE_U(7) EC_VCASE_U(8)
#undef EC_VCASE_U
#undef EC_VCASE
  }
}

extern "C" int isal_hip_launch_verify(const uint64_t* d_ptrs, int ptr_stride, int src_idx0,
                                      int dst_idx0, const uint32_t* d_tbl, int len, int k, int rows,
                                      long long col0, unsigned long long* slots, int* nslots,
                                      int vec16, const isal_hip_encmask* em, void* stream) {
  *nslots = 0;
  if (len <= 0 || rows <= 0) return 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  em = enc_xor_masks(em);
  const unsigned span = vec16 ? kTile : kBlock;
  const unsigned tiles = static_cast<unsigned>((static_cast<long long>(len) + span - 1) / span);
  const unsigned grid = tiles < EC_VERIFY_MAX_GRID ? tiles : EC_VERIFY_MAX_GRID;
  const int U = verify_group(k);
  for (int r0 = 0; r0 < rows; r0 += EC_MAX_ROWS_PER_PASS) {
    const int P = rows - r0 < EC_MAX_ROWS_PER_PASS ? rows - r0 : EC_MAX_ROWS_PER_PASS;
    const uint32_t* tbl = d_tbl + static_cast<size_t>(kTbl) * k * r0;
    const int dst0 = dst_idx0 + r0;
    const int g = r0 / EC_MAX_ROWS_PER_PASS;
    const bool x = em && g < EC_MAX_PASSES && ((em->ok >> g) & 1u);
    const unsigned long long r0m = x ? em->r0[g] : 0ull;
    const unsigned c0m = x ? em->c0[g] : 0u;
    unsigned long long* out = slots + *nslots;
    if (!vec16) {
      switch (P) {
#define EC_CASE(n)                                                                                      \
  case n:                                                                                               \
    ISAL_LAUNCH(ec_verify_b1<n>, dim3(grid), dim3(kBlock), 0, s, d_ptrs, ptr_stride, src_idx0, dst0, \
                       tbl, len, k, tiles, tiles, out, r0, col0);                                       \
    break;
        EC_CASE(1) EC_CASE(2) EC_CASE(3) EC_CASE(4) EC_CASE(5) EC_CASE(6) EC_CASE(7) EC_CASE(8)
#undef EC_CASE
      }
    } else {
      verify_pass_v16(P, U, x, grid, s, d_ptrs, ptr_stride, src_idx0, dst0, tbl, len, k, tiles, tiles, out, r0, col0,
                      r0m, c0m, nullptr);
    }
    *nslots += static_cast<int>(grid);
    isal_hip_count_launch();
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return static_cast<int>(e);
  }
  return 0;
}

extern "C" int isal_hip_launch_verify_batch(const uint64_t* d_ptrs, int ptr_stride, int src_idx0, int dst_idx0,
                                            const uint32_t* d_tbl, int len, int k, int rows, long long nstripes,
                                            const isal_hip_encmask* em, unsigned long long* bad, void* stream) {
  if (len <= 0 || rows <= 0 || nstripes <= 0) return 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipError_t e = hipMemsetAsync(bad, 0xff, static_cast<size_t>(nstripes) * 8, s);
  if (e != hipSuccess) return static_cast<int>(e);
  em = enc_xor_masks(em);
  const unsigned per = stripes_per_launch(len, true);
  const unsigned tiles = static_cast<unsigned>((static_cast<long long>(len) + kTile - 1) / kTile);
  const int U = verify_group(k);
  for (long long s0 = 0; s0 < nstripes; s0 += per) {
    const unsigned ns = static_cast<unsigned>(nstripes - s0 < per ? nstripes - s0 : per);
    const uint64_t* ptrs = d_ptrs + s0 * ptr_stride;
    for (int r0 = 0; r0 < rows; r0 += EC_MAX_ROWS_PER_PASS) {
      const int P = rows - r0 < EC_MAX_ROWS_PER_PASS ? rows - r0 : EC_MAX_ROWS_PER_PASS;
      const int g = r0 / EC_MAX_ROWS_PER_PASS;
      const bool x = em && g < EC_MAX_PASSES && ((em->ok >> g) & 1u);
      verify_pass_v16(P, U, x, ns * tiles, s, ptrs, ptr_stride, src_idx0, dst_idx0 + r0,
                      d_tbl + static_cast<size_t>(kTbl) * k * r0, len, k, ns * tiles, tiles, nullptr, r0, 0,
                      x ? em->r0[g] : 0ull, x ? em->c0[g] : 0u, bad + s0);
      isal_hip_count_launch();
      e = hipGetLastError();
      if (e != hipSuccess) return static_cast<int>(e);
    }
  }
  return 0;
}

extern "C" int isal_hip_launch_verify_karg(const isal_hip_karg* a, const isal_hip_kdone* d, int len, int k,
                                           int rows, const isal_hip_encmask* em, void* stream) {
  if (len <= 0 || rows <= 0) return 0;
  if (!d || !d->cnt || !d->res || !d->mail || rows > EC_MAX_ROWS_PER_PASS || k + rows > ISAL_HIP_KARG_PTRS ||
      static_cast<size_t>(kTbl) * k * rows > ISAL_HIP_KARG_TBL)
    return static_cast<int>(hipErrorInvalidValue);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const unsigned tiles = static_cast<unsigned>((static_cast<long long>(len) + kTile - 1) / kTile);
  em = enc_xor_masks(em);
  const bool x = em && (em->ok & 1u);
  const unsigned long long r0m = x ? em->r0[0] : 0ull;
  const unsigned c0m = x ? em->c0[0] : 0u;
  switch (rows * 64 + verify_group(k) * 2 + (x ? 1 : 0)) {
#define EC_VKARG(n, u)                                                                                             \
  case n * 64 + u * 2:                                                                                             \
    ISAL_LAUNCH((ec_verify_karg<n, EncPol<u, kBufNT, kBufNT, 0>, kEncLUT>), dim3(tiles), dim3(kBlock), 0, s, \
                       *a, *d, len, k, tiles, 0ull, 0u);                                                           \
    break;                                                                                                         \
  case n * 64 + u * 2 + 1:                                                                                         \
    ISAL_LAUNCH((ec_verify_karg<n, EncPol<u, kBufNT, kBufNT, 0>, kEncXor>), dim3(tiles), dim3(kBlock), 0, s, \
                       *a, *d, len, k, tiles, r0m, c0m);                                                           \
    break;
#define EC_VKARG_U(n) EC_VKARG(n, 10) EC_VKARG(n, 8) EC_VKARG(n, 6) EC_VKARG(n, 4)
    EC_VKARG_U(1) EC_VKARG_U(2) EC_VKARG_U(3) EC_VKARG_U(4) EC_VKARG_U(5) EC_VKARG_U(6) EC_VKARG_U(7) EC_VKARG_U(8)
#undef EC_VKARG_U
#undef EC_VKARG
    default: return static_cast<int>(hipErrorInvalidValue);
  }
  isal_hip_count_launch();
  return static_cast<int>(hipGetLastError());
}

extern "C" int isal_hip_launch_update(const uint64_t* d_ptrs, int ptr_stride, int src_idx,
                                      int dst_idx0, const uint32_t* d_tbl, int len, int k, int rows,
                                      int vec_i, long long nstripes, int vec16, void* stream) {
  if (len <= 0 || rows <= 0 || nstripes <= 0) return 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const unsigned per = stripes_per_launch(len, vec16 != 0, kUpdTile);
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
