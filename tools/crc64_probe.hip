// crc64_probe.hip — variants of the CRC64 checksum-only pass (crc64_shards_pre)
// on the C2 shape, timed side by side in one process, each checked bit-exact
// against the library's kernel (same partials). Not shipped.
//
//   usage: crc64_probe [ITERS] [NSTRIPES] [ROUNDS] [NAME...]   one JSON line per variant
//          (NAME: run only the variants named)
//
// Variants:
//   lib      crc64_shards_pre as the library launches it (2 items per
//            workgroup, chains interleaved, 4-tile register batches), tt = 64
//   lib128   the same at 128 tiles per item
//   ringR_N  the sources staged through a per-wave LDS-DMA ring of R 1-KiB
//            slots (global_load_lds, counted vmcnt: no VGPRs hold loads, R - 1
//            tiles in flight all the time), N items' chains interleaved
//
// Build: make -C isa-l_amd crc64_probe (includes csrc/crc64_kernels.hip).
#include "../isa-l_amd/csrc/crc64_kernels.hip"

#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

// the library pieces crc64_kernels.hip links against, stubbed for the probe
extern "C" void isal_hip_count_launch(void) {}
extern "C" void isal_hip_kreg_add(const void*, const char*) {}
#define FUSED64_STUB(p)                                                                              \
  extern "C" void isal_hip_fused64_part_##p(unsigned, hipStream_t, const uint64_t*, int, const uint32_t*, \
                                            int, int, const isal_hip_crc64_geom*, const isal_hip_xrows*, int, \
                                            const uint64_t*, uint64_t*) {}
FUSED64_STUB(1) FUSED64_STUB(2) FUSED64_STUB(3) FUSED64_STUB(4) FUSED64_STUB(5) FUSED64_STUB(6) FUSED64_STUB(7)
FUSED64_STUB(8)

namespace {

__device__ __forceinline__ void bt_offs8(uint32_t w, uint32_t (&o)[4]) {
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

__device__ __forceinline__ uint64_t bt_at(const uint64_t* t, int j, uint32_t o) {
  return *reinterpret_cast<const uint64_t*>(reinterpret_cast<const char*>(t) + j * 2048 + o);
}

__device__ __forceinline__ void bt_slice8(X64& acc, const uint64_t* t, uint32_t lo, uint32_t hi) {
  uint32_t o[4], q[4];
  bt_offs8(lo, o);
  bt_offs8(hi, q);
  acc.add2(bt_at(t, 0, o[0]), bt_at(t, 1, o[1]));
  acc.add2(bt_at(t, 2, o[2]), bt_at(t, 3, o[3]));
  acc.add2(bt_at(t, 4, q[0]), bt_at(t, 5, q[1]));
  acc.add2(bt_at(t, 6, q[2]), bt_at(t, 7, q[3]));
}

template <int OA>
__device__ __forceinline__ uint4 lds_rd16(uint32_t addr) {
  u32x4 x;
  asm volatile("ds_read_b128 %0, %1 offset:%2\n\ts_waitcnt lgkmcnt(0)" : "=v"(x) : "v"(addr), "i"(OA) : "memory");
  return make_uint4(x.x, x.y, x.z, x.w);
}

__device__ __forceinline__ void dma16(uint64_t base_, uint32_t voff, uint32_t m0) {
  const uint32_t hi = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(base_ >> 32)));
  const uint32_t lo = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(base_)));
  const uint64_t base = (static_cast<uint64_t>(hi) << 32) | lo;
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(base), "s"(m0)
               : "memory");
}

template <int N>
__device__ __forceinline__ void vmw() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// vmcnt(n) for a wave-uniform n < 16
__device__ __forceinline__ void vmw_rt(int n) {
  switch (n) {
#define W(i) \
  case i: vmw<i>(); break;
    W(0) W(1) W(2) W(3) W(4) W(5) W(6) W(7) W(8) W(9) W(10) W(11) W(12) W(13) W(14)
#undef W
    default: vmw<15>(); break;
  }
}

// Ring variant: NI items per workgroup, their steps interleaved
// (item q's tile i is step i * NI + q), one 1-KiB ring slot per wave and step.
template <int R, int NI>
__global__ __launch_bounds__(kBlock) void crc64_pre_ring(const uint64_t* __restrict__ ptrs, int ptr_stride, int nsh,
                                                         int len, unsigned nitems, unsigned nblk, unsigned tt,
                                                         unsigned nfull, int uswap, const uint64_t* __restrict__ tabs,
                                                         uint64_t* __restrict__ part) {
  __shared__ uint64_t lt[2 * kCE];  // F_u, F'_u
  extern __shared__ __attribute__((aligned(16))) uint8_t ring_lds[];
  load_lds<2 * kCE>(lt, tabs + ISAL_HIP_CRC64_PRE_TAB);
  __syncthreads();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t ring = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) uint8_t*)ring_lds)) +
                        wave * (R * 1024);
  const uint32_t mine = ring + (threadIdx.x & 63) * kVec;
  const uint32_t lane = threadIdx.x * kVec;
  auto step = [&](bool last, X64 b, const uint4& x) __attribute__((always_inline)) {
    X64 c{0u, 0u};
    if (last)
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
    const unsigned S = n * NI;  // ring steps
    vmw<0>();                   // the previous item's partial stores
    auto issue = [&](unsigned s) __attribute__((always_inline)) {
      const unsigned q = s % NI, i = s / NI;
      dma16(base[q], (t0[q] + i) * kTile + lane, ring + (s % R) * 1024);
    };
    for (unsigned s = 0; s < R && s < S; ++s) issue(s);
    for (unsigned s = 0; s < S; ++s) {
      const unsigned ahead = min(S - 1 - s, static_cast<unsigned>(R - 1));  // DMAs issued after step s's
      if (ahead == R - 1)
        vmw<R - 1>();
      else
        vmw_rt(static_cast<int>(ahead));
      const uint4 x = lds_rd16<0>(mine + (s % R) * 1024);
      if (s + R < S) issue(s + R);
      const unsigned q = s % NI, i = s / NI;
#pragma unroll
      for (int qq = 0; qq < NI; ++qq)
        if (qq == static_cast<int>(q)) bc[qq] = step(t0[qq] + i + 1 == t1[qq], bc[qq], x);
    }
    vmw<0>();
#pragma unroll
    for (int q = 0; q < NI; ++q) {
      for (unsigned j = t0[q] + n; j < t1[q]; ++j)
        bc[q] = step(j + 1 == t1[q], bc[q], load16<kBufNT>(base[q], static_cast<long long>(j) * kTile + lane, len));
      const unsigned w = NI * v + q;
      if (w < nitems) {
        const uint64_t r = bc[q].get();
        part[static_cast<size_t>(w) * kBlock + threadIdx.x] = uswap ? __builtin_bswap64(r) : r;
      }
    }
  }
}

// Rolling register batch: as crc64_shards_pre (NI items' chains interleaved,
// B tiles per item held in registers), but a register is refilled with tile
// i + B as soon as tile i has been read from it, so NI * B loads stay in
// flight all the time instead of one batch at a time.
template <int NI, int B>
__global__ __launch_bounds__(kBlock) void crc64_pre_roll(const uint64_t* __restrict__ ptrs, int ptr_stride, int nsh,
                                                         int len, unsigned nitems, unsigned nblk, unsigned tt,
                                                         unsigned nfull, int uswap, const uint64_t* __restrict__ tabs,
                                                         uint64_t* __restrict__ part) {
  __shared__ uint64_t lt[2 * kCE];  // F_u, F'_u
  load_lds<2 * kCE>(lt, tabs + ISAL_HIP_CRC64_PRE_TAB);
  __syncthreads();
  const long long lane = threadIdx.x * kVec;
  auto step = [&](bool last, X64 b, const uint4& x) __attribute__((always_inline)) {
    X64 c{0u, 0u};
    if (last)
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
    if (n >= B) {
      uint4 x[NI][B];
#pragma unroll
      for (int g = 0; g < B; ++g)
#pragma unroll
        for (int q = 0; q < NI; ++q)
          x[q][g] = load16<kBufNT>(base[q], static_cast<long long>(t0[q] + g) * kTile + lane, len);
      for (; i + 2 * B <= n; i += B) {
#pragma unroll
        for (int g = 0; g < B; ++g)
#pragma unroll
          for (int q = 0; q < NI; ++q) {
            const uint4 xx = x[q][g];
            x[q][g] = load16<kBufNT>(base[q], static_cast<long long>(t0[q] + i + B + g) * kTile + lane, len);
            bc[q] = step(t0[q] + i + g + 1 == t1[q], bc[q], xx);
          }
      }
#pragma unroll
      for (int g = 0; g < B; ++g)
#pragma unroll
        for (int q = 0; q < NI; ++q) bc[q] = step(t0[q] + i + g + 1 == t1[q], bc[q], x[q][g]);
      i += B;
    }
#pragma unroll
    for (int q = 0; q < NI; ++q) {
      for (unsigned j = t0[q] + i; j < t1[q]; ++j)
        bc[q] = step(j + 1 == t1[q], bc[q], load16<kBufNT>(base[q], static_cast<long long>(j) * kTile + lane, len));
      const unsigned w = NI * v + q;
      if (w < nitems) {
        const uint64_t r = bc[q].get();
        part[static_cast<size_t>(w) * kBlock + threadIdx.x] = uswap ? __builtin_bswap64(r) : r;
      }
    }
  }
}

// Byte tables instead of field tables (the fused kernel's chunk path,
// crc64_kernels.hip chain_step_sl): 16 byte-indexed lookups per chunk (one
// SDWA op each) into the u-domain slicing tables A / A' (8 x 256 entries
// each, 32 KiB), at ~3x bank conflicts — fewer VALU and LDS instructions than
// the 28 field lookups. NV lane groups of 256 share one table copy.
template <int PH>
__device__ __forceinline__ uint64_t bt_step(const uint64_t* lt, uint64_t b, uint32_t w0, uint32_t w1, uint32_t w2,
                                            uint32_t w3) {
  X64 u{0u, 0u};
  X64 c{0u, 0u};
  bt_slice8(u, lt, w0 ^ static_cast<uint32_t>(b), w1 ^ static_cast<uint32_t>(b >> 32));
  bt_slice8(c, lt + (PH == 1 ? 0 : 8 * 256), w2 ^ u.lo, w3 ^ u.hi);
  return c.get();
}

template <int NI, int B, int NV>
__global__ __launch_bounds__(kBlock* NV) void crc64_pre_bytes(const uint64_t* __restrict__ ptrs, int ptr_stride,
                                                              int nsh, int len, unsigned nitems, unsigned nblk,
                                                              unsigned tt, unsigned nfull, int uswap,
                                                              const uint64_t* __restrict__ tabs,
                                                              uint64_t* __restrict__ part) {
  __shared__ uint64_t lt[16 * 256];  // A, A'
  load_lds<16 * 256, NV>(lt, tabs + ISAL_HIP_CRC64_SLICE_TAB);
  __syncthreads();
  const unsigned tid = threadIdx.x % kBlock;
  const long long lane = tid * kVec;
  for (unsigned v = blockIdx.x * NV + threadIdx.x / kBlock; NI * v < nitems; v += gridDim.x * NV) {
    uint64_t base[NI];
    unsigned t0[NI], t1[NI], n = ~0u;
    uint64_t bc[NI];
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
      bc[q] = 0;
    }
    auto stp = [&](bool last, uint64_t b, const uint4& x) __attribute__((always_inline)) {
      return last ? bt_step<1>(lt, b, x.x, x.y, x.z, x.w) : bt_step<0>(lt, b, x.x, x.y, x.z, x.w);
    };
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
        for (int q = 0; q < NI; ++q) bc[q] = stp(t0[q] + i + g + 1 == t1[q], bc[q], x[q][g]);
    }
#pragma unroll
    for (int q = 0; q < NI; ++q) {
      for (unsigned j = t0[q] + i; j < t1[q]; ++j)
        bc[q] = stp(j + 1 == t1[q], bc[q], load16<kBufNT>(base[q], static_cast<long long>(j) * kTile + lane, len));
      const unsigned w = NI * v + q;
      if (w < nitems) part[static_cast<size_t>(w) * kBlock + tid] = uswap ? __builtin_bswap64(bc[q]) : bc[q];
    }
  }
}

// Compute only: crc64_pre_roll's arithmetic with the loads replaced by
// register-made chunks (2 VALU ops per dword): what the LDS lookups and VALU
// cost with no HBM traffic at all (results not comparable).
template <int NI>
__global__ __launch_bounds__(kBlock) void crc64_pre_nomem(const uint64_t* __restrict__ ptrs, int ptr_stride, int nsh,
                                                          int len, unsigned nitems, unsigned nblk, unsigned tt,
                                                          unsigned nfull, int uswap, const uint64_t* __restrict__ tabs,
                                                          uint64_t* __restrict__ part) {
  __shared__ uint64_t lt[2 * kCE];
  load_lds<2 * kCE>(lt, tabs + ISAL_HIP_CRC64_PRE_TAB);
  __syncthreads();
  auto step = [&](bool last, X64 b, const uint4& x) __attribute__((always_inline)) {
    X64 c{0u, 0u};
    if (last)
      chunk_acc(c, lt, x.x ^ b.lo, x.y ^ b.hi, x.z, x.w);
    else
      chunk_acc(c, lt + kCE, x.x ^ b.lo, x.y ^ b.hi, x.z, x.w);
    return c;
  };
  for (unsigned v = blockIdx.x; NI * v < nitems; v += gridDim.x) {
    X64 bc[NI];
    unsigned t1 = tt;
#pragma unroll
    for (int q = 0; q < NI; ++q) bc[q] = X64{threadIdx.x * 77u + q, v};
    for (unsigned i = 0; i < t1; ++i) {
#pragma unroll
      for (int q = 0; q < NI; ++q) {
        const uint32_t h = (i * 2654435761u) ^ (threadIdx.x + q);
        bc[q] = step(i + 1 == t1, bc[q], make_uint4(h, h * 3u, h + 12345u, h ^ 0x5bd1e995u));
      }
    }
#pragma unroll
    for (int q = 0; q < NI; ++q) {
      const unsigned w = NI * v + q;
      if (w < nitems) part[static_cast<size_t>(w) * kBlock + threadIdx.x] = bc[q].get();
    }
  }
}

}  // namespace

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

__global__ void fill(uint64_t* p, size_t n, uint64_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t x = (i + 1) * 0x9E3779B97F4A7C15ull ^ seed;
    x ^= x >> 31;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 29;
    p[i] = x;
  }
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 10;
  const int ns = argc > 2 ? atoi(argv[2]) : 1024;
  const int nsh = 14, len = 1 << 20, variant = 0; /* ISAL_HIP_CRC64_ECMA_REFL */
  const size_t total = static_cast<size_t>(ns) * nsh * len;
  uint8_t* d = nullptr;
  CK(hipMalloc(&d, total));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint64_t*>(d), total / 8, 12345ull);
  std::vector<uint64_t> hp(static_cast<size_t>(ns) * nsh);
  for (size_t i = 0; i < hp.size(); ++i) hp[i] = reinterpret_cast<uint64_t>(d + i * len);
  uint64_t* dp = nullptr;
  CK(hipMalloc(&dp, hp.size() * 8));
  CK(hipMemcpy(dp, hp.data(), hp.size() * 8, hipMemcpyHostToDevice));
  const int tts[2] = {64, 128};
  uint64_t* dtab[2];
  std::vector<uint64_t> ht(ISAL_HIP_CRC64_TAB_ENTRIES);
  for (int j = 0; j < 2; ++j) {
    isal_hip_crc64_tables(variant, len, tts[j], ht.data());
    CK(hipMalloc(&dtab[j], ht.size() * 8));
    CK(hipMemcpy(dtab[j], ht.data(), ht.size() * 8, hipMemcpyHostToDevice));
  }
  const size_t part_words = static_cast<size_t>(ns) * nsh * (256 / 64) * kBlock;
  uint64_t *pref = nullptr, *pv = nullptr;
  CK(hipMalloc(&pref, part_words * 8));
  CK(hipMalloc(&pv, part_words * 8));
  std::vector<uint64_t> href(part_words), hv(part_words);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double bytes = static_cast<double>(total);

  struct V {
    const char* name;
    int tt;
    void (*go)(const uint64_t*, int, int, int, unsigned, unsigned, unsigned, unsigned, const uint64_t*, uint64_t*);
  };
#define LIB(tt_)                                                                                                    \
  [](const uint64_t* p, int nsh_, int len_, int, unsigned nitems, unsigned nblk, unsigned tt, unsigned nfull,     \
     const uint64_t* t, uint64_t* part) {                                                                          \
    hipLaunchKernelGGL(crc64_shards_pre, dim3((nitems + kPreItems - 1) / kPreItems), dim3(kBlock), 0, 0, p, nsh_, \
                       nsh_, len_, nitems, nblk, tt, nfull, 0, t, part);                                           \
  }
#define RING(R, NI)                                                                                               \
  [](const uint64_t* p, int nsh_, int len_, int, unsigned nitems, unsigned nblk, unsigned tt, unsigned nfull,   \
     const uint64_t* t, uint64_t* part) {                                                                        \
    hipLaunchKernelGGL((crc64_pre_ring<R, NI>), dim3((nitems + NI - 1) / NI), dim3(kBlock), 4 * R * 1024, 0, p,  \
                       nsh_, nsh_, len_, nitems, nblk, tt, nfull, 0, t, part);                                   \
  }
#define ROLL(NI, B)                                                                                              \
  [](const uint64_t* p, int nsh_, int len_, int, unsigned nitems, unsigned nblk, unsigned tt, unsigned nfull,   \
     const uint64_t* t, uint64_t* part) {                                                                        \
    hipLaunchKernelGGL((crc64_pre_roll<NI, B>), dim3((nitems + NI - 1) / NI), dim3(kBlock), 0, 0, p, nsh_, nsh_,   \
                       len_, nitems, nblk, tt, nfull, 0, t, part);                                               \
  }
#define BYTES(NI, B, NV)                                                                                         \
  [](const uint64_t* p, int nsh_, int len_, int, unsigned nitems, unsigned nblk, unsigned tt, unsigned nfull,   \
     const uint64_t* t, uint64_t* part) {                                                                        \
    hipLaunchKernelGGL((crc64_pre_bytes<NI, B, NV>), dim3((nitems + NI * NV - 1) / (NI * NV)), dim3(kBlock * NV), 0, \
                       0, p, nsh_, nsh_, len_, nitems, nblk, tt, nfull, 0, t, part);                              \
  }
#define NOMEM(NI)                                                                                                 \
  [](const uint64_t* p, int nsh_, int len_, int, unsigned nitems, unsigned nblk, unsigned tt, unsigned nfull,   \
     const uint64_t* t, uint64_t* part) {                                                                        \
    hipLaunchKernelGGL((crc64_pre_nomem<NI>), dim3((nitems + NI - 1) / NI), dim3(kBlock), 0, 0, p, nsh_, nsh_,     \
                       len_, nitems, nblk, tt, nfull, 0, t, part);                                               \
  }
  const V vs[] = {
      {"lib", 64, LIB(64)},         {"lib128", 128, LIB(128)},      {"ring4_2", 64, RING(4, 2)},
      {"ring6_2", 64, RING(6, 2)},  {"ring8_2", 64, RING(8, 2)},    {"ring12_2", 64, RING(12, 2)},
      {"ring6_4", 64, RING(6, 4)},  {"ring8_4", 64, RING(8, 4)},    {"ring8_1", 64, RING(8, 1)},
      {"ring8_2_128", 128, RING(8, 2)}, {"ring6_2_128", 128, RING(6, 2)},
      {"roll2_4", 64, ROLL(2, 4)},  {"roll2_2", 64, ROLL(2, 2)},    {"roll2_3", 64, ROLL(2, 3)},
      {"roll1_4", 64, ROLL(1, 4)},  {"roll2_6", 64, ROLL(2, 6)},    {"roll3_2", 64, ROLL(3, 2)},
      {"roll2_4_128", 128, ROLL(2, 4)}, {"roll2_2_128", 128, ROLL(2, 2)},
      {"bytes2_4_1", 64, BYTES(2, 4, 1)}, {"bytes2_4_2", 64, BYTES(2, 4, 2)}, {"bytes1_4_2", 64, BYTES(1, 4, 2)},
      {"bytes2_2_2", 64, BYTES(2, 2, 2)}, {"bytes3_2_2", 64, BYTES(3, 2, 2)}, {"bytes2_4_2_128", 128, BYTES(2, 4, 2)},
      {"bytes4_2_2", 64, BYTES(4, 2, 2)},
      {"nomem2", 64, NOMEM(2)}, {"nomem1", 64, NOMEM(1)}, {"nomem4", 64, NOMEM(4)},
  };
  const int rounds = argc > 3 ? atoi(argv[3]) : 2;
  for (int round = 0; round < rounds; ++round)
    for (const V& v : vs) {
      bool pick = argc <= 4;
      for (int a = 4; a < argc; ++a) pick |= strcmp(argv[a], v.name) == 0;
      if (!pick) continue;
      isal_hip_crc64_geom g;
      isal_hip_crc64_geometry(len, v.tt, &g);
      const unsigned nitems = static_cast<unsigned>(ns * nsh * g.nblk);
      uint64_t* tab = dtab[v.tt == 128];
      // reference partials: the library kernel at the same geometry
      CK(hipMemset(pref, 0, part_words * 8));
      hipLaunchKernelGGL(crc64_shards_pre, dim3((nitems + kPreItems - 1) / kPreItems), dim3(kBlock), 0, 0, dp, nsh,
                         nsh, len, nitems, static_cast<unsigned>(g.nblk), static_cast<unsigned>(g.tt),
                         static_cast<unsigned>(g.nfull), 0, tab, pref);
      CK(hipMemset(pv, 0xA5, part_words * 8));
      v.go(dp, nsh, len, 0, nitems, g.nblk, g.tt, g.nfull, tab, pv);
      CK(hipDeviceSynchronize());
      CK(hipGetLastError());
      const size_t used = static_cast<size_t>(nitems) * kBlock;
      CK(hipMemcpy(href.data(), pref, used * 8, hipMemcpyDeviceToHost));
      CK(hipMemcpy(hv.data(), pv, used * 8, hipMemcpyDeviceToHost));
      const bool ok = memcmp(href.data(), hv.data(), used * 8) == 0;
      for (int w = 0; w < 2; ++w) v.go(dp, nsh, len, 0, nitems, g.nblk, g.tt, g.nfull, tab, pv);
      CK(hipEventRecord(e0, 0));
      for (int it = 0; it < iters; ++it) v.go(dp, nsh, len, 0, nitems, g.nblk, g.tt, g.nfull, tab, pv);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= iters;
      printf("{\"round\": %d, \"variant\": \"%s\", \"tt\": %d, \"ms\": %.4f, \"gb_s\": %.1f, \"frac\": %.4f, "
             "\"bit_exact\": %s}\n",
             round, v.name, v.tt, ms, bytes / ms / 1e6, bytes / ms / 1e6 / 8000.0, ok ? "true" : "false");
      fflush(stdout);
    }
  return 0;
}
