// ec_probe.hip — measurement tool, not part of libisal_hip.so.
//
// 1. Achievable HBM bandwidth for the encode access pattern: memory-only
//    kernels with exactly the addressing of ec_encode_v16 (R source streams
//    read, W parity streams written, XOR instead of GF math), plus a plain copy.
// 2. Policy variants of the real encode kernel (EncDefault vs others), checked
//    bit-exact against the default variant.
// Interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24);
// median and min per variant. Output: one line per variant + a JSON summary.
#include "../csrc/ec_kernels.hip"

// Work orders only the probe measures (the library launches 0 and 2,
// ec_kernels.hip EncOrder): 1 stripe fastest; 3 / 5 the XCD-contiguous order
// cut into 16 / 32 ranges (two / four per XCD); 4 XCD x streams whole stripes
// s = x (mod 8), tile fastest.
namespace {
template <>
struct EncOrder<1> {
  __device__ static void item(unsigned w, unsigned nitems, unsigned tiles, unsigned& stripe, unsigned& tile) {
    const unsigned nstripes = nitems / tiles;
    tile = w / nstripes;
    stripe = w - tile * nstripes;
  }
};

template <unsigned G>
struct EncOrderRanges {
  __device__ static void item(unsigned w, unsigned nitems, unsigned tiles, unsigned& stripe, unsigned& tile) {
    const unsigned per = nitems / G;
    const unsigned v = (nitems % G) ? w : (w % G) * per + w / G;
    stripe = v / tiles;
    tile = v - stripe * tiles;
  }
};
template <>
struct EncOrder<3> : EncOrderRanges<16> {};
template <>
struct EncOrder<5> : EncOrderRanges<32> {};

template <>
struct EncOrder<4> {
  __device__ static void item(unsigned w, unsigned nitems, unsigned tiles, unsigned& stripe, unsigned& tile) {
    const unsigned nstripes = nitems / tiles;
    const unsigned j = w >> 3, x = w & 7;
    const unsigned sj = j / tiles;
    stripe = (nstripes & 7) ? w / tiles : sj * 8 + x;
    tile = (nstripes & 7) ? w - (w / tiles) * tiles : j - sj * tiles;
  }
};
}  // namespace

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

extern "C" void gf_gen_rs_matrix(unsigned char* a, int m, int k);
extern "C" void ec_init_tables(int k, int rows, unsigned char* a, unsigned char* gftbls);
extern "C" void isal_hip_count_launch(void) {}
extern "C" long long isal_hip_knob(int) { return -1; }

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

namespace {

template <int R, int W, bool NT_LD, bool NT_ST>
__global__ __launch_bounds__(256) void mem_pattern(const uint64_t* __restrict__ ptrs, int stride,
                                                   int len, unsigned nitems, unsigned tiles,
                                                   uint32_t* __restrict__ sink) {
  for (unsigned w = blockIdx.x; w < nitems; w += gridDim.x) {
    const unsigned stripe = w / tiles, tile = w - stripe * tiles;
    const uint64_t* __restrict__ sp = ptrs + static_cast<size_t>(stripe) * stride;
    const long long off = static_cast<long long>(tile) * kTile + threadIdx.x * kVec;
    uint4 a = make_uint4(w, 1, 2, 3);
    uint4 x[R > 0 ? R : 1];
#pragma unroll
    for (int j = 0; j < R; ++j) x[j] = load16<NT_LD ? kNT : kPlain>(sp[j], off);
#pragma unroll
    for (int j = 0; j < R; ++j) {
      a.x ^= x[j].x;
      a.y ^= x[j].y;
      a.z ^= x[j].z;
      a.w ^= x[j].w;
    }
    if constexpr (W == 0) {
      if ((a.x ^ a.y ^ a.z ^ a.w) == 0x9E3779B9u) sink[threadIdx.x] = a.x;
    }
#pragma unroll
    for (int l = 0; l < W; ++l) {
      store16<NT_ST ? kNT : kPlain>(sp[10 + l], off, a);  // parity pointers (k = 10) only
      a.x += 1;
    }
  }
}

// Same pattern through buffer_load/store with explicit cache-policy bits
// (gfx950 CPol: sc0 = 1, nt = 2, sc1 = 16).
template <int R, int W, int AUX_LD, int AUX_ST>
__global__ __launch_bounds__(256) void mem_pattern_buf(const uint64_t* __restrict__ ptrs, int stride,
                                                       int len, unsigned nitems, unsigned tiles,
                                                       uint32_t* __restrict__ sink) {
  for (unsigned w = blockIdx.x; w < nitems; w += gridDim.x) {
    const unsigned stripe = w / tiles, tile = w - stripe * tiles;
    const uint64_t* __restrict__ sp = ptrs + static_cast<size_t>(stripe) * stride;
    const int off = static_cast<int>(tile) * kTile + threadIdx.x * kVec;
    typedef int v4i __attribute__((ext_vector_type(4)));
    v4i a = {static_cast<int>(w), 1, 2, 3};
    v4i x[R > 0 ? R : 1];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)sp[j], 0, len, 0x00020000);
      x[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, AUX_LD);
    }
#pragma unroll
    for (int j = 0; j < R; ++j) a ^= x[j];
    if constexpr (W == 0) {
      if ((a.x ^ a.y ^ a.z ^ a.w) == 0x1E3779B9) sink[threadIdx.x] = a.x;
    }
#pragma unroll
    for (int l = 0; l < W; ++l) {
      auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)sp[10 + l], 0, len, 0x00020000);
      __builtin_amdgcn_raw_buffer_store_b128(a, rs, off, 0, AUX_ST);
      a.x += 1;
    }
  }
}

// Two 4 KiB tiles per work item (each wave streams 2 KiB contiguous per shard).
template <int R, int W>
__global__ __launch_bounds__(256) void mem_pattern_2t(const uint64_t* __restrict__ ptrs, int stride,
                                                      int len, unsigned nitems, unsigned tiles,
                                                      uint32_t* __restrict__ sink) {
  const unsigned half = tiles / 2;
  for (unsigned w = blockIdx.x; w < nitems / 2; w += gridDim.x) {
    const unsigned stripe = w / half, tp = w - stripe * half;
    const uint64_t* __restrict__ sp = ptrs + static_cast<size_t>(stripe) * stride;
    // wave-contiguous: wave v covers bytes [tp*8K + v*2K, +2K)
    const unsigned wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const long long off0 = static_cast<long long>(tp) * 2 * kTile + wave * 2048 + lane * 16;
    uint4 a0 = make_uint4(w, 1, 2, 3), a1 = a0;
    uint4 x0[R], x1[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      x0[j] = load16<kNT>(sp[j], off0);
      x1[j] = load16<kNT>(sp[j], off0 + 1024);
    }
#pragma unroll
    for (int j = 0; j < R; ++j) {
      a0.x ^= x0[j].x; a0.y ^= x0[j].y; a0.z ^= x0[j].z; a0.w ^= x0[j].w;
      a1.x ^= x1[j].x; a1.y ^= x1[j].y; a1.z ^= x1[j].z; a1.w ^= x1[j].w;
    }
#pragma unroll
    for (int l = 0; l < W; ++l) {
      store16<kNT>(sp[10 + l], off0, a0);
      store16<kNT>(sp[10 + l], off0 + 1024, a1);
      a0.x += 1;
      a1.x += 1;
    }
  }
}

__global__ void copy16(const uint4* __restrict__ s, uint4* __restrict__ d, size_t n16) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16;
       i += (size_t)gridDim.x * blockDim.x)
    d[i] = s[i];
}

// Streaming copy between two separate buffers, U 16-byte loads in flight per
// lane (each wave-instruction one contiguous KiB), non-temporal buffer ops:
// the "float4 copy" the microarchitecture guide quotes (6.29 TB/s).
template <int U>
__global__ __launch_bounds__(256) void copy_nt(const uint8_t* __restrict__ s, uint8_t* __restrict__ d,
                                               size_t bytes) {
  typedef int v4i __attribute__((ext_vector_type(4)));
  const size_t step = static_cast<size_t>(gridDim.x) * 256 * 16;
  for (size_t base = (static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x) * 16; base < bytes;
       base += step * U) {
    v4i x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t o = base + u * step;
      const size_t chunk = o & ~((size_t(1) << 30) - 1);  // 1 GiB buffer windows
      auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(s + chunk), 0, 1 << 30, 0x00020000);
      x[u] = o < bytes ? __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(o - chunk), 0, 2)
                       : v4i{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t o = base + u * step;
      const size_t chunk = o & ~((size_t(1) << 30) - 1);
      auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(d + chunk), 0, 1 << 30, 0x00020000);
      if (o < bytes) __builtin_amdgcn_raw_buffer_store_b128(x[u], rs, static_cast<int>(o - chunk), 0, 2);
    }
  }
}

__global__ void fill_random(uint32_t* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ull + seed;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    p[i] = static_cast<uint32_t>(z ^ (z >> 31));
  }
}

template <int UU, bool NL, bool NS, int ORD>
using Pol = EncPol<UU, NL ? kNT : kPlain, NS ? kNT : kPlain, ORD>;

struct Variant {
  std::string name;
  double bytes;  // algorithmic bytes per launch
  std::function<void(hipStream_t)> run;
  std::vector<double> gbs;
  bool encode = false;
};

}  // namespace

int main(int argc, char** argv) {
  const int k = argc > 1 ? atoi(argv[1]) : 10;
  const int p = argc > 2 ? atoi(argv[2]) : 4;
  const int len = argc > 3 ? atoi(argv[3]) : (1 << 20);
  const int S = argc > 4 ? atoi(argv[4]) : 1024;
  const int rounds = argc > 5 ? atoi(argv[5]) : 5;
  const int iters = 10;
  if (k != 10 || p != 4) {
    fprintf(stderr, "memory patterns are instantiated for k=10 p=4 only\n");
    return 2;
  }
  const size_t shard = static_cast<size_t>(len);
  const size_t maxpad = 65536 + 4096;
  const size_t dbytes = shard * k * S, cbytes = shard * p * S;
  const size_t dalloc = (shard + maxpad) * k * S, calloc_ = (shard + maxpad) * p * S;
  uint8_t *data, *coding, *sinkp;
  CK(hipMalloc(&data, dalloc));
  CK(hipMalloc(&coding, calloc_));
  CK(hipMalloc(&sinkp, 4096));
  hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, (uint32_t*)data, dalloc / 4, 7u);
  CK(hipDeviceSynchronize());

  // pointer table [S][k+p] and coefficient tables (C2 Vandermonde)
  std::vector<uint64_t> h_ptrs(static_cast<size_t>(S) * (k + p));
  for (int s = 0; s < S; ++s) {
    for (int j = 0; j < k; ++j)
      h_ptrs[(size_t)s * (k + p) + j] = (uint64_t)(data + ((size_t)s * k + j) * shard);
    for (int l = 0; l < p; ++l)
      h_ptrs[(size_t)s * (k + p) + k + l] = (uint64_t)(coding + ((size_t)s * p + l) * shard);
  }
  std::vector<unsigned char> a((k + p) * k), g(32 * k * p);
  gf_gen_rs_matrix(a.data(), k + p, k);
  ec_init_tables(k, p, a.data() + k * k, g.data());
  std::vector<uint32_t> h_tbl(isal_hip_tables_dwords(k, p));
  isal_hip_build_tables(k, p, g.data(), h_tbl.data());
  uint64_t* d_ptrs;
  uint32_t* d_tbl;
  CK(hipMalloc(&d_ptrs, h_ptrs.size() * 8));
  CK(hipMalloc(&d_tbl, h_tbl.size() * 4 + 4));
  CK(hipMemcpy(d_ptrs, h_ptrs.data(), h_ptrs.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_tbl, h_tbl.data(), h_tbl.size() * 4, hipMemcpyHostToDevice));
  // padded layouts: shard stride len + pad (partition-camping check)
  const size_t pads[3] = {256, 4096, 65536 + 4096};
  uint64_t* d_pptrs[3];
  for (int q = 0; q < 3; ++q) {
    std::vector<uint64_t> hp(h_ptrs.size());
    const size_t st = shard + pads[q];
    for (int s2 = 0; s2 < S; ++s2) {
      for (int j = 0; j < k; ++j) hp[(size_t)s2 * (k + p) + j] = (uint64_t)(data + ((size_t)s2 * k + j) * st);
      for (int l = 0; l < p; ++l)
        hp[(size_t)s2 * (k + p) + k + l] = (uint64_t)(coding + ((size_t)s2 * p + l) * st);
    }
    CK(hipMalloc(&d_pptrs[q], hp.size() * 8));
    CK(hipMemcpy(d_pptrs[q], hp.data(), hp.size() * 8, hipMemcpyHostToDevice));
  }

  const unsigned tiles = (len + kTile - 1) / kTile;
  const unsigned nitems = S * tiles;
  const int stride = k + p;
  const double enc_bytes = (double)(k + p) * shard * S;
  std::vector<Variant> V;

#define PATTERN(R, W, NL, NS, NAME)                                                            \
  V.push_back({NAME, (double)((R) + (W)) * shard * S, [=](hipStream_t st) {                     \
                 hipLaunchKernelGGL((mem_pattern<R, W, NL, NS>), dim3(nitems), dim3(256), 0, st, \
                                    d_ptrs, stride, len, nitems, tiles, (uint32_t*)sinkp);      \
               }});
  PATTERN(10, 4, false, false, "mem read10+write4")
  PATTERN(10, 4, true, true, "mem read10+write4 nt/nt")
  PATTERN(10, 4, false, true, "mem read10+write4 ld/nt")
  PATTERN(10, 0, false, false, "mem read10 only")
#define PATTERNB(LD, ST, NAME)                                                                 \
  V.push_back({NAME, 14.0 * shard * S, [=](hipStream_t st) {                                    \
                 hipLaunchKernelGGL((mem_pattern_buf<10, 4, LD, ST>), dim3(nitems), dim3(256), 0, \
                                    st, d_ptrs, stride, len, nitems, tiles, (uint32_t*)sinkp);  \
               }});
  PATTERNB(2, 2, "buf r10w4 nt/nt")
  // the decode (C3) mix: 10 survivors read, 3 recovered shards written
  V.push_back({"buf r10w3 nt/nt (decode mix)", 13.0 * shard * S, [=](hipStream_t st) {
                 hipLaunchKernelGGL((mem_pattern_buf<10, 3, 2, 2>), dim3(nitems), dim3(256), 0, st,
                                    d_ptrs, stride, len, nitems, tiles, (uint32_t*)sinkp);
               }});
  PATTERNB(0x12, 0x12, "buf r10w4 sc1nt/sc1nt")
  PATTERNB(0x13, 0x13, "buf r10w4 sc0sc1nt/sc0sc1nt")
  PATTERNB(0x10, 0x10, "buf r10w4 sc1/sc1")
  PATTERNB(2, 0x12, "buf r10w4 nt/sc1nt")
  PATTERNB(3, 3, "buf r10w4 sc0nt/sc0nt")
  V.push_back({"mem r10w4 nt 2 tiles/item", 14.0 * shard * S, [=](hipStream_t st) {
                 hipLaunchKernelGGL((mem_pattern_2t<10, 4>), dim3(nitems / 2), dim3(256), 0, st,
                                    d_ptrs, stride, len, nitems, tiles, (uint32_t*)sinkp);
               }});
  PATTERN(0, 4, false, false, "mem write4 only")
  // first half of the parity buffer copied onto its second half: cbytes moved
  // (the source shards are never written, so encode outputs stay comparable)
  V.push_back({"copy16 (1 read : 1 write)", (double)cbytes, [=](hipStream_t st) {
                 hipLaunchKernelGGL(copy16, dim3(8192), dim3(256), 0, st, (const uint4*)coding,
                                    (uint4*)(coding + cbytes / 2), cbytes / 2 / 16);
               }});
#define COPYNT(U, GRID, NAME)                                                                  \
  V.push_back({NAME, 2.0 * (double)cbytes, [=](hipStream_t st) {                                \
                 hipLaunchKernelGGL((copy_nt<U>), dim3(GRID), dim3(256), 0, st, (const uint8_t*)data, \
                                    coding, cbytes);                                            \
               }});
  COPYNT(1, 16384, "copy nt data->coding 4 GiB U1 grid 16384")
  COPYNT(4, 16384, "copy nt data->coding 4 GiB U4 grid 16384")
  COPYNT(4, 2048, "copy nt data->coding 4 GiB U4 grid 2048")
  COPYNT(8, 2048, "copy nt data->coding 4 GiB U8 grid 2048")
  V.push_back({"buf r1w1 nt/nt (encode items, shard 0 -> parity 0)", 2.0 * shard * S, [=](hipStream_t st) {
                 hipLaunchKernelGGL((mem_pattern_buf<1, 1, 2, 2>), dim3(nitems), dim3(256), 0, st,
                                    d_ptrs, stride, len, nitems, tiles, (uint32_t*)sinkp);
               }});
  V.push_back({"hipMemcpyDtoD 4 GiB", 2.0 * (double)cbytes, [=](hipStream_t st) {
                 CK(hipMemcpyAsync(coding, data, cbytes, hipMemcpyDeviceToDevice, st));
               }});

#define ENC(POL, GRID, NAME)                                                                  \
  V.push_back({NAME, enc_bytes, [=](hipStream_t st) {                                          \
                 unsigned gr = (GRID) ? std::min<unsigned>((GRID), nitems) : nitems;          \
                 hipLaunchKernelGGL((ec_encode_v16<4, POL>), dim3(gr), dim3(256), 0, st, d_ptrs, \
                                    stride, 0, k, (const uint32_t*)d_tbl, len, k, nitems, tiles, 0ull, 0u); \
               }});                                                                           \
  V.back().encode = true;
  using PNB = Pol<4, true, true, 0>;
  using PNB10 = Pol<10, true, true, 0>;
  using PNB10X = Pol<10, true, true, 2>;
  using PBUF10 = EncPol<10, kBufNT, kBufNT, 0>;
  using PBUF10X = EncPol<10, kBufNT, kBufNT, 2>;
  using PBUF5 = EncPol<5, kBufNT, kBufNT, 0>;
  using PBUF10G16 = EncPol<10, kBufNT, kBufNT, 3>;
  using PBUF10G32 = EncPol<10, kBufNT, kBufNT, 5>;
  using PBUF10SX = EncPol<10, kBufNT, kBufNT, 4>;
  ENC(EncDefault, 0, "encode default (buf U4)")
  ENC(PNB, 0, "encode U4 nt-both")
  ENC(PNB10, 0, "encode U10 nt-both")
  ENC(PNB10X, 0, "encode U10 nt-both xcd-contig")
  ENC(PBUF10, 0, "encode U10 buf-nt")
  ENC(PBUF10X, 0, "encode U10 buf-nt xcd-contig")
  ENC(PBUF5, 0, "encode U5 buf-nt")
  ENC(PBUF10X, 2048, "encode U10 buf-nt xcd-contig grid 2048")
  ENC(PBUF10X, 4096, "encode U10 buf-nt xcd-contig grid 4096")
  ENC(PBUF10X, 16384, "encode U10 buf-nt xcd-contig grid 16384")
  ENC(PBUF10, 4096, "encode U10 buf-nt grid 4096")
  ENC(PBUF10G16, 0, "encode U10 buf-nt 16 ranges")
  ENC(PBUF10G32, 0, "encode U10 buf-nt 32 ranges")
  ENC(PBUF10SX, 0, "encode U10 buf-nt stripes mod 8 per XCD")
#define ENCP(POL, Q, NAME)                                                                     \
  V.push_back({NAME, enc_bytes, [=](hipStream_t st) {                                          \
                 hipLaunchKernelGGL((ec_encode_v16<4, POL>), dim3(nitems), dim3(256), 0, st,     \
                                    d_pptrs[Q], stride, 0, k, (const uint32_t*)d_tbl, len, k,    \
                                    nitems, tiles, 0ull, 0u);                                  \
               }});
  ENCP(PNB, 0, "encode U4 nt-both pad256 (unchecked)")
  ENCP(PNB, 1, "encode U4 nt-both pad4K (unchecked)")
  ENCP(PNB, 2, "encode U4 nt-both pad68K (unchecked)")
  ENCP(EncDefault, 1, "encode U4 pad4K (unchecked)")

  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));

  // reference parity from the default variant
  std::vector<uint8_t> want(cbytes / S * 2), got(cbytes / S * 2);
  auto grab = [&](std::vector<uint8_t>& out) {
    CK(hipStreamSynchronize(st));
    CK(hipMemcpy(out.data(), coding, cbytes / S, hipMemcpyDeviceToHost));
    CK(hipMemcpy(out.data() + cbytes / S, coding + cbytes - cbytes / S, cbytes / S,
                 hipMemcpyDeviceToHost));
  };
  // reference parity from the default encode variant
  for (auto& v : V)
    if (v.encode) {
      v.run(st);
      break;
    }
  grab(want);

  for (int r = 0; r < rounds; ++r) {
    for (auto& v : V) {
      v.run(st);  // warm
      CK(hipEventRecord(e0, st));
      for (int i = 0; i < iters; ++i) v.run(st);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.gbs.push_back(v.bytes / (ms / iters * 1e-3) / 1e9);
      if (v.encode) {
        CK(hipMemsetAsync(coding, 0, cbytes / S, st));
        v.run(st);
        grab(got);
        if (memcmp(got.data(), want.data(), want.size()) != 0) {
          fprintf(stderr, "MISMATCH in variant %s\n", v.name.c_str());
          return 3;
        }
      }
    }
  }
  printf("%-34s %10s %10s %8s\n", "variant", "median", "max", "%8TB/s");
  std::string json = "{";
  for (auto& v : V) {
    std::vector<double> s = v.gbs;
    std::sort(s.begin(), s.end());
    const double med = s[s.size() / 2], mx = s.back();
    printf("%-34s %10.1f %10.1f %8.1f\n", v.name.c_str(), med, mx, med / 80.0);
    json += "\"" + v.name + "\": " + std::to_string(med) + ", ";
  }
  json += "\"unit\": \"GB/s (algorithmic bytes / launch time, median of rounds)\"}";
  printf("%s\n", json.c_str());
  return 0;
}
