// update_probe.hip — measurement tool, not part of libisal_hip.so.
//
// Achievable HBM bandwidth for the update (gf_vect_mad / ec_encode_data_update)
// access pattern — per lane: read 16 B of one source and of every parity
// shard, write the parity back in place — as memory-only kernels (XOR instead
// of GF math) beside the engine's ec_update_v16<P> and update variants.
// Default shape C4: k=20 p=6, 4 MiB shards, 64 stripes. Interleaved rounds,
// median per variant; bytes counted (1 + 2p) * len per stripe.
#include "../csrc/ec_kernels.hip"

#include <algorithm>
#include <cstdio>
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

// read src + P parity, write P parity in place (XOR of the source as the "math")
template <int P, int LD, int ST>
__global__ __launch_bounds__(256) void mem_rmw(const uint64_t* __restrict__ ptrs, int stride,
                                               int src, int dst0, int len, unsigned nitems,
                                               unsigned tiles) {
  for (unsigned w = blockIdx.x; w < nitems; w += gridDim.x) {
    const unsigned stripe = w / tiles, tile = w - stripe * tiles;
    const uint64_t* __restrict__ sp = ptrs + static_cast<size_t>(stripe) * stride;
    const long long off = static_cast<long long>(tile) * kTile + threadIdx.x * kVec;
    const uint4 x = load16<LD>(sp[src], off, len);
    uint4 d[P];
#pragma unroll
    for (int l = 0; l < P; ++l) d[l] = load16<LD>(sp[dst0 + l], off, len);
#pragma unroll
    for (int l = 0; l < P; ++l) {
      d[l].x ^= x.x; d[l].y ^= x.y; d[l].z ^= x.z; d[l].w ^= x.w;
      store16<ST>(sp[dst0 + l], off, d[l], len);
    }
  }
}

// The update kernel with two 4 KiB tiles per work item: twice the bytes in
// flight per lane (the encode kernel's U = 10 loads vs the update's 7).
template <int P>
__global__ __launch_bounds__(kBlock) void update_2t(const uint64_t* __restrict__ ptrs,
                                                    int ptr_stride, int src_idx, int dst0,
                                                    const uint32_t* __restrict__ tbl, int len,
                                                    unsigned nitems, unsigned tiles) {
  const unsigned half = tiles / 2;
  for (unsigned w = blockIdx.x; w < nitems / 2; w += gridDim.x) {
    const unsigned stripe = w / half, tp = w - stripe * half;
    const uint64_t* __restrict__ sp = ptrs + static_cast<size_t>(stripe) * ptr_stride;
    const long long off0 = static_cast<long long>(tp) * 2 * kTile + threadIdx.x * kVec;
    const long long off1 = off0 + kTile;
    const uint4 x0 = load16<kBufNT>(sp[src_idx], off0, len);
    const uint4 x1 = load16<kBufNT>(sp[src_idx], off1, len);
    uint4 d0[P], d1[P];
#pragma unroll
    for (int l = 0; l < P; ++l) {
      d0[l] = load16<kBufNT>(sp[dst0 + l], off0, len);
      d1[l] = load16<kBufNT>(sp[dst0 + l], off1, len);
    }
    const Sel a0 = split(x0.x), a1 = split(x0.y), a2 = split(x0.z), a3 = split(x0.w);
    const Sel b0 = split(x1.x), b1 = split(x1.y), b2 = split(x1.z), b3 = split(x1.w);
#pragma unroll
    for (int l = 0; l < P; ++l) {
      const Coef c = load_coef(tbl + l * kTbl);
      d0[l].x ^= gf_mul4(c, a0); d0[l].y ^= gf_mul4(c, a1);
      d0[l].z ^= gf_mul4(c, a2); d0[l].w ^= gf_mul4(c, a3);
      d1[l].x ^= gf_mul4(c, b0); d1[l].y ^= gf_mul4(c, b1);
      d1[l].z ^= gf_mul4(c, b2); d1[l].w ^= gf_mul4(c, b3);
      store16<kBufNT>(sp[dst0 + l], off0, d0[l], len);
      store16<kBufNT>(sp[dst0 + l], off1, d1[l], len);
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

struct Variant {
  std::string name;
  std::function<void(hipStream_t)> run;
  std::vector<double> gbs;
};

}  // namespace

int main(int argc, char** argv) {
  const int k = argc > 1 ? atoi(argv[1]) : 20;
  const int len = argc > 2 ? atoi(argv[2]) : (4 << 20);
  const int S = argc > 3 ? atoi(argv[3]) : 64;
  const int rounds = argc > 4 ? atoi(argv[4]) : 5;
  constexpr int p = 6;
  const int iters = 10;
  const size_t shard = static_cast<size_t>(len);
  uint8_t *data, *coding;
  CK(hipMalloc(&data, shard * k * S));
  CK(hipMalloc(&coding, shard * p * S));
  hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, (uint32_t*)data, shard * k * S / 4, 7u);
  hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, (uint32_t*)coding, shard * p * S / 4, 9u);
  CK(hipDeviceSynchronize());
  std::vector<uint64_t> h_ptrs(static_cast<size_t>(S) * (k + p));
  for (int s = 0; s < S; ++s) {
    for (int j = 0; j < k; ++j) h_ptrs[(size_t)s * (k + p) + j] = (uint64_t)(data + ((size_t)s * k + j) * shard);
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
  const unsigned tiles = (len + kTile - 1) / kTile;
  const unsigned nitems = S * tiles;
  const int stride = k + p;
  const double bytes = (1.0 + 2 * p) * shard * S;
  const int vi = 3;  // the source folded in (any)
  const uint32_t* tb = d_tbl + static_cast<size_t>(vi) * p * kTbl;
  std::vector<Variant> V;
  V.push_back({"mem rmw buf-nt/buf-nt", [=](hipStream_t st) {
                 hipLaunchKernelGGL((mem_rmw<p, kBufNT, kBufNT>), dim3(nitems), dim3(256), 0, st,
                                    d_ptrs, stride, vi, k, len, nitems, tiles);
               }});
  V.push_back({"mem rmw plain/plain", [=](hipStream_t st) {
                 hipLaunchKernelGGL((mem_rmw<p, kPlain, kPlain>), dim3(nitems), dim3(256), 0, st,
                                    d_ptrs, stride, vi, k, len, nitems, tiles);
               }});
  V.push_back({"mem rmw plain/nt", [=](hipStream_t st) {
                 hipLaunchKernelGGL((mem_rmw<p, kPlain, kNT>), dim3(nitems), dim3(256), 0, st,
                                    d_ptrs, stride, vi, k, len, nitems, tiles);
               }});
  V.push_back({"ec_update_v16<6> (engine)", [=](hipStream_t st) {
                 hipLaunchKernelGGL(ec_update_v16<p>, dim3(nitems), dim3(kBlock), 0, st, d_ptrs,
                                    stride, vi, k, tb, len, nitems, tiles);
               }});
  V.push_back({"update 2 tiles/item", [=](hipStream_t st) {
                 hipLaunchKernelGGL(update_2t<p>, dim3(nitems / 2), dim3(kBlock), 0, st, d_ptrs,
                                    stride, vi, k, tb, len, nitems, tiles);
               }});
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int r = 0; r < rounds; ++r)
    for (auto& v : V) {
      v.run(st);
      CK(hipEventRecord(e0, st));
      for (int i = 0; i < iters; ++i) v.run(st);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.gbs.push_back(bytes / (ms / iters * 1e-3) / 1e9);
    }
  // the 2-tile variant must equal the engine kernel: apply engine then undo with 2t
  // (update is its own inverse: x ^= c*s twice restores x)
  {
    std::vector<uint8_t> before(shard), after(shard);
    CK(hipMemcpy(before.data(), coding, shard, hipMemcpyDeviceToHost));
    hipLaunchKernelGGL(ec_update_v16<p>, dim3(nitems), dim3(kBlock), 0, st, d_ptrs, stride, vi, k, tb,
                       len, nitems, tiles);
    hipLaunchKernelGGL(update_2t<p>, dim3(nitems / 2), dim3(kBlock), 0, st, d_ptrs, stride, vi, k,
                       tb, len, nitems, tiles);
    CK(hipStreamSynchronize(st));
    CK(hipMemcpy(after.data(), coding, shard, hipMemcpyDeviceToHost));
    if (before != after) {
      fprintf(stderr, "MISMATCH: update_2t is not the engine update\n");
      return 3;
    }
  }
  printf("%-30s %10s %10s %8s   (k=%d p=%d len=%d stripes=%d, bytes (1+2p)*len)\n", "variant",
         "median", "max", "%8TB/s", k, p, len, S);
  for (auto& v : V) {
    std::vector<double> s = v.gbs;
    std::sort(s.begin(), s.end());
    printf("%-30s %10.1f %10.1f %8.1f\n", v.name.c_str(), s[s.size() / 2], s.back(),
           s[s.size() / 2] / 80.0);
  }
  return 0;
}
