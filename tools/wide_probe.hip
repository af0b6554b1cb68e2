// wide_probe.hip — the wide encode passes (5-8 parity rows) with their GF
// products looked up in LDS instead of computed by v_perm (not shipped).
//
// The library's encode multiplies each source byte by each of the pass's P
// coefficients with three v_perm_b32 lookups (3+3+2-bit fields of the byte,
// 8-byte tables in SGPRs): ~4.5 VALU per (source dword, row), VALU-bound from
// ~6 rows on. Here one lookup returns the products of one source
// byte field with ALL P coefficients at once: per source j, a 32-entry table
// T5_j[v] (8 bytes: byte l = c[l][j] * v, v = bits 0-4) and an 8-entry table
// T3_j[v] (byte l = c[l][j] * (v << 5), bits 5-7) in LDS. A lane accumulates
// its 16 byte positions as 16 X64 words (byte l = row l's partial), two
// lookups and one XOR3 per half per source byte, and transposes them into the
// P parity rows before storing (v_perm, once per tile). Per source dword: 12
// offset ops (byte fields pre-scaled by 8, one SDWA add each) + 8 XOR3 + 8
// ds_read_b64, whatever P; the tables are conflict-free (32 entries x 8 B =
// one bank row).
//
// The library ships this as ec_encode_ldsx (7-8 row passes). Variants here:
//   glds        the library's encode with no product tables (ec_encode_glds)
//   ldsx_uU     ec_encode_ldsx<P, U>: U sources loaded, then folded
//   ldsx_pf2    pairs, the next pair's loads issued before the current is folded
//   ldsx_ringR  sources staged through a per-wave LDS-DMA ring of R slots
//
// Round-6 final form: the library's ec_encode_ldsx<P, 2> (double-buffered
// pairs) at several occupancy caps (dynamic LDS per workgroup) beside the
// library's encode, in bench.py's shard layout (LAYOUT 1) or with each
// stripe's shards back to back (0, the layout of the sweeps above).
//
//   usage: wide_probe [ITERS] [ROUNDS] [LAYOUT]   one JSON line per (shape, variant)
//          wide_probe ITERS ROUNDS LAYOUT matrix  the library's default over k x p
//          wide_probe ITERS ROUNDS 1 lanes        the product tables at 256 / 128 lanes x caps
//
// Build: make -C isa-l_amd wide_probe (includes csrc/ec_kernels.hip).
#include "../isa-l_amd/csrc/ec_kernels.hip"

#include <cstring>
#include <vector>

#include "erasure_code.h"

extern "C" void isal_hip_count_launch(void) {}
extern "C" void isal_hip_kreg_add(const void*, const char*) {}

namespace {

// ec_encode_ldsx with the next pair's loads issued before the current pair is
// folded (register double buffer: 4 loads in flight per wave instead of 2)
template <int P>
__global__ __launch_bounds__(kBlock) void ldsx_pf(const uint64_t* __restrict__ ptrs, int ptr_stride, int src0,
                                                  int dst0, const uint64_t* __restrict__ ltg, int len, int k,
                                                  unsigned nitems, unsigned tiles) {
  extern __shared__ uint64_t lt[];
  for (int i = threadIdx.x; i < k * ISAL_HIP_LDSX_ENTRIES; i += kBlock) lt[i] = ltg[i];
  __syncthreads();
  const uint32_t base5 = lds_off(lt), base3 = base5 + static_cast<uint32_t>(k) * 256u;
  for (unsigned w = blockIdx.x; w < nitems; w += gridDim.x) {
    const unsigned v = xcd_item(w, nitems, 1);
    const unsigned stripe = v / tiles, tile = v - stripe * tiles;
    const uint64_t* __restrict__ sp = ptrs + static_cast<size_t>(stripe) * ptr_stride;
    const long long off = static_cast<long long>(tile) * kTile + threadIdx.x * kVec;
    if (off + kVec > len) continue;  // the probe's shapes have len % 4096 == 0
    Acc64 acc[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = Acc64{0u, 0u};
    uint4 a0 = load16<kBufNT>(sp[src0], off, len);
    uint4 a1 = k > 1 ? load16<kBufNT>(sp[src0 + 1], off, len) : make_uint4(0, 0, 0, 0);
    for (int j = 0; j < k; j += 2) {
      uint4 b0 = make_uint4(0, 0, 0, 0), b1 = make_uint4(0, 0, 0, 0);
      if (j + 2 < k) b0 = load16<kBufNT>(sp[src0 + j + 2], off, len);
      if (j + 3 < k) b1 = load16<kBufNT>(sp[src0 + j + 3], off, len);
      ldsx_acc(acc, a0, base5 + j * 256u, base3 + j * 64u);
      if (j + 1 < k) ldsx_acc(acc, a1, base5 + (j + 1) * 256u, base3 + (j + 1) * 64u);
      a0 = b0;
      a1 = b1;
    }
    ldsx_store<P>(acc, sp, dst0, off, len);
  }
}

// ec_encode_ldsx with the sources staged through a per-wave LDS-DMA ring of R
// 1-KiB slots, as ec_encode_glds: R loads in flight all the time, no VGPRs
template <int P, int R>
__global__ __launch_bounds__(kBlock) void ldsx_ring(const uint64_t* __restrict__ ptrs, int ptr_stride, int src0,
                                                    int dst0, const uint64_t* __restrict__ ltg, int len, int k,
                                                    unsigned nitems, unsigned tiles) {
  static_assert(R % 2 == 0 && R >= 2 && R <= 8, "ring of 2..8 slots, folded in pairs");
  extern __shared__ uint64_t lt[];
  const int ltn = k * ISAL_HIP_LDSX_ENTRIES;
  for (int i = threadIdx.x; i < ltn; i += kBlock) lt[i] = ltg[i];
  __syncthreads();
  const uint32_t base5 = lds_off(lt), base3 = base5 + static_cast<uint32_t>(k) * 256u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t ring = base5 + ((static_cast<uint32_t>(ltn) * 8 + 1023) & ~1023u) + wave * (R * 1024);
  const uint32_t mine = ring + (threadIdx.x & 63) * kVec;
  for (unsigned w = blockIdx.x; w < nitems; w += gridDim.x) {
    const unsigned v = xcd_item(w, nitems, 1);
    const unsigned stripe = v / tiles, tile = v - stripe * tiles;
    const uint64_t* __restrict__ sp = ptrs + static_cast<size_t>(stripe) * ptr_stride;
    const long long off = static_cast<long long>(tile) * kTile + threadIdx.x * kVec;
    if (static_cast<long long>(tile + 1) * kTile > len) continue;  // full tiles only in the probe
    vm_wait<0>();
    const uint32_t voff = static_cast<uint32_t>(off);
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (r < k) glds16(sp[src0 + r], voff, ring + r * 1024);
    Acc64 acc[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = Acc64{0u, 0u};
    for (int j0 = 0; j0 < k; j0 += R) {
      auto step = [&](auto rc) {
        constexpr int r = decltype(rc)::value * 2;
        const int j = j0 + r;
        if (j >= k) return;
        uint4 x0, x1;
        if (j + 1 < k) {
          if (j + R <= k)
            vm_wait<R - 2>();
          else
            vm_wait_rt(k - 2 - j);
          lds_read2<r * 1024, (r + 1) * 1024>(x0, x1, mine);
          if (j + R < k) glds16(sp[src0 + j + R], voff, ring + r * 1024);
          if (j + 1 + R < k) glds16(sp[src0 + j + 1 + R], voff, ring + (r + 1) * 1024);
          __builtin_amdgcn_sched_barrier(0);
          ldsx_acc(acc, x0, base5 + j * 256u, base3 + j * 64u);
          ldsx_acc(acc, x1, base5 + (j + 1) * 256u, base3 + (j + 1) * 64u);
        } else {
          vm_wait<0>();
          lds_read1<r * 1024>(x0, mine);
          __builtin_amdgcn_sched_barrier(0);
          ldsx_acc(acc, x0, base5 + j * 256u, base3 + j * 64u);
        }
        __builtin_amdgcn_sched_barrier(0);
      };
      static_for(step, std::make_integer_sequence<int, R / 2>{});
    }
    vm_wait<0>();
    ldsx_store<P>(acc, sp, dst0, off, len);
  }
}

}  // namespace

#define CK(x)                                                                               \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));    \
      exit(1);                                                                              \
    }                                                                                       \
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

struct Shape {
  int k, p, len, ns;
};

// V: 1..5 the library's ec_encode_ldsx<P, V>; 10 + R the LDS-DMA ring of R slots; 20 the prefetch
template <int P>
static void launch_var(int V, unsigned grid, const uint64_t* dp, int stride, const uint32_t* dt, const uint64_t* dlt,
                       int len, int k, unsigned nitems, unsigned tiles, size_t cap) {
  const size_t lt0 = static_cast<size_t>(k) * ISAL_HIP_LDSX_ENTRIES * 8, ringb = (lt0 + 1023) & ~size_t(1023);
  const size_t lt = lt0 > cap ? lt0 : cap;  // dynamic LDS as an occupancy cap
  switch (V) {
#define LIB(u)                                                                                                   \
  case u:                                                                                                        \
    hipLaunchKernelGGL((ec_encode_ldsx<P, u>), dim3(grid), dim3(kBlock), lt, 0, dp, stride, 0, k, dt, dlt, len, k, \
                       nitems, tiles);                                                                           \
    return;
    LIB(1) LIB(2) LIB(3) LIB(4)
#undef LIB
#define RING(r)                                                                                                  \
  case 10 + r:                                                                                                   \
    hipLaunchKernelGGL((ldsx_ring<P, r>), dim3(grid), dim3(kBlock), ringb + 4 * r * 1024, 0, dp, stride, 0, k, dlt, \
                       len, k, nitems, tiles);                                                                   \
    return;
    RING(2) RING(4) RING(6) RING(8)
#undef RING
    case 20:
      hipLaunchKernelGGL((ldsx_pf<P>), dim3(grid), dim3(kBlock), lt, 0, dp, stride, 0, k, dlt, len, k, nitems, tiles);
      return;
  }
  fprintf(stderr, "no variant %d\n", V);
  exit(1);
}

static void ldsx(int P, int V, unsigned grid, const uint64_t* dp, int stride, const uint32_t* dt, const uint64_t* dlt,
                 int len, int k, unsigned nitems, unsigned tiles, size_t cap) {
  switch (P) {
    case 4: return launch_var<4>(V, grid, dp, stride, dt, dlt, len, k, nitems, tiles, cap);
    case 5: return launch_var<5>(V, grid, dp, stride, dt, dlt, len, k, nitems, tiles, cap);
    case 6: return launch_var<6>(V, grid, dp, stride, dt, dlt, len, k, nitems, tiles, cap);
    case 7: return launch_var<7>(V, grid, dp, stride, dt, dlt, len, k, nitems, tiles, cap);
    case 8: return launch_var<8>(V, grid, dp, stride, dt, dlt, len, k, nitems, tiles, cap);
  }
  fprintf(stderr, "no instantiation P=%d\n", P);
  exit(1);
}

// matrix mode: the library's default dispatch (product tables uploaded, as a
// batch does) over k x p shapes of 1 MiB shards, ~14 GiB per launch, in
// bench.py's layout; bit_exact = the same parity as the library without the
// product tables (the v_perm kernels, which the GPU suite checks against the
// oracle).
static int matrix_main(int iters, int rounds, int layout) {
  const int ks[] = {4, 6, 8, 10, 12, 16, 20, 24, 32}, ps[] = {1, 2, 3, 4, 5, 6, 7, 8};
  const int len = 1 << 20;
  const size_t shard = static_cast<size_t>(len);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int round = 0; round < rounds; ++round)
  for (int k : ks)
    for (int p : ps) {
      const int stride = k + p;
      const int ns = static_cast<int>((14ull << 30) / (static_cast<unsigned long long>(stride) * shard));
      uint8_t *d = nullptr, *c = nullptr;
      // layout 0: one buffer, each stripe's k + p shards back to back (c aliases d)
      CK(hipMalloc(&d, shard * (layout ? k : stride) * ns));
      if (layout)
        CK(hipMalloc(&c, shard * p * ns));
      else
        c = d;
      hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint64_t*>(d),
                         shard * (layout ? k : stride) * ns / 8, 977ull + k * 31 + p);
      std::vector<uint64_t> hp(static_cast<size_t>(stride) * ns);
      for (int st = 0; st < ns; ++st)
        for (int i = 0; i < stride; ++i)
          hp[static_cast<size_t>(st) * stride + i] = reinterpret_cast<uint64_t>(
              layout ? (i < k ? d + (static_cast<size_t>(st) * k + i) * shard
                              : c + (static_cast<size_t>(st) * p + i - k) * shard)
                     : (i < k ? d : c) + (static_cast<size_t>(st) * stride + i) * shard);
      uint64_t* dp = nullptr;
      CK(hipMalloc(&dp, hp.size() * 8));
      CK(hipMemcpy(dp, hp.data(), hp.size() * 8, hipMemcpyHostToDevice));
      std::vector<unsigned char> a(stride * k), g(32 * k * p);
      gf_gen_rs_matrix(a.data(), stride, k);
      ec_init_tables(k, p, a.data() + k * k, g.data());
      std::vector<uint32_t> ht(isal_hip_tables_dwords(k, p) + 1);
      isal_hip_build_tables(k, p, g.data(), ht.data());
      isal_hip_encmask em, em0;
      isal_hip_enc_masks(k, p, g.data(), &em);
      em0 = em;
      uint32_t* dt = nullptr;
      CK(hipMalloc(&dt, ht.size() * 4));
      CK(hipMemcpy(dt, ht.data(), ht.size() * 4, hipMemcpyHostToDevice));
      std::vector<uint64_t> hl(isal_hip_ldsx_words(k, p));
      isal_hip_build_ldsx_tables(k, p, g.data(), hl.data());
      uint64_t* dl = nullptr;
      CK(hipMalloc(&dl, hl.size() * 8));
      CK(hipMemcpy(dl, hl.data(), hl.size() * 8, hipMemcpyHostToDevice));
      em.ldsx = dl;
      uint8_t* last = reinterpret_cast<uint8_t*>(hp[static_cast<size_t>(ns - 1) * stride + k]);  // p shards apart by layout
      std::vector<uint8_t> ref(shard * p), got(shard * p);
      CK(static_cast<hipError_t>(isal_hip_launch_encode(dp, stride, 0, k, dt, len, k, p, ns, 1, &em0, nullptr)));
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(ref.data(), last, shard * p, hipMemcpyDeviceToHost));
      CK(hipMemset(last, 0xA5, shard * p));
      auto go = [&]() {
        CK(static_cast<hipError_t>(isal_hip_launch_encode(dp, stride, 0, k, dt, len, k, p, ns, 1, &em, nullptr)));
      };
      go();
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(got.data(), last, shard * p, hipMemcpyDeviceToHost));
      const bool ok = memcmp(ref.data(), got.data(), shard * p) == 0;
      for (int w = 0; w < 2; ++w) go();
      CK(hipEventRecord(e0, 0));
      for (int it = 0; it < iters; ++it) go();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= iters;
      const double bytes = static_cast<double>(stride) * shard * ns;
      printf("{\"round\": %d, \"layout\": %d, \"k\": %d, \"p\": %d, \"len\": %d, \"stripes\": %d, \"ms\": %.4f, "
             "\"frac\": %.4f, \"bit_exact\": %s}\n", round, layout, k, p, len, ns, ms, bytes / ms / 1e6 / 8000.0,
             ok ? "true" : "false");
      fflush(stdout);
      CK(hipFree(d));
      if (layout) CK(hipFree(c));
      CK(hipFree(dp));
      CK(hipFree(dt));
      CK(hipFree(dl));
    }
  return 0;
}

// ec_encode_ldsx's body at 128 lanes (2 KiB tiles)
template <int P>
__global__ __launch_bounds__(128) void ldsx_128(const uint64_t* __restrict__ ptrs, int ptr_stride,
                                                const uint32_t* __restrict__ tbl, const uint64_t* __restrict__ ltg,
                                                int len, int k, unsigned nitems, unsigned tiles) {
  ldsx_items<P, 2, kBufNT, 128>(ptrs, ptr_stride, 0, k, tbl, ltg, len, k, nitems, tiles);
}

// lanes mode: ec_encode_ldsx<P, 2> at 256 lanes against ldsx_items at 128 lanes
// under dynamic-LDS occupancy caps (0 = its tables only), bench.py's layout.
static int lanes_main(int iters, int rounds) {
  struct Sh { int k, p, len, ns; };
  const Sh shapes[] = {{20, 8, 4 << 20, 64}, {20, 6, 4 << 20, 64}, {16, 8, 1 << 20, 512}, {10, 8, 1 << 20, 1024}};
  // LANES_ORDER=1: 256 lanes only, cap 0 measured first and last (is the first
  // configuration of a shape slow only because it runs first?)
  const bool order = getenv("LANES_ORDER") != nullptr;
  const std::vector<int> caps = order ? std::vector<int>{0, 16384, 20480, 0, 16384, 0}
                                      : std::vector<int>{0, 8192, 10240, 13312, 16384, 20480};
  const std::vector<int> lane_set = order ? std::vector<int>{256} : std::vector<int>{256, 128};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int round = 0; round < rounds; ++round)
    for (const Sh& sh : shapes) {
      const int k = sh.k, p = sh.p, len = sh.len, ns = sh.ns, stride = k + p;
      const size_t shard = static_cast<size_t>(len);
      uint8_t *d = nullptr, *c = nullptr;
      CK(hipMalloc(&d, shard * k * ns));
      CK(hipMalloc(&c, shard * p * ns));
      hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint64_t*>(d), shard * k * ns / 8, 5ull + k);
      std::vector<uint64_t> hp(static_cast<size_t>(stride) * ns);
      for (int st = 0; st < ns; ++st)
        for (int i = 0; i < stride; ++i)
          hp[static_cast<size_t>(st) * stride + i] = reinterpret_cast<uint64_t>(
              i < k ? d + (static_cast<size_t>(st) * k + i) * shard : c + (static_cast<size_t>(st) * p + i - k) * shard);
      uint64_t* dp = nullptr;
      CK(hipMalloc(&dp, hp.size() * 8));
      CK(hipMemcpy(dp, hp.data(), hp.size() * 8, hipMemcpyHostToDevice));
      std::vector<unsigned char> a(stride * k), g(32 * k * p);
      gf_gen_rs_matrix(a.data(), stride, k);
      ec_init_tables(k, p, a.data() + k * k, g.data());
      std::vector<uint32_t> ht(isal_hip_tables_dwords(k, p) + 1);
      isal_hip_build_tables(k, p, g.data(), ht.data());
      uint32_t* dt = nullptr;
      CK(hipMalloc(&dt, ht.size() * 4));
      CK(hipMemcpy(dt, ht.data(), ht.size() * 4, hipMemcpyHostToDevice));
      std::vector<uint64_t> hl(isal_hip_ldsx_words(k, p));
      isal_hip_build_ldsx_tables(k, p, g.data(), hl.data());
      uint64_t* dl = nullptr;
      CK(hipMalloc(&dl, hl.size() * 8));
      CK(hipMemcpy(dl, hl.data(), hl.size() * 8, hipMemcpyHostToDevice));
      const size_t lt = static_cast<size_t>(k) * ISAL_HIP_LDSX_ENTRIES * 8;
      const uint8_t* last = c + static_cast<size_t>(ns - 1) * p * shard;
      std::vector<uint8_t> ref(shard * p), got(shard * p);
      const unsigned t256 = len / kTile, t128 = len / (128 * kVec);
      auto run = [&](int lanes, int cap) {
        const size_t dyn = lt > static_cast<size_t>(cap) ? lt : static_cast<size_t>(cap);
        if (lanes == 256) {
          if (p == 8)
            hipLaunchKernelGGL((ec_encode_ldsx<8, 2>), dim3(t256 * ns), dim3(256), dyn, 0, dp, stride, 0, k, dt, dl, len,
                               k, t256 * ns, t256);
          else
            hipLaunchKernelGGL((ec_encode_ldsx<6, 2>), dim3(t256 * ns), dim3(256), dyn, 0, dp, stride, 0, k, dt, dl, len,
                               k, t256 * ns, t256);
        } else {
          if (p == 8)
            hipLaunchKernelGGL((ldsx_128<8>), dim3(t128 * ns), dim3(128), dyn, 0, dp, stride, dt, dl, len, k, t128 * ns,
                               t128);
          else
            hipLaunchKernelGGL((ldsx_128<6>), dim3(t128 * ns), dim3(128), dyn, 0, dp, stride, dt, dl, len, k, t128 * ns,
                               t128);
        }
      };
      run(256, 0);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(ref.data(), last, shard * p, hipMemcpyDeviceToHost));
      for (int lanes : lane_set)
        for (int cap : caps) {
          CK(hipMemset(const_cast<uint8_t*>(last), 0xA5, shard * p));
          run(lanes, cap);
          CK(hipDeviceSynchronize());
          CK(hipGetLastError());
          CK(hipMemcpy(got.data(), last, shard * p, hipMemcpyDeviceToHost));
          const bool ok = memcmp(ref.data(), got.data(), shard * p) == 0;
          for (int w = 0; w < 2; ++w) run(lanes, cap);
          CK(hipEventRecord(e0, 0));
          for (int it = 0; it < iters; ++it) run(lanes, cap);
          CK(hipEventRecord(e1, 0));
          CK(hipEventSynchronize(e1));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, e0, e1));
          ms /= iters;
          const double bytes = static_cast<double>(stride) * shard * ns;
          printf("{\"round\": %d, \"k\": %d, \"p\": %d, \"lanes\": %d, \"cap\": %d, \"ms\": %.4f, \"frac\": %.4f, "
                 "\"bit_exact\": %s}\n", round, k, p, lanes, cap, ms, bytes / ms / 1e6 / 8000.0, ok ? "true" : "false");
          fflush(stdout);
        }
      CK(hipFree(d));
      CK(hipFree(c));
      CK(hipFree(dp));
      CK(hipFree(dt));
      CK(hipFree(dl));
    }
  return 0;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 10;
  if (argc > 4 && strcmp(argv[4], "lanes") == 0) return lanes_main(iters, argc > 2 ? atoi(argv[2]) : 1);
  if (argc > 4 && strcmp(argv[4], "matrix") == 0)
    return matrix_main(iters, argc > 2 ? atoi(argv[2]) : 1, argc > 3 ? atoi(argv[3]) : 1);
  const int rounds = argc > 2 ? atoi(argv[2]) : 2;
  // layout 1 (default): bench.py's — the sources of all stripes in one buffer
  // (stripe s, source j at (s k + j) len), the parity rows in another; layout
  // 0: each stripe's k + p shards back to back in one buffer
  const int layout = argc > 3 ? atoi(argv[3]) : 1;
  const Shape shapes[] = {{10, 4, 1 << 20, 1024}, {12, 4, 1 << 20, 1024}, {10, 6, 1 << 20, 1024},
                          {10, 8, 1 << 20, 1024}, {16, 8, 1 << 20, 512},  {13, 6, 1 << 20, 512},
                          {20, 6, 4 << 20, 64},   {20, 8, 4 << 20, 64}};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int round = 0; round < rounds; ++round)
    for (const Shape& s : shapes) {
      const int k = s.k, p = s.p, len = s.len, ns = s.ns, stride = k + p;
      const size_t shard = static_cast<size_t>(len);
      uint8_t *d = nullptr, *c = nullptr;
      CK(hipMalloc(&d, shard * (layout ? k : stride) * ns));
      if (layout) CK(hipMalloc(&c, shard * p * ns));
      hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint64_t*>(d),
                         shard * (layout ? k : stride) * ns / 8, 777ull + k * 31 + p);
      std::vector<uint64_t> hp(static_cast<size_t>(stride) * ns);
      auto at = [&](size_t st, int i) -> uint8_t* {
        if (!layout) return d + (st * stride + i) * shard;
        return i < k ? d + (st * k + i) * shard : c + (st * p + (i - k)) * shard;
      };
      for (int st = 0; st < ns; ++st)
        for (int i = 0; i < stride; ++i) hp[static_cast<size_t>(st) * stride + i] = reinterpret_cast<uint64_t>(at(st, i));
      uint64_t* dp = nullptr;
      CK(hipMalloc(&dp, hp.size() * 8));
      CK(hipMemcpy(dp, hp.data(), hp.size() * 8, hipMemcpyHostToDevice));
      std::vector<unsigned char> a(stride * k), g(32 * k * p);
      gf_gen_rs_matrix(a.data(), stride, k);
      ec_init_tables(k, p, a.data() + k * k, g.data());
      std::vector<uint32_t> ht(isal_hip_tables_dwords(k, p) + 1);
      isal_hip_build_tables(k, p, g.data(), ht.data());
      isal_hip_encmask em;
      isal_hip_enc_masks(k, p, g.data(), &em);
      uint32_t* dt = nullptr;
      CK(hipMalloc(&dt, ht.size() * 4));
      CK(hipMemcpy(dt, ht.data(), ht.size() * 4, hipMemcpyHostToDevice));
      std::vector<uint64_t> hl(isal_hip_ldsx_words(k, p));
      isal_hip_build_ldsx_tables(k, p, g.data(), hl.data());
      uint64_t* dl = nullptr;
      CK(hipMalloc(&dl, hl.size() * 8));
      CK(hipMemcpy(dl, hl.data(), hl.size() * 8, hipMemcpyHostToDevice));
      const unsigned tiles = len / kTile, nitems = tiles * ns;
      const double bytes = static_cast<double>(stride) * shard * ns;
      // reference parity: the library's encode without product tables
      std::vector<uint8_t> ref(shard * p), got(shard * p);
      CK(static_cast<hipError_t>(isal_hip_launch_encode(dp, stride, 0, k, dt, len, k, p, ns, 1, &em, nullptr)));
      CK(hipDeviceSynchronize());
      const size_t probe_stripe = ns - 1;
      for (int l = 0; l < p; ++l) CK(hipMemcpy(ref.data() + l * shard, at(probe_stripe, k + l), shard, hipMemcpyDeviceToHost));
      struct Var {
        const char* name;
        int U;
        size_t cap;
      };
      // lib: the library's encode without product tables (v16 / glds); ldsx_capN:
      // ec_encode_ldsx<P, 2> with N KiB of dynamic LDS (0: its tables only)
      const Var vars[] = {{"lib", 0, 0},           {"ldsx_cap0", 2, 0},       {"ldsx_cap20", 2, 20 << 10},
                          {"ldsx_cap24", 2, 24 << 10}, {"ldsx_cap32", 2, 32 << 10}, {"ldsx_cap40", 2, 40 << 10}};
      for (const Var& var : vars) {
        auto go = [&]() {
          if (!var.U)
            CK(static_cast<hipError_t>(isal_hip_launch_encode(dp, stride, 0, k, dt, len, k, p, ns, 1, &em, nullptr)));
          else
            ldsx(p, var.U, nitems, dp, stride, dt, dl, len, k, nitems, tiles, var.cap);
        };
        for (int l = 0; l < p; ++l) CK(hipMemset(at(probe_stripe, k + l), 0xA5, shard));
        go();
        CK(hipDeviceSynchronize());
        CK(hipGetLastError());
        for (int l = 0; l < p; ++l) CK(hipMemcpy(got.data() + l * shard, at(probe_stripe, k + l), shard, hipMemcpyDeviceToHost));
        const bool ok = memcmp(ref.data(), got.data(), shard * p) == 0;
        for (int w = 0; w < 2; ++w) go();
        CK(hipEventRecord(e0, 0));
        for (int it = 0; it < iters; ++it) go();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= iters;
        printf("{\"round\": %d, \"layout\": %d, \"k\": %d, \"p\": %d, \"len\": %d, \"stripes\": %d, \"variant\": \"%s\", "
               "\"ms\": %.4f, \"frac\": %.4f, \"bit_exact\": %s}\n",
               round, layout, k, p, len, ns, var.name, ms, bytes / ms / 1e6 / 8000.0, ok ? "true" : "false");
        fflush(stdout);
      }
      CK(hipFree(d));
      if (c) CK(hipFree(c));
      CK(hipFree(dp));
      CK(hipFree(dt));
      CK(hipFree(dl));
    }
  return 0;
}
