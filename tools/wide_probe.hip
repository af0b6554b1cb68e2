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
//   usage: wide_probe [ITERS] [ROUNDS]   one JSON line per (shape, variant)
//
// Build: make -C isa-l_amd wide_probe (includes csrc/ec_kernels.hip).
#include "../isa-l_amd/csrc/ec_kernels.hip"

#include <cstring>
#include <vector>

#include "erasure_code.h"

extern "C" void isal_hip_count_launch(void) {}
extern "C" void isal_hip_kreg_add(const void*, const char*) {}

namespace {

struct L64 {
  uint32_t lo, hi;
};

__device__ __forceinline__ uint32_t sdwa_add_b(uint32_t v, uint32_t base, int b) {
  uint32_t r;
  switch (b) {
    case 0:
      asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:DWORD"
          : "=v"(r) : "v"(v), "v"(base));
      break;
    case 1:
      asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD"
          : "=v"(r) : "v"(v), "v"(base));
      break;
    case 2:
      asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:DWORD"
          : "=v"(r) : "v"(v), "v"(base));
      break;
    default:
      asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:DWORD"
          : "=v"(r) : "v"(v), "v"(base));
      break;
  }
  return r;
}

__device__ __forceinline__ uint64_t lds64(uint32_t addr) {
  return *reinterpret_cast<const __attribute__((address_space(3))) uint64_t*>(static_cast<uintptr_t>(addr));
}

// acc[4d + b] ^= T5_j[field5(byte b of dword d)] ^ T3_j[field3(...)] for one 16-byte source chunk
__device__ __forceinline__ void ldsx_acc(L64 (&acc)[16], const uint4& x, uint32_t b5, uint32_t b3) {
  const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const uint32_t lo8 = (w[d] << 3) & 0xF8F8F8F8u;  // bits 0-4 of each byte, times 8
    const uint32_t hi8 = (w[d] >> 2) & 0x38383838u;  // bits 5-7 of each byte, times 8
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const uint64_t p = lds64(sdwa_add_b(lo8, b5, b));
      const uint64_t q = lds64(sdwa_add_b(hi8, b3, b));
      L64& a = acc[4 * d + b];
      a.lo = xor3(a.lo, static_cast<uint32_t>(p), static_cast<uint32_t>(q));
      a.hi = xor3(a.hi, static_cast<uint32_t>(p >> 32), static_cast<uint32_t>(q >> 32));
    }
  }
}

template <int P, int U>
__global__ __launch_bounds__(kBlock) void enc_ldsx(const uint64_t* __restrict__ ptrs, int ptr_stride, int src0,
                                                   int dst0, const uint64_t* __restrict__ ltg, int len, int k,
                                                   unsigned nitems, unsigned tiles) {
  extern __shared__ uint64_t lt[];  // [k][32] T5, then [k][8] T3
  for (int i = threadIdx.x; i < k * 40; i += kBlock) lt[i] = ltg[i];
  __syncthreads();
  const uint32_t lbase = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) uint64_t*)lt));
  for (unsigned w = blockIdx.x; w < nitems; w += gridDim.x) {
    const unsigned v = xcd_item(w, nitems, 1);
    const unsigned stripe = v / tiles, tile = v - stripe * tiles;
    const uint64_t* __restrict__ sp = ptrs + static_cast<size_t>(stripe) * ptr_stride;
    const long long off = static_cast<long long>(tile) * kTile + threadIdx.x * kVec;
    if (off + kVec > len) continue;  // the probe's shapes have len % 4096 == 0
    L64 acc[16];
#pragma unroll
    for (int p = 0; p < 16; ++p) acc[p] = L64{0u, 0u};
    int j = 0;
    for (; j + U <= k; j += U) {
      uint4 x[U];
#pragma unroll
      for (int u = 0; u < U; ++u) x[u] = load16<kBufNT>(sp[src0 + j + u], off, len);
#pragma unroll
      for (int u = 0; u < U; ++u)
        ldsx_acc(acc, x[u], lbase + (j + u) * 256u, lbase + k * 256u + (j + u) * 64u);
    }
    for (; j < k; ++j) {
      const uint4 x = load16<kBufNT>(sp[src0 + j], off, len);
      ldsx_acc(acc, x, lbase + j * 256u, lbase + k * 256u + j * 64u);
    }
    // transpose: row l, dword d = byte l of acc[4d..4d+3] (rows 0-3 in .lo, 4-7 in .hi)
    uint32_t out[P][4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (h == 1 && P <= 4) continue;
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
      store16<kBufNT>(sp[dst0 + l], off, make_uint4(out[l][0], out[l][1], out[l][2], out[l][3]), len);
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

template <int P, int U>
static void launch_ldsx(unsigned grid, const uint64_t* dp, int stride, const uint64_t* dlt, int len, int k,
                        unsigned nitems, unsigned tiles) {
  hipLaunchKernelGGL((enc_ldsx<P, U>), dim3(grid), dim3(kBlock), static_cast<size_t>(k) * 40 * 8, 0, dp, stride, 0, k,
                     dlt, len, k, nitems, tiles);
}

static void ldsx(int P, int U, unsigned grid, const uint64_t* dp, int stride, const uint64_t* dlt, int len, int k,
                 unsigned nitems, unsigned tiles) {
#define L(p, u) \
  if (P == p && U == u) return launch_ldsx<p, u>(grid, dp, stride, dlt, len, k, nitems, tiles);
#define LU(p) L(p, 1) L(p, 2) L(p, 3) L(p, 4) L(p, 5)
  LU(3) LU(4) LU(5) LU(6) LU(7) LU(8)
#undef LU
#undef L
  fprintf(stderr, "no instantiation P=%d U=%d\n", P, U);
  exit(1);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 10;
  const int rounds = argc > 2 ? atoi(argv[2]) : 2;
  const Shape shapes[] = {{10, 4, 1 << 20, 1024}, {10, 3, 1 << 20, 1024}, {10, 5, 1 << 20, 1024},
                          {10, 6, 1 << 20, 1024}, {10, 7, 1 << 20, 1024}, {10, 8, 1 << 20, 1024},
                          {20, 4, 4 << 20, 64},    {20, 5, 4 << 20, 64},    {20, 6, 4 << 20, 64},
                          {20, 7, 4 << 20, 64},    {20, 8, 4 << 20, 64},    {8, 6, 1 << 20, 1024},
                          {16, 8, 1 << 20, 512},   {12, 4, 1 << 20, 1024}};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int round = 0; round < rounds; ++round)
    for (const Shape& s : shapes) {
      const int k = s.k, p = s.p, len = s.len, ns = s.ns, stride = k + p;
      const size_t shard = static_cast<size_t>(len);
      uint8_t* d = nullptr;
      CK(hipMalloc(&d, shard * stride * ns));
      hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint64_t*>(d), shard * stride * ns / 8,
                         777ull + k * 31 + p);
      std::vector<uint64_t> hp(static_cast<size_t>(stride) * ns);
      for (size_t i = 0; i < hp.size(); ++i) hp[i] = reinterpret_cast<uint64_t>(d + i * shard);
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
      std::vector<uint64_t> hl(static_cast<size_t>(k) * 40, 0);
      for (int j = 0; j < k; ++j)
        for (int l = 0; l < p; ++l) {
          const unsigned char c = a[(k + l) * k + j];
          for (int v = 0; v < 32; ++v)
            hl[j * 32 + v] |= static_cast<uint64_t>(gf_mul(c, static_cast<unsigned char>(v))) << (8 * l);
          for (int v = 0; v < 8; ++v)
            hl[k * 32 + j * 8 + v] |= static_cast<uint64_t>(gf_mul(c, static_cast<unsigned char>(v << 5))) << (8 * l);
        }
      uint64_t* dl = nullptr;
      CK(hipMalloc(&dl, hl.size() * 8));
      CK(hipMemcpy(dl, hl.data(), hl.size() * 8, hipMemcpyHostToDevice));
      const unsigned tiles = len / kTile, nitems = tiles * ns;
      const double bytes = static_cast<double>(stride) * shard * ns;
      // reference parity: the library's encode
      std::vector<uint8_t> ref(shard * p), got(shard * p);
      CK(static_cast<hipError_t>(isal_hip_launch_encode(dp, stride, 0, k, dt, len, k, p, ns, 1, &em, nullptr)));
      CK(hipDeviceSynchronize());
      const size_t probe_stripe = ns - 1;
      for (int l = 0; l < p; ++l)
        CK(hipMemcpy(ref.data() + l * shard, d + (probe_stripe * stride + k + l) * shard, shard, hipMemcpyDeviceToHost));
      struct Var {
        const char* name;
        int U;
        unsigned grid;
      };
      const Var vars[] = {{"lib", 0, 0},         {"ldsx_u1", 1, nitems}, {"ldsx_u2", 2, nitems},
                          {"ldsx_u3", 3, nitems}, {"ldsx_u4", 4, nitems}, {"ldsx_u5", 5, nitems}};
      for (const Var& var : vars) {
        auto go = [&]() {
          if (!var.U)
            CK(static_cast<hipError_t>(isal_hip_launch_encode(dp, stride, 0, k, dt, len, k, p, ns, 1, &em, nullptr)));
          else
            ldsx(p, var.U, var.grid < nitems ? var.grid : nitems, dp, stride, dl, len, k, nitems, tiles);
        };
        CK(hipMemset(d + (probe_stripe * stride + k) * shard, 0xA5, shard * p));
        go();
        CK(hipDeviceSynchronize());
        CK(hipGetLastError());
        for (int l = 0; l < p; ++l)
          CK(hipMemcpy(got.data() + l * shard, d + (probe_stripe * stride + k + l) * shard, shard, hipMemcpyDeviceToHost));
        const bool ok = memcmp(ref.data(), got.data(), shard * p) == 0;
        for (int w = 0; w < 2; ++w) go();
        CK(hipEventRecord(e0, 0));
        for (int it = 0; it < iters; ++it) go();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= iters;
        printf("{\"round\": %d, \"k\": %d, \"p\": %d, \"len\": %d, \"stripes\": %d, \"variant\": \"%s\", \"ms\": %.4f, "
               "\"frac\": %.4f, \"bit_exact\": %s}\n",
               round, k, p, len, ns, var.name, ms, bytes / ms / 1e6 / 8000.0, ok ? "true" : "false");
        fflush(stdout);
      }
      CK(hipFree(d));
      CK(hipFree(dp));
      CK(hipFree(dt));
      CK(hipFree(dl));
    }
  return 0;
}
