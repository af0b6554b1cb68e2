// valu_probe.hip — issue rate of the VALU instructions the GF / CRC kernels
// are built from (v_perm_b32, v_bitop3_b32, SDWA shifts, ...) on gfx950, with
// several waves per SIMD, against v_add_u32 as the full-rate reference.
// Question it answers: at 0.67-0.77 VALU wave-instructions per CU-cycle
// (SQ_INSTS_VALU of the fused encode+CRC kernels), is the VALU saturated?
// Also times random-address ds_read_b64 from a 256-entry (2 KiB) and a
// 32-entry (256 B) table, with the kernels' 8-byte entries.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/valu_probe tools/valu_probe.hip
// Output: one JSON line per op: ns per launch, wave-instructions per CU per ns,
// and the rate relative to v_add_u32.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

constexpr int kIters = 2048;
constexpr int kAcc = 8;  // independent chains per lane

enum Op { ADD, PERM, BITOP3, XOR, SDWA_SHL, AND, BFE, LSHR, DS64_256, DS64_32, PERM_S, BITOP3_S,
          LDS_LIN, LDS_R256, LDS_R32, NOPS };
static const char* kName[NOPS] = {"v_add_u32",   "v_perm_b32", "v_bitop3_b32", "v_xor_b32",
                                  "v_lshlrev_b32_sdwa", "v_and_b32", "v_bfe_u32", "v_lshrrev_b32",
                                  "ds_read_b64 (256 x 8 B, random)", "ds_read_b64 (32 x 8 B, random)",
                                  "v_perm_b32 (table in an SGPR, as the GF kernels)",
                                  "v_bitop3_b32 (one SGPR operand)",
                                  "ds_read_b64 throughput, lane-linear (conflict-free)",
                                  "ds_read_b64 throughput, random entry of 256 x 8 B",
                                  "ds_read_b64 throughput, random entry of 32 x 8 B"};

template <int OP>
__global__ __launch_bounds__(256) void probe(uint32_t* out, uint32_t seed) {
  __shared__ uint64_t lt[256];
  lt[threadIdx.x] = 0x9E3779B97F4A7C15ull * (threadIdx.x + 1);
  __syncthreads();
  uint32_t a[kAcc];
#pragma unroll
  for (int i = 0; i < kAcc; ++i) a[i] = seed * (threadIdx.x + 17 * i + 1);
  const uint32_t b = seed ^ threadIdx.x, c = seed + 0x01020304u * threadIdx.x;
  // LDS byte offsets of the throughput modes (fixed per lane: the same bank
  // pattern every iteration): lane-linear, or random entries of a 2 KiB / 256 B table
  uint32_t o[kAcc];
#pragma unroll
  for (int q = 0; q < kAcc; ++q) {
    uint32_t h = (threadIdx.x * 8 + q + 1) * 0x9E3779B1u;
    h ^= h >> 15;
    h *= 0x85EBCA77u;
    h ^= h >> 13;
    o[q] = OP == LDS_LIN ? ((threadIdx.x & 31) * 8 + q * 256) % 2048 : OP == LDS_R256 ? (h & 0x7F8u) : (h & 0xF8u);
  }
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int i = 0; i < kAcc; ++i) {
      if constexpr (OP == ADD)
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
      else if constexpr (OP == PERM)
        asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(b), "v"(c));
      else if constexpr (OP == BITOP3)
        asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[i]) : "v"(b), "v"(c));
      else if constexpr (OP == XOR)
        asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
      else if constexpr (OP == SDWA_SHL)
        asm volatile("v_lshlrev_b32_sdwa %0, %1, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1"
                     : "+v"(a[i]) : "v"(b));
      else if constexpr (OP == AND)
        asm volatile("v_and_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
      else if constexpr (OP == BFE)
        asm volatile("v_bfe_u32 %0, %0, 3, 8" : "+v"(a[i]));
      else if constexpr (OP == LSHR)
        asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(a[i]));
      else if constexpr (OP == PERM_S)
        asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(a[i]) : "s"(seed), "v"(c));
      else if constexpr (OP == BITOP3_S)
        asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[i]) : "s"(seed), "v"(c));
      else if constexpr (OP == LDS_LIN || OP == LDS_R256 || OP == LDS_R32) {
        if (i == 0) {  // 8 independent reads in flight per wave, then one wait
          // volatile: re-read every iteration (the offsets do not change)
          typedef const volatile __attribute__((address_space(3))) char lchar;
          typedef const volatile __attribute__((address_space(3))) uint64_t lu64;
          lchar* lv = (lchar*)(lt);
          uint64_t v[kAcc];
#pragma unroll
          for (int q = 0; q < kAcc; ++q) v[q] = *(lu64*)(lv + o[q]);
#pragma unroll
          for (int q = 0; q < kAcc; ++q) a[q] ^= static_cast<uint32_t>(v[q]);
        }
      } else {
        // dependent chain through LDS: next offset from the loaded entry
        constexpr uint32_t mask = OP == DS64_256 ? 0x7F8u : 0xF8u;
        const uint64_t v = *reinterpret_cast<const uint64_t*>(reinterpret_cast<const char*>(lt) + (a[i] & mask));
        a[i] = static_cast<uint32_t>(v >> 17) ^ static_cast<uint32_t>(v) ^ a[i];
      }
    }
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < kAcc; ++i) r ^= a[i];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int OP>
static double run(uint32_t* d, int blocks, hipEvent_t e0, hipEvent_t e1) {
  hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(256), 0, 0, d, 12345u);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(256), 0, 0, d, 12345u + r);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  return best * 1e6;  // ns
}

int main(int argc, char** argv) {
  int dev = 0;
  hipDeviceProp_t pr;
  CHECK(hipGetDeviceProperties(&pr, dev));
  const int cus = pr.multiProcessorCount;
  const int wps = argc > 1 ? atoi(argv[1]) : 4;  // waves per SIMD
  const int blocks = cus * wps;                   // 4 waves per block = one per SIMD
  uint32_t* d;
  CHECK(hipMalloc(&d, sizeof(uint32_t) * 256 * blocks));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  double ns[NOPS];
  ns[ADD] = run<ADD>(d, blocks, e0, e1);
  ns[PERM] = run<PERM>(d, blocks, e0, e1);
  ns[BITOP3] = run<BITOP3>(d, blocks, e0, e1);
  ns[XOR] = run<XOR>(d, blocks, e0, e1);
  ns[SDWA_SHL] = run<SDWA_SHL>(d, blocks, e0, e1);
  ns[AND] = run<AND>(d, blocks, e0, e1);
  ns[BFE] = run<BFE>(d, blocks, e0, e1);
  ns[LSHR] = run<LSHR>(d, blocks, e0, e1);
  ns[DS64_256] = run<DS64_256>(d, blocks, e0, e1);
  ns[DS64_32] = run<DS64_32>(d, blocks, e0, e1);
  ns[PERM_S] = run<PERM_S>(d, blocks, e0, e1);
  ns[BITOP3_S] = run<BITOP3_S>(d, blocks, e0, e1);
  ns[LDS_LIN] = run<LDS_LIN>(d, blocks, e0, e1);
  ns[LDS_R256] = run<LDS_R256>(d, blocks, e0, e1);
  ns[LDS_R32] = run<LDS_R32>(d, blocks, e0, e1);
  const double winstr = static_cast<double>(blocks) * 4 * kIters * kAcc;  // per op kind
  for (int o = 0; o < NOPS; ++o)
    printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"cus\": %d, \"ns\": %.0f, "
           "\"wave_instr_per_cu_ns\": %.4f, \"rate_vs_v_add\": %.3f}\n",
           kName[o], wps, cus, ns[o], winstr / cus / ns[o], ns[ADD] / ns[o]);
  CHECK(hipFree(d));
  return 0;
}
