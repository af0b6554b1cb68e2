// copy_probe.hip — the achievable HBM rate on this GPU, for bench.py's
// roofline.copy_ceiling ("also measure achievable peak with a
// device copy kernel, and report both"). Measurement infrastructure, not part
// of libisal_hip.so: built by `make -C isa-l_amd tools` into
// tools/libcopy_probe.so and loaded by bench.py through ctypes after torch.
//
// The kernel is the encode's memory skeleton with no arithmetic: each lane
// moves 16 bytes per 4 KiB tile with non-temporal buffer loads and stores (the
// encode's access mode), one tile per workgroup, tiles handed out
// XCD-contiguously as the encode does. MI355X_MICROARCH.md quotes 6.29 TB/s for
// a float4 copy.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int kBlock = 256;
constexpr int kTile = kBlock * 16;

__global__ __launch_bounds__(kBlock) void copy_tiles(uint64_t dst, uint64_t src, unsigned ntiles, int chunk) {
  const unsigned per = ntiles / 8;
  const unsigned w = blockIdx.x;
  const unsigned t = (ntiles % 8) ? w : (w % 8) * per + w / 8;
  const long long base = static_cast<long long>(t) * kTile;
  // one buffer descriptor per chunk of at most 1 GiB so the 32-bit offset fits
  const long long cbase = base / chunk * chunk;
  const int off = static_cast<int>(base - cbase) + threadIdx.x * 16;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(src + cbase), 0, chunk, 0x00020000);
  const auto rd = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(dst + cbase), 0, chunk, 0x00020000);
  typedef int v4i __attribute__((ext_vector_type(4)));
  const v4i v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 2 /* nt */);
  __builtin_amdgcn_raw_buffer_store_b128(v, rd, off, 0, 2 /* nt */);
}

// The memory skeleton of one encode shape: K source shards read and P output
// shards written per stripe, 16 bytes per lane per shard, one 4 KiB column tile
// per workgroup, tiles of a stripe consecutive and the (stripe, tile) items
// handed out XCD-contiguously (the encode's EncOrder<2>), nt buffer loads and
// stores — the encode with its GF arithmetic replaced by one XOR fold. P = 0 is
// a read-only pass (the check kernels' shape). Layout as bench.py allocates it:
// data[S][K][len], coding[S][P][len].
// PT: the shard addresses come from a device pointer table (per stripe: K
// sources then P outputs), as the batch encode reads them, instead of being
// computed from the layout.
// T: consecutive 4 KiB tiles per workgroup (items = stripes x tiles / T), one
// after the other with the item's address arithmetic shared.
// B: threads per workgroup (a tile is B x 16 bytes; the encode's 256 by default).
template <int K, int P, bool PT, int T = 1, int B = kBlock>
__global__ __launch_bounds__(B) void skel_tiles(uint64_t data, uint64_t coding, int len, unsigned tiles,
                                                     unsigned nitems, const uint64_t* __restrict__ ptrs) {
  extern __shared__ unsigned lds_pad[];  // the encode's occupancy cap (dynamic LDS), unused
  const unsigned per = nitems / 8;
  const unsigned w = blockIdx.x;
  const unsigned item = (nitems % 8) ? w : (w % 8) * per + w / 8;
  const unsigned s = item / (tiles / T), t = (item % (tiles / T)) * T;
#pragma unroll
  for (int h = 0; h < T; ++h) {
  const int off = static_cast<int>(t + h) * (B * 16) + threadIdx.x * 16;
  typedef int v4i __attribute__((ext_vector_type(4)));
  v4i v[K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const auto r = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(PT ? ptrs[static_cast<size_t>(s) * (K + P) + j]
                                   : data + (static_cast<uint64_t>(s) * K + j) * static_cast<uint64_t>(len)),
        0, len,
        0x00020000);
    v[j] = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 2 /* nt */);
  }
  v4i acc = v[0];
#pragma unroll
  for (int j = 1; j < K; ++j) acc ^= v[j];
  if (P == 0) {
    if (acc.x == 0x7eadbeef && acc.y == 0x1234567 && acc.z == 0x89abcdef && acc.w == 0x0f1e2d3c) lds_pad[0] = 1;
    continue;
  }
#pragma unroll
  for (int l = 0; l < P; ++l) {
    const auto r = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(PT ? ptrs[static_cast<size_t>(s) * (K + P) + K + l]
                                   : coding + (static_cast<uint64_t>(s) * P + l) * static_cast<uint64_t>(len)),
        0, len, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(acc ^ l, r, off, 0, 2 /* nt */);
  }
  }
}

}  // namespace

// Runs the (K, P) skeleton over S stripes of len-byte shards `reps` times after
// two warm-ups with `lds` bytes of dynamic LDS per workgroup; returns the
// rate in GB/s of (K + P) * len * S bytes per pass, or a negative error.
// use_ptrs: bit 0 the pointer table; bits 8-15 T, tiles per workgroup (1, 2
// or 4; the xor_gen / pq_gen / C2 shapes only for T > 1); bits 16+ threads per
// workgroup other than 256 (128, 512 or 1024 for xor_gen and C2; 128 or 512
// for k20p6 / k20p8, the C4 update (7, 6), decode (10, 3) and pq_gen (10, 2);
// T = 1).
// Bytes between consecutive shards beyond len in the pointer table (0: the
// shards abut, every one len-aligned like bench.py's (S, k, len) tensors):
// whether the shards' alignment to each other changes the rate.
static unsigned long long g_shard_pad = 0;
extern "C" void skel_probe_set_pad(unsigned long long pad) { g_shard_pad = pad; }

extern "C" double skel_probe_gbs(void* data, void* coding, int len, int k, int p, unsigned stripes, int reps,
                                 unsigned lds, int use_ptrs) {
  const int tpi = ((use_ptrs >> 8) & 255) ? ((use_ptrs >> 8) & 255) : 1;
  const int blk = (use_ptrs >> 16) ? (use_ptrs >> 16) : kBlock;
  use_ptrs &= 1;
  if (len <= 0 || len % (blk * 16 * tpi) || reps <= 0 || stripes == 0) return -1.0;
  const unsigned tiles = static_cast<unsigned>(len / (blk * 16)), nitems = tiles * stripes / tpi;
  void (*kern)(uint64_t, uint64_t, int, unsigned, unsigned, const uint64_t*) = nullptr;
  switch (k * 100 + p + 100000 * (tpi - 1) + 1000000 * (blk == kBlock ? 0 : blk)) {
    case 128001001: kern = use_ptrs ? skel_tiles<10, 1, true, 1, 128> : skel_tiles<10, 1, false, 1, 128>; break;
    case 512001001: kern = use_ptrs ? skel_tiles<10, 1, true, 1, 512> : skel_tiles<10, 1, false, 1, 512>; break;
    case 1024001001: kern = use_ptrs ? skel_tiles<10, 1, true, 1, 1024> : skel_tiles<10, 1, false, 1, 1024>; break;
    case 128001004: kern = use_ptrs ? skel_tiles<10, 4, true, 1, 128> : skel_tiles<10, 4, false, 1, 128>; break;
    case 512001004: kern = use_ptrs ? skel_tiles<10, 4, true, 1, 512> : skel_tiles<10, 4, false, 1, 512>; break;
    case 1024001004: kern = use_ptrs ? skel_tiles<10, 4, true, 1, 1024> : skel_tiles<10, 4, false, 1, 1024>; break;
    case 128000706: kern = use_ptrs ? skel_tiles<7, 6, true, 1, 128> : skel_tiles<7, 6, false, 1, 128>; break;
    case 128001003: kern = use_ptrs ? skel_tiles<10, 3, true, 1, 128> : skel_tiles<10, 3, false, 1, 128>; break;
    case 128001002: kern = use_ptrs ? skel_tiles<10, 2, true, 1, 128> : skel_tiles<10, 2, false, 1, 128>; break;
    case 128002006: kern = use_ptrs ? skel_tiles<20, 6, true, 1, 128> : skel_tiles<20, 6, false, 1, 128>; break;
    case 512002006: kern = use_ptrs ? skel_tiles<20, 6, true, 1, 512> : skel_tiles<20, 6, false, 1, 512>; break;
    case 128002008: kern = use_ptrs ? skel_tiles<20, 8, true, 1, 128> : skel_tiles<20, 8, false, 1, 128>; break;
    case 512002008: kern = use_ptrs ? skel_tiles<20, 8, true, 1, 512> : skel_tiles<20, 8, false, 1, 512>; break;
    case 101001: kern = use_ptrs ? skel_tiles<10, 1, true, 2> : skel_tiles<10, 1, false, 2>; break;
    case 101002: kern = use_ptrs ? skel_tiles<10, 2, true, 2> : skel_tiles<10, 2, false, 2>; break;
    case 101004: kern = use_ptrs ? skel_tiles<10, 4, true, 2> : skel_tiles<10, 4, false, 2>; break;
    case 301001: kern = use_ptrs ? skel_tiles<10, 1, true, 4> : skel_tiles<10, 1, false, 4>; break;
    case 301002: kern = use_ptrs ? skel_tiles<10, 2, true, 4> : skel_tiles<10, 2, false, 4>; break;
    case 301004: kern = use_ptrs ? skel_tiles<10, 4, true, 4> : skel_tiles<10, 4, false, 4>; break;
    case 101: kern = use_ptrs ? skel_tiles<1, 1, true> : skel_tiles<1, 1, false>; break;
    case 1004: kern = use_ptrs ? skel_tiles<10, 4, true> : skel_tiles<10, 4, false>; break;
    case 1000: kern = use_ptrs ? skel_tiles<10, 0, true> : skel_tiles<10, 0, false>; break;
    case 1200: kern = use_ptrs ? skel_tiles<12, 0, true> : skel_tiles<12, 0, false>; break;
    case 1002: kern = use_ptrs ? skel_tiles<10, 2, true> : skel_tiles<10, 2, false>; break;
    case 1001: kern = use_ptrs ? skel_tiles<10, 1, true> : skel_tiles<10, 1, false>; break;
    case 1006: kern = use_ptrs ? skel_tiles<10, 6, true> : skel_tiles<10, 6, false>; break;
    case 1008: kern = use_ptrs ? skel_tiles<10, 8, true> : skel_tiles<10, 8, false>; break;
    case 2006: kern = use_ptrs ? skel_tiles<20, 6, true> : skel_tiles<20, 6, false>; break;
    case 2008: kern = use_ptrs ? skel_tiles<20, 8, true> : skel_tiles<20, 8, false>; break;
    case 1003: kern = use_ptrs ? skel_tiles<10, 3, true> : skel_tiles<10, 3, false>; break;
    case 706: kern = use_ptrs ? skel_tiles<7, 6, true> : skel_tiles<7, 6, false>; break;  // C4 update: 1 source + 6 parity read, 6 parity written
    default: return -4.0;
  }
  uint64_t* d_ptrs = nullptr;
  if (use_ptrs) {
    const size_t np = static_cast<size_t>(stripes) * (k + p);
    uint64_t* h = static_cast<uint64_t*>(malloc(np * 8));
    if (!h) return -5.0;
    for (unsigned st = 0; st < stripes; ++st) {
      for (int j = 0; j < k; ++j)
        h[st * (k + p) + j] = reinterpret_cast<uint64_t>(data) + (static_cast<uint64_t>(st) * k + j) * (len + g_shard_pad);
      for (int l = 0; l < p; ++l)
        h[st * (k + p) + k + l] =
            reinterpret_cast<uint64_t>(coding) + (static_cast<uint64_t>(st) * p + l) * (len + g_shard_pad);
    }
    const bool ok = hipMalloc(&d_ptrs, np * 8) == hipSuccess && hipMemcpy(d_ptrs, h, np * 8, hipMemcpyHostToDevice) == hipSuccess;
    free(h);
    if (!ok) return -5.0;
  }
  hipStream_t st;
  hipEvent_t e0, e1;
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return -2.0;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int i = 0; i < reps + 2; ++i) {
    if (i == 2) (void)hipEventRecord(e0, st);
    hipLaunchKernelGGL(kern, dim3(nitems), dim3(blk), lds, st, reinterpret_cast<uint64_t>(data),
                       reinterpret_cast<uint64_t>(coding), len, tiles, nitems, d_ptrs);
  }
  (void)hipEventRecord(e1, st);
  const hipError_t err = hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipStreamDestroy(st);
  if (d_ptrs) (void)hipFree(d_ptrs);
  if (err != hipSuccess || ms <= 0.f) return -3.0;
  return static_cast<double>(k + p) * len * stripes * reps / (ms * 1e-3) / 1e9;
}

// Copies n bytes (a multiple of 4 KiB, at most 2^40) from src to dst `reps`
// times after two warm-up copies, on a stream of its own; returns the copy
// rate in GB/s (read + write bytes), or a negative HIP error code.
extern "C" double copy_probe_gbs(void* dst, const void* src, unsigned long long n, int reps) {
  if (n == 0 || n % kTile || reps <= 0) return -1.0;
  const unsigned ntiles = static_cast<unsigned>(n / kTile);
  const int chunk = 1 << 30;
  hipStream_t s;
  hipEvent_t e0, e1;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return -2.0;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < reps + 2; ++i) {
    if (i == 2) hipEventRecord(e0, s);
    hipLaunchKernelGGL(copy_tiles, dim3(ntiles), dim3(kBlock), 0, s, reinterpret_cast<uint64_t>(dst),
                       reinterpret_cast<uint64_t>(src), ntiles, chunk);
  }
  hipEventRecord(e1, s);
  const hipError_t err = hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  hipStreamDestroy(s);
  if (err != hipSuccess || ms <= 0.f) return -3.0;
  return 2.0 * static_cast<double>(n) * reps / (ms * 1e-3) / 1e9;
}

// LDS bookkeeping for the encode's occupancy cap: the device's
// LDS per CU, and how many 256-lane copy_tiles workgroups (a few VGPRs, so
// LDS is the only limit) the runtime fits per CU with `dyn` bytes of dynamic
// LDS each.
extern "C" int copy_probe_lds_per_cu(void) {
  int v = -1, dev = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev);
  return v;
}

extern "C" int copy_probe_blocks_per_cu(unsigned long long dyn) {
  int n = -1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(copy_tiles), kBlock,
                                                   static_cast<size_t>(dyn)) != hipSuccess)
    return -1;
  return n;
}
