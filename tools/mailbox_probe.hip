// mailbox_probe.hip — where the drop-in encode kernel's extra 2.2 µs goes
// (DESIGN §2 "Completion through a host mailbox": 6.7 µs without the mailbox,
// 8.9 µs with it). The library's own kernel-argument encode
// (ec_encode_karg<4, EncPol<10, nt, ST, 2>, kEncXor>, C2 stripe: k = 10, p = 4,
// 1 MiB shards, 256 workgroups) is launched in four forms:
//   ST  = nt        plain non-temporal parity stores (the batch kernels')
//       = sc1nt     write-through stores (the library's drop-in kernel)
//   end = sync      no completion protocol; hipStreamSynchronize
//       = tree      every workgroup waits for its stores and counts itself on
//                   the counter tree, the last writes the host mailbox
//                   (isal_hip_kdone), the host spins on it
// Kernel durations come from rocprofv3 --kernel-trace of one form per process
// (the kernel name carries ST; `end` is the process argument).
//
//   usage: mailbox_probe FORM [ITERS]     FORM in nt-sync nt-tree sc1nt-sync sc1nt-tree
//
// Build: make -C isa-l_amd mailbox_probe (includes csrc/ec_kernels.hip). Not shipped.
#include "../isa-l_amd/csrc/ec_kernels.hip"

#include <chrono>
#include <cstring>
#include <vector>

#include "erasure_code.h"

extern "C" void isal_hip_count_launch(void) {}
extern "C" void isal_hip_kreg_add(const void*, const char*) {}

#define CK(x)                                                                               \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));    \
      exit(1);                                                                              \
    }                                                                                       \
  } while (0)

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <int ST>
static void launch(const isal_hip_karg& a, const isal_hip_kdone& d, int len, int k, unsigned tiles,
                   unsigned long long r0m, unsigned c0m, hipStream_t s) {
  hipLaunchKernelGGL((ec_encode_karg<4, EncPol<10, kBufNT, ST, 2>, kEncXor>), dim3(tiles), dim3(kBlock), 0, s, a, d,
                     len, k, tiles, r0m, c0m);
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: mailbox_probe nt-sync|nt-tree|sc1nt-sync|sc1nt-tree [ITERS]\n");
    return 2;
  }
  const bool sc1 = strncmp(argv[1], "sc1nt", 5) == 0, tree = strstr(argv[1], "tree") != nullptr;
  const int iters = argc > 2 ? atoi(argv[2]) : 2000;
  const int k = 10, p = 4, len = 1 << 20;
  std::vector<unsigned char> a((k + p) * k), g(32 * k * p);
  gf_gen_rs_matrix(a.data(), k + p, k);
  ec_init_tables(k, p, a.data() + k * k, g.data());
  isal_hip_karg ka{};
  isal_hip_build_tables(k, p, g.data(), ka.tbl);
  isal_hip_encmask em;
  isal_hip_enc_masks(k, p, g.data(), &em);
  unsigned char* d = nullptr;
  CK(hipMalloc(&d, static_cast<size_t>(k + p) * len));
  std::vector<unsigned char> h(static_cast<size_t>(k) * len);
  for (size_t i = 0; i < h.size(); ++i) h[i] = static_cast<unsigned char>(i * 2654435761u >> 13);
  CK(hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice));
  for (int i = 0; i < k + p; ++i) ka.ptrs[i] = reinterpret_cast<uint64_t>(d + static_cast<size_t>(i) * len);
  unsigned* cnt = nullptr;
  const size_t cnt_bytes = static_cast<size_t>(ISAL_HIP_KDONE_WORDS) * 4;
  CK(hipMalloc(&cnt, cnt_bytes + 64));
  CK(hipMemset(cnt, 0, cnt_bytes));
  void* hm = nullptr;
  CK(hipHostMalloc(&hm, 64, hipHostMallocCoherent));
  memset(hm, 0, 64);
  volatile unsigned long long* mail = static_cast<volatile unsigned long long*>(hm);
  unsigned long long* dmail = nullptr;
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dmail), hm, 0));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  const unsigned tiles = len / kTile;
  const unsigned long long r0m = (em.ok & 1u) ? em.r0[0] : 0ull;
  const unsigned c0m = (em.ok & 1u) ? em.c0[0] : 0u;
  isal_hip_kdone kd = {nullptr, nullptr, nullptr, 0ull};
  if (tree) {
    kd.cnt = cnt;
    kd.mail = dmail;
  }
  long long misses = 0;
  double t0 = 0;
  for (int it = -50; it < iters; ++it) {
    if (it == 0) t0 = now_us();
    kd.seq = static_cast<unsigned long long>(it + 100);
    if (sc1)
      launch<kBufSC1NT>(ka, kd, len, k, tiles, r0m, c0m, s);
    else
      launch<kBufNT>(ka, kd, len, k, tiles, r0m, c0m, s);
    if (tree) {
      const double st = now_us();
      while (mail[0] != kd.seq)
        if (now_us() - st > 100000.0) {
          ++misses;
          break;
        }
      if ((it & 63) == 63) CK(hipStreamSynchronize(s));
    } else {
      CK(hipStreamSynchronize(s));
    }
  }
  const double us = (now_us() - t0) / iters;
  CK(hipStreamSynchronize(s));
  // parity row 0 of a Vandermonde matrix is the XOR of the sources: check it
  std::vector<unsigned char> par(len);
  CK(hipMemcpy(par.data(), d + static_cast<size_t>(k) * len, len, hipMemcpyDeviceToHost));
  bool ok = true;
  for (int i = 0; i < len && ok; i += 4099) {
    unsigned char x = 0;
    for (int j = 0; j < k; ++j) x ^= h[static_cast<size_t>(j) * len + i];
    ok = x == par[i];
  }
  printf("{\"form\": \"%s\", \"iters\": %d, \"us_per_call\": %.3f, \"mail_misses\": %lld, \"row0_ok\": %s}\n", argv[1],
         iters, us, misses, ok ? "true" : "false");
  return ok && !misses ? 0 : 1;
}
