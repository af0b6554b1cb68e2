// launch_probe.hip — what one synchronous kernel call costs on this runtime
// before any data moves: hipLaunchKernel + completion for kernels whose only
// work is the completion protocol, by kernel-argument size, stream kind, grid
// size and completion method. It bounds what the drop-in ec_encode_data call
// (2 KiB of kernel arguments, 256-1024 workgroups, completion
// through a host mailbox) can reach.
//
//   usage: launch_probe [ITERS]    (one JSON line per configuration)
//
// completion:
//   sync    hipStreamSynchronize after the launch;
//   mail    every workgroup counts itself on ONE device-scope counter; the
//           last writes the call's sequence number into coherent page-locked
//           host memory (system-scope store); the host spins on it;
//   tree    the library's protocol (ec_kernels.hip:karg_done): groups of
//           max(32, n/256) workgroups count on their own counter (64-byte
//           lines apart), the last of each group counts on a top counter, the
//           last group writes the mailbox;
//   slots   groups as in tree, but the last workgroup of each group writes
//           the sequence number into its own host slot and the host waits
//           for every slot (no top counter on the device).
// Every spin is bounded (100 ms, then the stream is synchronised and the miss
// counted).
//
// Build: make -C isa-l_amd tools (not shipped).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>

namespace {

enum { kSync, kMail, kTree, kSlots };
constexpr int kGroups = 256, kStride = 16;  // as ISAL_HIP_KDONE_GROUPS / _STRIDE

template <int N>
struct Arg {
  unsigned w[N / 4];
};

template <int N>
__global__ void __launch_bounds__(256) probe(Arg<N> a, unsigned* cnt, unsigned long long* mail,
                                             unsigned long long seq, int mode, unsigned gmin) {
  // every lane reads one argument dword (the kernel-argument traffic of a real call)
  const unsigned v = a.w[threadIdx.x % (N / 4)];
  __syncthreads();
  if (threadIdx.x != 0 || mode == kSync) return;
  const unsigned n = gridDim.x, b = blockIdx.x;
  const unsigned long long out = seq + (v == 0xdeadbeefu);
  if (mode == kMail) {
    if (__hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == n - 1) {
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(mail, out, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    return;
  }
  const unsigned gsz = max(gmin, (n + kGroups - 1) / kGroups);
  const unsigned g = b / gsz, gn = min(gsz, n - g * gsz), ng = (n + gsz - 1) / gsz;
  unsigned* gc = cnt + g * kStride;
  if (__hip_atomic_fetch_add(gc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != gn - 1) return;
  __hip_atomic_store(gc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (mode == kSlots) {
    __hip_atomic_store(mail + g, out, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  unsigned* top = cnt + kGroups * kStride;
  if (__hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ng - 1) {
    __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(mail, out, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Ctx {
  unsigned* cnt;
  volatile unsigned long long* h_mail;  // kGroups slots
  unsigned long long* d_mail;
  unsigned long long seq;
  long long misses;
};

bool arrived(const Ctx& c, int mode, unsigned nslots, unsigned long long seq) {
  if (mode != kSlots) return c.h_mail[0] == seq;
  for (unsigned g = 0; g < nslots; g++)
    if (c.h_mail[g] != seq) return false;
  return true;
}

template <int N>
double run(Ctx& c, hipStream_t s, unsigned blocks, int mode, int iters, bool query0, unsigned gmin = 32) {
  Arg<N> a{};
  for (int i = 0; i < N / 4; i++) a.w[i] = i;
  const unsigned gsz = std::max(gmin, (blocks + kGroups - 1) / kGroups);  // as the kernel
  const unsigned nslots = (blocks + gsz - 1) / gsz;
  double t0 = 0;
  for (int it = -20; it < iters; it++) {
    if (it == 0) t0 = now_us();
    const unsigned long long seq = ++c.seq;
    if (query0 && hipStreamQuery(nullptr) != hipSuccess) c.misses += 1000000;  // the null stream is idle here
    hipLaunchKernelGGL((probe<N>), dim3(blocks), dim3(256), 0, s, a, c.cnt, c.d_mail, seq, mode, gmin);
    if (mode != kSync) {
      const double start = now_us();
      while (!arrived(c, mode, nslots, seq)) {
        if (now_us() - start > 100000.0) {
          c.misses++;
          break;
        }
      }
      if ((it & 63) == 63) (void)hipStreamSynchronize(s);
    } else {
      (void)hipStreamSynchronize(s);
    }
  }
  const double t = (now_us() - t0) / iters;
  (void)hipStreamSynchronize(s);
  return t;
}

}  // namespace

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 4000;
  static const char* const names[] = {"sync", "mail", "tree", "slots"};
  Ctx c{};
  const size_t cnt_bytes = (kGroups + 1) * kStride * 4;
  if (hipMalloc(&c.cnt, cnt_bytes) != hipSuccess || hipMemset(c.cnt, 0, cnt_bytes) != hipSuccess) return 1;
  void* h = nullptr;
  if (hipHostMalloc(&h, kGroups * 8, hipHostMallocCoherent) != hipSuccess) return 1;
  c.h_mail = static_cast<volatile unsigned long long*>(h);
  for (int g = 0; g < kGroups; g++) c.h_mail[g] = 0;
  if (hipHostGetDevicePointer(reinterpret_cast<void**>(&c.d_mail), h, 0) != hipSuccess) return 1;
  hipStream_t sb, snb;
  if (hipStreamCreate(&sb) != hipSuccess || hipStreamCreateWithFlags(&snb, hipStreamNonBlocking) != hipSuccess)
    return 1;
  // kind 2: the non-blocking stream, with hipStreamQuery(0) before every
  // launch (what ordering after the legacy default stream would cost without
  // a blocking stream)
  for (int kind = 0; kind < 3; kind++)
    for (unsigned blocks : {1u, 256u, 1024u})
      for (int mode = kSync; mode <= kTree; mode++)
        for (int bytes : {64, 2048}) {
          if (mode == kMail && blocks > 256) continue;  // one counter: contention (round 5: 18 us at 1024)
          hipStream_t s = kind ? snb : sb;
          const double us = bytes == 64 ? run<64>(c, s, blocks, mode, iters, kind == 2)
                                        : run<2048>(c, s, blocks, mode, iters, kind == 2);
          printf("{\"stream\": \"%s\", \"blocks\": %u, \"completion\": \"%s\", \"karg_bytes\": %d, \"iters\": %d, "
                 "\"us_per_call\": %.3f, \"mail_misses\": %lld}\n",
                 kind == 2 ? "nonblocking+query0" : kind ? "nonblocking" : "blocking", blocks, names[mode], bytes, iters, us, c.misses);
          fflush(stdout);
        }
  // tree group size sweep (the library uses max(32, n / 256)), blocking stream, 2 KiB
  for (unsigned blocks : {256u, 1024u})
    for (unsigned gmin : {4u, 8u, 16u, 32u, 64u}) {
      const double us = run<2048>(c, sb, blocks, kTree, iters, false, gmin);
      printf("{\"stream\": \"blocking\", \"blocks\": %u, \"completion\": \"tree\", \"group_min\": %u, "
             "\"karg_bytes\": 2048, \"iters\": %d, \"us_per_call\": %.3f, \"mail_misses\": %lld}\n",
             blocks, gmin, iters, us, c.misses);
      fflush(stdout);
    }
  // launch API: hipLaunchKernel (the <<<>>> path the library uses) vs
  // hipModuleLaunchKernel with the argument block passed as one buffer
  // (HIP_LAUNCH_PARAM_BUFFER_POINTER) on a function handle looked up once
  {
    hipFunction_t f = nullptr;
    if (hipGetFuncBySymbol(&f, reinterpret_cast<const void*>(probe<2048>)) == hipSuccess && f) {
      struct {
        Arg<2048> a;
        unsigned* cnt;
        unsigned long long* mail;
        unsigned long long seq;
        int mode;
        unsigned gmin;
      } buf{};
      for (int i = 0; i < 512; i++) buf.a.w[i] = i;
      buf.cnt = c.cnt;
      buf.mail = c.d_mail;
      buf.mode = kTree;
      buf.gmin = 32;
      size_t sz = sizeof(buf);
      for (unsigned blocks : {1u, 256u, 1024u}) {
        double t0 = 0;
        for (int it = -20; it < iters; it++) {
          if (it == 0) t0 = now_us();
          buf.seq = ++c.seq;
          void* extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &buf, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz,
                           HIP_LAUNCH_PARAM_END};
          if (hipModuleLaunchKernel(f, blocks, 1, 1, 256, 1, 1, 0, sb, nullptr, extra) != hipSuccess) {
            c.misses += 1000000;
            break;
          }
          const double start = now_us();
          while (c.h_mail[0] != buf.seq) {
            if (now_us() - start > 100000.0) {
              c.misses++;
              break;
            }
          }
          if ((it & 63) == 63) (void)hipStreamSynchronize(sb);
        }
        const double us = (now_us() - t0) / iters;
        (void)hipStreamSynchronize(sb);
        printf("{\"stream\": \"blocking\", \"blocks\": %u, \"completion\": \"tree\", \"launch\": "
               "\"hipModuleLaunchKernel+buffer\", \"karg_bytes\": 2048, \"iters\": %d, \"us_per_call\": %.3f, "
               "\"mail_misses\": %lld}\n",
               blocks, iters, us, c.misses);
        fflush(stdout);
        printf("{\"stream\": \"blocking\", \"blocks\": %u, \"completion\": \"tree\", \"launch\": "
               "\"hipLaunchKernel\", \"karg_bytes\": 2048, \"iters\": %d, \"us_per_call\": %.3f, "
               "\"mail_misses\": %lld}\n",
               blocks, iters, run<2048>(c, sb, blocks, kTree, iters, false, 32), c.misses);
        fflush(stdout);
      }
    }
  }
  (void)hipStreamDestroy(sb);
  (void)hipStreamDestroy(snb);
  (void)hipHostFree(h);
  (void)hipFree(c.cnt);
  return c.misses ? 1 : 0;
}
