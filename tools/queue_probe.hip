// queue_probe.hip — which HIP streams of one process share a hardware queue (study tool, round 6).
//
// Two streams share a hardware queue when work on the second cannot start while the first runs a kernel that waits:
// stream a runs k_hold (one wave, spins on a host-mapped release flag, bounded by a wall-clock timeout), stream b runs
// k_mark (stores a host-mapped flag).  If the mark lands while the hold spins, a and b are on different queues.
//   hipcc --offload-arch=gfx950 -O2 -o /tmp/queue_probe tools/queue_probe.hip && /tmp/queue_probe [streams]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                      \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

// flags[0]: the hold has started; flags[1]: release; flags[2]: the mark
__global__ void k_hold(uint32_t* flags, uint64_t max_ticks) {
  if (threadIdx.x != 0) return;
  __hip_atomic_store(&flags[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const uint64_t t0 = wall_clock64();
  while (__hip_atomic_load(&flags[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0u &&
         wall_clock64() - t0 < max_ticks)
    __builtin_amdgcn_s_sleep(8);
}

__global__ void k_mark(uint32_t* flags) {
  if (threadIdx.x == 0) __hip_atomic_store(&flags[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// 1: a and b are on different hardware queues (b ran while a was held), 0: shared
int disjoint(hipStream_t a, hipStream_t b, uint32_t* h, uint32_t* d) {
  h[0] = h[1] = h[2] = 0;
  __atomic_thread_fence(__ATOMIC_SEQ_CST);
  k_hold<<<1, 64, 0, a>>>(d, 100ull * 1000 * 50);  // wall clock 100 MHz: 50 ms at most
  CK(hipGetLastError());
  auto t0 = std::chrono::steady_clock::now();
  while (__atomic_load_n(&h[0], __ATOMIC_ACQUIRE) == 0 && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(5))
    ;
  k_mark<<<1, 64, 0, b>>>(d);
  CK(hipGetLastError());
  t0 = std::chrono::steady_clock::now();
  int r = 0;
  while (std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(10))
    if (__atomic_load_n(&h[2], __ATOMIC_ACQUIRE) != 0) {
      r = 1;
      break;
    }
  __atomic_store_n(&h[1], 1u, __ATOMIC_RELEASE);
  CK(hipStreamSynchronize(a));
  CK(hipStreamSynchronize(b));
  return r;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 7;
  uint32_t *h = nullptr, *d = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void**>(&h), 64, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&d), h, 0));
  std::vector<hipStream_t> s(1, nullptr);  // the null stream first
  for (int i = 1; i < n; ++i) {
    hipStream_t t;
    CK(hipStreamCreateWithFlags(&t, hipStreamNonBlocking));
    s.push_back(t);
  }
  const char* q = getenv("GPU_MAX_HW_QUEUES");
  printf("GPU_MAX_HW_QUEUES=%s; streams: 0 = null, 1.. created in order\n", q ? q : "(unset)");
  printf("disjoint[a][b] (1: b runs while a holds its queue)\n    ");
  for (int b = 0; b < n; ++b) printf("%3d", b);
  printf("\n");
  for (int a = 0; a < n; ++a) {
    printf("%3d ", a);
    for (int b = 0; b < n; ++b) printf("%3s", a == b ? "-" : (disjoint(s[a], s[b], h, d) ? "1" : "0"));
    printf("\n");
  }
  // destroy stream 1 and create a new one: which queue does it take?
  if (n > 3) {
    CK(hipStreamDestroy(s[1]));
    hipStream_t t;
    CK(hipStreamCreateWithFlags(&t, hipStreamNonBlocking));
    printf("after destroying stream 1, a new stream shares with:");
    for (int b = 0; b < n; ++b)
      if (b != 1 && !disjoint(t, s[b], h, d)) printf(" %d", b);
    printf("\n");
    s[1] = t;
  }
  for (int i = 1; i < n; ++i) CK(hipStreamDestroy(s[i]));
  CK(hipHostFree(h));
  return 0;
}
