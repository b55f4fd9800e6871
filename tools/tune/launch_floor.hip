// launch_floor.hip — the device-side floor under the round's small launches (round 6, VERDICT r05 item 4: "plan
// <= 6 us").  The plan launch (k_round_plan at config 4's shapes: 16 row chunks + 512 pair-list workgroups + the round
// check, 256 threads each) moves under 1.3 MB and measures 7-8 us.  This times launches of the same grid that do
// (almost) nothing, so the plan's own share can be told from the launch's:
//   empty1      1 workgroup, no work
//   empty577    577 workgroups of 256 threads, no work
//   touch577    577 x 256, each thread loads one 8-byte word and stores it elsewhere (1.2 MB moved)
//   pinned1     1 workgroup, one system-scope 8-byte store into pinned host memory (the plan's counts)
//   chain64     64 workgroups: a ticket atomic, one load, one agent-scope publish, a wait for the previous ticket's
//               publish (the plan chunks' look-back, one link), one store
//   spin           1024 x 256 workgroups that each spin 20 us on the wall clock (a stand-in for the worker scan: a full
//                  chip for a fixed time), back to back
//   spin+rec       the same with an event recorded after each launch (the round's `scanned` record, which the side
//                  stream waits on: DisableTiming | DisableSystemFence)
//   spin+rec+wait  and a second stream waiting on each record and running a one-wave kernel (the all-gather's start)
// Every case: 200 launches back to back on one stream, timed with events (mean per launch), three interleaved passes;
// run under `rocprofv3 --kernel-trace --stats` for the kernels' own durations.
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/launch_floor tools/tune/launch_floor.hip && tools/bin/launch_floor
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

__global__ __launch_bounds__(256) void k_empty(uint64_t* sink) {
  if (sink != nullptr && threadIdx.x == 0 && blockIdx.x == 0xFFFFFFFFu) sink[0] = 1;  // never taken
}

__global__ __launch_bounds__(256) void k_spin(uint64_t ticks) {
  const uint64_t t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

__global__ __launch_bounds__(256) void k_touch(const uint64_t* src, uint64_t* dst) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  dst[i] = src[i] + 1;
}

__global__ __launch_bounds__(64) void k_pinned(uint64_t* host_word, uint32_t seq) {
  if (threadIdx.x == 0)
    __hip_atomic_store(host_word, (static_cast<uint64_t>(seq) << 32) | 7u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ws[0] ticket (re-armed by the last), ws[1 + c] publish of chunk c tagged with seq
__global__ __launch_bounds__(256) void k_chain(uint64_t* ws, const uint64_t* src, uint64_t* dst, uint32_t seq) {
  __shared__ uint32_t s_c;
  if (threadIdx.x == 0)
    s_c = static_cast<uint32_t>(__hip_atomic_fetch_add(&ws[0], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  __syncthreads();
  const uint32_t c = s_c;
  const uint64_t i = static_cast<uint64_t>(c) * blockDim.x + threadIdx.x;
  const uint64_t v = src[i];
  const uint64_t tag = static_cast<uint64_t>(seq) << 32;
  if (threadIdx.x == 0) {
    __hip_atomic_store(&ws[1 + c], tag | c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (c > 0)
      while ((__hip_atomic_load(&ws[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 32) != seq)
        __builtin_amdgcn_s_sleep(1);
    if (c + 1 == gridDim.x) __hip_atomic_store(&ws[0], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  dst[i] = v + c;
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 200;
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  uint64_t *src, *dst, *ws, *host;
  const size_t words = 577 * 256;
  CK(hipMalloc(&src, words * 8));
  CK(hipMalloc(&dst, words * 8));
  CK(hipMalloc(&ws, 4096));
  CK(hipMemset(src, 0, words * 8));
  CK(hipMemset(ws, 0, 4096));
  CK(hipHostMalloc(&host, 4096, hipHostMallocMapped));
  uint64_t* host_d;
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&host_d), host, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  uint32_t seq = 0;
  const char* names[] = {"empty1", "empty577", "touch577", "pinned1", "chain64", "spin", "spin+rec", "spin+rec+wait"};
  constexpr int kCases = 8;
  double sum[kCases] = {};
  hipStream_t side;
  CK(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
  hipEvent_t rec;
  CK(hipEventCreateWithFlags(&rec, hipEventDisableTiming | hipEventDisableSystemFence));
  const uint64_t spin_ticks = 2000;  // 20 us at the wall clock's 100 MHz
  for (int pass = 0; pass < 3; ++pass) {
    for (int k = 0; k < kCases; ++k) {
      auto launch = [&]() {
        switch (k) {
          case 0: k_empty<<<1, 64, 0, st>>>(nullptr); break;
          case 1: k_empty<<<577, 256, 0, st>>>(nullptr); break;
          case 2: k_touch<<<577, 256, 0, st>>>(src, dst); break;
          case 3: k_pinned<<<1, 64, 0, st>>>(host_d, ++seq); break;
          case 4: k_chain<<<64, 256, 0, st>>>(ws, src, dst, ++seq == 0 ? ++seq : seq); break;
          default:
            k_spin<<<1024, 256, 0, st>>>(spin_ticks);
            if (k >= 6) CK(hipEventRecord(rec, st));
            if (k == 7) {
              CK(hipStreamWaitEvent(side, rec, 0));
              k_empty<<<1, 64, 0, side>>>(nullptr);
            }
            break;
        }
      };
      for (int i = 0; i < 10; ++i) launch();
      CK(hipStreamSynchronize(st));
      CK(hipEventRecord(e0, st));
      for (int i = 0; i < reps; ++i) launch();
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      CK(hipGetLastError());
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = 1000.0 * ms / reps;
      sum[k] += us;
      printf("pass %d %-13s %7.2f us per launch (events over %d back to back)\n", pass, names[k], us, reps);
    }
  }
  for (int k = 0; k < kCases; ++k) printf("mean %-13s %7.2f us\n", names[k], sum[k] / 3);
  CK(hipStreamSynchronize(side));
  CK(hipStreamSynchronize(st));
  return 0;
}
