// event_cost.hip — what a cross-stream dependency costs the producing stream on MI355X (diagnostic for the
// pipelined round).  Stream A runs a ~45 us HBM-bound kernel back to back; variants add, after each
// launch: nothing; an event record; an event record that stream B waits on before a small kernel; a device flag
// the kernel itself sets that stream B's small kernel spins on; hipStreamWriteValue32 / hipStreamWaitValue32.
// Prints the period of stream A per variant.
// Then the same record / wait with events created hipEventDisableSystemFence, and stream A waiting each iteration on
// an event of stream B that has long completed (the scan's wait for the plan three rounds back).
//   hipcc --offload-arch=gfx950 -O3 -o build/event_cost tools/event_cost.hip && build/event_cost
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

typedef float v4f __attribute__((ext_vector_type(4)));

// streaming read of n4 float4s (grid-stride), result kept live through a never-taken store; the last workgroup to
// finish stores `seq` to *flag (when flag != null) after a device-scope arrival count
__global__ void k_read(const v4f* x, uint64_t n4, float* sink, unsigned* arrive, unsigned* flag, unsigned seq) {
  v4f acc = {0, 0, 0, 0};
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * blockDim.x)
    acc += __builtin_nontemporal_load(x + i);
  if (acc.x == 1234.5f) sink[threadIdx.x] = acc.y;
  if (flag == nullptr) return;
  __syncthreads();
  if (threadIdx.x == 0) {
    __atomic_thread_fence(__ATOMIC_RELEASE);
    const unsigned old = __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (old == gridDim.x - 1) {
      __hip_atomic_store(arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__global__ void k_small(float* y) { y[threadIdx.x] += 1.0f; }

__global__ void k_spin(const unsigned* flag, unsigned seq, float* y) {
  if (threadIdx.x == 0)
    while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < seq) __builtin_amdgcn_s_sleep(2);
  __syncthreads();
  y[threadIdx.x] += 1.0f;
}

int main() {
  const uint64_t bytes = 256ull << 20, n4 = bytes / 16;
  v4f* x;
  float *sink, *y;
  unsigned *arrive, *flag;
  CK(hipMalloc(&x, bytes));
  CK(hipMemset(x, 0, bytes));
  CK(hipMalloc(&sink, 4096));
  CK(hipMalloc(&y, 4096));
  CK(hipMalloc(&arrive, 4));
  CK(hipMalloc(&flag, 4));
  CK(hipMemset(arrive, 0, 4));
  CK(hipMemset(flag, 0, 4));
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  hipEvent_t ev[4], evf[4];
  for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (auto& e : evf) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence));
  const int iters = 200;
  const char* names[] = {"kernel only", "+ event record", "+ record, stream B waits + small kernel",
                         "+ kernel-set flag, stream B spin kernel", "+ hipStreamWriteValue32 / WaitValue32",
                         "+ event record (no system fence)", "+ record, stream B waits + small kernel (no sys fence)",
                         "+ stream A waits a completed event of B", "+ stream A waits a completed event of B (no sys fence)"};
  unsigned seq = 0;
  for (int v = 0; v < 9; ++v) {
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipDeviceSynchronize());
      const auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < iters; ++i) {
        ++seq;
        k_read<<<2048, 256, 0, a>>>(x, n4, sink, arrive, v == 3 ? flag : nullptr, seq);
        if (v == 1 || v == 2) CK(hipEventRecord(ev[i % 4], a));
        if (v == 2) {
          CK(hipStreamWaitEvent(b, ev[i % 4], 0));
          k_small<<<1, 64, 0, b>>>(y);
        }
        if (v == 5 || v == 6) CK(hipEventRecord(evf[i % 4], a));
        if (v == 6) {
          CK(hipStreamWaitEvent(b, evf[i % 4], 0));
          k_small<<<1, 64, 0, b>>>(y);
        }
        if (v == 7 || v == 8) {  // B recorded its event long ago (three iterations back); A waits on it
          hipEvent_t* E = v == 7 ? ev : evf;
          if (i >= 3) CK(hipStreamWaitEvent(a, E[(i - 3) % 4], 0));
          k_small<<<1, 64, 0, b>>>(y);
          CK(hipEventRecord(E[i % 4], b));
        }
        if (v == 3) k_spin<<<1, 64, 0, b>>>(flag, seq, y);
        if (v == 4) {
          CK(hipStreamWriteValue32(a, flag, seq, 0));
          CK(hipStreamWaitValue32(b, flag, seq, hipStreamWaitValueGte, 0xffffffffu));
          k_small<<<1, 64, 0, b>>>(y);
        }
      }
      CK(hipDeviceSynchronize());
      const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      if (rep) printf("%-44s period %7.2f us\n", names[v], us / iters);
    }
  }
  return 0;
}
