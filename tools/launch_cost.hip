// launch_cost.hip — host time of the HIP calls a round issues (diagnostic for the round's host side).
// The round spends 5-8.5 us of host time per kernel launch and 3-8 us per event call (OMR_HOST_TRACE); this
// measures the same calls alone: a launch with a small and with a 256-byte argument struct, on one stream and
// round-robin over 3 and 6 streams (GPU_MAX_HW_QUEUES is 4 on the box: streams beyond that share hardware queues),
// fence-free event records, stream waits on such events, and hipEventQuery.  The kernels do nothing, and every
// block of calls is followed by a device sync outside the timed loop, so the host is never throttled by a full
// queue (128 calls per block).
// The same measurement as a library (lc_run) is called by tools/launch_cost_ctx.py inside a process that has torch,
// an RCCL communicator and the round's engine loaded, to see which of them makes the round's calls dearer.
//   hipcc --offload-arch=gfx950 -O3 -o build/launch_cost tools/launch_cost.hip && build/launch_cost
//   hipcc --offload-arch=gfx950 -O3 -fPIC -shared -o build/liblaunch_cost.so tools/launch_cost.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

struct Big {
  const void* p[24];
  unsigned long long n[8];
};

__global__ void k_small(int* sink, int v) {
  if (v == 0x7fffffff) sink[threadIdx.x] = v;
}
__global__ void k_big(Big b) {
  if (b.n[7] == 0x7fffffffull) static_cast<int*>(const_cast<void*>(b.p[0]))[threadIdx.x] = 1;
}

using Clock = std::chrono::steady_clock;
constexpr int kBlock = 128;
constexpr int kReps = 20;

template <typename F>
double per_call_us(F body) {
  std::vector<double> v;
  for (int r = 0; r < kReps; ++r) {
    CK(hipDeviceSynchronize());
    const auto t0 = Clock::now();
    for (int i = 0; i < kBlock; ++i) body(i);
    const auto t1 = Clock::now();
    CK(hipDeviceSynchronize());
    if (r > 1) v.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count() / kBlock);
  }
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

extern "C" int lc_run() {
  CK(hipSetDevice(0));
  int* sink;
  CK(hipMalloc(&sink, 4096));
  hipStream_t s[6];
  for (auto& x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
  hipEvent_t ev[kBlock];
  for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence));
  Big b{};
  b.p[0] = sink;
  struct Row {
    const char* name;
    double us;
  };
  std::vector<Row> rows;
  rows.push_back({"launch, 4+4 B args, 1 stream", per_call_us([&](int) { k_small<<<1, 64, 0, s[0]>>>(sink, 1); })});
  rows.push_back({"launch, 256 B args, 1 stream", per_call_us([&](int) { k_big<<<1, 64, 0, s[0]>>>(b); })});
  rows.push_back({"launch, 4+4 B args, 1024 workgroups", per_call_us([&](int) { k_small<<<1024, 256, 0, s[0]>>>(sink, 1); })});
  rows.push_back({"launch, round-robin 3 streams", per_call_us([&](int i) { k_small<<<1, 64, 0, s[i % 3]>>>(sink, 1); })});
  rows.push_back({"launch, round-robin 6 streams", per_call_us([&](int i) { k_small<<<1, 64, 0, s[i % 6]>>>(sink, 1); })});
  rows.push_back({"launch, null stream", per_call_us([&](int) { k_small<<<1, 64, 0, nullptr>>>(sink, 1); })});
  rows.push_back({"event record (no sys fence)", per_call_us([&](int i) { CK(hipEventRecord(ev[i], s[0])); })});
  rows.push_back({"launch + event record", per_call_us([&](int i) {
                    k_small<<<1, 64, 0, s[0]>>>(sink, 1);
                    CK(hipEventRecord(ev[i], s[0]));
                  })});
  rows.push_back({"launch A + record A + wait B + launch B", per_call_us([&](int i) {
                    k_small<<<1, 64, 0, s[0]>>>(sink, 1);
                    CK(hipEventRecord(ev[i], s[0]));
                    CK(hipStreamWaitEvent(s[1], ev[i], 0));
                    k_small<<<1, 64, 0, s[1]>>>(sink, 1);
                  })});
  rows.push_back({"hipEventQuery (completed)", per_call_us([&](int i) { (void)hipEventQuery(ev[i]); })});
  rows.push_back({"hipStreamWaitEvent (completed event)", per_call_us([&](int i) { CK(hipStreamWaitEvent(s[1], ev[i], 0)); })});
  for (const Row& r : rows) printf("%-44s %7.2f us host per call\n", r.name, r.us);
  fflush(stdout);
  for (auto& e : ev) CK(hipEventDestroy(e));
  for (auto& x : s) CK(hipStreamDestroy(x));
  CK(hipFree(sink));
  return 0;
}

int main() { return lc_run(); }
