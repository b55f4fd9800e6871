// lat_r04.hip — timing study (not the product; tools/tune_lat_r04.py): how long the first dependent load of a kernel
// takes when 1024 waves (one per SIMD, the shard sum's grid at config 4) issue it together, to place the round-3 shard
// sum's 4.9 us "index consumed" stamp.  Each wave stamps s_memrealtime (100 MHz) at entry, issues `nload` 8-byte loads
// per lane from `arrays` arrays (row = lane, like the shard sum's mask rows), waits, stamps again.
//   mode 0: every wave reads the same rows (the shard sum: 64 units of a 32-row band share their mask rows);
//   mode 1: every wave reads rows of its own (distinct lines);
//   mode 2: no load at all (entry + stamp cost only).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {
__global__ __launch_bounds__(256) void k_lat(const uint64_t* src, uint64_t stride, uint32_t arrays, int mode,
                                              uint64_t* tl, uint64_t* sink) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const int lane = threadIdx.x & 63;
  const uint64_t gw = static_cast<uint64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  uint64_t acc = 0;
  if (mode != 2) {
    const uint64_t row = mode == 0 ? static_cast<uint64_t>(lane) % 32 : gw * 64 + lane;
    uint64_t v[16];
#pragma unroll
    for (uint32_t a = 0; a < 16; ++a) v[a] = a < arrays ? src[a * stride + row] : 0ull;
#pragma unroll
    for (uint32_t a = 0; a < 16; ++a) acc |= v[a];
  }
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0) {
    tl[gw * 4 + 0] = t0;
    tl[gw * 4 + 1] = t1;
    tl[gw * 4 + 2] = static_cast<uint64_t>(__builtin_amdgcn_s_getreg((15 << 11) | 20));  // XCC id
  }
  if (acc == 0x123456789ull) sink[0] = acc;  // keep the loads
}
}  // namespace

extern "C" int tune_lat(const uint64_t* src, uint64_t stride, uint32_t arrays, int mode, unsigned grid, uint64_t* tl,
                        uint64_t* sink, hipStream_t st) {
  k_lat<<<grid, 256, 0, st>>>(src, stride, arrays, mode, tl, sink);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
