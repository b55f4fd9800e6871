// stream_probe.hip — timing-only study (not product code): how fast can one 256 MiB read stream go on MI355X,
// register loads (buffer_load_dwordx4 nt, the k_scan1f load) versus LDS-DMA (global_load_lds_dwordx4 nt into a
// per-wave LDS ring, then ds_read), at several occupancies and depths.  Every variant checksums all the words
// it read, so a variant that skips or mis-orders data is caught.  Build: hipcc --offload-arch=gfx950 -O3
// -std=c++17 -o build/stream_probe tools/tune/stream_probe.hip; run: build/stream_probe [MiB] [rounds].
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__global__ void k_fill(uint32_t* x, uint64_t n, uint32_t salt) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull)
    x[i] = static_cast<uint32_t>(i * 2654435761ull) ^ salt;
}

// One plain store per wave (a single atomic target would serialise thousands of waves at ~12 ns each).
__device__ __forceinline__ void publish(unsigned long long* sink, unsigned long long acc, uint32_t gw) {
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off);
  if ((threadIdx.x & 63) == 0) sink[gw] = acc;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, static_cast<int>(bytes), 0x00020000);
}

// Register stream: wave-contiguous groups of D pieces (1 KiB = one dwordx4 per lane), grid-stride over groups.
template <int W, int D>
__global__ __launch_bounds__(64 * W) void r_vgpr(const uint32_t* x, uint32_t pieces, unsigned long long* sink) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t groups = pieces / D;
  unsigned long long acc = 0;  // 64-bit: the total must not depend on which thread read a word
  for (uint32_t g = blockIdx.x * W + wave; g < groups; g += gridDim.x * W) {
    const __amdgpu_buffer_rsrc_t s = rsrc(x + static_cast<uint64_t>(g) * D * 256, D * 1024);
    v4u v[D];
#pragma unroll
    for (int i = 0; i < D; ++i)
      v[i] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(s, i * 1024 + lane * 16, 0, 2));
    __builtin_amdgcn_sched_barrier(0);  // every load issued before the first use (D pieces in flight)
#pragma unroll
    for (int i = 0; i < D; ++i) acc += (unsigned long long)v[i].x + v[i].y + (unsigned long long)v[i].z + v[i].w;
  }
  publish(sink, acc, blockIdx.x * W + wave);
}

// Register stream, persistent: each wave owns one contiguous range of pieces (the k_scan1f shape without columns).
template <int W, int D>
__global__ __launch_bounds__(64 * W) void r_vgpr_pers(const uint32_t* x, uint32_t pieces, unsigned long long* sink) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t tw = gridDim.x * W, gw = blockIdx.x * W + wave;
  const uint32_t per = pieces / tw;  // host guarantees divisibility by D
  unsigned long long acc = 0;  // 64-bit: the total must not depend on which thread read a word
  for (uint32_t p = gw * per; p < (gw + 1) * per; p += D) {
    const __amdgpu_buffer_rsrc_t s = rsrc(x + static_cast<uint64_t>(p) * 256, D * 1024);
    v4u v[D];
#pragma unroll
    for (int i = 0; i < D; ++i)
      v[i] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(s, i * 1024 + lane * 16, 0, 2));
    __builtin_amdgcn_sched_barrier(0);  // every load issued before the first use (D pieces in flight)
#pragma unroll
    for (int i = 0; i < D; ++i) acc += (unsigned long long)v[i].x + v[i].y + (unsigned long long)v[i].z + v[i].w;
  }
  publish(sink, acc, blockIdx.x * W + wave);
}

// LDS-DMA stream: each wave owns a contiguous range of pieces and a ring of D 1-KiB LDS slots; it keeps D pieces
// in flight (global_load_lds_dwordx4 nt), waits for the oldest with vmcnt(D-1), reads it with ds_read_b128,
// drains that read (lgkmcnt(0)) and refills the slot.  All DMA issue and the vmcnt waits are inline asm, so the
// compiler inserts no conservative vmcnt(0) before the LDS reads.
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off nt\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_dst)
      : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int W, int D>
__global__ __launch_bounds__(64 * W) void r_lds(const uint32_t* x, uint32_t pieces, unsigned long long* sink) {
  __shared__ v4u ring[W][D][64];
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t tw = gridDim.x * W, gw = blockIdx.x * W + wave;
  const uint32_t per = pieces / tw;  // multiple of D (host check)
  const uint32_t p0 = gw * per;
  const uint32_t lds0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(&ring[wave][0][0]));
  const char* src = reinterpret_cast<const char*>(x) + static_cast<uint64_t>(p0) * 1024 + lane * 16;
  unsigned long long acc = 0;  // 64-bit: the total must not depend on which thread read a word
#pragma unroll
  for (int i = 0; i < D; ++i) glds16(src + i * 1024, __builtin_amdgcn_readfirstlane(lds0 + i * 1024));
  for (uint32_t p = D; p < per; p += D) {
#pragma unroll
    for (int i = 0; i < D; ++i) {
      wait_vm<D - 1>();
      const v4u v = ring[wave][i][lane];
      acc += (unsigned long long)v.x + v.y + (unsigned long long)v.z + v.w;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      glds16(src + static_cast<uint64_t>(p + i) * 1024, __builtin_amdgcn_readfirstlane(lds0 + i * 1024));
    }
  }
  wait_vm<0>();
#pragma unroll
  for (int i = 0; i < D; ++i) {
    const v4u v = ring[wave][i][lane];
    acc += (unsigned long long)v.x + v.y + (unsigned long long)v.z + v.w;
  }
  publish(sink, acc, blockIdx.x * W + wave);
}

// Config-2 geometry (256 MiB: 8 partitions x 512 rows x 64 lanes of 1 KiB), 512 workgroups of 16 waves, each
// wave reads two batches of 16 KiB.  COL: a workgroup owns one (partition, lane) column (k_scan1f's split): a
// batch is 16 rows of the column, 1 KiB pieces 64 KiB apart.  TILE: a workgroup owns 16 lanes x 32 rows of one
// partition: a batch is one row's 16 consecutive blocks (16 KiB contiguous).  SPLIT: the wave's two batches lie
// in the two halves of the partition (everything in flight at once is one half of each partition) instead of
// being adjacent.  XCD: workgroup -> work permuted so one partition shares an XCD (k_scan1f's mapping).
template <int MODE>  // bit 0: TILE (else COL); bit 1: SPLIT; bit 2: XCD permutation
__global__ __launch_bounds__(1024) void r_geom(const uint32_t* x, uint32_t pieces, unsigned long long* sink) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t T = gridDim.x, bid = blockIdx.x;
  const uint32_t lin = (MODE & 4) ? (bid % 8) * (T / 8) + bid / 8 : bid;
  constexpr uint32_t kRow = 64 * 1024, kRpp = 512;
  unsigned long long acc = 0;
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    uint64_t base;
    uint32_t stride;
    if constexpr (MODE & 1) {  // TILE: lin = (p, g, k), k = 16 segments of 32 rows
      const uint32_t k = lin % 16, g = (lin / 16) % 4, p = lin / 64;
      const uint32_t r = (MODE & 2) ? b * 256 + k * 16 + wave : k * 32 + wave * 2 + (1 - b);
      base = (static_cast<uint64_t>(p) * kRpp + r) * kRow + g * 16384;
      stride = 1024;
    } else {  // COL: lin = (p, l)
      const uint32_t l = lin % 64, p = lin / 64;
      const uint32_t r = (MODE & 2) ? b * 256 + wave * 16 : wave * 32 + (1 - b) * 16;
      base = (static_cast<uint64_t>(p) * kRpp + r) * kRow + l * 1024;
      stride = kRow;
    }
    const __amdgpu_buffer_rsrc_t s = rsrc(reinterpret_cast<const char*>(x) + base, 15 * stride + 1024);
    v4u v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i)
      v[i] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(s, i * stride + lane * 16, 0, 2));
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 16; ++i) acc += (unsigned long long)v[i].x + v[i].y + (unsigned long long)v[i].z + v[i].w;
  }
  publish(sink, acc, blockIdx.x * 16 + wave);
}

using Kfn = void (*)(const uint32_t*, uint32_t, unsigned long long*);
struct Variant {
  const char* name;
  Kfn fn;
  int grid, threads, pers_div;  // pers_div: pieces must divide by grid*W*D (0 = grid-stride)
};

int main(int argc, char** argv) {
  const uint64_t bytes = (argc > 1 ? strtoull(argv[1], nullptr, 10) : 256ull) << 20;
  const int rounds = argc > 2 ? atoi(argv[2]) : 8;
  const int batch = 20, nbuf = 4;
  const uint32_t pieces = static_cast<uint32_t>(bytes / 1024);
  std::vector<uint32_t*> bufs(nbuf);
  for (int b = 0; b < nbuf; ++b) {
    CK(hipMalloc(&bufs[b], bytes));
    k_fill<<<4096, 256>>>(bufs[b], bytes / 4, 0x9e3779b9u * (b + 1));
  }
  unsigned long long* sink;
  constexpr int kMaxWaves = 1 << 15;
  CK(hipMalloc(&sink, 8 * kMaxWaves));
  CK(hipDeviceSynchronize());
#define V(name, k, grid, W, D, pers) Variant{name, k<W, D>, grid, 64 * W, pers ? grid * W * D : 0}
#define G(name, mode) Variant{name, r_geom<mode>, 512, 1024, 0}
  std::vector<Variant> vs = {
      V("vgpr W16 D16 g512 (k_scan1f occupancy)", r_vgpr, 512, 16, 16, 0),
      V("vgpr W8 D16 g1024", r_vgpr, 1024, 8, 16, 0),
      V("vgpr-pers W16 D16 g512", r_vgpr_pers, 512, 16, 16, 1),
      G("col contig (k_scan1f)", 0),
      G("col contig xcd (k_scan1f exact)", 4),
      G("col split", 2),
      G("col split xcd", 6),
      G("tile contig", 1),
      G("tile contig xcd", 5),
      G("tile split", 3),
      G("tile split xcd", 7),
      V("lds W2 D16 g1024", r_lds, 1024, 2, 16, 1),
  };
#undef V
#undef G
  // checksum reference: every variant must read every word exactly once
  unsigned long long ref = 0;
  for (size_t v = 0; v < vs.size(); ++v) {
    if (vs[v].pers_div && pieces % vs[v].pers_div) {
      fprintf(stderr, "%s: %u pieces not divisible by %d\n", vs[v].name, pieces, vs[v].pers_div);
      return 1;
    }
    const int waves = vs[v].grid * vs[v].threads / 64;
    vs[v].fn<<<vs[v].grid, vs[v].threads>>>(bufs[0], pieces, sink);
    CK(hipGetLastError());
    std::vector<unsigned long long> hs(waves);
    CK(hipMemcpy(hs.data(), sink, 8 * waves, hipMemcpyDeviceToHost));
    unsigned long long h = 0;
    for (auto w : hs) h += w;
    if (v == 0) ref = h;
    printf("check %-40s %s\n", vs[v].name, h == ref ? "ok" : "CHECKSUM MISMATCH");
    if (h != ref) return 2;
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<float>> us(vs.size());
  int k = 0;
  for (int r = 0; r < rounds; ++r)
    for (size_t v = 0; v < vs.size(); ++v) {
      CK(hipEventRecord(e0));
      for (int i = 0; i < batch; ++i, ++k) vs[v].fn<<<vs[v].grid, vs[v].threads>>>(bufs[k % nbuf], pieces, sink);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r > 0) us[v].push_back(ms * 1e3f / batch);  // round 0 = warm-up
    }
  for (size_t v = 0; v < vs.size(); ++v) {
    auto t = us[v];
    std::sort(t.begin(), t.end());
    const float med = t[t.size() / 2], best = t[0];
    printf("%-40s median %7.2f us  %6.0f GB/s   best %7.2f us  %6.0f GB/s\n", vs[v].name, med, bytes / med / 1e3,
           best, bytes / best / 1e3);
  }
  return 0;
}
