// scan_variants.hip — tuning harness (not the product): k_scan1 shape variants + HBM calibration kernels,
// timed side by side in one process by tools/tune_scan.py (interleaved rounds, guide §5.4 rule 24).
#include <hip/hip_runtime.h>

#include <cstdint>

typedef float v4f __attribute__((ext_vector_type(4)));
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t nz_bits(const v4f& v) {
  const v4u u = __builtin_bit_cast(v4u, v);
  return (u.x | u.y | u.z | u.w) & 0x7fffffffu;
}
template <bool NT>
__device__ __forceinline__ v4f ld4(const v4f* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT>
__device__ __forceinline__ void st4(v4f* p, v4f v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

struct TArgs {
  const float* x;
  float* out;
  int32_t* flags;
  uint64_t* masks;
  uint64_t rows;
  uint32_t lanes;
  uint32_t rows_per_part;
};

// MAP 0: one wave per row (grid-stride rows).  MAP 1: one wave per LOADS-KiB chunk (grid-stride chunks);
// 16-bit pieces of the row mask stored directly (VEC == 1, LOADS == 16 only).
template <int VEC, bool NT, int LOADS, int WPG, bool NTS, int MAP>
__global__ __launch_bounds__(64 * WPG) void t_scan1(TArgs a) {
  constexpr int B4 = 64 * VEC;
  constexpr int SUB = LOADS / VEC;
  const int lane = threadIdx.x & 63;
  const v4f* __restrict__ x = reinterpret_cast<const v4f*>(a.x);
  v4f* __restrict__ out = reinterpret_cast<v4f*>(a.out);
  const uint64_t nwaves = static_cast<uint64_t>(gridDim.x) * WPG;
  const uint64_t gw = static_cast<uint64_t>(blockIdx.x) * WPG + (threadIdx.x >> 6);
  if constexpr (MAP == 0) {
    for (uint64_t row = gw; row < a.rows; row += nwaves) {
      const bool head = (row % a.rows_per_part) == 0;
      const uint64_t rowbase = row * a.lanes * B4;
      uint64_t wm = 0;
      for (uint32_t l0 = 0; l0 < a.lanes; l0 += SUB) {
        v4f v[SUB][VEC];
        const v4f* src = x + rowbase + static_cast<uint64_t>(l0) * B4 + lane;
#pragma unroll
        for (int s = 0; s < SUB; ++s)
#pragma unroll
          for (int q = 0; q < VEC; ++q) v[s][q] = ld4<NT>(src + s * B4 + q * 64);
#pragma unroll
        for (int s = 0; s < SUB; ++s) {
          uint32_t o = 0;
#pragma unroll
          for (int q = 0; q < VEC; ++q) o |= nz_bits(v[s][q]);
          const bool nz = __ballot(o != 0) != 0;
          wm |= static_cast<uint64_t>(nz) << (l0 + s);
          if (nz || head) {
            v4f* dst = out + rowbase + static_cast<uint64_t>(l0 + s) * B4 + lane;
#pragma unroll
            for (int q = 0; q < VEC; ++q) st4<NTS>(dst + q * 64, v4f{0.f, 0.f, 0.f, 0.f} + v[s][q]);
          }
        }
      }
      if (lane == 0) a.masks[row] = wm;
      if (lane < static_cast<int>(a.lanes)) a.flags[row * a.lanes + lane] = static_cast<int32_t>((wm >> lane) & 1u);
    }
  } else {
    static_assert(VEC == 1 && LOADS == 16, "MAP 1 needs 16-block chunks");
    const uint64_t chunks = a.rows * (a.lanes / 16);
    for (uint64_t c = gw; c < chunks; c += nwaves) {
      const uint64_t row = c / (a.lanes / 16);
      const uint32_t l0 = static_cast<uint32_t>(c % (a.lanes / 16)) * 16;
      const bool head = (row % a.rows_per_part) == 0;
      const uint64_t base = c * 16 * B4;
      v4f v[16];
#pragma unroll
      for (int s = 0; s < 16; ++s) v[s] = ld4<NT>(x + base + s * B4 + lane);
      uint32_t bits = 0;
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const bool nz = __ballot(nz_bits(v[s]) != 0) != 0;
        bits |= static_cast<uint32_t>(nz) << s;
        if (nz || head) st4<NTS>(out + base + s * B4 + lane, v4f{0.f, 0.f, 0.f, 0.f} + v[s]);
      }
      if (lane == 0) reinterpret_cast<uint16_t*>(a.masks)[row * 4 + l0 / 16] = static_cast<uint16_t>(bits);
      if (lane < 16) a.flags[row * a.lanes + l0 + lane] = static_cast<int32_t>((bits >> lane) & 1u);
    }
  }
}


// chunk mapping, VEC=1: wave handles CH-block chunks (CH = 16 or 32), grid-stride; PIPE issues the next
// chunk's loads before processing the current one; STORE=false drops the block stores (cost probe).
template <int CH, int WPG, bool PIPE, bool STORE>
__global__ __launch_bounds__(64 * WPG) void t_chunk(TArgs a) {
  constexpr int B4 = 64;
  const int lane = threadIdx.x & 63;
  const v4f* __restrict__ x = reinterpret_cast<const v4f*>(a.x);
  v4f* __restrict__ out = reinterpret_cast<v4f*>(a.out);
  const uint64_t nwaves = static_cast<uint64_t>(gridDim.x) * WPG;
  const uint64_t gw = static_cast<uint64_t>(blockIdx.x) * WPG + (threadIdx.x >> 6);
  const uint32_t cpr = a.lanes / CH;  // chunks per row
  const uint64_t chunks = a.rows * cpr;
  v4f v[CH];
  uint64_t c = gw;
  if (c < chunks) {
#pragma unroll
    for (int s = 0; s < CH; ++s) v[s] = ld4<true>(x + c * CH * B4 + s * B4 + lane);
  }
  for (; c < chunks; c += nwaves) {
    v4f cur[CH];
#pragma unroll
    for (int s = 0; s < CH; ++s) cur[s] = v[s];
    const uint64_t cn = c + nwaves;
    if (!PIPE) {
      // nothing issued ahead
    } else if (cn < chunks) {
#pragma unroll
      for (int s = 0; s < CH; ++s) v[s] = ld4<true>(x + cn * CH * B4 + s * B4 + lane);
    }
    const uint64_t row = c / cpr;
    const uint32_t l0 = static_cast<uint32_t>(c % cpr) * CH;
    const bool head = (row % a.rows_per_part) == 0;
    const uint64_t base = c * CH * B4;
    uint32_t bits = 0;
#pragma unroll
    for (int s = 0; s < CH; ++s) {
      const bool nz = __ballot(nz_bits(cur[s]) != 0) != 0;
      bits |= static_cast<uint32_t>(nz) << s;
      if (STORE && (nz || head)) out[base + s * B4 + lane] = v4f{0.f, 0.f, 0.f, 0.f} + cur[s];
    }
    if (lane == 0) {
      if (CH == 16) reinterpret_cast<uint16_t*>(a.masks)[row * 4 + l0 / 16] = static_cast<uint16_t>(bits);
      else reinterpret_cast<uint32_t*>(a.masks)[row * 2 + l0 / 32] = bits;
    }
    if (lane < CH) a.flags[row * a.lanes + l0 + lane] = static_cast<int32_t>((bits >> lane) & 1u);
    if (!PIPE && cn < chunks) {
#pragma unroll
      for (int s = 0; s < CH; ++s) v[s] = ld4<true>(x + cn * CH * B4 + s * B4 + lane);
    }
  }
}


// chunk mapping with the block stores issued as buffer stores carrying a cache policy: SC1 = write-through
// (aux 16: the line leaves the XCD's L2, so nothing is left dirty for the kernel-boundary write-back),
// NT = aux 2.
template <int WPG, int AUX, int LAUX = -1>
__global__ __launch_bounds__(64 * WPG) void t_chunk_pol(TArgs a) {
  constexpr int CH = 16, B4 = 64;
  const int lane = threadIdx.x & 63;
  const v4f* __restrict__ x = reinterpret_cast<const v4f*>(a.x);
  const uint64_t nwaves = static_cast<uint64_t>(gridDim.x) * WPG;
  const uint64_t gw = static_cast<uint64_t>(blockIdx.x) * WPG + (threadIdx.x >> 6);
  const uint32_t cpr = a.lanes / CH;
  const uint64_t chunks = a.rows * cpr;
  for (uint64_t c = gw; c < chunks; c += nwaves) {
    const uint64_t row = c / cpr;
    const uint32_t l0 = static_cast<uint32_t>(c % cpr) * CH;
    const bool head = (row % a.rows_per_part) == 0;
    const uint64_t base = c * CH * B4;
    v4f v[CH];
    if constexpr (LAUX < 0) {
#pragma unroll
      for (int s = 0; s < CH; ++s) v[s] = ld4<true>(x + base + s * B4 + lane);
    } else {
      __amdgpu_buffer_rsrc_t ls = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.x) + base * 4, 0,
                                                                    CH * B4 * 16, 0x00020000);
#pragma unroll
      for (int s = 0; s < CH; ++s)
        v[s] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(ls, (s * B4 + lane) * 16, 0, LAUX));
    }
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(a.out + base * 4, 0, CH * B4 * 16, 0x00020000);
    uint32_t bits = 0;
#pragma unroll
    for (int s = 0; s < CH; ++s) {
      const bool nz = __ballot(nz_bits(v[s]) != 0) != 0;
      bits |= static_cast<uint32_t>(nz) << s;
      if (nz || head) {
        const v4f r = v4f{0.f, 0.f, 0.f, 0.f} + v[s];
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, r), rs, (s * B4 + lane) * 16, 0, AUX);
      }
    }
    if (lane == 0) reinterpret_cast<uint16_t*>(a.masks)[row * 4 + l0 / 16] = static_cast<uint16_t>(bits);
    if (lane < CH) a.flags[row * a.lanes + l0 + lane] = static_cast<int32_t>((bits >> lane) & 1u);
  }
}


// column mapping probe: a wave owns CH consecutive rows of ONE lane of one partition (CH blocks at a 64 KiB
// stride instead of CH consecutive blocks).  Flags only (no row masks): a bandwidth probe for a column-major
// work split in which next offsets would be wave-local.
template <int CH, int WPG, int SAUX>
__global__ __launch_bounds__(64 * WPG) void t_col(TArgs a) {
  constexpr int B4 = 64;
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * WPG;
  const uint32_t segs = a.rows / CH;              // column segments per lane (all partitions)
  const uint32_t units = segs * a.lanes;
  for (uint32_t u = blockIdx.x * WPG + wave; u < units; u += nwaves) {
    const uint32_t l = u % a.lanes, seg = u / a.lanes;
    const uint32_t r0 = seg * CH;
    v4f v[CH];
#pragma unroll
    for (int s = 0; s < CH; ++s) {
      const uint64_t blk = static_cast<uint64_t>(r0 + s) * a.lanes + l;
      v[s] = ld4<true>(reinterpret_cast<const v4f*>(a.x) + blk * B4 + lane);
    }
    uint32_t bits = 0;
#pragma unroll
    for (int s = 0; s < CH; ++s) {
      const uint64_t blk = static_cast<uint64_t>(r0 + s) * a.lanes + l;
      const bool nz = __ballot(nz_bits(v[s]) != 0) != 0;
      bits |= static_cast<uint32_t>(nz) << s;
      const bool head = ((r0 + s) % a.rows_per_part) == 0;
      if (nz || head) {
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(a.out + blk * 256, 0, 1024, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v4f{0.f, 0.f, 0.f, 0.f} + v[s]), rs,
                                               lane * 16, 0, SAUX);
      }
    }
    if (lane < CH) a.flags[static_cast<uint64_t>(r0 + lane) * a.lanes + l] = static_cast<int32_t>((bits >> lane) & 1u);
  }
}

// pure streaming read (OR-reduce, one store per wave) and float4 copy: the HBM ceilings on this box
template <bool NT, int LOADS>
__global__ __launch_bounds__(256) void t_read(const float* x, uint64_t n4, uint32_t* sink) {
  const v4f* p = reinterpret_cast<const v4f*>(x);
  const uint64_t nwaves = static_cast<uint64_t>(gridDim.x) * 4;
  const uint64_t gw = static_cast<uint64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  uint32_t acc = 0;
  for (uint64_t base = gw * LOADS * 64; base < n4; base += nwaves * LOADS * 64) {
    v4f v[LOADS];
#pragma unroll
    for (int s = 0; s < LOADS; ++s) v[s] = ld4<NT>(p + base + s * 64 + lane);
#pragma unroll
    for (int s = 0; s < LOADS; ++s) acc |= nz_bits(v[s]);
  }
  if (__ballot(acc != 0) == 0xdeadbeefull) sink[gw] = acc;
}

template <bool NT>
__global__ __launch_bounds__(256) void t_copy(const float* x, float* y, uint64_t n4) {
  const v4f* p = reinterpret_cast<const v4f*>(x);
  v4f* q = reinterpret_cast<v4f*>(y);
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * 256;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x; i < n4; i += stride)
    q[i] = ld4<NT>(p + i);
}

template <int VEC, bool NT, int LOADS, int WPG, bool NTS, int MAP>
static void launch(const TArgs& a, unsigned grid, hipStream_t st) {
  t_scan1<VEC, NT, LOADS, WPG, NTS, MAP><<<grid, 64 * WPG, 0, st>>>(a);
}

extern "C" {

// variant ids -> (NT, LOADS, WPG, NTS, MAP); grid = min(cap, work/WPG)
int tune_num_variants() { return 31; }

const char* tune_variant_name(int v) {
  static const char* names[] = {
      "row nt L16 w4",      "row plain L16 w4", "row nt L32 w4",    "row nt L8 w4",     "row nt L16 w8",
      "row nt L16 w4 ntst", "chunk nt L16 w4",  "chunk plain L16 w4", "row nt L16 w2", "chunk nt L16 w8",
      "c16 w8",            "c16 w16",          "c32 w8",           "c16 w8 pipe",      "c16 w4 pipe",
      "c32 w4",            "c16 w8 nostore",   "c16 w4 nostore",   "c16 w8 sc1st",     "c16 w8 ntst",
      "c16 w8 sc0sc1st",   "st19 sc01nt",     "st18 sc1nt",       "st1 sc0",          "st3 sc0nt",
      "st17 ld2buf",       "st17 ld0buf",     "st17 ld3buf",      "col16 w8",         "col16 w16",
      "col32 w8"};
  return (v >= 0 && v < 31) ? names[v] : "?";
}

int tune_scan(int v, const float* x, float* out, int32_t* flags, uint64_t* masks, uint64_t rows, uint32_t lanes,
              uint32_t rows_per_part, unsigned grid_cap, void* stream) {
  TArgs a{x, out, flags, masks, rows, lanes, rows_per_part};
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  auto grid = [&](uint64_t waves, int wpg) {
    uint64_t g = (waves + wpg - 1) / wpg;
    if (g > grid_cap) g = grid_cap;
    return static_cast<unsigned>(g ? g : 1);
  };
  const uint64_t chunks = rows * (lanes / 16);
  switch (v) {
    case 0: launch<1, true, 16, 4, false, 0>(a, grid(rows, 4), st); break;
    case 1: launch<1, false, 16, 4, false, 0>(a, grid(rows, 4), st); break;
    case 2: launch<1, true, 32, 4, false, 0>(a, grid(rows, 4), st); break;
    case 3: launch<1, true, 8, 4, false, 0>(a, grid(rows, 4), st); break;
    case 4: launch<1, true, 16, 8, false, 0>(a, grid(rows, 8), st); break;
    case 5: launch<1, true, 16, 4, true, 0>(a, grid(rows, 4), st); break;
    case 6: launch<1, true, 16, 4, false, 1>(a, grid(chunks, 4), st); break;
    case 7: launch<1, false, 16, 4, false, 1>(a, grid(chunks, 4), st); break;
    case 8: launch<1, true, 16, 2, false, 0>(a, grid(rows, 2), st); break;
    case 9: launch<1, true, 16, 8, false, 1>(a, grid(chunks, 8), st); break;
    case 10: t_chunk<16, 8, false, true><<<grid(chunks, 8), 512, 0, st>>>(a); break;
    case 11: t_chunk<16, 16, false, true><<<grid(chunks, 16), 1024, 0, st>>>(a); break;
    case 12: t_chunk<32, 8, false, true><<<grid(chunks / 2, 8), 512, 0, st>>>(a); break;
    case 13: t_chunk<16, 8, true, true><<<grid(chunks, 8), 512, 0, st>>>(a); break;
    case 14: t_chunk<16, 4, true, true><<<grid(chunks, 4), 256, 0, st>>>(a); break;
    case 15: t_chunk<32, 4, false, true><<<grid(chunks / 2, 4), 256, 0, st>>>(a); break;
    case 16: t_chunk<16, 8, false, false><<<grid(chunks, 8), 512, 0, st>>>(a); break;
    case 17: t_chunk<16, 4, false, false><<<grid(chunks, 4), 256, 0, st>>>(a); break;
    case 18: t_chunk_pol<8, 16><<<grid(chunks, 8), 512, 0, st>>>(a); break;
    case 19: t_chunk_pol<8, 2><<<grid(chunks, 8), 512, 0, st>>>(a); break;
    case 20: t_chunk_pol<8, 17><<<grid(chunks, 8), 512, 0, st>>>(a); break;
    case 21: t_chunk_pol<8, 19><<<grid(chunks, 8), 512, 0, st>>>(a); break;
    case 22: t_chunk_pol<8, 18><<<grid(chunks, 8), 512, 0, st>>>(a); break;
    case 23: t_chunk_pol<8, 1><<<grid(chunks, 8), 512, 0, st>>>(a); break;
    case 24: t_chunk_pol<8, 3><<<grid(chunks, 8), 512, 0, st>>>(a); break;
    case 25: t_chunk_pol<8, 17, 2><<<grid(chunks, 8), 512, 0, st>>>(a); break;
    case 26: t_chunk_pol<8, 17, 0><<<grid(chunks, 8), 512, 0, st>>>(a); break;
    case 27: t_chunk_pol<8, 17, 3><<<grid(chunks, 8), 512, 0, st>>>(a); break;
    case 28: t_col<16, 8, 17><<<grid(chunks, 8), 512, 0, st>>>(a); break;
    case 29: t_col<16, 16, 17><<<grid(chunks, 16), 1024, 0, st>>>(a); break;
    case 30: t_col<32, 8, 17><<<grid(chunks / 2, 8), 512, 0, st>>>(a); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

int tune_read(int nt, int loads, const float* x, uint64_t n, uint32_t* sink, unsigned grid, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const uint64_t n4 = n / 4;
  if (nt && loads == 16) t_read<true, 16><<<grid, 256, 0, st>>>(x, n4, sink);
  else if (nt && loads == 32) t_read<true, 32><<<grid, 256, 0, st>>>(x, n4, sink);
  else if (!nt && loads == 16) t_read<false, 16><<<grid, 256, 0, st>>>(x, n4, sink);
  else t_read<false, 32><<<grid, 256, 0, st>>>(x, n4, sink);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

int tune_copy(int nt, const float* x, float* y, uint64_t n, unsigned grid, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (nt) t_copy<true><<<grid, 256, 0, st>>>(x, y, n / 4);
  else t_copy<false><<<grid, 256, 0, st>>>(x, y, n / 4);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
}
