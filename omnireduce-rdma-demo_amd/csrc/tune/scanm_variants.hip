// scanm_variants.hip — tuning harness (not the product): the m-worker one-device sum, k_scanm shapes (SUB blocks x
// UW workers of loads in flight; the product launches SUB*VEC = 16, UW = 1) against the previous plain-load
// kernel, timed side by side by tools/tune_scanm.py.
#define OMR_NO_CAPI
#include "../omr_kernels.hip"

namespace {
constexpr int pow2floor(int x) {
  int r = 1;
  while (r * 2 <= x) r *= 2;
  return r;
}

// k_scanm_plain: the product's m-worker kernel before tools/tune_scanm.py (kept here as the baseline).
//
// Same row sweep; per sub-batch the m workers' blocks are read in rank order and accumulated from +0.0f
// (server.cc:148-150, :97-98).  Adding a zero-flagged worker's block (all +-0.0) to an accumulator that
// started at +0.0 never changes it, so summing every worker equals the reference, which only adds the
// workers that sent the block.  Lane w keeps worker w's row mask (no runtime-indexed register arrays).
template <int VEC, bool NT>
__global__ __launch_bounds__(kWGThreads) void k_scanm_plain(ScanArgs a) {
  constexpr int B4 = 64 * VEC;
  constexpr int SUB = pow2floor(8 / VEC);
  const int lane = threadIdx.x & 63;
  v4f* __restrict__ out = reinterpret_cast<v4f*>(a.out);
  const uint64_t nwaves = static_cast<uint64_t>(gridDim.x) * kWavesPerWG;
  for (uint64_t row = static_cast<uint64_t>(blockIdx.x) * kWavesPerWG + (threadIdx.x >> 6); row < a.rows;
       row += nwaves) {
    const bool head = (row % a.rows_per_part) == 0;
    const uint64_t rowbase = row * a.lanes * B4;
    uint64_t lane_wm = 0;  // lane w: worker w's mask
    uint64_t um = 0;       // union mask (wave-uniform)
    for (uint32_t l0 = 0; l0 < a.lanes; l0 += SUB) {
      v4f acc[SUB][VEC];
#pragma unroll
      for (int s = 0; s < SUB; ++s)
#pragma unroll
        for (int q = 0; q < VEC; ++q) acc[s][q] = v4f{0.f, 0.f, 0.f, 0.f};
      uint32_t sub_any = 0;

      for (uint32_t w = 0; w < a.m; ++w) {
        const v4f* src = reinterpret_cast<const v4f*>(a.x.p[w]) + rowbase +
                            static_cast<uint64_t>(l0) * B4 + lane;
        v4f v[SUB][VEC];
#pragma unroll
        for (int s = 0; s < SUB; ++s)
#pragma unroll
          for (int q = 0; q < VEC; ++q) v[s][q] = ld4<NT>(src + s * B4 + q * 64);
        uint32_t wbits = 0;
#pragma unroll
        for (int s = 0; s < SUB; ++s) {
          uint32_t o = 0;
#pragma unroll
          for (int q = 0; q < VEC; ++q) {
            o |= nz_bits(v[s][q]);
            acc[s][q] = add4(acc[s][q], v[s][q]);
          }
          wbits |= static_cast<uint32_t>(wave_ballot(o != 0) != 0) << s;
        }
        if (lane == static_cast<int>(w)) lane_wm |= static_cast<uint64_t>(wbits) << l0;
        sub_any |= wbits;
      }
      um |= static_cast<uint64_t>(sub_any) << l0;
      if (out != nullptr) {
#pragma unroll
        for (int s = 0; s < SUB; ++s) {
          if (((sub_any >> s) & 1u) || head) {
            v4f* dst = out + rowbase + static_cast<uint64_t>(l0 + s) * B4 + lane;
#pragma unroll
            for (int q = 0; q < VEC; ++q) dst[q * 64] = acc[s][q];
          }
        }
      }
    }
    if (lane < static_cast<int>(a.m)) a.masks[static_cast<uint64_t>(lane) * a.rows + row] = lane_wm;
    if (lane == 0) a.masks[static_cast<uint64_t>(a.m) * a.rows + row] = um;
    if (a.flags != nullptr) {
      for (uint32_t w = 0; w < a.m; ++w) {
        const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(lane_wm), w);
        const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(lane_wm >> 32), w);
        const uint64_t wmw = (static_cast<uint64_t>(hi) << 32) | lo;
        if (lane < static_cast<int>(a.lanes))
          a.flags[w * a.nb + row * a.lanes + lane] = static_cast<int32_t>((wmw >> lane) & 1u);
      }
    }
  }
}

template <int VEC, int SUB, int UW>
void go2(const ScanArgs& a, unsigned g, hipStream_t st) {
  k_scanm<VEC, SUB, UW><<<g, kWGThreads, 0, st>>>(a);
}
template <int VEC>
void go1(const ScanArgs& a, unsigned g, hipStream_t st) {
  k_scanm_plain<VEC, true><<<g, kWGThreads, 0, st>>>(a);
}
struct Variant {
  const char* name;
  void (*v1)(const ScanArgs&, unsigned, hipStream_t);
  void (*v4)(const ScanArgs&, unsigned, hipStream_t);
};
const Variant kVariants[] = {
    {"plain loads (previous)", go1<1>, go1<4>},
    {"SUB8 UW1", go2<1, 8, 1>, go2<4, 2, 1>},
    {"SUB8 UW2", go2<1, 8, 2>, go2<4, 2, 2>},
    {"SUB4 UW4", go2<1, 4, 4>, go2<4, 1, 4>},
    {"SUB4 UW2", go2<1, 4, 2>, go2<4, 1, 2>},
    {"SUB16 UW1", go2<1, 16, 1>, go2<4, 4, 1>},
    {"SUB8 UW4", go2<1, 8, 4>, go2<4, 2, 4>},
};
constexpr int kNum = sizeof(kVariants) / sizeof(kVariants[0]);
}  // namespace

extern "C" {
uint32_t omr_sentinel(uint32_t block_size, uint32_t num_lanes) {  // the product's, compiled out by OMR_NO_CAPI
  return (UINT32_MAX / block_size / num_lanes - 1u) * num_lanes * block_size;
}
int tune_scanm_count(void) { return kNum; }
const char* tune_scanm_name(int v) { return (v >= 0 && v < kNum) ? kVariants[v].name : "?"; }
int tune_scanm(int v, const float* const* xs, uint32_t m, float* out, int32_t* flags, uint64_t* masks, uint64_t n,
               uint32_t B, void* stream) {
  Layout L;
  if (v < 0 || v >= kNum || m < 2 || m > OMR_MAX_WORKERS) return -3;
  if (make_layout(n, B, 16384 / B, 8, &L)) return -1;
  ScanArgs a{};
  for (uint32_t w = 0; w < m; ++w) a.x.p[w] = xs[w];
  a.m = m;
  a.lanes = L.lanes;
  a.rows_per_part = L.rows_per_part;
  a.row_begin = 0;
  a.row_end = static_cast<uint32_t>(L.rows);
  a.rows = L.rows;
  a.nb = L.nb;
  a.flags = flags;
  a.masks = masks;
  a.out = out;
  const unsigned g = grid_for(L.rows);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (L.vec == 1) kVariants[v].v1(a, g, st);
  else if (L.vec == 4) kVariants[v].v4(a, g, st);
  else return -2;
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
}
