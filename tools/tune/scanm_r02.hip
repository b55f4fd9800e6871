// scanm_r02.hip — tuning harness (not the product): round-2 study of the m-worker one-device sum.
//
// Round 1's k_scanm (k_scanm_row below) gives one wave a whole row (64 KiB per worker at B=256): 4096 work units at 256 MiB, about
// 1.3 per wave slot, so the last third of the launch runs on a third of the machine, and the 8 workers' streams
// sit at identical offsets of their buffers.  k_scanm_g splits a row into units of G blocks (a unit = the blocks of
// G lanes of one row, every worker), sweeps units grid-stride with an XCD-contiguous unit order, optionally
// software-pipelines worker w+1's loads behind worker w's adds (PF), and stores each unit's piece of the row masks
// as a G/8-byte store.  tools/tune_scanm_r02.py times the variants side by side (and with worker buffers staggered
// inside one allocation, the channel-contention test) and checks every variant against the product bit for bit.
#define OMR_NO_CAPI
#include "../../omnireduce-rdma-demo_amd/csrc/omr_kernels.hip"
#include "scan1f_study.h"

namespace {

// k_scanm_row: round 1's product kernel (a wave per row), the study's baseline.
//
// One wave per row, rows swept grid-stride.  Per group of SUB blocks of the row, the m workers' blocks are read in
// rank order (buffer loads, nt; UW workers' SUB*VEC dwordx4 per lane in flight at once) and accumulated from
// +0.0f (server.cc:148-150, :97-98); each block's ballot gives the worker's flag bit.  Adding a zero-flagged
// worker's block (all +-0.0) to an accumulator that started at +0.0 never changes it, so summing every worker
// equals the reference, which only adds the workers that sent the block.  The aggregated blocks go out
// write-through with a static store schedule (a block outside the write set is pointed past the row's
// descriptor and dropped).  Lane w keeps worker w's row mask (no runtime-indexed register arrays).
// tools/tune_scanm.py: SUB*VEC = 16 loads per worker, UW = 1 is fastest (8 x 256 MiB: 391.5 vs 410.8 us for the
// previous plain-load form, tools/tune/scanm_variants.hip).
template <int VEC, int SUB, int UW>
__global__ __launch_bounds__(kWGThreads) void k_scanm_row(ScanArgs a) {
  constexpr uint32_t B4 = 64 * VEC;  // 16-byte vectors per block
  const int lane = threadIdx.x & 63;
  const uint32_t row_bytes = a.lanes * B4 * 16;
  const uint64_t nwaves = static_cast<uint64_t>(gridDim.x) * kWavesPerWG;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (uint64_t row = static_cast<uint64_t>(blockIdx.x) * kWavesPerWG + wave; row < a.rows; row += nwaves) {
    const bool head = (row % a.rows_per_part) == 0;
    const uint64_t rowbase = row * a.lanes * B4 * 4;  // float offset of the row
    const __amdgpu_buffer_rsrc_t dst = chunk_rsrc(a.out + rowbase, a.out != nullptr ? row_bytes : 0u);
    uint64_t lane_wm = 0;  // lane w: worker w's mask
    uint64_t um = 0;       // union mask (wave-uniform)
    for (uint32_t l0 = 0; l0 < a.lanes; l0 += SUB) {
      v4f acc[SUB][VEC];
#pragma unroll
      for (int s = 0; s < SUB; ++s)
#pragma unroll
        for (int q = 0; q < VEC; ++q) acc[s][q] = v4f{0.f, 0.f, 0.f, 0.f};
      uint32_t sub_any = 0;
      for (uint32_t w = 0; w < a.m; w += UW) {
        v4f v[UW][SUB][VEC];
#pragma unroll
        for (int j = 0; j < UW; ++j) {
          // workers past m read through an empty descriptor: zeros, no memory traffic
          const bool live = w + j < a.m;
          const __amdgpu_buffer_rsrc_t src =
              chunk_rsrc(a.x.p[live ? w + j : 0] + rowbase + static_cast<uint64_t>(l0) * B4 * 4, live ? SUB * B4 * 16 : 0u);
#pragma unroll
          for (int s = 0; s < SUB; ++s)
#pragma unroll
            for (int q = 0; q < VEC; ++q)
              v[j][s][q] = __builtin_bit_cast(
                  v4f, __builtin_amdgcn_raw_buffer_load_b128(src, (s * B4 + q * 64 + lane) * 16, 0, kLoadAux));
        }
        __builtin_amdgcn_sched_barrier(0);  // every load of the group in flight before the first use
#pragma unroll
        for (int j = 0; j < UW; ++j) {
          uint32_t wbits = 0;
#pragma unroll
          for (int s = 0; s < SUB; ++s) {
            uint32_t o = 0;
#pragma unroll
            for (int q = 0; q < VEC; ++q) {
              o |= nz_bits(v[j][s][q]);
              acc[s][q] = add4(acc[s][q], v[j][s][q]);  // rank order: worker w+j after w+j-1 (server.cc:97-98)
            }
            wbits |= static_cast<uint32_t>(wave_ballot(o != 0) != 0) << s;
          }
          if (lane == static_cast<int>(w + j)) lane_wm |= static_cast<uint64_t>(wbits) << l0;
          sub_any |= wbits;
        }
      }
      um |= static_cast<uint64_t>(sub_any) << l0;
#pragma unroll
      for (int s = 0; s < SUB; ++s) {
        const uint32_t drop = (((sub_any >> s) & 1u) || head) ? 0u : kDropStore;
#pragma unroll
        for (int q = 0; q < VEC; ++q)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, acc[s][q]), dst,
                                                 (((l0 + s) * B4 + q * 64 + lane) * 16) | drop, 0, kStoreAux);
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

template <int VEC, int SUB, int LAUX = kLoadAux>
__device__ __forceinline__ void load_group(v4f (&v)[SUB][VEC], const float* base, bool live, int lane) {
  constexpr uint32_t B4 = 64 * VEC;
  const __amdgpu_buffer_rsrc_t src = chunk_rsrc(base, live ? SUB * B4 * 16 : 0u);
#pragma unroll
  for (int s = 0; s < SUB; ++s)
#pragma unroll
    for (int q = 0; q < VEC; ++q)
      v[s][q] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(src, (s * B4 + q * 64 + lane) * 16, 0,
                                                                              LAUX));
}

// acc += v in rank order; returns the group's non-zero bits of this worker (bit s = block l0 + s)
template <int VEC, int SUB>
__device__ __forceinline__ uint32_t add_group(v4f (&acc)[SUB][VEC], const v4f (&v)[SUB][VEC]) {
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
  return wbits;
}

// the unit's piece [g0, g0 + gl) of one row mask (gl = 8, 16, 32 or 64 bits; bits of lanes >= NB stay zero)
__device__ __forceinline__ void store_mask_piece(uint64_t* masks, uint64_t row, uint32_t g0, uint32_t gl,
                                                 uint32_t lanes, uint64_t bits) {
  uint8_t* mp = reinterpret_cast<uint8_t*>(masks + row) + g0 / 8;
  if (gl == 64 || lanes == gl) {
    masks[row] = bits;  // the unit is the whole row
  } else if (gl == 32) {
    *reinterpret_cast<uint32_t*>(mp) = static_cast<uint32_t>(bits);
    if (g0 + gl == lanes && lanes < 64) *reinterpret_cast<uint32_t*>(mp + 4) = 0;
  } else if (gl == 16) {
    *reinterpret_cast<uint16_t*>(mp) = static_cast<uint16_t>(bits);
    if (g0 + gl == lanes)
      for (uint32_t b = lanes / 8; b < 8; ++b) reinterpret_cast<uint8_t*>(masks + row)[b] = 0;
  } else {
    *mp = static_cast<uint8_t>(bits);
    if (g0 + gl == lanes)
      for (uint32_t b = lanes / 8; b < 8; ++b) reinterpret_cast<uint8_t*>(masks + row)[b] = 0;
  }
}

// PF: 0 = one worker's loads at a time; 1 = two register sets (worker w+1's loads in flight while worker w is added);
// 2 = as 1 with scheduling barriers between the phases (no hoisting of the set after next); 3 = three sets.
// A worker past m reads through an empty descriptor (zeros, no traffic); adding +0.0 to an accumulator that is never
// -0.0 (it starts at +0.0, and a round-to-nearest sum is -0.0 only if both terms are) leaves it unchanged.
template <int VEC, int SUB, int G, int WAVES, int PF, bool XCD, int SAUX = kStoreAux, int LAUX = kLoadAux>
__global__ __launch_bounds__(64 * WAVES) void k_scanm_g(ScanArgs a) {
  constexpr uint32_t B4 = 64 * VEC;
  static_assert(G % SUB == 0 && G <= 64, "unit = whole sub-groups of one row");
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t gl = a.lanes < static_cast<uint32_t>(G) ? a.lanes : static_cast<uint32_t>(G);
  const uint32_t upr = a.lanes / gl;  // units per row
  const uint64_t units = a.rows * upr;
  const uint32_t T = gridDim.x, bid = blockIdx.x;
  const uint32_t lin = (XCD && T % 8 == 0) ? (bid % 8) * (T / 8) + bid / 8 : bid;
  const uint64_t stride = static_cast<uint64_t>(T) * WAVES;
  for (uint64_t u = static_cast<uint64_t>(lin) * WAVES + wave; u < units; u += stride) {
    const uint64_t row = u / upr;
    const uint32_t g0 = static_cast<uint32_t>(u % upr) * gl;
    const bool head = (row % a.rows_per_part) == 0;
    const uint64_t rowbase = row * a.lanes * B4 * 4;  // float offset of the row
    const __amdgpu_buffer_rsrc_t dst = chunk_rsrc(a.out + rowbase, a.out != nullptr ? a.lanes * B4 * 16 : 0u);
    uint64_t lane_wm = 0;  // lane w: worker w's bits of this unit (bit i = lane g0 + i)
    uint64_t um = 0;
    for (uint32_t l0 = g0; l0 < g0 + gl; l0 += SUB) {
      v4f acc[SUB][VEC];
#pragma unroll
      for (int s = 0; s < SUB; ++s)
#pragma unroll
        for (int q = 0; q < VEC; ++q) acc[s][q] = v4f{0.f, 0.f, 0.f, 0.f};
      uint32_t sub_any = 0;
      const uint64_t goff = rowbase + static_cast<uint64_t>(l0) * B4 * 4;
      auto take = [&](const v4f (&v)[SUB][VEC], uint32_t w) {
        const uint32_t b = add_group<VEC, SUB>(acc, v);
        if (lane == static_cast<int>(w)) lane_wm |= static_cast<uint64_t>(b) << (l0 - g0);
        sub_any |= b;
      };
      auto ld = [&](v4f (&v)[SUB][VEC], uint32_t w) {
        const bool live = w < a.m;
        load_group<VEC, SUB, LAUX>(v, a.x.p[live ? w : 0] + goff, live, lane);
      };
      if constexpr (PF == 1 || PF == 2) {
        v4f va[SUB][VEC], vb[SUB][VEC];
        ld(va, 0);
        for (uint32_t w = 0; w < a.m; w += 2) {
          ld(vb, w + 1);
          if constexpr (PF == 2) __builtin_amdgcn_sched_barrier(0);
          take(va, w);
          if constexpr (PF == 2) __builtin_amdgcn_sched_barrier(0);
          if (w + 2 < a.m) ld(va, w + 2);
          if constexpr (PF == 2) __builtin_amdgcn_sched_barrier(0);
          take(vb, w + 1);
          if constexpr (PF == 2) __builtin_amdgcn_sched_barrier(0);
        }
      } else if constexpr (PF == 3) {
        v4f va[SUB][VEC], vb[SUB][VEC], vc[SUB][VEC];
        ld(va, 0);
        ld(vb, 1);
        for (uint32_t w = 0; w < a.m; w += 3) {
          ld(vc, w + 2);
          __builtin_amdgcn_sched_barrier(0);
          take(va, w);
          __builtin_amdgcn_sched_barrier(0);
          if (w + 3 < a.m) ld(va, w + 3);
          __builtin_amdgcn_sched_barrier(0);
          take(vb, w + 1);
          __builtin_amdgcn_sched_barrier(0);
          if (w + 4 < a.m) ld(vb, w + 4);
          __builtin_amdgcn_sched_barrier(0);
          take(vc, w + 2);
          __builtin_amdgcn_sched_barrier(0);
        }
      } else {
        for (uint32_t w = 0; w < a.m; ++w) {
          v4f v[SUB][VEC];
          ld(v, w);
          __builtin_amdgcn_sched_barrier(0);
          take(v, w);
        }
      }
      um |= static_cast<uint64_t>(sub_any) << (l0 - g0);
#pragma unroll
      for (int s = 0; s < SUB; ++s) {
        const uint32_t drop = (((sub_any >> s) & 1u) || head) ? 0u : kDropStore;
#pragma unroll
        for (int q = 0; q < VEC; ++q)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, acc[s][q]), dst,
                                                 (((l0 + s) * B4 + q * 64 + lane) * 16) | drop, 0, SAUX);
      }
    }
    if (lane < static_cast<int>(a.m))
      store_mask_piece(a.masks + static_cast<uint64_t>(lane) * a.rows, row, g0, gl, a.lanes, lane_wm);
    if (lane == static_cast<int>(a.m)) store_mask_piece(a.masks + static_cast<uint64_t>(a.m) * a.rows, row, g0, gl,
                                                        a.lanes, um);
    if (a.flags != nullptr) {
      for (uint32_t w = 0; w < a.m; ++w) {
        const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(lane_wm), w);
        const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(lane_wm >> 32), w);
        const uint64_t wmw = (static_cast<uint64_t>(hi) << 32) | lo;
        if (static_cast<uint32_t>(lane) < gl)
          a.flags[w * a.nb + row * a.lanes + g0 + lane] = static_cast<int32_t>((wmw >> lane) & 1u);
      }
    }
  }
}

unsigned g_cap = 0;  // grid cap (workgroups); 0 = one unit per wave
unsigned g_occ = 0;  // workgroups per CU forced through dynamic LDS (0 = registers decide)

template <int VEC, int SUB, int G, int WAVES, int PF, bool XCD, int SAUX = kStoreAux, int LAUX = kLoadAux>
void gog(const ScanArgs& a, hipStream_t st) {
  const uint64_t gl = a.lanes < G ? a.lanes : G;
  const uint64_t units = a.rows * (a.lanes / gl);
  uint64_t g = (units + WAVES - 1) / WAVES;
  if (g_cap && g > g_cap) g = g_cap;
  unsigned lds = 0;
  if (g_occ) {
    lds = (160u * 1024u / g_occ - 512u) & ~255u;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_scanm_g<VEC, SUB, G, WAVES, PF, XCD, SAUX, LAUX>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
  }
  k_scanm_g<VEC, SUB, G, WAVES, PF, XCD, SAUX, LAUX><<<static_cast<unsigned>(g), 64 * WAVES, lds, st>>>(a);
}
void go_row(const ScanArgs& a, hipStream_t st) { k_scanm_row<1, 16, 1><<<grid_for(a.rows), kWGThreads, 0, st>>>(a); }
void go_prod(const ScanArgs& a, hipStream_t st) {
  k_scanm<1, 32, kScanmUnitLanes><<<static_cast<unsigned>(a.rows * 2 / kWavesPerWG), kWGThreads, 0, st>>>(a);
}

// ablations (timing only, not checked): the product's loads and masks without the sums' stores, and without the
// sums' and the flags' stores
void go_prod_nosum(const ScanArgs& a0, hipStream_t st) {
  ScanArgs a = a0;
  a.out = nullptr;  // every sum store dropped by the empty descriptor
  go_prod(a, st);
}
void go_prod_read(const ScanArgs& a0, hipStream_t st) {
  ScanArgs a = a0;
  a.out = nullptr;
  a.flags = nullptr;
  go_prod(a, st);
}

struct Variant {
  const char* name;
  void (*fn)(const ScanArgs&, hipStream_t);
};
const Variant kVariants[] = {
    {"product k_scanm (G32 SUB32 nt-st)", go_prod},
    {"G32 SUB32 W4 nt-st ld-nt", gog<1, 32, 32, 4, 0, true, 2, 2>},
    {"G32 SUB32 W4 nt-st ld-plain", gog<1, 32, 32, 4, 0, true, 2, 0>},
    {"G32 SUB32 W4 nt-st ld-sc1", gog<1, 32, 32, 4, 0, true, 2, 16>},
    {"G32 SUB32 W4 plain-st ld-nt", gog<1, 32, 32, 4, 0, true, 0, 2>},
    {"G32 SUB32 W4 nt-st noxcd", gog<1, 32, 32, 4, 0, false, 2, 2>},
    {"G64 SUB32 W4 nt-st", gog<1, 32, 64, 4, 0, true, 2, 2>},
    {"ablation: product without sum stores", go_prod_nosum},
    {"ablation: product, reads + masks only", go_prod_read},
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
               uint32_t B, uint32_t cap, uint32_t occ, void* stream) {
  Layout L;
  if (v < 0 || v >= kNum || m < 2 || m > OMR_MAX_WORKERS) return -3;
  if (B != 256) return -2;  // the study's variants are instantiated for B = 256 (VEC = 1) only
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
  g_cap = cap;
  g_occ = occ;
  kVariants[v].fn(a, reinterpret_cast<hipStream_t>(stream));
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
}
