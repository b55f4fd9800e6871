// plan_v5_study.hip — timing-study copies (not the product) of round 5's row-chunk plan (csrc/omr_kernels.hip
// plan_chunk): where its 6-8 us at config 4's shapes go.  Variants V:
//   0  the product's form (ticket, look-back with s_sleep between polls)
//   1  the chunk's rows loaded for chunk = blockIdx.x while the ticket is in flight (used when they match)
//   2  no ticket: chunk = blockIdx.x (relies on in-order workgroup dispatch)
//   3  no wait in the look-back (WRONG prefixes: timing only, what the hand-over costs)
//   4  1 + polls without s_sleep
// Built by tools/tune_plan_v5.py into tools/tune/libplan_v5.so (before a GPU call); tests/test_tune_build.py checks that it compiles.
#define OMR_NO_CAPI
#include "../../omnireduce-rdma-demo_amd/csrc/omr_kernels.hip"

namespace {
template <int W, int V>
__device__ __forceinline__ void plan_chunk_study(const PlanArgs& a) {
  constexpr uint32_t NA = W + 1;  // arrays unrolled: W workers, then the write set
  __shared__ uint32_t s_wtot[kPlanWaves][NA];
  __shared__ uint32_t s_base[NA];
  __shared__ uint32_t s_chunk;
  __shared__ uint64_t s_bounds[OMR_MAX_WORKERS + 2];
  const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const uint32_t cnt = a.count;
  const uint64_t all_lanes = a.lanes >= 64 ? ~0ull : ((1ull << a.lanes) - 1ull);
  const uint64_t tag = static_cast<uint64_t>(a.seq) << 32;
  if (t == 0) {
    if constexpr (V == 2) s_chunk = blockIdx.x;
    else s_chunk = static_cast<uint32_t>(__hip_atomic_fetch_add(&a.ws[0], 1ull, __ATOMIC_RELAXED,
                                                                __HIP_MEMORY_SCOPE_AGENT));
  }
  if (t < a.nbounds) s_bounds[t] = a.bounds[t];
  if (t < NA) s_base[t] = 0;
  [[maybe_unused]] uint64_t spec[W];
  if constexpr (V == 1 || V == 4) {  // rows of chunk blockIdx.x loaded while the ticket is in flight
#pragma unroll
    for (int k = 0; k < W; ++k) {
      const uint64_t r = static_cast<uint64_t>(blockIdx.x) * a.tiles * kPlanThreads + t;
      spec[k] = (static_cast<uint32_t>(k) < cnt && r < a.rows) ? a.masks[static_cast<uint64_t>(k) * a.mstride + r] : 0;
    }
  }
  __syncthreads();
  const uint32_t c = s_chunk;
  if (c == 0 && a.zero_cnt != nullptr && t < a.zero_cnt_n) a.zero_cnt[t] = 0;
  const uint64_t row0 = static_cast<uint64_t>(c) * a.tiles * kPlanThreads;
  __amdgpu_buffer_rsrc_t src[W];
#pragma unroll
  for (int k = 0; k < W; ++k)
    src[k] = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint64_t*>(a.masks + static_cast<uint64_t>(static_cast<uint32_t>(k) < cnt ? k : 0) * a.mstride), 0,
        static_cast<uint32_t>(k) < cnt ? static_cast<int>(a.rows * 8) : 0, 0x00020000);
  auto load_row = [&](uint64_t r, uint64_t (&mk)[W]) {
#pragma unroll
    for (int k = 0; k < W; ++k) {
      const v2u v = __builtin_bit_cast(v2u, __builtin_amdgcn_raw_buffer_load_b64(src[k], static_cast<uint32_t>(r) * 8u,
                                                                                 0, 0));
      mk[k] = static_cast<uint64_t>(v.x) | (static_cast<uint64_t>(v.y) << 32);
    }
  };
  auto write_set_of = [&](uint64_t r, const uint64_t (&mk)[W], uint64_t* u) {
    uint64_t x = 0;
#pragma unroll
    for (int k = 0; k < W; ++k) x |= mk[k];
    *u = x;
    return (r < a.rows && r % a.rpp == 0) ? (x | all_lanes) : x;
  };
  // ---- 2. the chunk's totals (its rows kept in registers when it is one tile)
  uint64_t mk[W], un = 0, wsr = 0;
  uint32_t tot[NA];
#pragma unroll
  for (uint32_t k = 0; k < NA; ++k) tot[k] = 0;
  for (uint32_t i = 0; i < a.tiles; ++i) {
    const uint64_t r = row0 + static_cast<uint64_t>(i) * kPlanThreads + t;
    if ((V == 1 || V == 4) && a.tiles == 1 && c == blockIdx.x) {
#pragma unroll
      for (int k = 0; k < W; ++k) mk[k] = spec[k];
    } else {
      load_row(r, mk);
    }
    wsr = write_set_of(r, mk, &un);
#pragma unroll
    for (uint32_t k = 0; k < NA; ++k)
      tot[k] += static_cast<uint32_t>(__builtin_popcountll(k < static_cast<uint32_t>(W) ? mk[k] : wsr));
  }
#pragma unroll
  for (uint32_t k = 0; k < NA; ++k) {
    const uint32_t inc = wave_incl_scan(tot[k]);
    if (lane == 63) s_wtot[wave][k] = inc;
  }
  __syncthreads();
  // ---- 3. publish, then add the lower chunks' totals (tagged with seq: a stale word from an earlier launch is not it)
  if (t < NA) {
    uint32_t sum = 0;
#pragma unroll
    for (uint32_t w = 0; w < kPlanWaves; ++w) sum += s_wtot[w][t];
    __hip_atomic_store(&a.ws[1 + static_cast<uint64_t>(c) * kPlanArrays + t], tag | sum, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  for (uint32_t j = t; j < c * NA; j += kPlanThreads) {
    const uint32_t i = j / NA, k = j - i * NA;
    uint64_t v;
    if constexpr (V == 3) {  // timing only: no wait (wrong prefixes)
      v = __hip_atomic_load(&a.ws[1 + static_cast<uint64_t>(i) * kPlanArrays + k], __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_AGENT);
    } else {
      while (((v = __hip_atomic_load(&a.ws[1 + static_cast<uint64_t>(i) * kPlanArrays + k], __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT)) >> 32) != a.seq)
        if constexpr (V != 4) __builtin_amdgcn_s_sleep(1);
    }
    atomicAdd(&s_base[k], static_cast<uint32_t>(v));
  }
  if (c + 1 == a.nchunks && t == 0)  // every chunk has taken its ticket: re-arm the counter for the next launch
    __hip_atomic_store(&a.ws[0], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  uint32_t carry[NA];  // the array's set bits before the tile
#pragma unroll
  for (uint32_t k = 0; k < NA; ++k) carry[k] = s_base[k];
  // ---- 4. the rows' prefixes and stores, tile by tile
  for (uint32_t i = 0; i < a.tiles; ++i) {
    const uint64_t r = row0 + static_cast<uint64_t>(i) * kPlanThreads + t;
    if (a.tiles > 1) {  // (a one-tile chunk still holds its rows from step 2)
      load_row(r, mk);
      wsr = write_set_of(r, mk, &un);
    }
    uint32_t ex[NA];
    if (i > 0) __syncthreads();  // (s_wtot is refilled)
#pragma unroll
    for (uint32_t k = 0; k < NA; ++k) {
      const uint32_t v = static_cast<uint32_t>(__builtin_popcountll(k < static_cast<uint32_t>(W) ? mk[k] : wsr));
      const uint32_t inc = wave_incl_scan(v);
      ex[k] = inc - v;
      if (lane == 63) s_wtot[wave][k] = inc;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < NA; ++k) {
      uint32_t before = 0, all = 0;
#pragma unroll
      for (uint32_t w = 0; w < kPlanWaves; ++w) {
        const uint32_t x = s_wtot[w][k];
        before += w < wave ? x : 0u;
        all += x;
      }
      ex[k] += carry[k] + before;
      carry[k] += all;
    }
    if (r < a.rows) {
      a.write_set[r] = wsr;
      if (a.union_masks != nullptr) a.union_masks[r] = un;
      if (a.zero_masks != nullptr) a.zero_masks[r] = 0;
#pragma unroll
      for (uint32_t k = 0; k < NA; ++k) {
        if (k < static_cast<uint32_t>(W) && k >= cnt) continue;
        const uint32_t arr = k < static_cast<uint32_t>(W) ? k : cnt;
        a.prefix[static_cast<uint64_t>(arr) * (a.rows + 1) + r] = ex[k];
      }
      for (uint32_t s = 0; s < a.nbounds; ++s)  // (a row at a shard bound: its counts; empty shards repeat a bound)
        if (s_bounds[s] == r)
#pragma unroll
          for (uint32_t k = 0; k < NA; ++k) {
            if (k < static_cast<uint32_t>(W) && k >= cnt) continue;
            const uint32_t arr = k < static_cast<uint32_t>(W) ? k : cnt;
            __hip_atomic_store(&a.counts[arr * a.nbounds + s], tag | ex[k], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
          }
    }
  }
  // the totals: prefix[a][rows], and the counts of every bound at or past the end (the last chunk)
  if (c + 1 == a.nchunks && t < NA && (t == static_cast<uint32_t>(W) || t < cnt)) {
    uint32_t total = 0;
#pragma unroll
    for (uint32_t k = 0; k < NA; ++k) total = k == t ? carry[k] : total;
    const uint32_t arr = t < static_cast<uint32_t>(W) ? t : cnt;
    a.prefix[static_cast<uint64_t>(arr) * (a.rows + 1) + a.rows] = total;
    for (uint32_t s = 0; s < a.nbounds; ++s)
      if (s_bounds[s] >= a.rows)
        __hip_atomic_store(&a.counts[arr * a.nbounds + s], tag | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}


template <int W, int V>
__global__ __launch_bounds__(kPlanThreads) void k_round_plan_study(PlanArgs a) {
  if (blockIdx.x < a.nchunks) {
    plan_chunk_study<W, V>(a);
    return;
  }
  const uint32_t b = blockIdx.x - a.nchunks;
  const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  build_sum_list(a.list, static_cast<uint64_t>(b) * kPlanWaves + w, static_cast<uint64_t>(a.list_wgs) * kPlanWaves);
}

template <int V>
void launch_study(const PlanArgs& a, unsigned grid, hipStream_t st) {
  if (a.count <= 2) k_round_plan_study<2, V><<<grid, kPlanThreads, 0, st>>>(a);
  else if (a.count <= 4) k_round_plan_study<4, V><<<grid, kPlanThreads, 0, st>>>(a);
  else if (a.count <= 8) k_round_plan_study<8, V><<<grid, kPlanThreads, 0, st>>>(a);
  else k_round_plan_study<OMR_MAX_WORKERS, V><<<grid, kPlanThreads, 0, st>>>(a);
}
}  // namespace

// omr_round_plan_list without union_next (the round's call), variant V of the chunks
extern "C" int tune_plan_v5(int variant, const uint64_t* row_masks, uint32_t count, uint64_t mask_stride, uint64_t rows,
                            uint32_t rows_per_part, uint32_t num_lanes, const uint64_t* bounds, uint32_t num_bounds,
                            uint64_t* write_set, uint64_t* union_masks, uint32_t* prefix, uint64_t* counts,
                            uint64_t* zero_masks, uint32_t* zero_counters, uint32_t num_zero_counters,
                            uint64_t* workspace, uint32_t seq, uint32_t block_size, const omr_sum_list* list,
                            omr_stream_t stream) {
  PlanArgs a;
  memset(&a, 0, sizeof(a));
  a.masks = row_masks;
  a.mstride = mask_stride;
  a.zero_cnt = zero_counters;
  a.zero_cnt_n = num_zero_counters;
  a.count = count;
  a.rpp = rows_per_part;
  a.lanes = num_lanes;
  a.nbounds = num_bounds;
  a.rows = rows;
  a.bounds = bounds;
  a.write_set = write_set;
  a.union_masks = union_masks;
  a.prefix = prefix;
  a.counts = counts;
  a.zero_masks = zero_masks;
  a.ws = workspace;
  a.seq = seq;
  const uint64_t tiles_all = (rows + kPlanThreads - 1) / kPlanThreads;
  a.tiles = static_cast<uint32_t>((tiles_all + kPlanChunksMax - 1) / kPlanChunksMax);
  a.nchunks = static_cast<uint32_t>((tiles_all + a.tiles - 1) / a.tiles);
  if (list != nullptr) {
    Layout L;
    if (int rc = make_layout(rows * num_lanes * block_size, block_size, num_lanes,
                             static_cast<uint32_t>(rows / rows_per_part), &L))
      return rc;
    if (int rc = make_list_args(L, row_masks, count, mask_stride, list, &a.list)) return rc;
    const uint64_t wgs = (list_units_host(a.list) + kPlanWaves - 1) / kPlanWaves;
    a.list_wgs = static_cast<uint32_t>(wgs < 512 ? wgs : 512);
  }
  const unsigned grid = a.nchunks + a.list_wgs;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  switch (variant) {
    case 0: launch_study<0>(a, grid, st); break;
    case 1: launch_study<1>(a, grid, st); break;
    case 2: launch_study<2>(a, grid, st); break;
    case 3: launch_study<3>(a, grid, st); break;
    default: launch_study<4>(a, grid, st); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" uint32_t omr_sentinel(uint32_t block_size, uint32_t num_lanes) {  // the product's, compiled out by OMR_NO_CAPI
  if (block_size == 0 || num_lanes == 0) return 0;
  return (UINT32_MAX / block_size / num_lanes - 1u) * num_lanes * block_size;
}
