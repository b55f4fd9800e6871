// plan_r04.hip — timing-study copies (not the product): the round's bookkeeping and shard-sum forms that lost.
// Moved out of csrc/omr_kernels.hip in round 5 (the product library keeps its default forms only):
//   k_round_plan_r04   round 3/4's plan launch: one 1024-thread workgroup per mask array (the write-set workgroup re-reads
//                      every worker's masks), arrival counter + completion notice; + aggregator chain + pair list
//   k_round_plan2_r04  round 4's row-chunk form (256-thread workgroups, decoupled look-back): slower (13.4 vs 11.95 us)
//   k_shard_sum_r04    the shard sum with its column-stream branch (round 3's default, omr_shard_sum_cols_f32): slower
//                      than the pair-list sum (11.8 vs 9.3 us at config 4's 8-worker shard)
// Built by tools/tune/build.sh into tools/tune/libplan_r04.so for tools/tune_round_r03.py and tools/tune_plan_r05.py;
// tests/test_tune_build.py checks that it still compiles against the product source.
#define OMR_NO_CAPI
#include "../../omnireduce-rdma-demo_amd/csrc/omr_kernels.hip"

namespace {
constexpr int kPlanThreadsR04 = 1024;
constexpr uint64_t kPlanLdsRowsR04 = 8192;  // 64 KiB of dynamic LDS
constexpr uint64_t kRowStreams = ~0ull;  // SumArgsR04.pos_off of row streams

__device__ __forceinline__ uint64_t plan_row(const uint64_t* masks, uint32_t a, uint32_t count, uint64_t mstride,
                                             uint64_t r, uint32_t rpp, uint64_t all_lanes, uint64_t* uni) {
  if (a < count) return masks[static_cast<uint64_t>(a) * mstride + r];
  uint64_t u = 0;
  for (uint32_t c = 0; c < count; ++c) u |= masks[static_cast<uint64_t>(c) * mstride + r];
  *uni = u;
  return (r % rpp == 0) ? (u | all_lanes) : u;
}

struct PlanArgsR04 {
  const uint64_t* masks;  // worker c's row masks at masks + c * mstride
  uint32_t count, rpp, lanes, nbounds;
  uint64_t rows, mstride;
  uint32_t* zero_cnt;     // [zero_cnt_n] cleared by the write-set workgroup (the next round's pack counters), or null
  uint32_t zero_cnt_n;
  const uint64_t* bounds;
  uint64_t* write_set;
  uint64_t* union_masks;
  uint32_t* prefix;
  uint32_t* counts;     // device or host-mapped memory: stored at system scope
  uint64_t* zero_masks;
  uint32_t* arrive;     // device arrival counter (zero between launches) or null
  uint32_t* done_flag;  // receives `seq` once every workgroup's counts are visible system-wide, or null
  uint32_t seq;
  NextArgs chain;       // union_next: the aggregator chain over the union, by workgroups count+1.. (chain.next null: none)
  uint32_t chain_wgs;
  uint32_t list_wgs;    // the shard sum's pair list, by the workgroups after the chain's (0: none)
  ListArgs list;
};

__global__ __launch_bounds__(kPlanThreadsR04) void k_round_plan_r04(PlanArgsR04 a) {
  if (blockIdx.x > a.count + a.chain_wgs) {  // the shard sum's pair list, one unit per wave
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    constexpr uint32_t kW = kPlanThreadsR04 / 64;
    build_sum_list(a.list, static_cast<uint64_t>(blockIdx.x - a.count - 1 - a.chain_wgs) * kW + w,
                   static_cast<uint64_t>(a.list_wgs) * kW);
    return;
  }
  if (blockIdx.x > a.count) {  // the aggregator chain (server.cc:86-96 min_next) over the union, one segment each
    const uint64_t* m = a.masks;
    const uint32_t cnt = a.count;
    const uint64_t ms = a.mstride;
    next_segment<kPlanThreadsR04 / 64>(a.chain, blockIdx.x - a.count - 1, [&](uint64_t r) {
      uint64_t u = 0;
      for (uint32_t c = 0; c < cnt; ++c) u |= m[static_cast<uint64_t>(c) * ms + r];
      return u;
    }, a.chain.next);
    return;
  }
  extern __shared__ uint64_t s_val[];  // [rows] when rows <= kPlanLdsRowsR04
  __shared__ uint32_t s_wave[kPlanThreadsR04 / 64];
  __shared__ uint64_t s_bounds[OMR_MAX_WORKERS + 2];
  const uint32_t arr = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const uint64_t all_lanes = a.lanes >= 64 ? ~0ull : ((1ull << a.lanes) - 1ull);
  const bool ws = arr == a.count;
  const bool keep = a.rows <= kPlanLdsRowsR04;
  if (t < a.nbounds) s_bounds[t] = a.bounds[t];
  if (ws && a.zero_cnt != nullptr && t < a.zero_cnt_n) a.zero_cnt[t] = 0;
  // pass 1: coalesced row reads, 4 rows per thread per step
  for (uint64_t r0 = t; r0 < a.rows; r0 += 4 * kPlanThreadsR04) {
    uint64_t v[4], u[4] = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint64_t r = r0 + static_cast<uint64_t>(i) * kPlanThreadsR04;
      v[i] = r < a.rows ? plan_row(a.masks, arr, a.count, a.mstride, r, a.rpp, all_lanes, &u[i]) : 0;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint64_t r = r0 + static_cast<uint64_t>(i) * kPlanThreadsR04;
      if (r >= a.rows) break;
      if (keep) s_val[r] = v[i];
      if (ws) {
        a.write_set[r] = v[i];
        a.union_masks[r] = u[i];
        if (a.zero_masks != nullptr) a.zero_masks[r] = 0;
      }
    }
  }
  __syncthreads();  // LDS rows (and, when re-read, this workgroup's write-set stores) visible to every thread
  const uint64_t per = (a.rows + kPlanThreadsR04 - 1) / kPlanThreadsR04;
  const uint64_t rb = t * per < a.rows ? t * per : a.rows;
  const uint64_t re = rb + per < a.rows ? rb + per : a.rows;
  auto row = [&](uint64_t r) -> uint64_t {
    if (keep) return s_val[r];
    if (ws) return a.write_set[r];
    return a.masks[static_cast<uint64_t>(arr) * a.mstride + r];
  };
  uint32_t sum = 0;
  for (uint64_t r = rb; r < re; ++r) sum += static_cast<uint32_t>(__builtin_popcountll(row(r)));
  // block-wide exclusive scan of the per-thread sums (wave shuffles, then the 16 wave totals)
  uint32_t inc = sum;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(inc, d, 64);
    if (lane >= static_cast<uint32_t>(d)) inc += o;
  }
  if (lane == 63) s_wave[wave] = inc;
  __syncthreads();
  uint32_t wbase = 0, total = 0;
  for (uint32_t w = 0; w < kPlanThreadsR04 / 64; ++w) {
    if (w < wave) wbase += s_wave[w];
    total += s_wave[w];
  }
  uint32_t run = wbase + inc - sum;  // exclusive prefix at row rb
  uint32_t* pre = a.prefix + static_cast<uint64_t>(arr) * (a.rows + 1);
  for (uint64_t r = rb; r < re; ++r) {
    for (uint32_t s = 0; s < a.nbounds; ++s)
      if (s_bounds[s] == r)
        __hip_atomic_store(&a.counts[arr * a.nbounds + s], run, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    pre[r] = run;
    run += static_cast<uint32_t>(__builtin_popcountll(row(r)));
  }
  if (t == 0) {
    pre[a.rows] = total;
    for (uint32_t s = 0; s < a.nbounds; ++s)
      if (s_bounds[s] >= a.rows)
        __hip_atomic_store(&a.counts[arr * a.nbounds + s], total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (a.arrive == nullptr) return;
  // completion notice for a host that polls instead of waiting on an event.  The counts went out as system-scope
  // (write-through) stores; once every thread has seen them acknowledged (vmcnt(0)) and passed the barrier, the
  // workgroup arrives, and the last arrival stores the round's sequence number and re-arms the counter.  No L2
  // write-back is needed: nothing the host reads sits in an L2.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    const uint32_t old = __hip_atomic_fetch_add(a.arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == a.count) {
      __hip_atomic_store(a.arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.done_flag, a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// ---------------------------------------------------------------- the round plan in row chunks (round 4)
// k_round_plan above gives each mask array ONE 1024-thread workgroup: 16 waves that cannot share a CU with a running
// scan workgroup (VGPRs), so the plan waits for the scan's workgroups to drain, and its write-set workgroup alone reads
// every worker's every row.  Here 256-thread workgroups (one wave per SIMD) each take a chunk of 256 rows of EVERY
// array: one round trip loads the chunk's rows of the count workers' masks; the union, the write set, every array's
// popcounts and their exclusive scans over the chunk come from registers; the chunk's per-array totals are published
// (a flag per chunk) and each workgroup sums its predecessors' totals, which they all publish at about the same time
// (no chain of look-backs).  A workgroup's chunk is a ticket taken when it starts, so every lower chunk belongs to a
// workgroup that is already running (the look-back never waits on one that is not resident).  A total is published as
// total + 1, so its word doubles as its flag.  Workspace (uint32): [0] the arrival counter, [1] the ticket counter,
// [2, 2 + kPlanChunksMaxR04) reserved, then the totals [chunk][array]; the launch's last arrival zeroes them again.
constexpr uint32_t kPlan2ThreadsR04 = kWGThreads;
constexpr uint32_t kPlanChunksMaxR04 = 64;  // rows <= 64 * 256 (larger plans keep k_round_plan)
constexpr uint32_t kPlanArraysR04 = OMR_MAX_WORKERS + 1;
constexpr uint64_t kPlan2WorkspaceWordsR04 = 2 + kPlanChunksMaxR04 + static_cast<uint64_t>(kPlanChunksMaxR04) * kPlanArraysR04;

// W >= count: the per-array loops are unrolled over W workers + the write set (the launch picks 2, 4, 8 or 16)
template <bool LIST, int W>
__global__ __launch_bounds__(kPlan2ThreadsR04) void k_round_plan2_r04(PlanArgsR04 a, uint32_t nchunks, uint32_t* ws) {
  const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
  constexpr uint32_t kW = kPlan2ThreadsR04 / 64;
  if constexpr (LIST) {
    if (blockIdx.x >= nchunks + a.chain_wgs) {  // the shard sum's pair list, one unit per wave
      const uint32_t w = __builtin_amdgcn_readfirstlane(wave);
      build_sum_list(a.list, static_cast<uint64_t>(blockIdx.x - nchunks - a.chain_wgs) * kW + w,
                     static_cast<uint64_t>(a.list_wgs) * kW);
      return;
    }
  }
  if (blockIdx.x >= nchunks) {  // the aggregator chain (server.cc:86-96 min_next) over the union, one segment each
    const uint64_t* m = a.masks;
    const uint32_t cnt = a.count;
    const uint64_t ms = a.mstride;
    next_segment<kW>(a.chain, blockIdx.x - nchunks, [&](uint64_t r) {
      uint64_t u = 0;
      for (uint32_t c = 0; c < cnt; ++c) u |= m[static_cast<uint64_t>(c) * ms + r];
      return u;
    }, a.chain.next);
    return;
  }
  constexpr uint32_t NW = W + 1;  // arrays unrolled: W workers, then the write set
  __shared__ uint32_t s_wtot[kW][NW];
  __shared__ uint32_t s_base[NW];
  __shared__ uint32_t s_ticket;
  __shared__ uint64_t s_bounds[OMR_MAX_WORKERS + 2];
  if (t == 0) s_ticket = __hip_atomic_fetch_add(&ws[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (t < a.nbounds) s_bounds[t] = a.bounds[t];
  __syncthreads();
  const uint32_t c = s_ticket;
  const uint32_t NA = a.count + 1;  // the workers' arrays, then the write set
  const uint64_t all_lanes = a.lanes >= 64 ? ~0ull : ((1ull << a.lanes) - 1ull);
  uint32_t* const totals = ws + 2 + kPlanChunksMaxR04;  // (words [2, 2 + kPlanChunksMaxR04): reserved)
  if (c == 0 && a.zero_cnt != nullptr && t < a.zero_cnt_n) a.zero_cnt[t] = 0;
  // ---- one round trip: row r = c * 256 + t of every worker's masks; union, write set, every array's popcount
  const uint64_t r = static_cast<uint64_t>(c) * kPlan2ThreadsR04 + t;
  const bool in = r < a.rows;
  uint64_t mk[W];
#pragma unroll
  for (uint32_t w = 0; w < W; ++w)
    mk[w] = (w < a.count && in) ? a.masks[static_cast<uint64_t>(w) * a.mstride + r] : 0ull;
  uint64_t u = 0;
#pragma unroll
  for (uint32_t w = 0; w < W; ++w) u |= mk[w];
  const uint64_t wsr = in ? ((r % a.rpp == 0) ? (u | all_lanes) : u) : 0ull;  // union + lane heads (client.cc:201-205)
  // ---- per array: the chunk's exclusive prefix at this row (wave scan, then the earlier waves' totals), the total
  uint32_t pfx[NW];
#pragma unroll
  for (uint32_t arr = 0; arr < NW; ++arr) {  // (the row's popcounts first: the masks are dead after this)
    const uint64_t bits = arr < W ? mk[arr] : 0ull;
    pfx[arr] = arr < NA ? static_cast<uint32_t>(__builtin_popcountll(arr == a.count ? wsr : bits)) : 0u;
  }
#pragma unroll
  for (uint32_t arr = 0; arr < NW; ++arr) {
    const uint32_t v = pfx[arr];
    uint32_t inc = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t o = __shfl_up(inc, d, 64);
      if (lane >= static_cast<uint32_t>(d)) inc += o;
    }
    pfx[arr] = inc - v;
    if (lane == 63) s_wtot[wave][arr] = inc;
  }
  if (t < NW) s_base[t] = 0;
  __syncthreads();
  uint32_t ctot[NW];
#pragma unroll
  for (uint32_t arr = 0; arr < NW; ++arr) {
    uint32_t before = 0, all = 0;
#pragma unroll
    for (uint32_t w = 0; w < kW; ++w) {
      const uint32_t x = s_wtot[w][arr];
      before += w < wave ? x : 0u;
      all += x;
    }
    pfx[arr] += before;
    ctot[arr] = all;
  }
  // ---- publish the chunk's totals (stored + 1: a zero word is "not yet"), then add the predecessors': thread
  // (i, arr) waits for chunk i's total of array arr, whose workgroup took its ticket first (it is running or done)
  if (t < NA) {
    uint32_t v = 0;
#pragma unroll
    for (uint32_t arr = 0; arr < NW; ++arr) v = arr == t ? ctot[arr] : v;
    __hip_atomic_store(&totals[c * kPlanArraysR04 + t], v + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  for (uint32_t idx = t; idx < c * NA; idx += kPlan2ThreadsR04) {
    const uint32_t i = idx / NA, arr = idx - i * NA;
    uint32_t v;
    while ((v = __hip_atomic_load(&totals[i * kPlanArraysR04 + arr], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0u)
      __builtin_amdgcn_s_sleep(1);
    atomicAdd(&s_base[arr], v - 1u);
  }
  __syncthreads();
  // ---- this chunk's rows: write set, union, own masks cleared, prefixes, the counts at the shard bounds
  //      (system-scope stores: the host reads them), the totals
  if (in) {
    a.write_set[r] = wsr;
    a.union_masks[r] = u;
    if (a.zero_masks != nullptr) a.zero_masks[r] = 0;
  }
  uint32_t bnd = kNone;  // the shard bound this row starts, if any (bounds are distinct except empty shards)
  for (uint32_t s = 0; s < a.nbounds; ++s)
    if (s_bounds[s] == r && in) bnd = s;
  if (in) {
#pragma unroll
    for (uint32_t arr = 0; arr < NW; ++arr) {
      if (arr >= NA) continue;
      const uint32_t pv = s_base[arr] + pfx[arr];
      a.prefix[static_cast<uint64_t>(arr) * (a.rows + 1) + r] = pv;
      if (bnd != kNone)  // (every bound equal to this row: empty shards repeat a bound)
        for (uint32_t s = 0; s < a.nbounds; ++s)
          if (s_bounds[s] == r)
            __hip_atomic_store(&a.counts[arr * a.nbounds + s], pv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  if (c + 1 == nchunks && t == 0) {
#pragma unroll
    for (uint32_t arr = 0; arr < NW; ++arr) {
      if (arr >= NA) continue;
      const uint32_t total = s_base[arr] + ctot[arr];
      a.prefix[static_cast<uint64_t>(arr) * (a.rows + 1) + a.rows] = total;
      for (uint32_t s = 0; s < a.nbounds; ++s)
        if (s_bounds[s] >= a.rows)
          __hip_atomic_store(&a.counts[arr * a.nbounds + s], total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  // ---- completion: every chunk's counts acknowledged (write-through, system scope), then the last arrival re-arms
  // the workspace (every chunk is past its look-back: nothing reads the totals any more) and posts the sequence number
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __shared__ uint32_t s_last;
  __syncthreads();
  if (t == 0) s_last = __hip_atomic_fetch_add(&ws[0], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) + 1 == nchunks;
  __syncthreads();
  if (s_last) {
    for (uint32_t idx = t; idx < nchunks * kPlanArraysR04; idx += kPlan2ThreadsR04)
      __hip_atomic_store(&totals[idx], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
      __hip_atomic_store(&ws[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&ws[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (a.done_flag != nullptr) __hip_atomic_store(a.done_flag, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// omr_round_plan_list (v2 false: k_round_plan, `arrive` one word) and omr_round_plan_ws (v2 true: k_round_plan2_r04 on
// plans of up to kPlanChunksMaxR04 * 256 rows, `arrive` its workspace; larger plans use k_round_plan with word 0)
int round_plan_launch_r04(const uint64_t* row_masks, uint32_t count, uint64_t mask_stride, uint64_t rows,
                      uint32_t rows_per_part, uint32_t num_lanes, const uint64_t* bounds, uint32_t num_bounds,
                      uint64_t* write_set, uint64_t* union_masks, uint32_t* prefix, uint32_t* counts,
                      uint64_t* zero_masks, uint32_t* zero_counters, uint32_t num_zero_counters, uint32_t* arrive,
                      uint32_t* done_flag, uint32_t seq, uint32_t* union_next, uint32_t block_size,
                      const omr_sum_list* list, bool v2, hipStream_t st) {
  if (mask_stride < rows) return fail("round_plan: mask_stride %llu < rows", static_cast<unsigned long long>(mask_stride));
  if (num_zero_counters > kPlanThreadsR04 || (num_zero_counters > 0 && zero_counters == nullptr))
    return fail("round_plan: zero_counters");
  if (count == 0 || count > OMR_MAX_WORKERS) return fail("round_plan: count %u out of range", count);
  if (rows == 0 || rows_per_part == 0 || rows % rows_per_part != 0) return fail("round_plan: bad rows");
  if (num_lanes == 0 || num_lanes > 64) return fail("round_plan: num_lanes %u out of range", num_lanes);
  if (row_masks == nullptr || write_set == nullptr || union_masks == nullptr || prefix == nullptr ||
      (num_bounds > 0 && (bounds == nullptr || counts == nullptr)))
    return fail("round_plan: NULL pointer");
  if (rows > 0xFFFFFFFFull / 64) return fail("round_plan: too many rows");
  if (num_bounds > OMR_MAX_WORKERS + 2) return fail("round_plan: %u bounds > %d", num_bounds, OMR_MAX_WORKERS + 2);
  PlanArgsR04 a;
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
  if (!v2 && (arrive == nullptr) != (done_flag == nullptr)) return fail("round_plan: arrive and done_flag go together");
  if (v2 && arrive == nullptr) return fail("round_plan_ws: NULL workspace");
  a.arrive = arrive;
  a.done_flag = done_flag;
  a.seq = seq;
  memset(&a.chain, 0, sizeof(a.chain));
  uint32_t chain_wgs = 0;
  if (union_next != nullptr) {
    if (block_size != 256 && block_size != 512 && block_size != 1024)
      return fail("round_plan: block_size %u unsupported", block_size);
    if ((num_lanes & (num_lanes - 1)) != 0) return fail("round_plan: num_lanes %u", num_lanes);
    const uint64_t parts = rows / rows_per_part;
    a.chain.next = union_next;
    a.chain.rows = rows;
    a.chain.nb = rows * num_lanes;
    a.chain.rows_per_part = rows_per_part;
    a.chain.segs_per_part = (rows_per_part + 63) / 64;
    a.chain.lanes = num_lanes;
    a.chain.block = block_size;
    a.chain.sentinel = omr_sentinel(block_size, num_lanes);
    chain_wgs = static_cast<uint32_t>(parts * a.chain.segs_per_part);
  }
  a.chain_wgs = chain_wgs;
  a.list_wgs = 0;
  if (list != nullptr) {
    if (block_size != 256 && block_size != 512 && block_size != 1024)
      return fail("round_plan: block_size %u unsupported", block_size);
    Layout L;
    if (int rc = make_layout(rows * num_lanes * block_size, block_size, num_lanes,
                             static_cast<uint32_t>(rows / rows_per_part), &L))
      return rc;
    if (int rc = make_list_args(L, row_masks, count, mask_stride, list, &a.list)) return rc;
    const uint64_t units = list_units_host(a.list);
    const uint64_t wgs = (units + kPlanThreadsR04 / 64 - 1) / (kPlanThreadsR04 / 64);
    a.list_wgs = static_cast<uint32_t>(wgs < 512 ? wgs : 512);
  }
  const uint64_t nchunks = (rows + kPlan2ThreadsR04 - 1) / kPlan2ThreadsR04;
  if (v2 && nchunks <= kPlanChunksMaxR04) {
    if (arrive == nullptr) return fail("round_plan_ws: NULL workspace");
    if (num_zero_counters > kPlan2ThreadsR04) return fail("round_plan_ws: zero_counters > %u", kPlan2ThreadsR04);
    if (list != nullptr) {  // (k_round_plan's list workgroups had 16 waves each: the same units, 4 waves per workgroup)
      const uint64_t units = list_units_host(a.list);
      const uint64_t wgs = (units + kPlan2ThreadsR04 / 64 - 1) / (kPlan2ThreadsR04 / 64);
      a.list_wgs = static_cast<uint32_t>(wgs < 2048 ? wgs : 2048);
    }
    a.arrive = nullptr;  // (k_round_plan2_r04 counts its arrivals in the workspace)
    const unsigned grid = static_cast<unsigned>(nchunks + chain_wgs + a.list_wgs);
    const uint32_t nc = static_cast<uint32_t>(nchunks);
    if (list != nullptr) {
      if (count <= 8) k_round_plan2_r04<true, 8><<<grid, kPlan2ThreadsR04, 0, st>>>(a, nc, arrive);
      else k_round_plan2_r04<true, OMR_MAX_WORKERS><<<grid, kPlan2ThreadsR04, 0, st>>>(a, nc, arrive);
    } else if (count <= 2) {
      k_round_plan2_r04<false, 2><<<grid, kPlan2ThreadsR04, 0, st>>>(a, nc, arrive);
    } else if (count <= 4) {
      k_round_plan2_r04<false, 4><<<grid, kPlan2ThreadsR04, 0, st>>>(a, nc, arrive);
    } else if (count <= 8) {
      k_round_plan2_r04<false, 8><<<grid, kPlan2ThreadsR04, 0, st>>>(a, nc, arrive);
    } else {
      k_round_plan2_r04<false, OMR_MAX_WORKERS><<<grid, kPlan2ThreadsR04, 0, st>>>(a, nc, arrive);
    }
    return launch_status("k_round_plan2_r04");
  }
  const size_t lds = rows <= kPlanLdsRowsR04 ? rows * sizeof(uint64_t) : 0;
  k_round_plan_r04<<<count + 1 + chain_wgs + a.list_wgs, kPlanThreadsR04, lds, st>>>(a);
  return launch_status("k_round_plan");
}
}  // namespace

extern "C" {

int tune_round_plan_list_r04(const uint64_t* row_masks, uint32_t count, uint64_t mask_stride, uint64_t rows,
                             uint32_t rows_per_part, uint32_t num_lanes, const uint64_t* bounds, uint32_t num_bounds,
                             uint64_t* write_set, uint64_t* union_masks, uint32_t* prefix, uint32_t* counts,
                             uint64_t* zero_masks, uint32_t* zero_counters, uint32_t num_zero_counters, uint32_t* arrive,
                             uint32_t* done_flag, uint32_t seq, uint32_t* union_next, uint32_t block_size,
                             const omr_sum_list* list, hipStream_t stream) {
  return round_plan_launch_r04(row_masks, count, mask_stride, rows, rows_per_part, num_lanes, bounds, num_bounds,
                               write_set, union_masks, prefix, counts, zero_masks, zero_counters, num_zero_counters,
                               arrive, done_flag, seq, union_next, block_size, list, false, stream);
}

uint64_t tune_round_plan_workspace_words_r04(void) { return kPlan2WorkspaceWordsR04; }

int tune_round_plan_ws_r04(const uint64_t* row_masks, uint32_t count, uint64_t mask_stride, uint64_t rows,
                           uint32_t rows_per_part, uint32_t num_lanes, const uint64_t* bounds, uint32_t num_bounds,
                           uint64_t* write_set, uint64_t* union_masks, uint32_t* prefix, uint32_t* counts,
                           uint64_t* zero_masks, uint32_t* zero_counters, uint32_t num_zero_counters, uint32_t* workspace,
                           uint32_t* done_flag, uint32_t seq, uint32_t* union_next, uint32_t block_size,
                           const omr_sum_list* list, hipStream_t stream) {
  return round_plan_launch_r04(row_masks, count, mask_stride, rows, rows_per_part, num_lanes, bounds, num_bounds,
                               write_set, union_masks, prefix, counts, zero_masks, zero_counters, num_zero_counters,
                               workspace, done_flag, seq, union_next, block_size, list, true, stream);
}

}  // extern "C"

namespace {
struct SumArgsR04 {
  const float* own;
  const float* recv;
  uint64_t recv_off[OMR_MAX_WORKERS];
  const uint64_t* masks;   // worker c's row masks at masks + c * mstride
  uint64_t mstride;
  const uint32_t* prefix;  // [count + 1][rows + 1]: the workers' row-stream prefixes, then the write set's
  uint64_t pos_off;        // column streams: worker c's position table at (const uint32_t*)(masks + c * mstride) + pos_off
  const uint64_t* write_set;
  float* out;
  uint64_t rows, r0, r1;
  uint32_t count, me, lanes, block, packed_out;
  uint32_t S, gps;         // column streams: segment rows (shards are whole segments), 64-row groups per segment
  // set by the launch, so a unit's coordinates are 32-bit shifts and two 32-bit divisions (round 3's 64-bit divisions
  // by runtime values were ~1,000 scalar instructions before a wave's first load)
  uint32_t units, lane_shift, seg0;
};


// W >= count: the contributor loops are unrolled W times (the launch picks 2, 4, 8 or 16), so an 8-worker shard does
// half the per-row work of a 16-way unroll.  UR: rows per unit.
template <int VEC, int W, uint32_t UR = kShardUnitRows>
__global__ __launch_bounds__(kWGThreads) void k_shard_sum_r04(SumArgsR04 a) {
  constexpr int P = 32 / VEC;  // pair slots per window
  constexpr int kSlotGroup = P < 8 ? P : 8;
  constexpr uint32_t kRecCap = UR * W;
  constexpr uint32_t QU = kPackGroupRows / UR;  // units per 64-row group (column streams)
  __shared__ uint64_t s_rec[kWavesPerWG][kRecCap];
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool cols = a.pos_off != kRowStreams;
  const uint32_t nw = gridDim.x * kWavesPerWG;
  const uint32_t* const pws = a.prefix + static_cast<uint64_t>(a.count) * (a.rows + 1);
  const uint32_t wpre0 = a.packed_out ? pws[a.r0] : 0u;
  const uint32_t bbytes = a.block * 4;
  for (uint32_t u = blockIdx.x * kWavesPerWG + wave; u < a.units; u += nw) {
    const uint32_t l = u & (a.lanes - 1);
    uint64_t g0, gidx = 0;  // first row the lanes load (lane i: row g0 + i); column streams: the group's table index
    uint32_t nload, h0, h1;  // rows loaded; the unit's rows are lanes [h0, h1)
    if (cols) {
      uint32_t t = u >> a.lane_shift;
      const uint32_t h = t % QU;
      t /= QU;
      const uint32_t j = t % a.gps;
      const uint64_t seg = a.seg0 + t / a.gps;
      g0 = seg * a.S + static_cast<uint64_t>(j) * kPackGroupRows;
      nload = a.S - j * kPackGroupRows < kPackGroupRows ? a.S - j * kPackGroupRows : kPackGroupRows;
      h0 = h * UR;
      h1 = nload < h0 + UR ? nload : h0 + UR;
      gidx = seg * a.gps + j;
      if (h0 >= h1) continue;
    } else {
      g0 = a.r0 + static_cast<uint64_t>(u >> a.lane_shift) * UR;
      nload = a.r1 - g0 < UR ? static_cast<uint32_t>(a.r1 - g0) : UR;
      h0 = 0;
      h1 = nload;
    }
    // ---- index loads, all issued together (one round trip)
    const bool rl = static_cast<uint32_t>(lane) < nload;
    const uint64_t r = g0 + (rl ? static_cast<uint32_t>(lane) : 0u);
    const uint64_t w = rl ? a.write_set[r] : 0ull;
    const uint32_t wpre = (rl && a.packed_out) ? pws[r] : 0u;
    uint64_t mk[W];
    uint32_t pre[W];
#pragma unroll
    for (uint32_t c = 0; c < W; ++c) {
      mk[c] = (c < a.count && rl) ? a.masks[c * a.mstride + r] : 0ull;
      pre[c] = (!cols && c < a.count && rl) ? a.prefix[c * (a.rows + 1) + r] : 0u;
    }
    // lane c < count: worker c's group position (column streams) or its stream prefix at r0 (row streams)
    const bool cl = static_cast<uint32_t>(lane) < a.count;
    const uint32_t base_c =
        !cl ? 0u
            : cols ? reinterpret_cast<const uint32_t*>(a.masks + lane * a.mstride)[a.pos_off + gidx * a.lanes + l]
                   : a.prefix[static_cast<uint64_t>(lane) * (a.rows + 1) + a.r0];
    // ---- (block, contributor) pairs of the unit's write-set blocks, rank order within a block
    const bool mine = static_cast<uint32_t>(lane) >= h0 && static_cast<uint32_t>(lane) < h1;
    const bool wb = mine && ((w >> l) & 1ull);
    uint32_t cb = 0;
#pragma unroll
    for (uint32_t c = 0; c < W; ++c) cb |= static_cast<uint32_t>((mk[c] >> l) & 1ull) << c;
    const uint32_t np = wb ? (cb ? static_cast<uint32_t>(__builtin_popcount(cb)) : 1u) : 0u;
    uint32_t inc = np;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t o = __shfl_up(inc, d, 64);
      if (lane >= d) inc += o;
    }
    const uint32_t total = __builtin_amdgcn_readlane(inc, 63);
    if (total == 0) continue;
    uint64_t ccol[W];  // column streams: worker c's bits of column l over the loaded rows
#pragma unroll
    for (uint32_t c = 0; c < W; ++c) ccol[c] = (cols && c < a.count) ? __ballot((mk[c] >> l) & 1ull) : 0ull;
    if (np != 0) {
      uint32_t k = inc - np;
      const uint32_t first = k, last = inc - 1;
      const uint64_t dst = a.packed_out ? static_cast<uint64_t>(wpre - wpre0) +
                                              static_cast<uint64_t>(__builtin_popcountll(w & below(l)))
                                        : r * a.lanes + l;
      const uint64_t hdr = dst << 32;
      if (cb == 0) {
        s_rec[wave][k] = hdr | kRecZero | kRecFirst | kRecLast;
      } else {
#pragma unroll
        for (uint32_t c = 0; c < W; ++c) {
          if (!((cb >> c) & 1u)) continue;
          uint64_t rec;
          if (c == a.me) {
            rec = (r * a.lanes + l) | kRecOwn;
          } else {
            const uint32_t bc = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(base_c), c));
            const uint64_t pos = cols ? static_cast<uint64_t>(bc) + static_cast<uint64_t>(__builtin_popcountll(
                                                                        ccol[c] & below(static_cast<uint32_t>(lane))))
                                      : static_cast<uint64_t>(pre[c] - bc) +
                                            static_cast<uint64_t>(__builtin_popcountll(mk[c] & below(l)));
            rec = (a.recv_off[c] + pos) & 0xFFFFFFFFull;
          }
          rec |= hdr | (k == first ? kRecFirst : 0ull) | (k == last ? kRecLast : 0ull);
          s_rec[wave][k++] = rec;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // the wave's record stores land before its reads
    // ---- the pairs, P at a time: every load of the window in flight, then the segmented rank-order sum
    v4f acc[VEC];
#pragma unroll
    for (int q = 0; q < VEC; ++q) acc[q] = v4f{0.f, 0.f, 0.f, 0.f};
    for (uint32_t wbase = 0; wbase < total; wbase += P) {
      const uint32_t nv = total - wbase < static_cast<uint32_t>(P) ? total - wbase : static_cast<uint32_t>(P);
      const uint64_t myrec = static_cast<uint32_t>(lane) < nv ? s_rec[wave][wbase + lane] : 0ull;
      v4f v[P][VEC];
      // every load of the window issued before the first use; slots in groups of kSlotGroup, a group past the
      // window's last pair skipped by a wave-uniform branch (a sparse unit issues only what it needs)
#pragma unroll
      for (int g = 0; g < P; g += kSlotGroup) {
        if (static_cast<uint32_t>(g) < nv) {
#pragma unroll
          for (int j = g; j < g + kSlotGroup; ++j) {
            const uint64_t rc = readlane64(myrec, j);
            const bool load = static_cast<uint32_t>(j) < nv && !(rc & kRecZero);
            const float* const sb = (rc & kRecOwn) ? a.own : a.recv;
            const __amdgpu_buffer_rsrc_t src =
                chunk_rsrc(sb + static_cast<uint64_t>(static_cast<uint32_t>(rc)) * a.block, load ? bbytes : 0u);
#pragma unroll
            for (int q = 0; q < VEC; ++q)
              v[j][q] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(src, (q * 64 + lane) * 16, 0,
                                                                                     kLoadAux));
          }
        }
      }
      // the segmented sums first, every pair's running sum kept in its slot's registers; then the stores of the blocks
      // the window completed.  (A store between two adds makes every later wait count it: on gfx9 vmcnt counts loads
      // and stores together, so the waits before the adds of the next slot group also waited for the stores' acks --
      // up to four store round trips per window, measured as a 3 us tail at config 4's shard; round 4.)
      // (every slot is consumed on every path, a slot past the window's last pair by a discarded add: a register whose
      // load might still be pending on some path would make the compiler wait again before its store)
#pragma unroll
      for (int j = 0; j < P; ++j) {
        const uint64_t rc = readlane64(myrec, j);
        const bool use = static_cast<uint32_t>(j) < nv;
#pragma unroll
        for (int q = 0; q < VEC; ++q) {  // (0.0f + x_first) + ...: a block's first pair restarts from +0.0f
          const v4f sum = add4((rc & kRecFirst) ? v4f{0.f, 0.f, 0.f, 0.f} : acc[q], v[j][q]);
          acc[q] = use ? sum : acc[q];
          v[j][q] = acc[q];
        }
      }
      // (pins every add above the stores: left to itself the compiler sinks slot j+1's add below slot j's conditional
      // store, and its wait then counts that store again)
#pragma unroll
      for (int j = 0; j < P; ++j)
#pragma unroll
        for (int q = 0; q < VEC; ++q) asm volatile("" : "+v"(v[j][q]));
#pragma unroll
      for (int j = 0; j < P; ++j) {
        if (static_cast<uint32_t>(j) < nv) {
          const uint64_t rc = readlane64(myrec, j);
          if (rc & kRecLast) {
            store_block_wt<VEC>(a.out + ((rc >> 32) & 0x0FFFFFFFull) * a.block, v[j], lane);
          }
        }
      }
    }
  }
}

template <int W>
void launch_shard_sum_w_r04(const SumArgsR04& a, unsigned g, hipStream_t st) {
  switch (a.block / 256) {
    case 1: k_shard_sum_r04<1, W><<<g, kWGThreads, 0, st>>>(a); break;
    case 2: k_shard_sum_r04<2, W><<<g, kWGThreads, 0, st>>>(a); break;
    default: k_shard_sum_r04<4, W><<<g, kWGThreads, 0, st>>>(a); break;
  }
}

int launch_shard_sum_r04(const SumArgsR04& a0, const uint64_t* recv_offsets, hipStream_t st) {
  SumArgsR04 a = a0;
  if (a.count == 0 || a.count > OMR_MAX_WORKERS) return fail("shard_sum: count %u out of range", a.count);
  if (a.block != 256 && a.block != 512 && a.block != 1024) return fail("shard_sum: block_size %u unsupported", a.block);
  if (a.lanes == 0 || a.lanes > 64 || (a.lanes & (a.lanes - 1)) != 0) return fail("shard_sum: num_lanes %u", a.lanes);
  if (a.r0 > a.r1 || a.r1 > a.rows) return fail("shard_sum: bad row range");
  if (a.r1 == a.r0) return 0;
  if (a.masks == nullptr || a.prefix == nullptr || a.write_set == nullptr || a.out == nullptr ||
      (a.me < a.count && a.own == nullptr) || (a.count > 1 && a.recv == nullptr) || recv_offsets == nullptr)
    return fail("shard_sum: NULL pointer");
  if (reinterpret_cast<uintptr_t>(a.out) % 16 != 0 || reinterpret_cast<uintptr_t>(a.own) % 16 != 0 ||
      reinterpret_cast<uintptr_t>(a.recv) % 16 != 0)
    return fail("shard_sum: buffers must be 16-byte aligned");
  for (uint32_t c = 0; c < OMR_MAX_WORKERS; ++c) {
    a.recv_off[c] = c < a.count ? recv_offsets[c] : 0;
    if (c < a.count && c != a.me && a.recv_off[c] > 0xFFFFFFFFull) return fail("shard_sum: recv offset beyond 2^32 blocks");
  }
  const uint64_t srows = a.r1 - a.r0;
  const uint64_t units = a.pos_off != kRowStreams ? (srows / a.S) * a.gps * (kPackGroupRows / kShardUnitRows) * a.lanes
                                                 : ((srows + kShardUnitRows - 1) / kShardUnitRows) * a.lanes;
  if (units > 0xFFFFFFFFull) return fail("shard_sum: %llu units", static_cast<unsigned long long>(units));
  a.units = static_cast<uint32_t>(units);
  a.lane_shift = static_cast<uint32_t>(__builtin_ctz(a.lanes));
  a.seg0 = a.pos_off != kRowStreams ? static_cast<uint32_t>(a.r0 / a.S) : 0u;
  const unsigned g = grid_for(units);
  if (a.count <= 2) launch_shard_sum_w_r04<2>(a, g, st);
  else if (a.count <= 4) launch_shard_sum_w_r04<4>(a, g, st);
  else if (a.count <= 8) launch_shard_sum_w_r04<8>(a, g, st);
  else launch_shard_sum_w_r04<OMR_MAX_WORKERS>(a, g, st);
  return launch_status("k_shard_sum");
}
}  // namespace

extern "C" {

int tune_shard_sum_cols_r04(const float* own, uint32_t me, const float* recv, const uint64_t* recv_offsets,
                           const uint64_t* row_masks, uint32_t count, uint64_t mask_stride, uint64_t pos_offset,
                           const uint32_t* prefix, const uint64_t* write_set, uint64_t n, uint32_t block_size,
                           uint32_t num_lanes, uint32_t num_parts, uint64_t row_begin, uint64_t row_end,
                           int packed_out, float* out, hipStream_t stream) {
  Layout L;
  if (int rc = make_layout(n, block_size, num_lanes, num_parts, &L)) return rc;
  const FusedShape f = fused_shape(L);
  if (row_begin % f.S != 0 || row_end % f.S != 0)
    return fail("shard_sum_cols: rows [%llu, %llu) are not whole %u-row column segments",
                static_cast<unsigned long long>(row_begin), static_cast<unsigned long long>(row_end), f.S);
  const uint64_t words = mask_stride * 2;  // the position table must lie inside each worker's array
  if (mask_stride < L.rows || pos_offset < L.rows * 2 || pos_offset + pack_table_entries(L, f) > words)
    return fail("shard_sum_cols: position table outside the mask arrays (stride %llu, offset %llu)",
                static_cast<unsigned long long>(mask_stride), static_cast<unsigned long long>(pos_offset));
  SumArgsR04 a{};
  a.own = own;
  a.recv = recv;
  a.masks = row_masks;
  a.mstride = mask_stride;
  a.prefix = prefix;
  a.pos_off = pos_offset;
  a.write_set = write_set;
  a.out = out;
  a.rows = L.rows;
  a.r0 = row_begin;
  a.r1 = row_end;
  a.count = count;
  a.me = me;
  a.lanes = L.lanes;
  a.block = L.block;
  a.packed_out = packed_out ? 1u : 0u;
  a.S = f.S;
  a.gps = pack_groups(f);
  return launch_shard_sum_r04(a, recv_offsets, stream);
}

}  // extern "C"

extern "C" uint32_t omr_sentinel(uint32_t block_size, uint32_t num_lanes) {  // the product's, compiled out by OMR_NO_CAPI
  if (block_size == 0 || num_lanes == 0) return 0;
  return (UINT32_MAX / block_size / num_lanes - 1u) * num_lanes * block_size;
}
