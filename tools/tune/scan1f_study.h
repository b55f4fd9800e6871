// scan1f_study.h — the timing-study form of the single-pass worker step (not the product; built only into the
// tools/tune harnesses, after omr_kernels.hip in the same translation unit).  It is the round-2 product kernel
// k_scan1f plus the study knobs that were measured with it:
//   ABL   bit 0 drops the data stores, bit 1 the flag/next stores, bit 2 sends every data store of a batch to the same
//         block at the start of `out` (the same store count, no scattered HBM writes), bit 3 records per-workgroup
//         timestamps {start, loop end, end with stores acknowledged, XCC} in place of the row masks
//         (tools/wg_timeline.py), bit 4 rotates the workgroup -> column map by one XCD;
//   MINW  the amdgpu_waves_per_eu floor (occupancy study; 1 = the compiler's choice);
//   SAUX  the block stores' cache policy (store-policy study; the product's is kStoreAux);
//   SKIP  a batch with no block to write skips its (dropped) data stores (the product's choice at B = 1024);
//   MAUX  the flag / next stores through buffer stores with cache policy MAUX (-1: the product's plain stores).
// The product (omr_kernels.hip) keeps none of these branches.
#pragma once

namespace {

template <int VEC, int WAVES, int LOADS = 16, int ABL = 0, int MINW = 1, int SAUX = kStoreAux, int SKIP = 0,
          int MAUX = -1>
__global__ __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(MINW))) void k_scan1f_study(FusedArgs a) {
  constexpr int RB = LOADS / VEC;  // rows per batch (<= 32)
  static_assert(RB >= 1 && RB <= 32, "batch bits are 32-bit");
  __shared__ uint32_t s_wfirst[WAVES], s_wlast[WAVES];
  __shared__ int s_fix;
  __shared__ uint32_t s_carry[64];
  __shared__ uint32_t s_seg_last[64];
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t T = gridDim.x, bid = blockIdx.x;
  const uint32_t lin0 = (T % 8 == 0) ? (bid % 8) * (T / 8) + bid / 8 : bid;
  const uint32_t lin = (ABL & 16) ? (lin0 + T / 8) % T : lin0;  // ABL bit 4: every XCD takes the next XCD's columns
  const uint32_t k = lin % a.K, col = lin / a.K + a.part0 * a.lanes;  // col: global (partition, lane) index
  const uint32_t l = col % a.lanes, p = col / a.lanes;
  const uint32_t r0 = k * a.S;                                  // segment's first row within the partition
  const uint64_t row0 = static_cast<uint64_t>(p) * a.rpp + r0;  // its global row
  uint64_t* const tl = (ABL & 8) ? a.masks : nullptr;           // timing-only: per-workgroup timestamps
  uint64_t* const masks = (ABL & 8) ? nullptr : a.masks;
  if ((ABL & 8) && threadIdx.x == 0) tl[bid * 4] = __builtin_amdgcn_s_memrealtime();
  const uint32_t row_bytes = a.lanes * a.block * 4;
  const uint32_t lane_b = l * a.block;
  const uint32_t row_stride = a.lanes * a.block;
  const bool last_seg = (k + 1 == a.K);
  // the wave's rows [lo, hi) of the segment: whole batches, except possibly the last nonempty wave's top one
  const uint32_t rw = ((a.S + WAVES * RB - 1) / (WAVES * RB)) * RB;
  const uint32_t lo = wave * rw < a.S ? wave * rw : a.S;
  const uint32_t hi = lo + rw < a.S ? lo + rw : a.S;
  uint32_t carry = kNone, wlast = kNone;
  for (uint32_t nb_ = (hi - lo + RB - 1) / RB; nb_ > 0; --nb_) {
    const uint32_t rr = lo + (nb_ - 1) * RB;
    const uint32_t nrow = (hi - rr < static_cast<uint32_t>(RB)) ? hi - rr : RB;
    const uint64_t blk0 = (row0 + rr) * a.lanes + l;  // block of the batch's first row
    const __amdgpu_buffer_rsrc_t src = chunk_rsrc(a.x + blk0 * a.block, nrow * row_bytes);
    v4f v[RB][VEC];
#pragma unroll
    for (int s = 0; s < RB; ++s)
#pragma unroll
      for (int q = 0; q < VEC; ++q)
        v[s][q] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(
                                              src, s * row_bytes + (q * 64 + lane) * 16, 0, kLoadAux));
    const __amdgpu_buffer_rsrc_t dst =
        chunk_rsrc((ABL & 4) ? a.out : a.out + blk0 * a.block, (a.out != nullptr && !(ABL & 1)) ? nrow * row_bytes : 0u);
    const uint32_t row_step = (ABL & 4) ? 0u : row_bytes;  // ABL bit 2: every row's store to the same block
    uint32_t bits = 0;
#pragma unroll
    for (int s = 0; s < RB; ++s) {
      uint32_t o = 0;
#pragma unroll
      for (int q = 0; q < VEC; ++q) o |= nz_bits(v[s][q]);
      const bool nz = wave_ballot(o != 0) != 0 && static_cast<uint32_t>(s) < nrow;
      bits |= static_cast<uint32_t>(nz) << s;
      if constexpr (!SKIP) {
        const bool head = (r0 + rr + s) == 0;  // lane head: row 0 of the partition, always sent (client.cc:201-205)
        // aggregated block 0.0f + x (server.cc:148-150 zero, :97-98 add), written in place (client.cc:89)
        const uint32_t drop = (nz || head) ? 0u : kDropStore;
#pragma unroll
        for (int q = 0; q < VEC; ++q)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, add4(v4f{0.f, 0.f, 0.f, 0.f}, v[s][q])),
                                                 dst, (s * row_step + (q * 64 + lane) * 16) | drop, 0, SAUX);
      }
    }
    if constexpr (SKIP) {
      // the batch's stores only when it has a block to write (a wave-uniform branch; inside it, the static schedule)
      if (bits != 0 || rr + r0 == 0) {
#pragma unroll
        for (int s = 0; s < RB; ++s) {
          const bool head = (r0 + rr + s) == 0;
          const uint32_t drop = (((bits >> s) & 1u) || head) ? 0u : kDropStore;
#pragma unroll
          for (int q = 0; q < VEC; ++q)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, add4(v4f{0.f, 0.f, 0.f, 0.f}, v[s][q])),
                                                   dst, (s * row_step + (q * 64 + lane) * 16) | drop, 0, SAUX);
        }
      }
    }
    if (!(ABL & 2) && static_cast<uint32_t>(lane) < nrow) {
      const uint64_t blk = blk0 + static_cast<uint64_t>(lane) * a.lanes;
      // successor of row rr+lane: next set bit above it in this batch, else the carry (client.cc:19-31)
      const uint32_t above = static_cast<uint32_t>(static_cast<uint64_t>(bits) >> (lane + 1));
      const uint32_t nr = above != 0 ? rr + lane + 1 + static_cast<uint32_t>(__builtin_ctz(above)) : carry;
      if constexpr (MAUX < 0) {
        if (a.flags != nullptr) a.flags[blk] = static_cast<int32_t>((bits >> lane) & 1u);
        if (nr != kNone) a.next[blk] = static_cast<uint32_t>(row0 + nr) * row_stride + lane_b;
      } else {  // study: the flag / next stores with cache policy MAUX (byte offsets < 2^31 in the study's sizes)
        const __amdgpu_buffer_rsrc_t rf = __builtin_amdgcn_make_buffer_rsrc(a.flags, 0, a.flags ? 0x7FFFFFFF : 0, 0x00020000);
        const __amdgpu_buffer_rsrc_t rn = __builtin_amdgcn_make_buffer_rsrc(a.next, 0, 0x7FFFFFFF, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b32((bits >> lane) & 1u, rf, static_cast<uint32_t>(blk * 4), 0, MAUX);
        if (nr != kNone)
          __builtin_amdgcn_raw_buffer_store_b32(static_cast<uint32_t>(row0 + nr) * row_stride + lane_b, rn,
                                                static_cast<uint32_t>(blk * 4), 0, MAUX);
      }
      if (masks != nullptr && ((bits >> lane) & 1u))
        (void)__hip_atomic_fetch_or(&masks[row0 + rr + lane], 1ull << l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (bits != 0) {
      if (wlast == kNone) wlast = rr + 31 - static_cast<uint32_t>(__builtin_clz(bits));
      carry = rr + static_cast<uint32_t>(__builtin_ctz(bits));
    }
  }
  if (lane == 0) {
    s_wfirst[wave] = carry;  // first non-zero row of the wave's range (kNone: all zero)
    s_wlast[wave] = wlast;   // last one
  }
  __syncthreads();
  if ((ABL & 8) && threadIdx.x == 0) tl[bid * 4 + 1] = __builtin_amdgcn_s_memrealtime();
  // tail rows [wlast or lo, hi): successor = first non-zero row of a later wave, else of a later segment
  uint32_t succ = kNone;
  for (uint32_t w2 = wave + 1; w2 < WAVES; ++w2)
    if (s_wfirst[w2] != kNone) {
      succ = s_wfirst[w2];
      break;
    }
  if (!(ABL & 2) && (succ != kNone || last_seg)) {
    const uint32_t val = succ != kNone ? static_cast<uint32_t>(row0 + succ) * row_stride + lane_b : a.sentinel + lane_b;
    for (uint32_t i = (wlast == kNone ? lo : wlast) + lane; i < hi; i += 64) a.next[(row0 + i) * a.lanes + l] = val;
  }
  if constexpr ((ABL & 8) != 0) {  // every store of the workgroup acknowledged
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      tl[bid * 4 + 2] = __builtin_amdgcn_s_memrealtime();
      tl[bid * 4 + 3] = static_cast<uint64_t>(__builtin_amdgcn_s_getreg((15 << 11) | 20));  // HW_REG_XCC_ID
    }
  }
  if (a.K == 1) return;
  // multi-segment column: publish {first, last}, count arrivals; the last arriver fixes every tail row
  if (threadIdx.x == 0) {
    uint32_t first = kNone, last = 0;
    for (int w2 = 0; w2 < WAVES; ++w2) {
      if (first == kNone) first = s_wfirst[w2];
      if (s_wlast[w2] != kNone) last = s_wlast[w2];
    }
    const uint64_t sm = (static_cast<uint64_t>(first) << 32) | (first == kNone ? kNone : last);
    (void)__hip_atomic_exchange(&a.summary[static_cast<uint64_t>(col) * a.K + k], sm, __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t old = __hip_atomic_fetch_add(&a.cnt[col], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_fix = (old == a.K - 1);
  }
  __syncthreads();
  if (!s_fix) return;
  if (threadIdx.x < a.K) {  // read every segment's summary at the coherence point (atomic RMW), K <= 64
    const uint64_t sm = __hip_atomic_fetch_or(&a.summary[static_cast<uint64_t>(col) * a.K + threadIdx.x], 0ull,
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_carry[threadIdx.x] = static_cast<uint32_t>(sm >> 32);  // first (temporarily)
    s_seg_last[threadIdx.x] = static_cast<uint32_t>(sm);
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // carry[k'] = first non-zero row (partition-relative) in segments after k'
    uint32_t c = kNone;
    for (int kk = static_cast<int>(a.K) - 1; kk >= 0; --kk) {
      const uint32_t first = s_carry[kk];
      s_carry[kk] = c;
      if (first != kNone) c = static_cast<uint32_t>(kk) * a.S + first;
    }
    __hip_atomic_store(&a.cnt[col], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // ready for the next launch
  }
  __syncthreads();
  const uint64_t part_row0 = static_cast<uint64_t>(p) * a.rpp;
  const uint32_t tail_total = (a.K - 1) * a.S;
  for (uint32_t t = threadIdx.x; t < tail_total; t += blockDim.x) {
    const uint32_t kk = t / a.S, i = t % a.S;
    const uint32_t last = s_seg_last[kk];  // kNone when the segment is all zero
    if (last != kNone && i < last) continue;  // a later non-zero row of its own segment follows: done locally
    const uint32_t c = s_carry[kk];
    const uint32_t val = (c != kNone) ? static_cast<uint32_t>(part_row0 + c) * row_stride + lane_b
                                      : a.sentinel + lane_b;
    a.next[(part_row0 + static_cast<uint64_t>(kk) * a.S + i) * a.lanes + l] = val;
  }
}

}  // namespace
