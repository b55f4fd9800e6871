// fused_r02.hip — tuning harness (not the product), round 2: variants of the single-pass worker step, each checked
// bit for bit against the product k_scan1f (or marked timing-only) and timed side by side, in place, by
// tools/tune_r02.py; per-workgroup timelines by tools/wg_timeline.py.  All measured slower or equal:
//   k_scan1d  stores issued after the next batch's loads
//   k_scan1g  a workgroup per row range owning all 16 lanes (B = 1024), contiguous flag/next runs
//   k_scan1w  a writer wave: 15 waves only read, the 16th issues every store (LDS rings)
//   k_scan1e  the workgroup's stores stashed in LDS and written after its last read
//   k_scan1q  persistent waves and per-XCD work queues with stealing (XCD balancing)
//   k_scan1s  K = 2 segments split unequally over an XCD pair (XCD balancing)
// plus the product's ablations (ABL bits: no data stores, no flag/next stores, data stores to one block,
// per-workgroup timestamps, rotated XCD map), flag/next store policies (MAUX), the pure read of the geometry and
// flat mixed read/write probes.
#define OMR_NO_CAPI
#include "../../omnireduce-rdma-demo_amd/csrc/omr_kernels.hip"
#include "scan1f_study.h"

namespace {
// k_scan1d — k_scan1f with decoupled stores (study; slower on MI355X: profiles/r02/tune_r02_*.log).
//
// Same work split, outputs and next-offset resolution as k_scan1f; only the ORDER of the memory operations differs.
// On gfx9 a wave's vmcnt counts loads and stores together and retires them in issue order, so in k_scan1f the wait
// for batch i+1's first load also waits for batch i's stores (data and flag/next) to be acknowledged — and a
// write-through store queued behind a saturating read stream is acknowledged late (the memory side favours reads).
// Here the blocks a batch must write (non-zero blocks and lane heads) are copied into P spare register slots, the
// NEXT batch's loads are issued, and only then are the batch's stores issued: the next wait covers the loads alone.
// A batch with more than P blocks to write stores the extra ones before the next loads (k_scan1f's behaviour, for
// those batches only).  Every store slot is issued every batch (unused slots and masked lanes are pointed past their
// descriptor's range and dropped), so the number of memory operations after each batch's loads is static and the
// compiler's vmcnt for a load never includes a younger store.
template <int VEC, int WAVES, int LOADS = 16, int P = 4, bool MASKS = false, int ABL = 0>
__global__ __launch_bounds__(64 * WAVES) void k_scan1d(FusedArgs a) {
  constexpr int RB = LOADS / VEC;  // rows per batch (<= 32)
  static_assert(RB >= 1 && RB <= 32, "batch bits are 32-bit");
  static_assert(P >= 1 && P <= RB, "spare slots");
  __shared__ uint32_t s_wfirst[WAVES], s_wlast[WAVES];
  __shared__ int s_fix;
  __shared__ uint32_t s_carry[64];
  __shared__ uint32_t s_seg_last[64];
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t T = gridDim.x, bid = blockIdx.x;
  const uint32_t lin = (T % 8 == 0) ? (bid % 8) * (T / 8) + bid / 8 : bid;
  const uint32_t k = lin % a.K, col = lin / a.K;
  const uint32_t l = col % a.lanes, p = col / a.lanes;
  const uint32_t r0 = k * a.S;                                  // segment's first row within the partition
  const uint64_t row0 = static_cast<uint64_t>(p) * a.rpp + r0;  // its global row
  const uint32_t row_bytes = a.lanes * a.block * 4;
  const uint32_t lane_b = l * a.block;
  const uint32_t row_stride = a.lanes * a.block;
  const uint32_t meta_stride = a.lanes * 4;  // bytes between one column's consecutive flag / next entries
  const bool last_seg = (k + 1 == a.K);
  const uint32_t rw = ((a.S + WAVES * RB - 1) / (WAVES * RB)) * RB;
  const uint32_t lo = wave * rw < a.S ? wave * rw : a.S;
  const uint32_t hi = lo + rw < a.S ? lo + rw : a.S;
  const uint32_t nbt = (hi - lo + RB - 1) / RB;
  const uint32_t lane16 = static_cast<uint32_t>(lane) * 16u;
  const bool data_out = a.out != nullptr && !(ABL & 1);
  uint32_t carry = kNone, wlast = kNone;

  v4f v[RB][VEC];
  auto load_batch = [&](uint32_t nb_) {
    const uint32_t rr = lo + (nb_ - 1) * RB;
    const uint32_t nrow = (hi - rr < static_cast<uint32_t>(RB)) ? hi - rr : RB;
    const __amdgpu_buffer_rsrc_t src = chunk_rsrc(a.x + ((row0 + rr) * a.lanes + l) * a.block, nrow * row_bytes);
#pragma unroll
    for (int s = 0; s < RB; ++s)
#pragma unroll
      for (int q = 0; q < VEC; ++q)
        v[s][q] = __builtin_bit_cast(
            v4f, __builtin_amdgcn_raw_buffer_load_b128(src, s * row_bytes + q * 1024 + lane16, 0, kLoadAux));
  };

  // the previous batch's stores, issued after the next batch's loads
  v4f sp[P][VEC];
  uint32_t sp_row[P];  // wave-uniform: row of slot j within its batch, kNone = slot unused
  __amdgpu_buffer_rsrc_t p_dst = chunk_rsrc(a.out, 0u);
  __amdgpu_buffer_rsrc_t p_flags = __builtin_amdgcn_make_buffer_rsrc(a.flags, 0, 0, 0x00020000);
  __amdgpu_buffer_rsrc_t p_next = __builtin_amdgcn_make_buffer_rsrc(a.next, 0, 0, 0x00020000);
  uint32_t p_flag_off = kDropStore, p_next_off = kDropStore, p_flag = 0, p_next_val = 0;
  uint64_t p_mask_row = 0;
  bool p_mask = false;
#pragma unroll
  for (int j = 0; j < P; ++j) {
    sp_row[j] = kNone;
#pragma unroll
    for (int q = 0; q < VEC; ++q) sp[j][q] = v4f{0.f, 0.f, 0.f, 0.f};  // defined data: the prologue's stores stay
  }
  auto issue_stores = [&]() {
    if constexpr (MASKS) {
      if (p_mask) (void)__hip_atomic_fetch_or(&a.masks[p_mask_row], 1ull << l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __builtin_amdgcn_raw_buffer_store_b32(p_flag, p_flags, p_flag_off, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32(p_next_val, p_next, p_next_off, 0, 0);
#pragma unroll
    for (int j = 0; j < P; ++j)
#pragma unroll
      for (int q = 0; q < VEC; ++q)
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(v4u, sp[j][q]), p_dst,
            (sp_row[j] != kNone ? sp_row[j] * row_bytes : kDropStore + j * VEC * 1024) + q * 1024 + lane16, 0,
            kStoreAux);
  };

  if (nbt > 0) load_batch(nbt);
  issue_stores();  // every slot dropped: the same operation count follows every batch's loads
  for (uint32_t nb_ = nbt; nb_ > 0; --nb_) {
    const uint32_t rr = lo + (nb_ - 1) * RB;
    const uint32_t nrow = (hi - rr < static_cast<uint32_t>(RB)) ? hi - rr : RB;
    const uint64_t blk0 = (row0 + rr) * a.lanes + l;  // block of the batch's first row
    uint32_t bits = 0;
#pragma unroll
    for (int s = 0; s < RB; ++s) {
      uint32_t o = 0;
#pragma unroll
      for (int q = 0; q < VEC; ++q) o |= nz_bits(v[s][q]);
      bits |= static_cast<uint32_t>(wave_ballot(o != 0) != 0 && static_cast<uint32_t>(s) < nrow) << s;
    }
    // blocks to write: non-zero ones and the lane head (row 0 of the partition, always sent: client.cc:201-205);
    // aggregated block 0.0f + x (server.cc:148-150 zero, :97-98 add), in place (client.cc:89)
    const uint32_t need = bits | ((r0 + rr) == 0 ? 1u : 0u);
    const __amdgpu_buffer_rsrc_t dst = chunk_rsrc(a.out + blk0 * a.block, data_out ? nrow * row_bytes : 0u);
    uint32_t cnt = 0;
#pragma unroll
    for (int j = 0; j < P; ++j) sp_row[j] = kNone;
#pragma unroll
    for (int s = 0; s < RB; ++s) {
      if ((need >> s) & 1u) {
        if (cnt < static_cast<uint32_t>(P)) {
#pragma unroll
          for (int j = 0; j < P; ++j)
            if (cnt == static_cast<uint32_t>(j)) {
#pragma unroll
              for (int q = 0; q < VEC; ++q) sp[j][q] = add4(v4f{0.f, 0.f, 0.f, 0.f}, v[s][q]);
              sp_row[j] = static_cast<uint32_t>(s);
            }
          ++cnt;
        } else {  // more blocks than spare slots: stored before the next loads
#pragma unroll
          for (int q = 0; q < VEC; ++q)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, add4(v4f{0.f, 0.f, 0.f, 0.f}, v[s][q])),
                                                   dst, s * row_bytes + q * 1024 + lane16, 0, kStoreAux);
        }
      }
    }
    // flag and next offset of row rr+lane: successor = next set bit above it in this batch, else the carry
    // (client.cc:19-31)
    const bool mine = static_cast<uint32_t>(lane) < nrow && !(ABL & 2);
    const uint32_t above = static_cast<uint32_t>(static_cast<uint64_t>(bits) >> (lane + 1));
    const uint32_t nr = above != 0 ? rr + lane + 1 + static_cast<uint32_t>(__builtin_ctz(above)) : carry;
    p_flag = (bits >> lane) & 1u;
    p_flag_off = (mine && a.flags != nullptr) ? static_cast<uint32_t>(lane) * meta_stride : kDropStore;
    p_next_val = static_cast<uint32_t>(row0 + nr) * row_stride + lane_b;
    p_next_off = (mine && nr != kNone) ? static_cast<uint32_t>(lane) * meta_stride : kDropStore;
    p_flags = __builtin_amdgcn_make_buffer_rsrc(a.flags + blk0, 0, a.flags != nullptr ? static_cast<int>(nrow * meta_stride) : 0,
                                                0x00020000);
    p_next = __builtin_amdgcn_make_buffer_rsrc(a.next + blk0, 0, static_cast<int>(nrow * meta_stride), 0x00020000);
    p_dst = dst;
    if constexpr (MASKS) {
      p_mask = mine && ((bits >> lane) & 1u);
      p_mask_row = row0 + rr + lane;
    }
    if (bits != 0) {
      if (wlast == kNone) wlast = rr + 31 - static_cast<uint32_t>(__builtin_clz(bits));
      carry = rr + static_cast<uint32_t>(__builtin_ctz(bits));
    }
    if (nb_ > 1) load_batch(nb_ - 1);
    issue_stores();
  }
  if (lane == 0) {
    s_wfirst[wave] = carry;  // first non-zero row of the wave's range (kNone: all zero)
    s_wlast[wave] = wlast;   // last one
  }
  __syncthreads();
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

// Pure read with k_scan1f's geometry and workgroup -> column mapping: the floor of the fused kernel's read stream.
template <int VEC, int W>
__global__ __launch_bounds__(64 * W) void k_read_geom2(FusedArgs a) {
  constexpr int RB = 16 / VEC;
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t T = gridDim.x, bid = blockIdx.x;
  const uint32_t lin = (T % 8 == 0) ? (bid % 8) * (T / 8) + bid / 8 : bid;
  const uint32_t k = lin % a.K, col = lin / a.K;
  const uint32_t l = col % a.lanes, p = col / a.lanes;
  const uint64_t row0 = static_cast<uint64_t>(p) * a.rpp + k * a.S;
  const uint32_t row_bytes = a.lanes * a.block * 4;
  const uint32_t rw = ((a.S + W * RB - 1) / (W * RB)) * RB;
  const uint32_t lo = wave * rw < a.S ? wave * rw : a.S;
  const uint32_t hi = lo + rw < a.S ? lo + rw : a.S;
  uint32_t acc = 0;
  for (uint32_t nb_ = (hi - lo + RB - 1) / RB; nb_ > 0; --nb_) {
    const uint32_t rr = lo + (nb_ - 1) * RB;
    const uint32_t nrow = (hi - rr < static_cast<uint32_t>(RB)) ? hi - rr : RB;
    const uint64_t blk0 = (row0 + rr) * a.lanes + l;
    const __amdgpu_buffer_rsrc_t src = chunk_rsrc(a.x + blk0 * a.block, nrow * row_bytes);
    v4f v[RB][VEC];
#pragma unroll
    for (int s = 0; s < RB; ++s)
#pragma unroll
      for (int q = 0; q < VEC; ++q)
        v[s][q] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(
                                              src, s * row_bytes + (q * 64 + lane) * 16, 0, kLoadAux));
#pragma unroll
    for (int s = 0; s < RB; ++s)
#pragma unroll
      for (int q = 0; q < VEC; ++q) acc |= nz_bits(v[s][q]);
  }
  if (acc == 0x12345678u) a.next[0] = acc;  // never true for the generator's data; keeps the loads
}

// k_scan1g — the single-pass worker step for NB = 16 lanes (B = 1024), with a workgroup per (partition, row
// segment) owning ALL 16 lane columns of its rows: wave w streams column w of the segment backwards (as k_scan1f's
// waves do), and each batch's flags / next offsets (RB rows x 16 lanes) are staged in LDS and stored by the workgroup
// as contiguous 64-byte row runs, instead of 4-byte stores 64 bytes apart from 16 different workgroups.  The row
// masks (multi-rank round) become one plain 8-byte store per row.  A row whose successor lies in a later segment is
// left to that column's fix-up, as in k_scan1f (no double writes).
constexpr uint32_t kUnset = 0xFFFFFFFFu;  // "successor in a later segment": stored by the fix-up, not here
template <int VEC, int LOADS = 16>
__global__ __launch_bounds__(1024) void k_scan1g(FusedArgs a) {
  constexpr int W = 16;            // waves = lane columns
  constexpr int RB = LOADS / VEC;  // rows per batch
  static_assert(RB >= 1 && RB <= 32 && 2 * RB * W + RB <= 1024, "batch");
  __shared__ uint32_t s_next[2][RB][W];
  __shared__ int32_t s_flag[2][RB][W];
  __shared__ uint32_t s_first[W][64], s_last[W][64];
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t T = gridDim.x, bid = blockIdx.x;
  const uint32_t lin = (T % 8 == 0) ? (bid % 8) * (T / 8) + bid / 8 : bid;
  const uint32_t k = lin % a.K, p = lin / a.K + a.part0;
  const uint32_t l = wave, col = p * a.lanes + l;
  const uint32_t r0 = k * a.S;
  const uint64_t row0 = static_cast<uint64_t>(p) * a.rpp + r0;
  const uint32_t row_bytes = a.lanes * a.block * 4;
  const uint32_t lane_b = l * a.block;
  const uint32_t row_stride = a.lanes * a.block;
  const bool last_seg = (k + 1 == a.K);
  uint32_t carry = kNone, wlast = kNone;
  int buf = 0;
  for (uint32_t nb_ = (a.S + RB - 1) / RB; nb_ > 0; --nb_, buf ^= 1) {
    const uint32_t rr = (nb_ - 1) * RB;
    const uint32_t nrow = (a.S - rr < static_cast<uint32_t>(RB)) ? a.S - rr : RB;
    const uint64_t blk0 = (row0 + rr) * a.lanes + l;
    const __amdgpu_buffer_rsrc_t src = chunk_rsrc(a.x + blk0 * a.block, nrow * row_bytes);
    v4f v[RB][VEC];
#pragma unroll
    for (int s = 0; s < RB; ++s)
#pragma unroll
      for (int q = 0; q < VEC; ++q)
        v[s][q] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(
                                              src, s * row_bytes + (q * 64 + lane) * 16, 0, kLoadAux));
    const __amdgpu_buffer_rsrc_t dst = chunk_rsrc(a.out + blk0 * a.block, a.out != nullptr ? nrow * row_bytes : 0u);
    uint32_t bits = 0;
#pragma unroll
    for (int s = 0; s < RB; ++s) {
      uint32_t o = 0;
#pragma unroll
      for (int q = 0; q < VEC; ++q) o |= nz_bits(v[s][q]);
      const bool nz = wave_ballot(o != 0) != 0 && static_cast<uint32_t>(s) < nrow;
      bits |= static_cast<uint32_t>(nz) << s;
      const bool head = (r0 + rr + s) == 0;
      const uint32_t drop = (nz || head) ? 0u : kDropStore;
#pragma unroll
      for (int q = 0; q < VEC; ++q)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, add4(v4f{0.f, 0.f, 0.f, 0.f}, v[s][q])), dst,
                                               (s * row_bytes + (q * 64 + lane) * 16) | drop, 0, kStoreAux);
    }
    if (static_cast<uint32_t>(lane) < nrow) {
      const uint32_t above = static_cast<uint32_t>(static_cast<uint64_t>(bits) >> (lane + 1));
      const uint32_t nr = above != 0 ? rr + lane + 1 + static_cast<uint32_t>(__builtin_ctz(above)) : carry;
      s_flag[buf][lane][l] = static_cast<int32_t>((bits >> lane) & 1u);
      s_next[buf][lane][l] = nr != kNone ? static_cast<uint32_t>(row0 + nr) * row_stride + lane_b
                                         : (last_seg ? a.sentinel + lane_b : kUnset);
    }
    if (bits != 0) {
      if (wlast == kNone) wlast = rr + 31 - static_cast<uint32_t>(__builtin_clz(bits));
      carry = rr + static_cast<uint32_t>(__builtin_ctz(bits));
    }
    __syncthreads();  // the batch's RB x 16 flags / next offsets are in LDS (double-buffered: one barrier per batch)
    const uint32_t t = threadIdx.x;
    if (t < nrow * W) {
      const uint64_t g = (row0 + rr + t / W) * a.lanes + t % W;
      if (a.flags != nullptr) a.flags[g] = s_flag[buf][t / W][t % W];
    } else if (t >= 256 && t < 256 + nrow * W) {
      const uint32_t u = t - 256;
      const uint32_t nv = s_next[buf][u / W][u % W];
      if (nv != kUnset) a.next[(row0 + rr + u / W) * a.lanes + u % W] = nv;
    } else if (a.masks != nullptr && t >= 512 && t < 512 + nrow) {
      const uint32_t r = t - 512;
      uint64_t m = 0;
#pragma unroll
      for (int c = 0; c < W; ++c) m |= static_cast<uint64_t>(s_flag[buf][r][c] & 1) << c;
      a.masks[row0 + rr + r] = m;
    }
  }
  if (a.K == 1) return;
  // multi-segment columns: every store of this workgroup done, then each wave publishes its column's {first, last}
  // and counts arrivals; the wave whose arrival completes its column fixes the rows whose successor lies in a later
  // segment (k_scan1f's fix-up, one wave per column)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  uint32_t fix = 0;
  if (lane == 0) {
    const uint64_t sm = (static_cast<uint64_t>(carry) << 32) | (carry == kNone ? kNone : wlast);
    (void)__hip_atomic_exchange(&a.summary[static_cast<uint64_t>(col) * a.K + k], sm, __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t old = __hip_atomic_fetch_add(&a.cnt[col], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    fix = (old == a.K - 1) ? 1u : 0u;
  }
  fix = __builtin_amdgcn_readfirstlane(fix);
  if (!fix) return;
  if (static_cast<uint32_t>(lane) < a.K) {
    const uint64_t sm = __hip_atomic_fetch_or(&a.summary[static_cast<uint64_t>(col) * a.K + lane], 0ull,
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_first[l][lane] = static_cast<uint32_t>(sm >> 32);
    s_last[l][lane] = static_cast<uint32_t>(sm);
  }
  __builtin_amdgcn_wave_barrier();
  if (lane == 0) {  // s_first[l][kk] := first non-zero row (partition-relative) in segments after kk
    uint32_t c = kNone;
    for (int kk = static_cast<int>(a.K) - 1; kk >= 0; --kk) {
      const uint32_t first = s_first[l][kk];
      s_first[l][kk] = c;
      if (first != kNone) c = static_cast<uint32_t>(kk) * a.S + first;
    }
    __hip_atomic_store(&a.cnt[col], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __builtin_amdgcn_wave_barrier();
  const uint64_t part_row0 = static_cast<uint64_t>(p) * a.rpp;
  const uint32_t tail_total = (a.K - 1) * a.S;
  for (uint32_t t = lane; t < tail_total; t += 64) {
    const uint32_t kk = t / a.S, i = t % a.S;
    const uint32_t last = s_last[l][kk];
    if (last != kNone && i < last) continue;
    const uint32_t c = s_first[l][kk];
    a.next[(part_row0 + static_cast<uint64_t>(kk) * a.S + i) * a.lanes + l] =
        (c != kNone) ? static_cast<uint32_t>(part_row0 + c) * row_stride + lane_b : a.sentinel + lane_b;
  }
}

// Mixed read/write ceiling probes (timing only): what the HBM gives for the kernel's byte mix without any of its
// logic.  Every probe is one grid-stride kernel of 256-thread workgroups, 16 one-KiB pieces in flight per wave.
//   MODE 0  write only: the blocks whose flag is set (the kernel's scattered 1 KiB writes), nothing read but flags
//   MODE 1  write only: the same number of 1 KiB blocks, packed into the first tenth of the buffer (contiguous)
//   MODE 2  read everything + write the flagged blocks (flat address order: the cheapest schedule of the same bytes)
//   MODE 3  read everything, write nothing (flat address order)
template <int MODE, int SAUX = kStoreAux>
__global__ __launch_bounds__(256) void k_mix_probe(FusedArgs a, uint64_t nb) {
  const int lane = threadIdx.x & 63;
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * 4;
  const uint64_t w0 = static_cast<uint64_t>(blockIdx.x) * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const v4f val = v4f{0.01f, 0.01f, 0.01f, 0.01f};
  for (uint64_t c = w0; c * 16 < nb; c += nw) {  // chunk c = blocks [16c, 16c + 16)
    const uint64_t b0 = c * 16;
    uint32_t fl = 0;
    if (lane < 16) fl = a.flags[b0 + lane] != 0 ? 1u : 0u;
    const uint32_t fbits = static_cast<uint32_t>(__ballot(fl != 0));
    if constexpr (MODE >= 2) {
      const __amdgpu_buffer_rsrc_t src = chunk_rsrc(a.x + b0 * 256, 16 * 1024);
      v4f v[16];
#pragma unroll
      for (int s = 0; s < 16; ++s)
        v[s] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(src, s * 1024 + lane * 16, 0, kLoadAux));
      uint32_t acc = 0;
#pragma unroll
      for (int s = 0; s < 16; ++s) acc |= nz_bits(v[s]);
      if constexpr (MODE == 2) {
        const __amdgpu_buffer_rsrc_t dst = chunk_rsrc(a.out + b0 * 256, 16 * 1024);
#pragma unroll
        for (int s = 0; s < 16; ++s)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v[s]), dst,
                                                 (((fbits >> s) & 1u) ? 0u : kDropStore) + s * 1024 + lane * 16, 0,
                                                 SAUX);
      }
      if (acc == 0x12345678u) a.next[0] = acc;  // keeps the loads
    } else {
      const uint64_t wb = MODE == 0 ? b0 : b0 / 10;  // MODE 1: flagged block b goes to block b / 10
      const __amdgpu_buffer_rsrc_t dst = chunk_rsrc(a.out + wb * 256, 16 * 1024);
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const uint32_t off = MODE == 0 ? s * 1024 : static_cast<uint32_t>((b0 + s) / 10 - b0 / 10) * 1024;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, val), dst,
                                               (((fbits >> s) & 1u) ? 0u : kDropStore) + off + lane * 16, 0,
                                               kStoreAux);
      }
    }
  }
}

// k_scan1w — k_scan1f with a WRITER WAVE (study).  Waves 0..WAVES-2 only read: loads, ballots, and LDS.  The last
// wave of the workgroup issues every global store of the workgroup.  On gfx9 a wave's vmcnt counts its loads and
// stores together, in issue order, so in k_scan1f (and in k_scan1d, one batch later) a wave that stores a block
// waits for that store's acknowledgement before it can use its next batch's first load.  At config 3 that costs
// 8.7 us for 11 MB of block writes (DESIGN.md §3.1 ablations): far more than their bandwidth.  Here a reader copies
// its batch's blocks to write (non-zero + lane head) into an LDS ring, and one record per batch {rows, flag bits,
// carry, blocks} into a record ring (one 64-bit LDS atomic hands out both tickets, so records and ring slots are
// consumed in the same order).  The writer takes the records in ticket order and stores the blocks (META = 0) or the
// blocks and the batch's flags / next offsets / row-mask bits (META = 1).  Readers wait only when a ring is full.
template <int VEC, int WAVES, int LOADS = 16, int META = 1, int RING_KB = 32>
__global__ __launch_bounds__(64 * WAVES) void k_scan1w(FusedArgs a) {
  constexpr int RB = LOADS / VEC;
  constexpr uint32_t R = WAVES - 1;  // reader waves; wave R is the writer
  constexpr int BLK4 = 64 * VEC;     // 16-byte vectors per block
  constexpr uint32_t NSLOT = RING_KB * 1024 / (BLK4 * 16);
  constexpr uint32_t NREC = 64;
  static_assert(NSLOT >= static_cast<uint32_t>(RB) && (NSLOT & (NSLOT - 1)) == 0, "ring holds a batch");
  __shared__ v4f s_ring[NSLOT * BLK4];
  __shared__ uint32_t s_rec[NREC][5];  // rr, nrow, bits, carry, wmask
  __shared__ uint32_t s_rready[NREC];
  __shared__ uint64_t s_head;          // records << 32 | ring slots handed out
  __shared__ uint32_t s_rtail, s_btail, s_done;
  __shared__ uint32_t s_wfirst[WAVES], s_wlast[WAVES];
  __shared__ int s_fix;
  __shared__ uint32_t s_carry[64];
  __shared__ uint32_t s_seg_last[64];
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t T = gridDim.x, bid = blockIdx.x;
  const uint32_t lin = (T % 8 == 0) ? (bid % 8) * (T / 8) + bid / 8 : bid;
  const uint32_t k = lin % a.K, col = lin / a.K + a.part0 * a.lanes;
  const uint32_t l = col % a.lanes, p = col / a.lanes;
  const uint32_t r0 = k * a.S;
  const uint64_t row0 = static_cast<uint64_t>(p) * a.rpp + r0;
  const uint32_t row_bytes = a.lanes * a.block * 4;
  const uint32_t lane_b = l * a.block;
  const uint32_t row_stride = a.lanes * a.block;
  const bool last_seg = (k + 1 == a.K);
  const bool data_out = a.out != nullptr;
  if (threadIdx.x == 0) {
    s_head = 0;
    s_rtail = s_btail = s_done = 0;
  }
  if (threadIdx.x < NREC) s_rready[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t rw = ((a.S + R * RB - 1) / (R * RB)) * RB;
  const uint32_t lo = wave < R ? (wave * rw < a.S ? wave * rw : a.S) : a.S;
  const uint32_t hi = wave < R ? (lo + rw < a.S ? lo + rw : a.S) : a.S;
  uint32_t carry = kNone, wlast = kNone;
  // the batch's flag / next / mask stores (k_scan1f's, by whichever wave issues them)
  auto meta_stores = [&](uint32_t rr, uint32_t nrow, uint32_t bits, uint32_t c) {
    if (static_cast<uint32_t>(lane) < nrow) {
      const uint64_t blk = (row0 + rr) * a.lanes + l + static_cast<uint64_t>(lane) * a.lanes;
      if (a.flags != nullptr) a.flags[blk] = static_cast<int32_t>((bits >> lane) & 1u);
      const uint32_t above = static_cast<uint32_t>(static_cast<uint64_t>(bits) >> (lane + 1));
      const uint32_t nr = above != 0 ? rr + lane + 1 + static_cast<uint32_t>(__builtin_ctz(above)) : c;
      if (nr != kNone) a.next[blk] = static_cast<uint32_t>(row0 + nr) * row_stride + lane_b;
      if (a.masks != nullptr && ((bits >> lane) & 1u))
        (void)__hip_atomic_fetch_or(&a.masks[row0 + rr + lane], 1ull << l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  };
  if (wave < R) {
    for (uint32_t nb_ = (hi - lo + RB - 1) / RB; nb_ > 0; --nb_) {
      const uint32_t rr = lo + (nb_ - 1) * RB;
      const uint32_t nrow = (hi - rr < static_cast<uint32_t>(RB)) ? hi - rr : RB;
      const uint64_t blk0 = (row0 + rr) * a.lanes + l;
      const __amdgpu_buffer_rsrc_t src = chunk_rsrc(a.x + blk0 * a.block, nrow * row_bytes);
      v4f v[RB][VEC];
#pragma unroll
      for (int s = 0; s < RB; ++s)
#pragma unroll
        for (int q = 0; q < VEC; ++q)
          v[s][q] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(
                                                src, s * row_bytes + (q * 64 + lane) * 16, 0, kLoadAux));
      uint32_t bits = 0;
#pragma unroll
      for (int s = 0; s < RB; ++s) {
        uint32_t o = 0;
#pragma unroll
        for (int q = 0; q < VEC; ++q) o |= nz_bits(v[s][q]);
        const bool nz = wave_ballot(o != 0) != 0 && static_cast<uint32_t>(s) < nrow;
        bits |= static_cast<uint32_t>(nz) << s;
      }
      const uint32_t wmask = data_out ? (bits | ((r0 + rr) == 0 ? 1u : 0u)) : 0u;
      if (META || wmask != 0) {
        const uint32_t n = static_cast<uint32_t>(__builtin_popcount(wmask));
        uint64_t tk = 0;
        if (lane == 0)
          tk = __hip_atomic_fetch_add(&s_head, (1ull << 32) | n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint32_t rt = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(tk >> 32));
        const uint32_t bt = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(tk));
        while (rt - __hip_atomic_load(&s_rtail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= NREC ||
               bt + n - __hip_atomic_load(&s_btail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) > NSLOT)
          __builtin_amdgcn_s_sleep(1);
        asm volatile("" ::: "memory");  // the ring writes stay behind the space check
        uint32_t t = bt;
#pragma unroll
        for (int s = 0; s < RB; ++s)
          if ((wmask >> s) & 1u) {
            const uint32_t slot = t % NSLOT;
#pragma unroll
            for (int q = 0; q < VEC; ++q) s_ring[slot * BLK4 + q * 64 + lane] = add4(v4f{0.f, 0.f, 0.f, 0.f}, v[s][q]);
            ++t;
          }
        if (lane == 0) {
          uint32_t* rec = s_rec[rt % NREC];
          rec[0] = rr; rec[1] = nrow; rec[2] = bits; rec[3] = carry; rec[4] = wmask;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the record and its blocks are in LDS
        if (lane == 0) __hip_atomic_store(&s_rready[rt % NREC], rt + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      if (!META) meta_stores(rr, nrow, bits, carry);
      if (bits != 0) {
        if (wlast == kNone) wlast = rr + 31 - static_cast<uint32_t>(__builtin_clz(bits));
        carry = rr + static_cast<uint32_t>(__builtin_ctz(bits));
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) (void)__hip_atomic_fetch_add(&s_done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  } else {
    // the writer: records in ticket order until every reader is done and the record ring is drained
    uint32_t rt = 0, bt = 0;
    for (;;) {
      const uint32_t slot = rt % NREC;
      bool have = false;
      for (;;) {
        if (__hip_atomic_load(&s_rready[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == rt + 1) {
          have = true;
          break;
        }
        if (__hip_atomic_load(&s_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == R) {
          have = __hip_atomic_load(&s_rready[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == rt + 1;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (!have) break;
      asm volatile("" ::: "memory");  // the record and ring reads stay behind the ready flag (LDS is in order)
      const uint32_t* rec = s_rec[slot];
      const uint32_t rr = __builtin_amdgcn_readfirstlane(rec[0]);
      const uint32_t nrow = __builtin_amdgcn_readfirstlane(rec[1]);
      const uint32_t bits = __builtin_amdgcn_readfirstlane(rec[2]);
      const uint32_t c = __builtin_amdgcn_readfirstlane(rec[3]);
      uint32_t wm = __builtin_amdgcn_readfirstlane(rec[4]);
      const uint64_t blk0 = (row0 + rr) * a.lanes + l;
      const __amdgpu_buffer_rsrc_t dst = chunk_rsrc(a.out + blk0 * a.block, data_out ? nrow * row_bytes : 0u);
      while (wm != 0) {
        const uint32_t s = static_cast<uint32_t>(__builtin_ctz(wm));
        wm &= wm - 1;
        const uint32_t bslot = bt % NSLOT;
        v4f d[VEC];
#pragma unroll
        for (int q = 0; q < VEC; ++q) d[q] = s_ring[bslot * BLK4 + q * 64 + lane];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        ++bt;
        if (lane == 0) __hip_atomic_store(&s_btail, bt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
        for (int q = 0; q < VEC; ++q)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, d[q]), dst,
                                                 s * row_bytes + (q * 64 + lane) * 16, 0, kStoreAux);
      }
      if (META) meta_stores(rr, nrow, bits, c);
      ++rt;
      if (lane == 0) __hip_atomic_store(&s_rtail, rt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  if (lane == 0) {
    s_wfirst[wave] = carry;
    s_wlast[wave] = wlast;
  }
  __syncthreads();
  uint32_t succ = kNone;
  for (uint32_t w2 = wave + 1; w2 < WAVES; ++w2)
    if (s_wfirst[w2] != kNone) {
      succ = s_wfirst[w2];
      break;
    }
  if (wave < R && (succ != kNone || last_seg)) {
    const uint32_t val = succ != kNone ? static_cast<uint32_t>(row0 + succ) * row_stride + lane_b : a.sentinel + lane_b;
    for (uint32_t i = (wlast == kNone ? lo : wlast) + lane; i < hi; i += 64) a.next[(row0 + i) * a.lanes + l] = val;
  }
  if (a.K == 1) return;
  if (threadIdx.x == 0) {
    uint32_t first = kNone, last = 0;
    for (uint32_t w2 = 0; w2 < WAVES; ++w2) {
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
  if (threadIdx.x < a.K) {
    const uint64_t sm = __hip_atomic_fetch_or(&a.summary[static_cast<uint64_t>(col) * a.K + threadIdx.x], 0ull,
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_carry[threadIdx.x] = static_cast<uint32_t>(sm >> 32);
    s_seg_last[threadIdx.x] = static_cast<uint32_t>(sm);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t c = kNone;
    for (int kk = static_cast<int>(a.K) - 1; kk >= 0; --kk) {
      const uint32_t first = s_carry[kk];
      s_carry[kk] = c;
      if (first != kNone) c = static_cast<uint32_t>(kk) * a.S + first;
    }
    __hip_atomic_store(&a.cnt[col], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  const uint64_t part_row0 = static_cast<uint64_t>(p) * a.rpp;
  const uint32_t tail_total = (a.K - 1) * a.S;
  for (uint32_t t = threadIdx.x; t < tail_total; t += blockDim.x) {
    const uint32_t kk = t / a.S, i = t % a.S;
    const uint32_t last = s_seg_last[kk];
    if (last != kNone && i < last) continue;
    const uint32_t c = s_carry[kk];
    a.next[(part_row0 + static_cast<uint64_t>(kk) * a.S + i) * a.lanes + l] =
        (c != kNone) ? static_cast<uint32_t>(part_row0 + c) * row_stride + lane_b : a.sentinel + lane_b;
  }
}

// k_scan1e — k_scan1f with the workgroup's stores STASHED in LDS and written at its end (study).  The writer-wave
// variant above takes the stores out of the readers' vmcnt queue and still pays ~9 us for config 3's 11 MB of block
// writes: the cost is on the memory side (writes interleaved one block at a time into a saturating read stream),
// not in the waves.  Here every wave keeps reading; the blocks to write (STASH bit 0) and the flag / next values
// (bit 1, segments of <= kStashRows rows) go to LDS, and the workgroup writes them out after its last read — so
// at config 3 (one workgroup per CU, all ending together) the chip's writes form one phase after the reads.  A
// batch whose blocks no longer fit stores them directly, as k_scan1f does.
constexpr uint32_t kStashRows = 2048;
constexpr uint32_t kUnsetNext = 0xFFFFFFFEu;  // successor in a later segment: the column's fix-up stores it
template <int VEC, int WAVES, int LOADS = 16, int STASH = 1, int CAP_KB = 96>
__global__ __launch_bounds__(64 * WAVES) void k_scan1e(FusedArgs a) {
  constexpr int RB = LOADS / VEC;
  constexpr uint32_t BLK4 = 64 * VEC;
  constexpr uint32_t NSLOT = CAP_KB * 1024 / (BLK4 * 16);
  constexpr uint32_t MR = (STASH & 2) ? kStashRows : 1;
  __shared__ v4f s_blk[NSLOT * BLK4];
  __shared__ uint32_t s_bdst[NSLOT];
  __shared__ uint32_t s_mflag[MR], s_mnext[MR];
  __shared__ uint32_t s_bcnt;
  __shared__ uint32_t s_wfirst[WAVES], s_wlast[WAVES];
  __shared__ int s_fix;
  __shared__ uint32_t s_carry[64];
  __shared__ uint32_t s_seg_last[64];
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t T = gridDim.x, bid = blockIdx.x;
  const uint32_t lin = (T % 8 == 0) ? (bid % 8) * (T / 8) + bid / 8 : bid;
  const uint32_t k = lin % a.K, col = lin / a.K + a.part0 * a.lanes;
  const uint32_t l = col % a.lanes, p = col / a.lanes;
  const uint32_t r0 = k * a.S;
  const uint64_t row0 = static_cast<uint64_t>(p) * a.rpp + r0;
  const uint32_t row_bytes = a.lanes * a.block * 4;
  const uint32_t lane_b = l * a.block;
  const uint32_t row_stride = a.lanes * a.block;
  const bool last_seg = (k + 1 == a.K);
  const bool data_out = a.out != nullptr && (STASH & 1);
  const bool mstash = (STASH & 2) && a.S <= MR;
  if (threadIdx.x == 0) s_bcnt = 0;
  __syncthreads();
  const uint32_t rw = ((a.S + WAVES * RB - 1) / (WAVES * RB)) * RB;
  const uint32_t lo = wave * rw < a.S ? wave * rw : a.S;
  const uint32_t hi = lo + rw < a.S ? lo + rw : a.S;
  uint32_t carry = kNone, wlast = kNone;
  for (uint32_t nb_ = (hi - lo + RB - 1) / RB; nb_ > 0; --nb_) {
    const uint32_t rr = lo + (nb_ - 1) * RB;
    const uint32_t nrow = (hi - rr < static_cast<uint32_t>(RB)) ? hi - rr : RB;
    const uint64_t blk0 = (row0 + rr) * a.lanes + l;
    const __amdgpu_buffer_rsrc_t src = chunk_rsrc(a.x + blk0 * a.block, nrow * row_bytes);
    v4f v[RB][VEC];
#pragma unroll
    for (int s = 0; s < RB; ++s)
#pragma unroll
      for (int q = 0; q < VEC; ++q)
        v[s][q] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(
                                              src, s * row_bytes + (q * 64 + lane) * 16, 0, kLoadAux));
    uint32_t bits = 0;
#pragma unroll
    for (int s = 0; s < RB; ++s) {
      uint32_t o = 0;
#pragma unroll
      for (int q = 0; q < VEC; ++q) o |= nz_bits(v[s][q]);
      bits |= static_cast<uint32_t>(wave_ballot(o != 0) != 0 && static_cast<uint32_t>(s) < nrow) << s;
    }
    const uint32_t wmask = (a.out != nullptr) ? (bits | ((r0 + rr) == 0 ? 1u : 0u)) : 0u;
    if (wmask != 0) {
      const uint32_t n = static_cast<uint32_t>(__builtin_popcount(wmask));
      uint32_t t0 = NSLOT;
      if (data_out) {
        uint32_t tk = 0;
        if (lane == 0) tk = __hip_atomic_fetch_add(&s_bcnt, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        t0 = __builtin_amdgcn_readfirstlane(tk);
      }
      if (t0 + n <= NSLOT) {
        uint32_t t = t0;
#pragma unroll
        for (int s = 0; s < RB; ++s)
          if ((wmask >> s) & 1u) {
#pragma unroll
            for (int q = 0; q < VEC; ++q) s_blk[t * BLK4 + q * 64 + lane] = add4(v4f{0.f, 0.f, 0.f, 0.f}, v[s][q]);
            if (lane == 0) s_bdst[t] = static_cast<uint32_t>(blk0 + static_cast<uint64_t>(s) * a.lanes);
            ++t;
          }
      } else {
        if (t0 < NSLOT && static_cast<uint32_t>(lane) < NSLOT - t0) s_bdst[t0 + lane] = kNone;
        const __amdgpu_buffer_rsrc_t dst = chunk_rsrc(a.out + blk0 * a.block, nrow * row_bytes);
#pragma unroll
        for (int s = 0; s < RB; ++s)
          if ((wmask >> s) & 1u) {
#pragma unroll
            for (int q = 0; q < VEC; ++q)
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, add4(v4f{0.f, 0.f, 0.f, 0.f}, v[s][q])),
                                                     dst, s * row_bytes + (q * 64 + lane) * 16, 0, kStoreAux);
          }
      }
    }
    if (static_cast<uint32_t>(lane) < nrow) {
      const uint64_t blk = blk0 + static_cast<uint64_t>(lane) * a.lanes;
      const uint32_t fl = (bits >> lane) & 1u;
      const uint32_t above = static_cast<uint32_t>(static_cast<uint64_t>(bits) >> (lane + 1));
      const uint32_t nr = above != 0 ? rr + lane + 1 + static_cast<uint32_t>(__builtin_ctz(above)) : carry;
      const uint32_t nv = static_cast<uint32_t>(row0 + nr) * row_stride + lane_b;
      if (mstash) {
        s_mflag[rr + lane] = fl;
        s_mnext[rr + lane] = nr != kNone ? nv : kUnsetNext;
      } else {
        if (a.flags != nullptr) a.flags[blk] = static_cast<int32_t>(fl);
        if (nr != kNone) a.next[blk] = nv;
      }
      if (a.masks != nullptr && fl)
        (void)__hip_atomic_fetch_or(&a.masks[row0 + rr + lane], 1ull << l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (bits != 0) {
      if (wlast == kNone) wlast = rr + 31 - static_cast<uint32_t>(__builtin_clz(bits));
      carry = rr + static_cast<uint32_t>(__builtin_ctz(bits));
    }
  }
  if (lane == 0) {
    s_wfirst[wave] = carry;
    s_wlast[wave] = wlast;
  }
  __syncthreads();
  uint32_t succ = kNone;
  for (uint32_t w2 = wave + 1; w2 < WAVES; ++w2)
    if (s_wfirst[w2] != kNone) {
      succ = s_wfirst[w2];
      break;
    }
  if (succ != kNone || last_seg) {
    const uint32_t val = succ != kNone ? static_cast<uint32_t>(row0 + succ) * row_stride + lane_b : a.sentinel + lane_b;
    for (uint32_t i = (wlast == kNone ? lo : wlast) + lane; i < hi; i += 64) {
      if (mstash) s_mnext[i] = val;
      else a.next[(row0 + i) * a.lanes + l] = val;
    }
  }
  __syncthreads();
  // the workgroup's stash, written after its last read
  const uint32_t cnt = s_bcnt < NSLOT ? s_bcnt : NSLOT;
  for (uint32_t j = wave; j < cnt; j += WAVES) {
    const uint32_t d = __builtin_amdgcn_readfirstlane(s_bdst[j]);
    if (d == kNone) continue;
    const __amdgpu_buffer_rsrc_t dst = chunk_rsrc(a.out + static_cast<uint64_t>(d) * a.block, a.block * 4);
#pragma unroll
    for (int q = 0; q < VEC; ++q)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, s_blk[j * BLK4 + q * 64 + lane]), dst,
                                             (q * 64 + lane) * 16, 0, kStoreAux);
  }
  if (mstash) {
    for (uint32_t i = threadIdx.x; i < a.S; i += blockDim.x) {
      const uint64_t blk = (row0 + i) * a.lanes + l;
      if (a.flags != nullptr) a.flags[blk] = static_cast<int32_t>(s_mflag[i]);
      if (s_mnext[i] != kUnsetNext) a.next[blk] = s_mnext[i];
    }
  }
  if (a.K == 1) return;
  if (threadIdx.x == 0) {
    uint32_t first = kNone, last = 0;
    for (uint32_t w2 = 0; w2 < WAVES; ++w2) {
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
  if (threadIdx.x < a.K) {
    const uint64_t sm = __hip_atomic_fetch_or(&a.summary[static_cast<uint64_t>(col) * a.K + threadIdx.x], 0ull,
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_carry[threadIdx.x] = static_cast<uint32_t>(sm >> 32);
    s_seg_last[threadIdx.x] = static_cast<uint32_t>(sm);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t c = kNone;
    for (int kk = static_cast<int>(a.K) - 1; kk >= 0; --kk) {
      const uint32_t first = s_carry[kk];
      s_carry[kk] = c;
      if (first != kNone) c = static_cast<uint32_t>(kk) * a.S + first;
    }
    __hip_atomic_store(&a.cnt[col], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  const uint64_t part_row0 = static_cast<uint64_t>(p) * a.rpp;
  const uint32_t tail_total = (a.K - 1) * a.S;
  for (uint32_t t = threadIdx.x; t < tail_total; t += blockDim.x) {
    const uint32_t kk = t / a.S, i = t % a.S;
    const uint32_t last = s_seg_last[kk];
    if (last != kNone && i < last) continue;
    const uint32_t c = s_carry[kk];
    a.next[(part_row0 + static_cast<uint64_t>(kk) * a.S + i) * a.lanes + l] =
        (c != kNone) ? static_cast<uint32_t>(part_row0 + c) * row_stride + lane_b : a.sentinel + lane_b;
  }
}

// k_scan1q — k_scan1f with the work balanced across XCDs at run time (study).  Workgroups go to XCDs round-robin
// by ID, so a static column split gives every XCD the same bytes; tools/wg_timeline.py shows the XCDs then finish up
// to 20 % apart (config 3: the last workgroup of the fastest XCD ends 135.7 us after the start, of the slowest
// 170.4 us), and the launch lasts as long as the slowest.  Here persistent waves take items (CR rows of one column)
// from eight queues, one per XCD and starting with their own (a partition per queue, its items chunk by chunk so
// that the waves of one XCD stream the same rows of all lanes), and move to the next queue when theirs runs dry.
// A wave streams its item as k_scan1f's waves stream their ranges (backwards, next offsets in-stream with a carry),
// publishes the item's {first, last} non-zero row with a device-scope atomic, and counts the column's arrivals; the
// wave that completes a column writes every next offset whose successor lies in a later item (a suffix minimum
// over the column's items, one lane per item).  The last wave out re-arms the queues for the next launch.
// FusedArgs reuse: K = partitions; cnt = [cols] arrival counters, then 8 queue counters and the exit counter;
// summary = [cols][rpp / CR].
template <int VEC, int WAVES, int LOADS = 16, int NBATCH = 2, int SKIP = 0>
__global__ __launch_bounds__(64 * WAVES) void k_scan1q(FusedArgs a) {
  constexpr int RB = LOADS / VEC;
  constexpr uint32_t CR = RB * NBATCH;  // rows per item
  const int lane = threadIdx.x & 63;
  const uint32_t parts = a.K;
  const uint32_t ncol = parts * a.lanes;
  const uint32_t nch = a.rpp / CR;  // items per column (<= 64)
  const uint32_t per_p = a.lanes * nch;
  const uint32_t total = ncol * nch;
  const uint32_t per_q = (total + 7) / 8;
  uint32_t* qc = a.cnt + ncol;
  uint32_t* exits = qc + 8;
  const uint32_t row_bytes = a.lanes * a.block * 4;
  const uint32_t row_stride = a.lanes * a.block;
  uint32_t q = static_cast<uint32_t>(__builtin_amdgcn_s_getreg((15 << 11) | 20)) & 7u;  // HW_REG_XCC_ID
  uint32_t tried = 0;
  for (;;) {
    uint32_t i = kNone;
    while (tried < 8) {
      uint32_t j = 0;
      if (lane == 0) j = __hip_atomic_fetch_add(&qc[q], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      j = __builtin_amdgcn_readfirstlane(j);
      if (j < per_q && q * per_q + j < total) {
        i = q * per_q + j;
        break;
      }
      q = (q + 1) & 7u;
      ++tried;
    }
    if (i == kNone) break;
    const uint32_t p = i / per_p, rem = i % per_p;
    const uint32_t chunk = rem / a.lanes, l = rem % a.lanes;
    const uint32_t col = p * a.lanes + l;
    const uint32_t r0 = chunk * CR;                               // partition-relative first row of the item
    const uint64_t prow0 = static_cast<uint64_t>(p) * a.rpp;      // the partition's first global row
    const uint64_t row0 = prow0 + r0;
    const uint32_t lane_b = l * a.block;
    uint32_t carry = kNone, wlast = kNone;  // item-relative rows
#pragma unroll 1
    for (uint32_t nb_ = NBATCH; nb_ > 0; --nb_) {
      const uint32_t rr = (nb_ - 1) * RB;
      const uint64_t blk0 = (row0 + rr) * a.lanes + l;
      const __amdgpu_buffer_rsrc_t src = chunk_rsrc(a.x + blk0 * a.block, RB * row_bytes);
      v4f v[RB][VEC];
#pragma unroll
      for (int s = 0; s < RB; ++s)
#pragma unroll
        for (int qq = 0; qq < VEC; ++qq)
          v[s][qq] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(
                                                 src, s * row_bytes + (qq * 64 + lane) * 16, 0, kLoadAux));
      const __amdgpu_buffer_rsrc_t dst = chunk_rsrc(a.out + blk0 * a.block, a.out != nullptr ? RB * row_bytes : 0u);
      uint32_t bits = 0;
#pragma unroll
      for (int s = 0; s < RB; ++s) {
        uint32_t o = 0;
#pragma unroll
        for (int qq = 0; qq < VEC; ++qq) o |= nz_bits(v[s][qq]);
        bits |= static_cast<uint32_t>(wave_ballot(o != 0) != 0) << s;
      }
      const uint32_t need = bits | ((r0 + rr) == 0 ? 1u : 0u);  // + the lane head (client.cc:201-205)
      if (!SKIP || need != 0) {
#pragma unroll
        for (int s = 0; s < RB; ++s) {
          const uint32_t drop = ((need >> s) & 1u) ? 0u : kDropStore;
#pragma unroll
          for (int qq = 0; qq < VEC; ++qq)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, add4(v4f{0.f, 0.f, 0.f, 0.f}, v[s][qq])),
                                                   dst, (s * row_bytes + (qq * 64 + lane) * 16) | drop, 0, kStoreAux);
        }
      }
      if (static_cast<uint32_t>(lane) < static_cast<uint32_t>(RB)) {
        const uint64_t blk = blk0 + static_cast<uint64_t>(lane) * a.lanes;
        if (a.flags != nullptr) a.flags[blk] = static_cast<int32_t>((bits >> lane) & 1u);
        const uint32_t above = static_cast<uint32_t>(static_cast<uint64_t>(bits) >> (lane + 1));
        const uint32_t nr = above != 0 ? rr + lane + 1 + static_cast<uint32_t>(__builtin_ctz(above)) : carry;
        if (nr != kNone) a.next[blk] = static_cast<uint32_t>(row0 + nr) * row_stride + lane_b;
        if (a.masks != nullptr && ((bits >> lane) & 1u))
          (void)__hip_atomic_fetch_or(&a.masks[row0 + rr + lane], 1ull << l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (bits != 0) {
        if (wlast == kNone) wlast = rr + 31 - static_cast<uint32_t>(__builtin_clz(bits));
        carry = rr + static_cast<uint32_t>(__builtin_ctz(bits));
      }
    }
    // the item's {first, last} non-zero row (partition-relative), then its arrival; the arrival waits for the
    // summary's return, so the column's last arriver reads every item's summary
    const uint32_t f_abs = carry == kNone ? kNone : r0 + carry;
    const uint32_t l_abs = wlast == kNone ? kNone : r0 + wlast;
    uint32_t old = 0;
    if (lane == 0) {
      const uint64_t prev = __hip_atomic_exchange(&a.summary[static_cast<uint64_t>(col) * nch + chunk],
                                                  (static_cast<uint64_t>(f_abs) << 32) | l_abs, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
      old = __hip_atomic_fetch_add(&a.cnt[col], 1u + static_cast<uint32_t>(prev == 0x5a5a5a5a5a5a5a5aull),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    old = __builtin_amdgcn_readfirstlane(old);
    if (old != nch - 1) continue;
    // the column's last item: next offsets of every row whose successor lies in a later item
    uint64_t sm = ~0ull;
    if (static_cast<uint32_t>(lane) < nch)
      sm = __hip_atomic_fetch_or(&a.summary[static_cast<uint64_t>(col) * nch + lane], 0ull, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t first = static_cast<uint32_t>(sm >> 32), last = static_cast<uint32_t>(sm);
    uint32_t suf = first;  // inclusive suffix minimum over items >= lane
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t o = __shfl_down(suf, off, 64);
      if (lane + off < 64) suf = o < suf ? o : suf;
    }
    uint32_t cy = __shfl_down(suf, 1, 64);  // first non-zero row in a later item
    if (lane == 63) cy = kNone;
    const uint32_t start = last == kNone ? static_cast<uint32_t>(lane) * CR : last;
    for (uint32_t j = 0; j < nch; ++j) {
      const uint32_t cj = __builtin_amdgcn_readlane(cy, j), sj = __builtin_amdgcn_readlane(start, j);
      const uint32_t val = cj != kNone ? static_cast<uint32_t>(prow0 + cj) * row_stride + lane_b : a.sentinel + lane_b;
      for (uint32_t r = sj + lane; r < (j + 1) * CR; r += 64) a.next[(prow0 + r) * a.lanes + l] = val;
    }
    if (lane == 0) __hip_atomic_store(&a.cnt[col], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (lane == 0) {
    const uint32_t o = __hip_atomic_fetch_add(exits, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (o == gridDim.x * WAVES - 1) {  // every wave is out of the queues: re-arm them for the next launch
      for (int k2 = 0; k2 < 8; ++k2) __hip_atomic_store(&qc[k2], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(exits, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// k_scan1s — k_scan1f at K = 2 with the two segments of a column on an XCD pair (study).  tools/wg_timeline.py shows
// the odd XCDs stream 10-15 % slower than the even ones at config 3 whatever partition they read (the rotated map
// moves the partitions, not the slowness).  Here XCD 2i takes segment 0 (rows [0, S0)) and XCD 2i+1 segment 1
// (rows [S0, rpp)) of the same columns, with S0 = rpp * PM / 1000, so the slower XCD of each pair streams fewer rows.
// K = 2 only; the column's second arriver writes the rows of segment 0 whose successor lies in segment 1.
template <int VEC, int WAVES, int PM, int SKIP>
__global__ __launch_bounds__(64 * WAVES) void k_scan1s(FusedArgs a) {
  constexpr int RB = 16 / VEC;
  __shared__ uint32_t s_wfirst[WAVES], s_wlast[WAVES];
  __shared__ int s_fix;
  __shared__ uint64_t s_sm[2];
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t T = gridDim.x, bid = blockIdx.x;
  const uint32_t x = bid % 8, jw = bid / 8;
  const uint32_t k = x & 1u, col = (x >> 1) * (T / 8) + jw;
  const uint32_t l = col % a.lanes, p = col / a.lanes;
  const uint32_t S0 = ((a.rpp * PM / 1000) / RB) * RB;
  const uint32_t r0 = k ? S0 : 0u, S = k ? a.rpp - S0 : S0;
  const uint64_t row0 = static_cast<uint64_t>(p) * a.rpp + r0;
  const uint32_t row_bytes = a.lanes * a.block * 4;
  const uint32_t lane_b = l * a.block;
  const uint32_t row_stride = a.lanes * a.block;
  const uint32_t rw = ((S + WAVES * RB - 1) / (WAVES * RB)) * RB;
  const uint32_t lo = wave * rw < S ? wave * rw : S;
  const uint32_t hi = lo + rw < S ? lo + rw : S;
  uint32_t carry = kNone, wlast = kNone;
  for (uint32_t nb_ = (hi - lo + RB - 1) / RB; nb_ > 0; --nb_) {
    const uint32_t rr = lo + (nb_ - 1) * RB;
    const uint32_t nrow = (hi - rr < static_cast<uint32_t>(RB)) ? hi - rr : RB;
    const uint64_t blk0 = (row0 + rr) * a.lanes + l;
    const __amdgpu_buffer_rsrc_t src = chunk_rsrc(a.x + blk0 * a.block, nrow * row_bytes);
    v4f v[RB][VEC];
#pragma unroll
    for (int s = 0; s < RB; ++s)
#pragma unroll
      for (int q = 0; q < VEC; ++q)
        v[s][q] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(
                                              src, s * row_bytes + (q * 64 + lane) * 16, 0, kLoadAux));
    const __amdgpu_buffer_rsrc_t dst = chunk_rsrc(a.out + blk0 * a.block, a.out != nullptr ? nrow * row_bytes : 0u);
    uint32_t bits = 0;
#pragma unroll
    for (int s = 0; s < RB; ++s) {
      uint32_t o = 0;
#pragma unroll
      for (int q = 0; q < VEC; ++q) o |= nz_bits(v[s][q]);
      bits |= static_cast<uint32_t>(wave_ballot(o != 0) != 0 && static_cast<uint32_t>(s) < nrow) << s;
    }
    const uint32_t need = bits | ((r0 + rr) == 0 ? 1u : 0u);
    if (!SKIP || need != 0) {
#pragma unroll
      for (int s = 0; s < RB; ++s) {
        const uint32_t drop = ((need >> s) & 1u) ? 0u : kDropStore;
#pragma unroll
        for (int q = 0; q < VEC; ++q)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, add4(v4f{0.f, 0.f, 0.f, 0.f}, v[s][q])),
                                                 dst, (s * row_bytes + (q * 64 + lane) * 16) | drop, 0, kStoreAux);
      }
    }
    if (static_cast<uint32_t>(lane) < nrow) {
      const uint64_t blk = blk0 + static_cast<uint64_t>(lane) * a.lanes;
      if (a.flags != nullptr) a.flags[blk] = static_cast<int32_t>((bits >> lane) & 1u);
      const uint32_t above = static_cast<uint32_t>(static_cast<uint64_t>(bits) >> (lane + 1));
      const uint32_t nr = above != 0 ? rr + lane + 1 + static_cast<uint32_t>(__builtin_ctz(above)) : carry;
      if (nr != kNone) a.next[blk] = static_cast<uint32_t>(row0 + nr) * row_stride + lane_b;
    }
    if (bits != 0) {
      if (wlast == kNone) wlast = rr + 31 - static_cast<uint32_t>(__builtin_clz(bits));
      carry = rr + static_cast<uint32_t>(__builtin_ctz(bits));
    }
  }
  if (lane == 0) {
    s_wfirst[wave] = carry;
    s_wlast[wave] = wlast;
  }
  __syncthreads();
  uint32_t succ = kNone;
  for (uint32_t w2 = wave + 1; w2 < WAVES; ++w2)
    if (s_wfirst[w2] != kNone) {
      succ = s_wfirst[w2];
      break;
    }
  if (succ != kNone || k == 1) {
    const uint32_t val = succ != kNone ? static_cast<uint32_t>(row0 + succ) * row_stride + lane_b : a.sentinel + lane_b;
    for (uint32_t i = (wlast == kNone ? lo : wlast) + lane; i < hi; i += 64) a.next[(row0 + i) * a.lanes + l] = val;
  }
  if (threadIdx.x == 0) {
    uint32_t first = kNone, last = 0;
    for (uint32_t w2 = 0; w2 < WAVES; ++w2) {
      if (first == kNone) first = s_wfirst[w2];
      if (s_wlast[w2] != kNone) last = s_wlast[w2];
    }
    const uint64_t sm = (static_cast<uint64_t>(first) << 32) | (first == kNone ? kNone : last);
    (void)__hip_atomic_exchange(&a.summary[static_cast<uint64_t>(col) * 2 + k], sm, __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t old = __hip_atomic_fetch_add(&a.cnt[col], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_fix = (old == 1);
    if (old == 1) {
      s_sm[0] = __hip_atomic_fetch_or(&a.summary[static_cast<uint64_t>(col) * 2], 0ull, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
      s_sm[1] = __hip_atomic_fetch_or(&a.summary[static_cast<uint64_t>(col) * 2 + 1], 0ull, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&a.cnt[col], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  if (!s_fix) return;
  // rows of segment 0 at or after its last non-zero row: successor = segment 1's first non-zero row, else sentinel
  const uint32_t last0 = static_cast<uint32_t>(s_sm[0]), first1 = static_cast<uint32_t>(s_sm[1] >> 32);
  const uint64_t prow0 = static_cast<uint64_t>(p) * a.rpp;
  const uint32_t val = first1 != kNone ? static_cast<uint32_t>(prow0 + S0 + first1) * row_stride + lane_b
                                       : a.sentinel + lane_b;
  for (uint32_t i = (last0 == kNone ? 0u : last0) + threadIdx.x; i < S0; i += blockDim.x)
    a.next[(prow0 + i) * a.lanes + l] = val;
}

using Launch = void (*)(const Layout&, const FusedShape&, FusedArgs, hipStream_t);

unsigned grid_of(const Layout& L, const FusedShape& f) {
  return static_cast<unsigned>(static_cast<uint64_t>(L.parts) * L.lanes * f.K);
}
unsigned g_occ = 0;  // workgroups per CU forced through dynamic LDS (0 = registers and workgroup size decide)

template <typename K>
unsigned occ_lds(K kern) {
  if (!g_occ) return 0;
  const unsigned lds = (160u * 1024u / g_occ - 4096u) & ~255u;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                            static_cast<int>(lds));
  return lds;
}
template <int VEC, int W, int LD, int ABL, int SAUX = kStoreAux, int SKIP = 0>
void go_f(const Layout& L, const FusedShape& f, FusedArgs a, hipStream_t st) {
  const unsigned lds = occ_lds(&k_scan1f_study<VEC, W, LD, ABL, 1, SAUX, SKIP>);
  k_scan1f_study<VEC, W, LD, ABL, 1, SAUX, SKIP><<<grid_of(L, f), 64 * W, lds, st>>>(a);
}
template <int VEC, int W, int SKIP, int MAUX>
void go_fm(const Layout& L, const FusedShape& f, FusedArgs a, hipStream_t st) {
  k_scan1f_study<VEC, W, 16, 0, 1, kStoreAux, SKIP, MAUX><<<grid_of(L, f), 64 * W, 0, st>>>(a);
}
template <int VEC, int W, int LD, int P, int ABL>
void go_d(const Layout& L, const FusedShape& f, FusedArgs a, hipStream_t st) {
  k_scan1d<VEC, W, LD, P, false, ABL><<<grid_of(L, f), 64 * W, 0, st>>>(a);
}
template <int VEC, int W, int LD, int META>
void go_w(const Layout& L, const FusedShape& f, FusedArgs a, hipStream_t st) {
  k_scan1w<VEC, W, LD, META><<<grid_of(L, f), 64 * W, 0, st>>>(a);
}
template <int VEC, int W, int ST, int CAP>
void go_e(const Layout& L, const FusedShape& f, FusedArgs a, hipStream_t st) {
  k_scan1e<VEC, W, 16, ST, CAP><<<grid_of(L, f), 64 * W, 0, st>>>(a);
}
template <int VEC, int W, int NBATCH, int SKIP>
void go_q(const Layout& L, const FusedShape&, FusedArgs a, hipStream_t st) {
  constexpr int RB = 16 / VEC;
  if (L.rows_per_part % (RB * NBATCH) != 0 || L.rows_per_part / (RB * NBATCH) > 64) return;
  int per_cu = 0, dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(&k_scan1q<VEC, W, 16, NBATCH, SKIP>),
                                                     64 * W, 0);
  // K = partitions; arrival + queue counters at 128 KiB into the workspace (clear of the product's K > 1 state),
  // summaries at 256 KiB
  a.K = L.parts;
  a.summary = reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(a.cnt) + (256u << 10));
  a.cnt = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(a.cnt) + (128u << 10));
  k_scan1q<VEC, W, 16, NBATCH, SKIP><<<static_cast<unsigned>(cus * (per_cu > 0 ? per_cu : 1)), 64 * W, 0, st>>>(a);
}
template <int VEC, int W, int PM, int SKIP>
void go_s(const Layout& L, const FusedShape&, FusedArgs a, hipStream_t st) {
  const uint64_t cols = static_cast<uint64_t>(L.parts) * L.lanes;
  if (cols % 32 != 0) return;  // every XCD pair takes cols / 4 columns
  a.cnt = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(a.cnt) + (384u << 10));
  a.summary = reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(a.cnt) + (64u << 10));
  k_scan1s<VEC, W, PM, SKIP><<<static_cast<unsigned>(cols * 2), 64 * W, 0, st>>>(a);
}
template <int VEC, int W>
void go_r(const Layout& L, const FusedShape& f, FusedArgs a, hipStream_t st) {
  k_read_geom2<VEC, W><<<grid_of(L, f), 64 * W, 0, st>>>(a);
}
template <int VEC, int LD>
void go_g(const Layout& L, const FusedShape& f, FusedArgs a, hipStream_t st) {
  if (L.lanes != 16) return;  // B = 1024 only
  k_scan1g<VEC, LD><<<static_cast<unsigned>(static_cast<uint64_t>(L.parts) * f.K), 1024, 0, st>>>(a);
}
template <int MODE, int SAUX = kStoreAux>
void go_m(const Layout& L, const FusedShape&, FusedArgs a, hipStream_t st) {
  if (L.block != 256) return;  // B = 256 probes only
  k_mix_probe<MODE, SAUX><<<2048, 256, 0, st>>>(a, L.nb);
}

struct Variant {
  const char* name;
  bool checked;  // produces the full outputs (ablations do not)
  Launch v1, v4;
};
const Variant kVariants[] = {
    {"f w16 L16 (product)", true, go_f<1, 16, 16, 0>, go_f<4, 16, 16, 0>},
    {"f w16 L16 skip-empty-batch stores", true, go_f<1, 16, 16, 0, kStoreAux, 1>, go_f<4, 16, 16, 0, kStoreAux, 1>},
    {"g rowgroup L16 (B=1024)", true, go_f<1, 16, 16, 0>, go_g<4, 16>},
    {"f w4 L32", true, go_f<1, 4, 32, 0>, go_f<4, 4, 32, 0>},
    {"f w8 L32", true, go_f<1, 8, 32, 0>, go_f<4, 8, 32, 0>},
    {"f w4 L16", true, go_f<1, 4, 16, 0>, go_f<4, 4, 16, 0>},
    {"f w8 L16", true, go_f<1, 8, 16, 0>, go_f<4, 8, 16, 0>},
    {"f w16 L16 nt-st", true, go_f<1, 16, 16, 0, 2>, go_f<4, 16, 16, 0, 2>},
    {"f w4 L32 nt-st", true, go_f<1, 4, 32, 0, 2>, go_f<4, 4, 32, 0, 2>},
    {"pure read", false, go_r<1, 16>, go_r<4, 16>},
    {"d w16 L16 P4/P2", true, go_d<1, 16, 16, 4, 0>, go_d<4, 16, 16, 2, 0>},
    {"d w16 L16 P2/P1", true, go_d<1, 16, 16, 2, 0>, go_d<4, 16, 16, 1, 0>},
    {"d w16 L16 P4/P2 -data", false, go_d<1, 16, 16, 4, 1>, go_d<4, 16, 16, 2, 1>},
    {"f w16 L16 -data-meta", false, go_f<1, 16, 16, 3>, go_f<4, 16, 16, 3>},
    {"f w16 L16 -data", false, go_f<1, 16, 16, 1>, go_f<4, 16, 16, 1>},
    {"f w16 L16 -meta", false, go_f<1, 16, 16, 2>, go_f<4, 16, 16, 2>},
    {"probe write scattered flagged blocks", false, go_m<0>, go_m<0>},
    {"probe write same count contiguous", false, go_m<1>, go_m<1>},
    {"probe flat read + write flagged", false, go_m<2>, go_m<2>},
    {"probe flat read", false, go_m<3>, go_m<3>},
    {"probe flat read + write flagged, plain st", false, go_m<2, 0>, go_m<2, 0>},
    {"probe flat read + write flagged, nt st", false, go_m<2, 2>, go_m<2, 2>},
    {"probe flat read + write flagged, sc1 st", false, go_m<2, 16>, go_m<2, 16>},
    {"w16 writer wave: blocks", true, go_w<1, 16, 16, 0>, go_w<4, 16, 16, 0>},
    {"w16 writer wave: blocks + meta", true, go_w<1, 16, 16, 1>, go_w<4, 16, 16, 1>},
    {"w8 writer wave: blocks + meta", true, go_w<1, 8, 16, 1>, go_w<4, 8, 16, 1>},
    {"e stash blocks 96K", true, go_e<1, 16, 1, 96>, go_e<4, 16, 1, 96>},
    {"e stash blocks + meta 96K", true, go_e<1, 16, 3, 96>, go_e<4, 16, 3, 96>},
    {"e stash meta only", true, go_e<1, 16, 2, 4>, go_e<4, 16, 2, 4>},
    {"e stash blocks + meta 128K", true, go_e<1, 16, 3, 128>, go_e<4, 16, 3, 128>},
    {"f meta st plain (buffer)", true, go_fm<1, 16, 0, 0>, go_fm<4, 16, 1, 0>},
    {"f meta st sc0 sc1", true, go_fm<1, 16, 0, 17>, go_fm<4, 16, 1, 17>},
    {"f meta st nt", true, go_fm<1, 16, 0, 2>, go_fm<4, 16, 1, 2>},
    {"f meta st sc1", true, go_fm<1, 16, 0, 16>, go_fm<4, 16, 1, 16>},
    {"f meta st sc0", true, go_fm<1, 16, 0, 1>, go_fm<4, 16, 1, 1>},
    {"f meta st nt sc1", true, go_fm<1, 16, 0, 18>, go_fm<4, 16, 1, 18>},
    {"f skip data st to one block (ablation)", false, go_f<1, 16, 16, 4, kStoreAux, 0>, go_f<4, 16, 16, 4, kStoreAux, 1>},
    {"f skip -meta", false, go_f<1, 16, 16, 2, kStoreAux, 0>, go_f<4, 16, 16, 2, kStoreAux, 1>},
    {"f skip -data", false, go_f<1, 16, 16, 1, kStoreAux, 0>, go_f<4, 16, 16, 1, kStoreAux, 1>},
    {"f skip plain st", true, go_f<1, 16, 16, 0, 0, 0>, go_f<4, 16, 16, 0, 0, 1>},
    {"f skip data to one block, plain st (ablation)", false, go_f<1, 16, 16, 4, 0, 0>, go_f<4, 16, 16, 4, 0, 1>},
    {"timeline product", false, go_f<1, 16, 16, 8, kStoreAux, 0>, go_f<4, 16, 16, 8, kStoreAux, 1>},
    {"timeline -data", false, go_f<1, 16, 16, 9, kStoreAux, 0>, go_f<4, 16, 16, 9, kStoreAux, 1>},
    {"timeline -data-meta", false, go_f<1, 16, 16, 11, kStoreAux, 0>, go_f<4, 16, 16, 11, kStoreAux, 1>},
    {"timeline -data-meta rotated", false, go_f<1, 16, 16, 27, kStoreAux, 0>, go_f<4, 16, 16, 27, kStoreAux, 1>},
    {"s xcd pair 500", true, go_s<1, 16, 500, 0>, go_s<4, 16, 500, 1>},
    {"s xcd pair 530", true, go_s<1, 16, 530, 0>, go_s<4, 16, 530, 1>},
    {"s xcd pair 545", true, go_s<1, 16, 545, 0>, go_s<4, 16, 545, 1>},
    {"s xcd pair 560", true, go_s<1, 16, 560, 0>, go_s<4, 16, 560, 1>},
    {"q queues w4 CR32", true, go_q<1, 4, 2, 0>, go_q<4, 4, 8, 1>},
    {"q queues w16 CR32", true, go_q<1, 16, 2, 0>, go_q<4, 16, 8, 1>},
    {"q queues w4 CR64/32", true, go_q<1, 4, 4, 0>, go_q<4, 4, 8, 1>},
};
constexpr int kNumVariants = sizeof(kVariants) / sizeof(kVariants[0]);
}  // namespace

extern "C" {
uint32_t omr_sentinel(uint32_t block_size, uint32_t num_lanes) {  // the product's, compiled out by OMR_NO_CAPI
  return (UINT32_MAX / block_size / num_lanes - 1u) * num_lanes * block_size;
}
int tune_count(void) { return kNumVariants; }
const char* tune_name(int v) { return (v >= 0 && v < kNumVariants) ? kVariants[v].name : "?"; }
int tune_checked(int v) { return (v >= 0 && v < kNumVariants) ? kVariants[v].checked : 0; }
int tune_run(int v, const float* x, float* out, int32_t* flags, uint32_t* next, void* ws, uint64_t n, uint32_t B,
             uint32_t K, uint32_t occ, void* stream) {
  g_occ = occ;
  Layout L;
  if (v < 0 || v >= kNumVariants) return -3;
  if (make_layout(n, B, 16384 / B, 8, &L)) return -1;
  FusedShape f;
  f.K = K;
  f.S = L.rows_per_part / K;
  FusedArgs a{};
  a.x = x; a.out = out; a.flags = flags; a.next = next;
  const uint64_t cols = static_cast<uint64_t>(L.parts) * L.lanes;
  a.cnt = static_cast<uint32_t*>(ws);
  a.summary = reinterpret_cast<uint64_t*>(static_cast<char*>(ws) + ((cols * 4 + 15) / 16) * 16);
  a.lanes = L.lanes; a.rpp = L.rows_per_part; a.K = f.K; a.S = f.S; a.block = L.block;
  a.sentinel = omr_sentinel(L.block, L.lanes);
  // timeline variants: per-workgroup timestamps in the second half of the workspace (in place of the row masks)
  if (strncmp(kVariants[v].name, "timeline", 8) == 0) a.masks = reinterpret_cast<uint64_t*>(static_cast<char*>(ws) + (512u << 10));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (L.vec == 4) kVariants[v].v4(L, f, a, st);
  else if (L.vec == 1) kVariants[v].v1(L, f, a, st);
  else return -2;
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
}
