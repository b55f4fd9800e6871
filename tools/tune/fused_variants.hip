// fused_variants.hip — tuning harness (not the product): k_scan1f shapes (waves per workgroup, loads in flight,
// occupancy floor), timing-only ablations (ABL bit 0: no data stores, bit 1: no flag/next stores) from the product
// source, and the split-batch study kernel k_scan1s, timed side by side by tools/tune_fused.py
// (profiles/r01/tune_round1_session4.md).
#define OMR_NO_CAPI
#include "../../omnireduce-rdma-demo_amd/csrc/omr_kernels.hip"
#include "scan1f_study.h"

namespace {
// k_scan1s — k_scan1f with SPLIT batch ownership (study): batch j (RB rows of the column segment) belongs to wave
// j % WAVES, so the batches in flight at any moment are one contiguous stretch of every column (tools/tune/
// stream_probe.hip: "col split" read 2-3 % faster than the contiguous per-wave ranges).  In-batch successors
// are stored in stream; every batch's tail (rows at and after its last non-zero row) gets its successor after
// one barrier, from an LDS bitmap of non-empty batches (ds_or_b64) and the batches' 16-bit row masks.
template <int VEC, int WAVES, int LOADS = 16, int ABL = 0>
__global__ __launch_bounds__(64 * WAVES) void k_scan1s(FusedArgs a) {
  constexpr int RB = LOADS / VEC;  // rows per batch
  static_assert(RB >= 1 && RB <= 16, "batch bits are 16-bit");
  constexpr uint32_t kMaxBatches = 4096;
  __shared__ uint16_t s_bits[kMaxBatches];
  __shared__ uint64_t s_ne[kMaxBatches / 64];
  __shared__ int s_fix;
  __shared__ uint32_t s_carry[64];
  __shared__ uint32_t s_seg_last[64];
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t T = gridDim.x, bid = blockIdx.x;
  const uint32_t lin = (T % 8 == 0) ? (bid % 8) * (T / 8) + bid / 8 : bid;
  const uint32_t k = lin % a.K, col = lin / a.K;
  const uint32_t l = col % a.lanes, p = col / a.lanes;
  const uint32_t r0 = k * a.S;
  const uint64_t row0 = static_cast<uint64_t>(p) * a.rpp + r0;
  const uint32_t row_bytes = a.lanes * a.block * 4;
  const uint32_t lane_b = l * a.block;
  const uint32_t row_stride = a.lanes * a.block;
  const bool last_seg = (k + 1 == a.K);
  const uint32_t nbt = (a.S + RB - 1) / RB;  // host: nbt <= kMaxBatches
  const uint32_t nw = (nbt + 63) / 64;
  for (uint32_t i = threadIdx.x; i < nw; i += blockDim.x) s_ne[i] = 0;
  __syncthreads();
  for (uint32_t j = wave; j < nbt; j += WAVES) {
    const uint32_t rr = j * RB;
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
    const __amdgpu_buffer_rsrc_t dst =
        chunk_rsrc(a.out + blk0 * a.block, (a.out != nullptr && !(ABL & 1)) ? nrow * row_bytes : 0u);
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
    if (!(ABL & 2) && static_cast<uint32_t>(lane) < nrow) {
      const uint64_t blk = blk0 + static_cast<uint64_t>(lane) * a.lanes;
      if (a.flags != nullptr) a.flags[blk] = static_cast<int32_t>((bits >> lane) & 1u);
      const uint32_t above = bits >> (lane + 1);
      if (above != 0)
        a.next[blk] = static_cast<uint32_t>(row0 + rr + lane + 1 + static_cast<uint32_t>(__builtin_ctz(above))) *
                          row_stride + lane_b;
      if (a.masks != nullptr && ((bits >> lane) & 1u))
        (void)__hip_atomic_fetch_or(&a.masks[row0 + rr + lane], 1ull << l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) {
      s_bits[j] = static_cast<uint16_t>(bits);
      if (bits != 0)
        (void)__hip_atomic_fetch_or(&s_ne[j / 64], 1ull << (j % 64), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  __syncthreads();
  // batch tails: successor = first non-zero row of a later batch of the segment (else a later segment's)
  for (uint32_t j = wave; j < nbt; j += WAVES) {
    const uint32_t rr = j * RB;
    const uint32_t nrow = (a.S - rr < static_cast<uint32_t>(RB)) ? a.S - rr : RB;
    const uint32_t bits = s_bits[j];
    uint32_t succ = kNone;
    uint32_t wi = (j + 1) / 64;
    uint64_t m = wi < nw ? s_ne[wi] & (~0ull << ((j + 1) % 64)) : 0ull;
    while (wi < nw) {
      if (m != 0) {
        const uint32_t j2 = wi * 64 + static_cast<uint32_t>(__builtin_ctzll(m));
        succ = j2 * RB + static_cast<uint32_t>(__builtin_ctz(static_cast<uint32_t>(s_bits[j2])));
        break;
      }
      if (++wi < nw) m = s_ne[wi];
    }
    const uint32_t t0 = bits != 0 ? 31u - static_cast<uint32_t>(__builtin_clz(bits)) : 0u;
    if (!(ABL & 2) && (succ != kNone || last_seg) && static_cast<uint32_t>(lane) >= t0 &&
        static_cast<uint32_t>(lane) < nrow) {
      const uint32_t val = succ != kNone ? static_cast<uint32_t>(row0 + succ) * row_stride + lane_b : a.sentinel + lane_b;
      a.next[(row0 + rr + lane) * a.lanes + l] = val;
    }
  }
  if (a.K == 1) return;
  if (threadIdx.x == 0) {
    uint32_t first = kNone, last = kNone;
    for (uint32_t wi = 0; wi < nw; ++wi)
      if (s_ne[wi] != 0) {
        const uint32_t j2 = wi * 64 + static_cast<uint32_t>(__builtin_ctzll(s_ne[wi]));
        first = j2 * RB + static_cast<uint32_t>(__builtin_ctz(static_cast<uint32_t>(s_bits[j2])));
        break;
      }
    for (uint32_t wi = nw; wi-- > 0;)
      if (s_ne[wi] != 0) {
        const uint32_t j2 = wi * 64 + 63u - static_cast<uint32_t>(__builtin_clzll(s_ne[wi]));
        last = j2 * RB + 31u - static_cast<uint32_t>(__builtin_clz(static_cast<uint32_t>(s_bits[j2])));
        break;
      }
    const uint64_t sm = (static_cast<uint64_t>(first) << 32) | last;
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
    const uint32_t val = (c != kNone) ? static_cast<uint32_t>(part_row0 + c) * row_stride + lane_b
                                      : a.sentinel + lane_b;
    a.next[(part_row0 + static_cast<uint64_t>(kk) * a.S + i) * a.lanes + l] = val;
  }
}

template <int VEC, int W, int LOADS, int ABL>
void go_s(const Layout& L, const FusedShape& f, FusedArgs a, hipStream_t st) {
  const unsigned grid = static_cast<unsigned>(static_cast<uint64_t>(L.parts) * L.lanes * f.K);
  k_scan1s<VEC, W, LOADS, ABL><<<grid, 64 * W, 0, st>>>(a);
}
}  // namespace

namespace {
// Pure read with k_scan1f's geometry and workgroup -> column mapping (no ballots, stores or barrier): the floor
// the fused kernel's read stream could reach (tools/tune/stream_probe.hip "col contig xcd").  Timing only.
template <int VEC, int W>
__global__ __launch_bounds__(64 * W) void k_read_geom(FusedArgs a) {
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
  if (acc == 0x12345678u) a.next[0] = acc;  // never true for nz_bits of the generator's data; keeps the loads
}

template <int VEC, int W, int LOADS, int ABL>
void go_r(const Layout& L, const FusedShape& f, FusedArgs a, hipStream_t st) {
  const unsigned grid = static_cast<unsigned>(static_cast<uint64_t>(L.parts) * L.lanes * f.K);
  k_read_geom<VEC, W><<<grid, 64 * W, 0, st>>>(a);
}
}  // namespace

namespace {
// k_scan1p — k_scan1f with the next batch's loads issued BEFORE the current batch's stores (study).  On gfx9
// stores count in vmcnt, so in k_scan1f the wait for batch i+1's first load also waits for batch i's stores to be
// acknowledged; here the prefetched loads are older than those stores and the wait covers the loads only.  Two
// register sets (LOADS x 2 dwordx4 per lane).  Same outputs as k_scan1f (next offsets in stream, K = 1 only).
template <int VEC, int WAVES, int LOADS, int ABL>
__global__ __launch_bounds__(64 * WAVES) void k_scan1p(FusedArgs a) {
  constexpr int RB = LOADS / VEC;
  static_assert(RB >= 1 && RB <= 32, "batch bits are 32-bit");
  __shared__ uint32_t s_wfirst[WAVES], s_wlast[WAVES];
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t T = gridDim.x, bid = blockIdx.x;
  const uint32_t col = (T % 8 == 0) ? (bid % 8) * (T / 8) + bid / 8 : bid;  // K = 1
  const uint32_t l = col % a.lanes, p = col / a.lanes;
  const uint64_t row0 = static_cast<uint64_t>(p) * a.rpp;
  const uint32_t row_bytes = a.lanes * a.block * 4;
  const uint32_t lane_b = l * a.block;
  const uint32_t row_stride = a.lanes * a.block;
  const uint32_t rw = ((a.S + WAVES * RB - 1) / (WAVES * RB)) * RB;
  const uint32_t lo = wave * rw < a.S ? wave * rw : a.S;
  const uint32_t hi = lo + rw < a.S ? lo + rw : a.S;
  uint32_t carry = kNone, wlast = kNone;
  auto load = [&](uint32_t nb_, v4f (&v)[RB][VEC]) {
    const uint32_t rr = lo + (nb_ - 1) * RB;
    const uint32_t nrow = (hi - rr < static_cast<uint32_t>(RB)) ? hi - rr : RB;
    const uint64_t blk0 = (row0 + rr) * a.lanes + l;
    const __amdgpu_buffer_rsrc_t src = chunk_rsrc(a.x + blk0 * a.block, nrow * row_bytes);
#pragma unroll
    for (int s = 0; s < RB; ++s)
#pragma unroll
      for (int q = 0; q < VEC; ++q)
        v[s][q] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(
                                              src, s * row_bytes + (q * 64 + lane) * 16, 0, kLoadAux));
  };
  auto ballots = [&](uint32_t nb_, const v4f (&v)[RB][VEC]) -> uint32_t {
    const uint32_t rr = lo + (nb_ - 1) * RB;
    const uint32_t nrow = (hi - rr < static_cast<uint32_t>(RB)) ? hi - rr : RB;
    uint32_t bits = 0;
#pragma unroll
    for (int s = 0; s < RB; ++s) {
      uint32_t o = 0;
#pragma unroll
      for (int q = 0; q < VEC; ++q) o |= nz_bits(v[s][q]);
      bits |= static_cast<uint32_t>(wave_ballot(o != 0) != 0 && static_cast<uint32_t>(s) < nrow) << s;
    }
    return bits;
  };
  auto store = [&](uint32_t nb_, const v4f (&v)[RB][VEC], uint32_t bits) {
    const uint32_t rr = lo + (nb_ - 1) * RB;
    const uint32_t nrow = (hi - rr < static_cast<uint32_t>(RB)) ? hi - rr : RB;
    const uint64_t blk0 = (row0 + rr) * a.lanes + l;
    const __amdgpu_buffer_rsrc_t dst =
        chunk_rsrc(a.out + blk0 * a.block, (a.out != nullptr && !(ABL & 1)) ? nrow * row_bytes : 0u);
#pragma unroll
    for (int s = 0; s < RB; ++s) {
      const uint32_t drop = (((bits >> s) & 1u) || (rr + s) == 0) ? 0u : kDropStore;
#pragma unroll
      for (int q = 0; q < VEC; ++q)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, add4(v4f{0.f, 0.f, 0.f, 0.f}, v[s][q])), dst,
                                               (s * row_bytes + (q * 64 + lane) * 16) | drop, 0, kStoreAux);
    }
    if (!(ABL & 2) && static_cast<uint32_t>(lane) < nrow) {
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
  };
  v4f va[RB][VEC], vb[RB][VEC];
  const uint32_t nbt = (hi - lo + RB - 1) / RB;
  if (nbt > 0) load(nbt, va);
  for (uint32_t nb_ = nbt; nb_ > 0;) {
    uint32_t bits = ballots(nb_, va);
    if (nb_ > 1) load(nb_ - 1, vb);  // issued before this batch's stores
    store(nb_, va, bits);
    if (--nb_ == 0) break;
    bits = ballots(nb_, vb);
    if (nb_ > 1) load(nb_ - 1, va);
    store(nb_, vb, bits);
    --nb_;
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
  if (!(ABL & 2)) {
    const uint32_t val = succ != kNone ? static_cast<uint32_t>(row0 + succ) * row_stride + lane_b : a.sentinel + lane_b;
    for (uint32_t i = (wlast == kNone ? lo : wlast) + lane; i < hi; i += 64) a.next[(row0 + i) * a.lanes + l] = val;
  }
}

template <int VEC, int W, int LOADS, int ABL>
void go_p(const Layout& L, const FusedShape& f, FusedArgs a, hipStream_t st) {
  if (f.K != 1) return;  // study kernel: one segment per column only
  const unsigned grid = static_cast<unsigned>(static_cast<uint64_t>(L.parts) * L.lanes);
  k_scan1p<VEC, W, LOADS, ABL><<<grid, 64 * W, 0, st>>>(a);
}
}  // namespace

namespace {
template <int VEC, int W, int LOADS, int ABL, int MINW = 1, int SAUX = kStoreAux>
void go_f(const Layout& L, const FusedShape& f, FusedArgs a, hipStream_t st) {
  const unsigned grid = static_cast<unsigned>(static_cast<uint64_t>(L.parts) * L.lanes * f.K);
  k_scan1f_study<VEC, W, LOADS, ABL, MINW, SAUX><<<grid, 64 * W, 0, st>>>(a);
}

// the product's B = 1024 form (SKIP: a batch with no block to write skips its dropped stores)
template <int VEC, int W, int LOADS>
void go_fs(const Layout& L, const FusedShape& f, FusedArgs a, hipStream_t st) {
  const unsigned grid = static_cast<unsigned>(static_cast<uint64_t>(L.parts) * L.lanes * f.K);
  k_scan1f_study<VEC, W, LOADS, 0, 1, kStoreAux, 1><<<grid, 64 * W, 0, st>>>(a);
}

struct Variant {
  const char* name;
  bool checked;  // produces the full outputs (ablations do not)
  void (*v1)(const Layout&, const FusedShape&, FusedArgs, hipStream_t);
  void (*v4)(const Layout&, const FusedShape&, FusedArgs, hipStream_t);
};

#define VF(W, LD, A) go_f<1, W, LD, A>, go_f<4, W, LD, A>
#define VS(W, LD, A) go_s<1, W, LD, A>, go_s<4, W, LD, A>
#define VO(W, LD, A, O) go_f<1, W, LD, A, O>, go_f<4, W, LD, A, O>
#define VR(W) go_r<1, W, 16, 0>, go_r<4, W, 16, 0>
#define VP(W, LD, A) go_p<1, W, LD, A>, go_p<4, W, LD, A>
#define VA(SA) go_f<1, 16, 16, 0, 1, SA>, go_f<4, 16, 16, 0, 1, SA>
const Variant kVariants[] = {
    {"pipe w16 L8", true, VP(16, 8, 0)},
    {"pipe w8 L16", true, VP(8, 16, 0)},
    {"pipe w16 L16", true, VP(16, 16, 0)},
    {"pipe w8 L8", true, VP(8, 8, 0)},
    {"pipe w16 L8 -data-meta", false, VP(16, 8, 3)},
    {"w16 L8", true, VF(16, 8, 0)},
    {"pure read, k_scan1f geometry", false, VR(16)},
    {"w16 L16", true, VF(16, 16, 0)},
    {"w16 L16 -data", false, VF(16, 16, 1)},
    {"w16 L16 -meta", false, VF(16, 16, 2)},
    {"w16 L16 -data-meta", false, VF(16, 16, 3)},
    {"w16 L16 st plain", true, VA(0)},
    {"w16 L16 st sc0", true, VA(1)},
    {"w16 L16 st sc1", true, VA(16)},
    {"w16 L16 st nt", true, VA(2)},
    {"w16 L16 st sc0sc1nt", true, VA(19)},
    {"w16 L16 st sc0sc1 (product)", true, VA(17)},
    {"w16 L16 st sc1nt", true, VA(18)},
    {"w16 L16 skip (product at B=1024)", true, go_fs<1, 16, 16>, go_fs<4, 16, 16>},
    {"w8 L16 skip", true, go_fs<1, 8, 16>, go_fs<4, 8, 16>},
};
constexpr int kNumVariants = sizeof(kVariants) / sizeof(kVariants[0]);
}  // namespace

extern "C" {
uint32_t omr_sentinel(uint32_t block_size, uint32_t num_lanes) {  // the product's, compiled out by OMR_NO_CAPI
  return (UINT32_MAX / block_size / num_lanes - 1u) * num_lanes * block_size;
}
int tune_fused_count(void) { return kNumVariants; }
const char* tune_fused_name(int v) { return (v >= 0 && v < kNumVariants) ? kVariants[v].name : "?"; }
int tune_fused_checked(int v) { return (v >= 0 && v < kNumVariants) ? kVariants[v].checked : 0; }
int tune_fused(int v, const float* x, float* out, int32_t* flags, uint32_t* next, void* ws, uint64_t n, uint32_t B,
               uint32_t K, void* stream) {
  Layout L;
  if (v < 0 || v >= kNumVariants) return -3;
  if (make_layout(n, B, 16384 / B, 8, &L)) return -1;
  FusedShape f;
  f.K = K;
  f.S = L.rows_per_part / K;
  FusedArgs a{};  // every field zero: masks = nullptr unless set (k_scan1f ORs row masks when non-null)
  a.x = x; a.out = out; a.flags = flags; a.next = next;
  const uint64_t cols = static_cast<uint64_t>(L.parts) * L.lanes;
  a.cnt = static_cast<uint32_t*>(ws);
  a.summary = reinterpret_cast<uint64_t*>(static_cast<char*>(ws) + ((cols * 4 + 15) / 16) * 16);
  a.lanes = L.lanes; a.rpp = L.rows_per_part; a.K = f.K; a.S = f.S; a.block = L.block;
  a.sentinel = omr_sentinel(L.block, L.lanes);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (L.vec == 4) kVariants[v].v4(L, f, a, st);
  else if (L.vec == 1) kVariants[v].v1(L, f, a, st);
  else return -2;
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
}
