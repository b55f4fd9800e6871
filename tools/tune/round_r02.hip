// round_r02.hip — tuning harness (not the product): the multi-rank round's aggregator shard sum.
//
// The product's k_shard_sum loads one contributor's blocks of a batch, waits, adds, then the next contributor's:
// with m workers a batch costs m dependent round trips.  k_shard_sum_all issues every contributor's loads of the
// batch at once (MC contributors x SL blocks, a contributor without the block reads through a dropped offset: a zero
// that leaves a sum started at +0.0 unchanged), then adds in rank order, so a batch costs one round trip whatever m.
// tools/tune_round_r02.py times both (and the product's pack, k_move) at an 8-worker shard and at world 1, and checks
// the variant against the product bit for bit.
#define OMR_NO_CAPI
#include "../../omnireduce-rdma-demo_amd/csrc/omr_kernels.hip"
#include "scan1f_study.h"

namespace {
// The round-2 product shard sum (kept here as the comparison point; the product's k_shard_sum since round 3 builds a
// flat (block, contributor) list per unit and issues all its loads at once).
// Aggregator shard sum over rows [r0, r1) of the write set (server.cc:83-99 with the RDMA hop replaced by the
// transport): for every write-set block, ((0.0f + x_a0) + x_a1) + ... over the workers whose mask has it, in
// rank order.  Worker `me`'s contribution is read in place from its dense tensor `own`; worker a's from its
// received stream at recv + recv_off[a] blocks (its shard blocks in block order).  Output dense (block
// position, in place) or packed (write-set order of the shard, for the sums' return trip).
struct ShardArgs {
  const float* own;
  const float* recv;
  uint64_t recv_off[OMR_MAX_WORKERS];
  const uint64_t* masks;  // [count][rows]
  const uint32_t* prefix;  // [count + 1][rows + 1]; index count = write set
  const uint64_t* write_set;
  float* out;
  uint64_t rows, r0, r1;
  uint32_t count, me, lanes, block, packed_out, lg;
};

template <int VEC>
__global__ __launch_bounds__(kWGThreads) void k_shard_sum_r02(ShardArgs a) {
  constexpr int SL = (8 / VEC) < 2 ? 2 : 8 / VEC;  // blocks per batch
  const int lane = threadIdx.x & 63;
  const uint32_t groups = a.lanes / a.lg;
  const uint32_t bbytes = a.block * 4;
  const uint64_t units = (a.r1 - a.r0) * groups;
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * kWavesPerWG;
  const uint32_t* pws = a.prefix + static_cast<uint64_t>(a.count) * (a.rows + 1);
  const uint64_t cmask = a.count >= 64 ? ~0ull : ((1ull << a.count) - 1ull);
  for (uint64_t u = static_cast<uint64_t>(blockIdx.x) * kWavesPerWG + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
       u < units; u += nw) {
    const uint64_t r = a.r0 + u / groups;
    const uint32_t g0 = static_cast<uint32_t>(u % groups) * a.lg;
    // every index load of the unit issued together (one round trip before the data loads): the write-set row and
    // its prefix, and on lane c < count worker c's mask and stream prefixes
    const bool cl = static_cast<uint32_t>(lane) < a.count;
    const uint32_t* pc = a.prefix + static_cast<uint64_t>(cl ? lane : 0) * (a.rows + 1);
    const uint64_t w = a.write_set[r];
    const uint64_t mc = cl ? a.masks[static_cast<uint64_t>(lane) * a.rows + r] : 0ull;
    const uint32_t pcr = pc[r], pcr0 = pc[a.r0];
    const uint32_t pwr = pws[r], pwr0 = pws[a.r0];
    uint64_t rem = w & (below(g0 + a.lg) & ~below(g0));
    if (rem == 0) continue;
    // lane c: the first block of row r in worker c's stream
    const uint64_t kc0 = cl ? a.recv_off[lane] + (pcr - pcr0) : 0ull;
    uint64_t kw = pwr - pwr0 + static_cast<uint64_t>(__builtin_popcountll(w & below(g0)));
    float* orow = a.out + r * a.lanes * a.block;
    while (rem != 0) {
      uint32_t lj[SL];
      uint64_t bm;
      const uint32_t nv = take_bits<SL>(rem, lj, bm);
      v4f acc[SL][VEC];
#pragma unroll
      for (int j = 0; j < SL; ++j)
#pragma unroll
        for (int q = 0; q < VEC; ++q) acc[j][q] = v4f{0.f, 0.f, 0.f, 0.f};
      // contributors of the batch in rank order; each worker's (up to SL) blocks loaded at once
      uint64_t cont = __ballot((mc & bm) != 0) & cmask;
      while (cont != 0) {
        const uint32_t c = static_cast<uint32_t>(__builtin_ctzll(cont));
        cont &= cont - 1;
        const uint64_t m_c = readlane64(mc, c);
        const bool mine = c == a.me;
        const __amdgpu_buffer_rsrc_t src =
            mine ? chunk_rsrc(a.own + r * a.lanes * a.block, a.lanes * bbytes)
                 : chunk_rsrc(a.recv + readlane64(kc0, c) * a.block,
                              static_cast<uint32_t>(__builtin_popcountll(m_c)) * bbytes);
        v4f v[SL][VEC];
#pragma unroll
        for (int j = 0; j < SL; ++j) {
          const bool has = static_cast<uint32_t>(j) < nv && ((m_c >> lj[j]) & 1u);
          const uint32_t off = (mine ? lj[j] : static_cast<uint32_t>(__builtin_popcountll(m_c & below(lj[j])))) * bbytes;
#pragma unroll
          for (int q = 0; q < VEC; ++q)
            v[j][q] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(
                                                  src, (off + (q * 64 + lane) * 16) | (has ? 0u : kDropStore), 0,
                                                  kLoadAux));
        }
#pragma unroll
        for (int j = 0; j < SL; ++j)
          if (static_cast<uint32_t>(j) < nv && ((m_c >> lj[j]) & 1u)) {
#pragma unroll
            for (int q = 0; q < VEC; ++q) acc[j][q] = add4(acc[j][q], v[j][q]);
          }
      }
      const __amdgpu_buffer_rsrc_t dst = a.packed_out ? chunk_rsrc(a.out + kw * a.block, nv * bbytes)
                                                      : chunk_rsrc(orow, a.lanes * bbytes);
#pragma unroll
      for (int j = 0; j < SL; ++j) {
        const uint32_t off = (a.packed_out ? static_cast<uint32_t>(j) : lj[j]) * bbytes;
        const uint32_t drop = static_cast<uint32_t>(j) < nv ? 0u : kDropStore;
#pragma unroll
        for (int q = 0; q < VEC; ++q)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, acc[j][q]), dst,
                                                 (off + (q * 64 + lane) * 16) | drop, 0, 0);
      }
      kw += nv;
    }
  }
}

}  // namespace

namespace {

template <int VEC, int MC, int SL>
__global__ __launch_bounds__(kWGThreads) void k_shard_sum_all(ShardArgs a) {
  const int lane = threadIdx.x & 63;
  const uint32_t groups = a.lanes / a.lg;
  const uint32_t bbytes = a.block * 4;
  const uint64_t units = (a.r1 - a.r0) * groups;
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * kWavesPerWG;
  const uint32_t* pws = a.prefix + static_cast<uint64_t>(a.count) * (a.rows + 1);
  for (uint64_t u = static_cast<uint64_t>(blockIdx.x) * kWavesPerWG + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
       u < units; u += nw) {
    const uint64_t r = a.r0 + u / groups;
    const uint32_t g0 = static_cast<uint32_t>(u % groups) * a.lg;
    const bool cl = static_cast<uint32_t>(lane) < a.count;
    const uint32_t* pc = a.prefix + static_cast<uint64_t>(cl ? lane : 0) * (a.rows + 1);
    const uint64_t w = a.write_set[r];
    const uint64_t mc = cl ? a.masks[static_cast<uint64_t>(lane) * a.rows + r] : 0ull;
    const uint32_t pcr = pc[r], pcr0 = pc[a.r0];
    const uint32_t pwr = pws[r], pwr0 = pws[a.r0];
    uint64_t rem = w & (below(g0 + a.lg) & ~below(g0));
    if (rem == 0) continue;
    const uint64_t kc0 = cl ? a.recv_off[lane] + (pcr - pcr0) : 0ull;
    uint64_t kw = pwr - pwr0 + static_cast<uint64_t>(__builtin_popcountll(w & below(g0)));
    // per contributor (static index): its mask and its stream's descriptor for this row
    uint64_t m_c[MC];
    __amdgpu_buffer_rsrc_t src[MC];
#pragma unroll
    for (int c = 0; c < MC; ++c) {
      const bool live = static_cast<uint32_t>(c) < a.count;
      m_c[c] = live ? readlane64(mc, c) : 0ull;
      const bool mine = static_cast<uint32_t>(c) == a.me;
      src[c] = !live ? chunk_rsrc(a.own, 0u)
               : mine ? chunk_rsrc(a.own + r * a.lanes * a.block, a.lanes * bbytes)
                      : chunk_rsrc(a.recv + readlane64(kc0, c) * a.block,
                                   static_cast<uint32_t>(__builtin_popcountll(m_c[c])) * bbytes);
    }
    float* orow = a.out + r * a.lanes * a.block;
    while (rem != 0) {
      uint32_t lj[SL];
      uint64_t bm;
      const uint32_t nv = take_bits<SL>(rem, lj, bm);
      v4f v[MC][SL][VEC];
#pragma unroll
      for (int c = 0; c < MC; ++c) {
        const bool mine = static_cast<uint32_t>(c) == a.me;
#pragma unroll
        for (int j = 0; j < SL; ++j) {
          const bool has = static_cast<uint32_t>(j) < nv && ((m_c[c] >> lj[j]) & 1u);
          const uint32_t off = (mine ? lj[j] : static_cast<uint32_t>(__builtin_popcountll(m_c[c] & below(lj[j])))) * bbytes;
#pragma unroll
          for (int q = 0; q < VEC; ++q)
            v[c][j][q] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(
                                                     src[c], (off + (q * 64 + lane) * 16) | (has ? 0u : kDropStore), 0,
                                                     kLoadAux));
        }
      }
      // rank-order sums from +0.0f (server.cc:148-150, :97-98); a dropped load is +0.0, which leaves them unchanged
      const __amdgpu_buffer_rsrc_t dst =
          a.packed_out ? chunk_rsrc(a.out + kw * a.block, nv * bbytes) : chunk_rsrc(orow, a.lanes * bbytes);
#pragma unroll
      for (int j = 0; j < SL; ++j) {
        v4f acc[VEC];
#pragma unroll
        for (int q = 0; q < VEC; ++q) acc[q] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < MC; ++c)
#pragma unroll
          for (int q = 0; q < VEC; ++q) acc[q] = add4(acc[q], v[c][j][q]);
        const uint32_t off = (a.packed_out ? static_cast<uint32_t>(j) : lj[j]) * bbytes;
        const uint32_t drop = static_cast<uint32_t>(j) < nv ? 0u : kDropStore;
#pragma unroll
        for (int q = 0; q < VEC; ++q)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, acc[q]), dst, (off + (q * 64 + lane) * 16) | drop,
                                                 0, 0);
      }
      kw += nv;
    }
  }
}

// k_move with SL slots per batch and prefetched index loads: a wave sweeps several units (grid-stride) and issues
// the next unit's mask + prefix loads before the current unit's data loads are consumed.
template <int VEC, int SL, bool PF>
__global__ __launch_bounds__(kWGThreads) void k_move_v(MoveArgs a) {
  const int lane = threadIdx.x & 63;
  const uint32_t groups = a.lanes / a.lg;
  const uint32_t bbytes = a.block * 4;
  const uint64_t units = a.rows * groups;
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * kWavesPerWG;
  const uint32_t skip_cnt = a.prefix[a.skip_e] - a.prefix[a.skip_b];
  uint64_t u = static_cast<uint64_t>(blockIdx.x) * kWavesPerWG + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint64_t m_n = 0;
  uint32_t pr_n = 0;
  if (PF && u < units) {
    m_n = a.masks[u / groups];
    pr_n = a.prefix[u / groups];
  }
  for (; u < units; u += nw) {
    const uint64_t r = u / groups;
    const uint32_t g0 = static_cast<uint32_t>(u % groups) * a.lg;
    uint64_t m;
    uint32_t pr;
    if constexpr (PF) {
      m = m_n;
      pr = pr_n;
      const uint64_t un = u + nw;
      if (un < units) {  // the next unit's index loads, in flight under this unit's data
        m_n = a.masks[un / groups];
        pr_n = a.prefix[un / groups];
      }
    } else {
      m = a.masks[r];
      pr = a.prefix[r];
    }
    if (r >= a.skip_b && r < a.skip_e) continue;
    uint64_t rem = m & (below(g0 + a.lg) & ~below(g0));
    if (rem == 0) continue;
    uint64_t k = pr + static_cast<uint64_t>(__builtin_popcountll(m & below(g0))) - (r >= a.skip_e ? skip_cnt : 0u);
    float* dense = const_cast<float*>(a.dir == 0 ? a.src : a.dst) + r * a.lanes * a.block;
    const __amdgpu_buffer_rsrc_t rd = chunk_rsrc(dense, a.lanes * bbytes);
    while (rem != 0) {
      uint32_t lj[SL];
      uint64_t bm;
      const uint32_t nv = take_bits<SL>(rem, lj, bm);
      float* packed = const_cast<float*>(a.dir == 0 ? a.dst : a.src) + k * a.block;
      const __amdgpu_buffer_rsrc_t rp = chunk_rsrc(packed, nv * bbytes);
      const __amdgpu_buffer_rsrc_t rs = a.dir == 0 ? rd : rp;
      const __amdgpu_buffer_rsrc_t rt = a.dir == 0 ? rp : rd;
      v4f v[SL][VEC];
#pragma unroll
      for (int j = 0; j < SL; ++j) {
        const uint32_t off = (a.dir == 0 ? lj[j] : static_cast<uint32_t>(j)) * bbytes;
        const uint32_t drop = static_cast<uint32_t>(j) < nv ? 0u : kDropStore;
#pragma unroll
        for (int q = 0; q < VEC; ++q)
          v[j][q] = __builtin_bit_cast(
              v4f, __builtin_amdgcn_raw_buffer_load_b128(rs, (off + (q * 64 + lane) * 16) | drop, 0, kLoadAux));
      }
#pragma unroll
      for (int j = 0; j < SL; ++j) {
        const uint32_t off = (a.dir == 0 ? static_cast<uint32_t>(j) : lj[j]) * bbytes;
        const uint32_t drop = static_cast<uint32_t>(j) < nv ? 0u : kDropStore;
#pragma unroll
        for (int q = 0; q < VEC; ++q)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v[j][q]), rt,
                                                 (off + (q * 64 + lane) * 16) | drop, 0, 0);
      }
      k += nv;
    }
  }
}

struct Shape {
  uint32_t lg;
  unsigned grid;
};
Shape shape_of(const ShardArgs& a, uint32_t lg_override) {
  Shape s;
  s.lg = lg_override ? lg_override : unit_lanes(a.r1 - a.r0, a.lanes);
  s.grid = grid_for((a.r1 - a.r0) * (a.lanes / s.lg));
  return s;
}

template <int MC, int SL>
void go_all(ShardArgs a, uint32_t lg, hipStream_t st) {
  const Shape s = shape_of(a, lg);
  a.lg = s.lg;
  k_shard_sum_all<1, MC, SL><<<s.grid, kWGThreads, 0, st>>>(a);
}
void go_prod(ShardArgs a, uint32_t lg, hipStream_t st) {
  const Shape s = shape_of(a, lg);
  a.lg = s.lg;
  k_shard_sum_r02<1><<<s.grid, kWGThreads, 0, st>>>(a);
}

struct Variant {
  const char* name;
  void (*fn)(ShardArgs, uint32_t, hipStream_t);
  uint32_t max_count;
};
const Variant kVariants[] = {
    {"round-2 k_shard_sum", go_prod, 16},
    {"all-contributors MC8 SL4", go_all<8, 4>, 8},
    {"all-contributors MC8 SL2", go_all<8, 2>, 8},
    {"all-contributors MC1 SL16", go_all<1, 16>, 1},
    {"all-contributors MC1 SL8", go_all<1, 8>, 1},
    {"all-contributors MC4 SL8", go_all<4, 8>, 4},
};
constexpr int kNum = sizeof(kVariants) / sizeof(kVariants[0]);

struct MoveVariant {
  const char* name;
  void (*fn)(const MoveArgs&, unsigned, hipStream_t);
};
template <int SL, bool PF>
void gm(const MoveArgs& a, unsigned g, hipStream_t st) {
  k_move_v<1, SL, PF><<<g, kWGThreads, 0, st>>>(a);
}
const MoveVariant kMoves[] = {
    {"move SL16 (product shape)", gm<16, false>}, {"move SL8", gm<8, false>}, {"move SL4", gm<4, false>},
    {"move SL16 prefetch", gm<16, true>},          {"move SL8 prefetch", gm<8, true>},
};
constexpr int kNumMoves = sizeof(kMoves) / sizeof(kMoves[0]);
}  // namespace

extern "C" {
int tune_move_count(void) { return kNumMoves; }
const char* tune_move_name(int v) { return (v >= 0 && v < kNumMoves) ? kMoves[v].name : "?"; }
// the pack (dir 0) of rows outside [skip_b, skip_e), B = 256; lg lanes per unit (0: the product's choice); grid cap
int tune_move(int v, const float* src, float* dst, const uint64_t* masks, const uint32_t* prefix, uint64_t rows,
              uint32_t lanes, uint64_t skip_b, uint64_t skip_e, uint32_t lg, uint32_t grid, void* stream) {
  if (v < 0 || v >= kNumMoves) return -3;
  MoveArgs a;
  a.src = src;
  a.dst = dst;
  a.masks = masks;
  a.prefix = prefix;
  a.rows = rows;
  a.skip_b = skip_b;
  a.skip_e = skip_e;
  a.lanes = lanes;
  a.block = 256;
  a.dir = 0;
  a.lg = lg ? lg : unit_lanes(rows, lanes);
  const unsigned g = grid ? grid : grid_for(rows * (lanes / a.lg));
  kMoves[v].fn(a, g, reinterpret_cast<hipStream_t>(stream));
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
uint32_t omr_sentinel(uint32_t block_size, uint32_t num_lanes) {  // the product's, compiled out by OMR_NO_CAPI
  return (UINT32_MAX / block_size / num_lanes - 1u) * num_lanes * block_size;
}
int tune_count(void) { return kNum; }
const char* tune_name(int v) { return (v >= 0 && v < kNum) ? kVariants[v].name : "?"; }
uint32_t tune_max_count(int v) { return (v >= 0 && v < kNum) ? kVariants[v].max_count : 0; }
// B = 256 only (VEC = 1)
int tune_shard_sum(int v, const float* own, uint32_t me, const float* recv, const uint64_t* recv_offsets,
                   const uint64_t* masks, uint32_t count, const uint32_t* prefix, const uint64_t* write_set,
                   uint64_t rows, uint64_t r0, uint64_t r1, uint32_t lanes, int packed_out, float* out, uint32_t lg,
                   void* stream) {
  if (v < 0 || v >= kNum || count == 0 || count > kVariants[v].max_count) return -3;
  ShardArgs a;
  a.own = own;
  a.recv = recv;
  for (uint32_t c = 0; c < OMR_MAX_WORKERS; ++c) a.recv_off[c] = c < count ? recv_offsets[c] : 0;
  a.masks = masks;
  a.prefix = prefix;
  a.write_set = write_set;
  a.out = out;
  a.rows = rows;
  a.r0 = r0;
  a.r1 = r1;
  a.count = count;
  a.me = me;
  a.lanes = lanes;
  a.block = 256;
  a.packed_out = packed_out ? 1u : 0u;
  a.lg = 0;
  kVariants[v].fn(a, lg, reinterpret_cast<hipStream_t>(stream));
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
}
