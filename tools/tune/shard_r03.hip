// shard_r03.hip — timing study of the round-3 product k_shard_sum (not the product; tools/tune_shard_r03.py): the same
// kernel with a window of PP/VEC pair slots (the product's PP is 32) and, with STAMP, per-wave s_memrealtime stamps
// {start, index data consumed, pair list written, first window summed, end with stores acknowledged, units, XCC} so the
// phases of a unit can be seen.  Built from the product source's kernel text (copied here when the study was made).
#include "plan_r04.hip"  // (the product kernels + the round-4 SumArgsR04 with its column-stream fields)

namespace {
constexpr uint32_t kR03UnitRows = 32;  // round 3's unit (the product's kSumUnitRows has changed since)
template <int VEC, int PP, int STAMP>
__global__ __launch_bounds__(kWGThreads) void k_shard_sum_s(SumArgsR04 a, uint64_t* tl) {
  constexpr int P = PP / VEC;  // pair slots per window
  constexpr int kSlotGroup = P < 8 ? P : 8;
  constexpr uint32_t kRecCap = kR03UnitRows * OMR_MAX_WORKERS;
  __shared__ uint64_t s_rec[kWavesPerWG][kRecCap];
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool cols = a.pos_off != kRowStreams;
  const uint64_t srows = a.r1 - a.r0;
  const uint64_t units = cols ? (srows / a.S) * a.gps * 2 * a.lanes
                              : ((srows + kR03UnitRows - 1) / kR03UnitRows) * a.lanes;
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * kWavesPerWG;
  const uint32_t* const pws = a.prefix + static_cast<uint64_t>(a.count) * (a.rows + 1);
  const uint32_t wpre0 = a.packed_out ? pws[a.r0] : 0u;
  const uint32_t bbytes = a.block * 4;
  const uint64_t gw = static_cast<uint64_t>(blockIdx.x) * kWavesPerWG + wave;
  uint64_t t0 = STAMP ? __builtin_amdgcn_s_memrealtime() : 0, t1 = 0, t2 = 0, t3 = 0;
  uint32_t nunits = 0;
  for (uint64_t u = static_cast<uint64_t>(blockIdx.x) * kWavesPerWG + wave; u < units; u += nw) {
    const uint32_t l = static_cast<uint32_t>(u % a.lanes);
    uint64_t g0, gidx = 0;  // first row the lanes load (lane i: row g0 + i); column streams: the group's table index
    uint32_t nload, h0, h1;  // rows loaded; the unit's rows are lanes [h0, h1)
    if (cols) {
      uint64_t t = u / a.lanes;
      const uint32_t h = static_cast<uint32_t>(t & 1u);
      t >>= 1;
      const uint32_t j = static_cast<uint32_t>(t % a.gps);
      const uint64_t seg = a.r0 / a.S + t / a.gps;
      g0 = seg * a.S + static_cast<uint64_t>(j) * kPackGroupRows;
      nload = a.S - j * kPackGroupRows < kPackGroupRows ? a.S - j * kPackGroupRows : kPackGroupRows;
      h0 = h * kR03UnitRows;
      h1 = nload < h0 + kR03UnitRows ? nload : h0 + kR03UnitRows;
      gidx = seg * a.gps + j;
      if (h0 >= h1) continue;
    } else {
      g0 = a.r0 + (u / a.lanes) * kR03UnitRows;
      nload = a.r1 - g0 < kR03UnitRows ? static_cast<uint32_t>(a.r1 - g0) : kR03UnitRows;
      h0 = 0;
      h1 = nload;
    }
    // ---- index loads, all issued together (one round trip)
    const bool rl = static_cast<uint32_t>(lane) < nload;
    const uint64_t r = g0 + (rl ? static_cast<uint32_t>(lane) : 0u);
    const uint64_t w = rl ? a.write_set[r] : 0ull;
    const uint32_t wpre = (rl && a.packed_out) ? pws[r] : 0u;
    uint64_t mk[OMR_MAX_WORKERS];
    uint32_t pre[OMR_MAX_WORKERS];
#pragma unroll
    for (uint32_t c = 0; c < OMR_MAX_WORKERS; ++c) {
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
    for (uint32_t c = 0; c < OMR_MAX_WORKERS; ++c) cb |= static_cast<uint32_t>((mk[c] >> l) & 1ull) << c;
    const uint32_t np = wb ? (cb ? static_cast<uint32_t>(__builtin_popcount(cb)) : 1u) : 0u;
    uint32_t inc = np;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t o = __shfl_up(inc, d, 64);
      if (lane >= d) inc += o;
    }
    const uint32_t total = __builtin_amdgcn_readlane(inc, 63);
    if (STAMP && nunits == 0) t1 = __builtin_amdgcn_s_memrealtime();
    ++nunits;
    if (total == 0) continue;
    uint64_t ccol[OMR_MAX_WORKERS];  // column streams: worker c's bits of column l over the loaded rows
#pragma unroll
    for (uint32_t c = 0; c < OMR_MAX_WORKERS; ++c) ccol[c] = (cols && c < a.count) ? __ballot((mk[c] >> l) & 1ull) : 0ull;
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
        for (uint32_t c = 0; c < OMR_MAX_WORKERS; ++c) {
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
    if (STAMP && t2 == 0) t2 = __builtin_amdgcn_s_memrealtime();
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
#pragma unroll
      for (int j = 0; j < P; ++j) {
        if (static_cast<uint32_t>(j) < nv) {  // (wave-uniform)
          const uint64_t rc = readlane64(myrec, j);
#pragma unroll
          for (int q = 0; q < VEC; ++q)  // (0.0f + x_first) + ...: a block's first pair restarts from +0.0f
            acc[q] = add4((rc & kRecFirst) ? v4f{0.f, 0.f, 0.f, 0.f} : acc[q], v[j][q]);
          if (rc & kRecLast) {
            v4f* const d = reinterpret_cast<v4f*>(a.out + ((rc >> 32) & 0x0FFFFFFFull) * a.block);
#pragma unroll
            for (int q = 0; q < VEC; ++q) d[q * 64 + lane] = acc[q];
          }
        }
      }
      if (STAMP && t3 == 0) t3 = __builtin_amdgcn_s_memrealtime();
    }
  }
  if (STAMP && lane == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint64_t t4 = __builtin_amdgcn_s_memrealtime();
    uint64_t* r = tl + gw * 8;
    r[0] = t0; r[1] = t1; r[2] = t2; r[3] = t3; r[4] = t4; r[5] = nunits;
    r[6] = static_cast<uint64_t>(__builtin_amdgcn_s_getreg((15 << 11) | 20));
  }
}
}  // namespace

extern "C" {
// variant v: 0 = PP 32 (the product's window), 1 = PP 16, 2 = PP 64 (VEC = 1 only); stamp 1 records the timeline
int tune_shard(int v, int stamp, const float* own, uint32_t me, const float* recv, const uint64_t* recv_off,
               const uint64_t* masks, uint32_t count, uint64_t mstride, uint64_t pos_off, const uint32_t* prefix,
               const uint64_t* write_set, uint64_t rows, uint64_t r0, uint64_t r1, uint32_t lanes, uint32_t S,
               uint32_t gps, float* out, uint64_t* tl, unsigned grid, hipStream_t st) {
  SumArgsR04 a{};
  a.own = own; a.recv = recv; a.masks = masks; a.mstride = mstride; a.prefix = prefix; a.pos_off = pos_off;
  a.write_set = write_set; a.out = out; a.rows = rows; a.r0 = r0; a.r1 = r1; a.count = count; a.me = me;
  a.lanes = lanes; a.block = 256; a.packed_out = 0; a.S = S; a.gps = gps;
  for (uint32_t c = 0; c < OMR_MAX_WORKERS; ++c) a.recv_off[c] = c < count ? recv_off[c] : 0;
  const uint64_t srows = r1 - r0;
  const uint64_t units = pos_off != kRowStreams ? (srows / S) * gps * 2 * lanes : ((srows + 31) / 32) * lanes;
  if (grid == 0) grid = grid_for(units);
#define GO(PP, ST) k_shard_sum_s<1, PP, ST><<<grid, kWGThreads, 0, st>>>(a, tl)
  if (stamp) {
    if (v == 0) GO(32, 1); else if (v == 1) GO(16, 1); else GO(64, 1);
  } else {
    if (v == 0) GO(32, 0); else if (v == 1) GO(16, 0); else GO(64, 0);
  }
#undef GO
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
unsigned tune_shard_units(uint64_t r0, uint64_t r1, uint32_t lanes, uint32_t S, uint32_t gps, int cols) {
  return cols ? static_cast<unsigned>(((r1 - r0) / S) * gps * 2 * lanes)
              : static_cast<unsigned>(((r1 - r0 + 31) / 32) * lanes);
}
}
