// omr_kernels.hip — CDNA4 (gfx950) kernels + C ABI for the OmniReduce sparse-block hot path.
//
// Reference behaviour implemented here (Phlix1/OmniReduce-RDMA-Demo, read-only at /root/reference):
//   worker scan    client.cc:19-31 find_next_nonzero_block, drivers client.cc:87-102 and :191-205
//   aggregator sum server.cc:83-99 (block_next_offset / min_next bookkeeping :84-96, the add :97-98)
//   layout         common.h:27-42 (BLOCK_SIZE, NUM_BLOCKS lanes, NUM_THREADS partitions)
//   generator      client.cc:396-421
// Design: the hot path is HBM-bound byte/integer work plus one fp32 add per element; no MFMA.
//   k_scan1f          : the single-pass m = 1 worker step.  A workgroup owns one (partition, lane) column — one
//                       reference next-offset chain — streams its 1 KiB blocks (16 dwordx4 loads per wave in
//                       flight), ballots the flags, stores the aggregated non-zero blocks write-through, and
//                       resolves every next offset from the column's bit vector in LDS (segments of a column, when
//                       there are few columns, meet through device-scope atomics).
//   k_scan1 / k_scanm : two-pass variant (plus row masks for the multi-GPU exchange) and the m-worker sum;
//                       16 KiB chunks / rows swept grid-stride, same loads, ballots and stores.
//   k_next            : next-offset chains from uint64 row masks (64x64 wave bit transposes).
//   exchange kernels  : mask union, popcount prefixes, compaction, block gather/scatter, sparse shard sum.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstring>

#include "omr.h"

namespace {

thread_local char g_err[512] = "";

int fail(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return OMR_EINVAL;
}

int launch_status(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
    return static_cast<int>(e);
  }
  return 0;
}

// Native 16-byte vectors: one dwordx4 per lane, a wave-wide load moves 1 KiB = one 256-float block.
typedef float v4f __attribute__((ext_vector_type(4)));
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));

struct WorkerPtrs {
  const float* p[OMR_MAX_WORKERS];
};

constexpr int kWavesPerWG = 4;
constexpr int kWGThreads = 64 * kWavesPerWG;
constexpr int kMaxGrid = 2048;  // 8 workgroups per CU over 256 CUs; grid-stride beyond (guide G11)

// ---------------------------------------------------------------- device helpers

// Non-zero test of 4 floats: x != 0.0f for any of them, with -0.0 zero and NaN non-zero.  OR-ing the raw
// bits and then clearing bit 31 is the bitwise OR of the four |x| bit patterns, so it is exact.
__device__ __forceinline__ uint32_t nz_bits(const v4f& v) {
  const v4u u = __builtin_bit_cast(v4u, v);
  return (u.x | u.y | u.z | u.w) & 0x7fffffffu;
}

template <bool NT>
__device__ __forceinline__ v4f ld4(const v4f* p) {
  if constexpr (NT) {
    return __builtin_nontemporal_load(p);
  } else {
    return *p;
  }
}

__device__ __forceinline__ v4f add4(const v4f& a, const v4f& b) { return a + b; }

__device__ __forceinline__ uint64_t wave_ballot(bool p) { return __ballot(p); }

constexpr uint32_t kNone = 0xFFFFFFFFu;  // "no row" marker

struct ScanArgs {
  WorkerPtrs x;
  uint32_t m;
  uint32_t lanes;          // NUM_BLOCKS
  uint32_t rows_per_part;  // rows per partition
  uint32_t row_begin;      // k_scan1 sweeps rows [row_begin, row_end) (a pipelined chunk, or everything)
  uint32_t row_end;
  uint32_t pad;
  uint64_t rows;           // total rows
  uint64_t nb;             // total blocks
  int32_t* flags;          // [m][nb] or null
  uint64_t* masks;         // [m (+1 union)][rows]
  float* out;              // dense or null
};

// ---------------------------------------------------------------- k_scan1: one worker, fused scan + sum
//
// Work unit = a chunk of CH consecutive blocks of one row (CH = 16 blocks = 16 KiB at B=256; 8 blocks at
// B=512/1024), swept grid-stride by 8-wave workgroups so that the waves in flight at any moment cover one
// contiguous stretch of HBM.  A wave issues all CH*VEC 16-byte-per-lane loads of its chunk (non-temporal:
// the gradient is read once) before the first use.  Per block: ballot(any element non-zero) -> flag bit; if
// the block is non-zero (or sits in a lane-head row, which the reference always sends: client.cc:201-205)
// the aggregated block 0.0f + x (server.cc:148-150 zero, :97-98 add) is stored straight from registers.
// The chunk's CH flag bits are one byte-aligned piece of the row's uint64 mask, stored directly.
constexpr int kScanWaves = 8;  // 512-thread workgroups (tools/tune_scan.py: fastest of 4/8/16 on MI355X)

template <int VEC>
constexpr int scan_chunk_blocks() {
  return (16 / VEC) > 8 ? (16 / VEC) : 8;
}

// Cache policy (tools/tune_scan.py, MI355X): loads are buffer loads with aux 2 (nt: read-once stream); the
// aggregated blocks are buffer stores with aux 17 (sc0 sc1: system-scope write-through), which leaves no
// dirty lines in the XCD L2s for the kernel-boundary write-back to flush before k_next can start.
constexpr int kLoadAux = 2;
constexpr int kStoreAux = 17;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t chunk_rsrc(const float* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, static_cast<int>(bytes), 0x00020000);
}

// A wave's store of one block (VEC dwordx4 per lane) at a wave-uniform address, with kStoreAux (write-through): the
// packed and summed blocks of the round's kernels leave no dirty lines in the XCD L2s either.  Plain stores did, and
// the kernel-end write-back of them ran after the last wave: the shard sum took 15.3 us with these stores against
// 16.8 with plain ones (stamped copies, profiles/r04/shard/shard_store_policy.log).
#ifndef OMR_BLOCK_STORE_AUX  // (tools: a study build may pick another policy, e.g. 2 = nt)
#define OMR_BLOCK_STORE_AUX kStoreAux
#endif
template <int VEC>
__device__ __forceinline__ void store_block_wt(float* dst, const v4f* v, int lane) {
  const uint64_t a = reinterpret_cast<uint64_t>(dst);
  const uint64_t u = (static_cast<uint64_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a >> 32))) << 32) |
                     static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a)));
  const __amdgpu_buffer_rsrc_t r = chunk_rsrc(reinterpret_cast<float*>(u), VEC * 1024u);
#pragma unroll
  for (int q = 0; q < VEC; ++q)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v[q]), r, (q * 64 + lane) * 16, 0,
                                           OMR_BLOCK_STORE_AUX);
}

template <int VEC>
__global__ __launch_bounds__(64 * kScanWaves) void k_scan1(ScanArgs a) {
  constexpr int B4 = 64 * VEC;  // 16-byte vectors per block
  constexpr int CH = scan_chunk_blocks<VEC>();
  constexpr uint32_t kChunkBytes = CH * B4 * 16;
  const int lane = threadIdx.x & 63;
  // wave index made provably uniform so the buffer descriptors below live in SGPRs (no waterfall loops, T20)
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const float* x = a.x.p[0];  // no __restrict__: out may alias x (in-place result, client.cc:89)
  float* out = a.out;
  uint8_t* __restrict__ mask_bytes = reinterpret_cast<uint8_t*>(a.masks);
  // rows < 2^18 for any n below the uint32 sentinel, so chunk/row indices are 32-bit (cheap scalar math)
  const uint32_t cpr_shift = static_cast<uint32_t>(__builtin_ctz(a.lanes / CH));  // chunks per row = 2^shift
  const uint32_t chunks = a.row_end << cpr_shift;
  const uint32_t nwaves = gridDim.x * kScanWaves;
  for (uint32_t c = (a.row_begin << cpr_shift) + blockIdx.x * kScanWaves + wave; c < chunks; c += nwaves) {
    const uint32_t row = c >> cpr_shift;
    const uint32_t l0 = (c & ((1u << cpr_shift) - 1u)) * CH;
    const bool head = (row % a.rows_per_part) == 0;
    const uint64_t base = static_cast<uint64_t>(c) * CH * B4 * 4;  // float offset of chunk c (= block c*CH)
    const __amdgpu_buffer_rsrc_t src = chunk_rsrc(x + base, kChunkBytes);
    v4f v[CH][VEC];
#pragma unroll
    for (int s = 0; s < CH; ++s)
#pragma unroll
      for (int q = 0; q < VEC; ++q)
        v[s][q] = __builtin_bit_cast(
            v4f, __builtin_amdgcn_raw_buffer_load_b128(src, ((s * B4 + q * 64 + lane) * 16), 0, kLoadAux));
    uint32_t bits = 0;
    const __amdgpu_buffer_rsrc_t dst = chunk_rsrc(out + base, out != nullptr ? kChunkBytes : 0u);
#pragma unroll
    for (int s = 0; s < CH; ++s) {
      uint32_t o = 0;
#pragma unroll
      for (int q = 0; q < VEC; ++q) o |= nz_bits(v[s][q]);
      const bool nz = wave_ballot(o != 0) != 0;
      bits |= static_cast<uint32_t>(nz) << s;
      if (out != nullptr && (nz || head)) {
        const v4f z = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < VEC; ++q)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, add4(z, v[s][q])), dst,
                                                 (s * B4 + q * 64 + lane) * 16, 0, kStoreAux);
      }
    }
    if (lane == 0) {
      uint8_t* mp = mask_bytes + static_cast<uint64_t>(row) * 8 + l0 / 8;
      if constexpr (CH == 16) {
        *reinterpret_cast<uint16_t*>(mp) = static_cast<uint16_t>(bits);
      } else {
        *mp = static_cast<uint8_t>(bits);
      }
    } else if (l0 + CH == a.lanes && lane < 8 && static_cast<uint32_t>(lane) >= a.lanes / 8) {
      mask_bytes[static_cast<uint64_t>(row) * 8 + lane] = 0;  // bits of lanes >= NB (rows narrower than 64)
    }
    if (a.flags != nullptr && lane < CH)
      a.flags[static_cast<uint64_t>(row) * a.lanes + l0 + lane] = static_cast<int32_t>((bits >> lane) & 1u);
  }
}

// ---------------------------------------------------------------- k_scan1f: single-pass scan + sum + next
//
// One launch for the whole m = 1 worker step.  Work is split by COLUMN instead of by address: a workgroup owns
// one lane l of one partition p (or a segment of its rows, when there are too few columns to fill the chip),
// i.e. exactly the blocks one find_next_nonzero_block chain walks (client.cc:19-31).  Each wave owns a
// CONTIGUOUS range of the segment's rows and streams it last batch first, LOADS dwordx4 loads per lane in flight
// (RB rows of the column: 1 KiB pieces 64 KiB apart at B=256), ballots the flags and stores the aggregated
// non-zero blocks write-through.  Because the rows are visited backwards, every row's successor lies either in
// its own batch (a ctz over the batch's ballot bits) or among the wave's already-scanned rows (a running carry
// = first non-zero row seen so far), so next offsets are stored as the stream goes, with no epilogue pass.
// Only the wave's tail rows (at and after its last non-zero row) need a later wave's first non-zero row: one
// barrier and one store per wave.  With K > 1 segments per column, each segment publishes {first, last}
// non-zero row through device-scope atomics; the segment whose arrival count completes the column writes the
// rows whose successor lies in a later segment.  Workgroup -> (p, l, k) is permuted so that one partition's
// columns share an XCD, letting the L2 merge their 4-byte flag/next stores into whole lines (speed only).
//
// Stores: every row issues its stores; a zero block's are pointed past the descriptor's range and discarded by
// the buffer range check.  The number of memory operations per batch is then static, so the compiler's vmcnt
// wait for a load never includes a younger, data-dependent store (tools/tune_fused.py: 2-4 % faster than
// branching around the stores; write-through sc0 sc1 beat plain, sc1-only and nt stores).
// SKIP (the product's choice at B = 1024): a batch with no block to write skips its (dropped) data stores through a
// wave-uniform branch.  (The timing-study form of this kernel, with its ablation / store-policy / timeline knobs, is
// tools/tune/scan1f_study.h; it is not built into libomr.so.)
//
// PACK (the multi-rank round's worker scan): the scan also packs the worker's non-zero blocks of the other shards
// for their aggregators (common.cc:399-407), so no separate pack pass re-reads them from HBM.  A shard is a row range
// made of whole column segments; its send stream is its segments' non-zero blocks, segment by segment, each segment's
// blocks in row order.  A segment's place in the stream is taken by ONE device atomic on the shard's counter once the
// workgroup knows its count (segments land in completion order, not in a fixed order: no workgroup ever waits for
// another).  Until then the blocks stay on chip: each wave keeps its range's non-zero blocks, highest row first, in
// `wcap` LDS slots of its own (the rest, its lowest rows, are re-read at the end: none at config 4's density).  The
// aggregator finds a block from pos[(segment, 64-row group), lane] = its stream position of the group's first block
// in that column, plus the column's set bits of the group below the row.
struct FusedArgs {
  const float* x;
  float* out;
  int32_t* flags;
  uint32_t* next;
  uint32_t* cnt;       // [parts*lanes] arrival counters (K > 1), zero between launches
  uint64_t* summary;   // [parts*lanes*K] {first << 32 | last} per segment (K > 1)
  uint64_t* masks;     // [rows] row masks, zero on entry, non-zero blocks OR-ed in (multi-rank round), or null
  uint32_t lanes, rpp, K, S, block, sentinel;
  uint32_t part0;      // first partition of the launch (a per-partition call scans partitions [part0, part0 + grid))
  // PACK
  float* send;         // shard s's stream starts at float send_row[s] * lanes * block (the streams in shard order,
                       // own_shard's left out: n floats less its rows)
  uint32_t* shard_cnt; // [nshards] blocks taken so far in each shard's stream (zero on entry)
  uint32_t* pos;       // [parts * K * gps * lanes] stream position of (segment, group, lane)'s first block
  uint32_t bounds[OMR_MAX_WORKERS + 1];  // shard s = rows [bounds[s], bounds[s + 1]), whole segments
  uint32_t send_row[OMR_MAX_WORKERS];
  uint32_t nshards, gps, wcap;
  int32_t own_shard;   // this rank's own shard (read in place by its aggregator, not packed); -1: none
  // TALLY (the one-rank round): workgroup b stores tally[b] = {non-zero blocks, zero lane-head blocks} of its segment
  // (one slot per workgroup: no atomic, so no queue of 512 of them on one address at the launch's end); workgroup 0's
  // first wave also publishes an earlier launch's slots, pub_src (pub_slots of them), to pub_dst (publish_tally)
  uint64_t* tally;
  const uint64_t* pub_src;
  uint32_t* pub_dst;
  uint32_t pub_seq, pub_slots;
  // CHK (the multi-rank round's worker scan, round 6): workgroup b stores chk[b] = (chk_seq << 32) | its non-zero
  // blocks, the count its row-mask bits must add up to; the plan launch checks every worker's (omr_round_plan_check)
  uint64_t* chk;
  uint32_t chk_seq;
  // ... and the launch's completion (round 6): done[0] counts workgroups out (zero between launches), the last one
  // stores chk_seq into done[1]; null: no signal
  uint32_t* done;
};

// CHK: the launch's completion signalled on the device.  Every workgroup counts itself out at its end and the last one
// stores the launch's seq into done[1] (and re-arms the counter).  The multi-rank round's side stream waits for that
// word with a one-wave kernel (omr_dist.hip k_wait_seq) instead of for an event recorded on the caller's stream after
// the scan: such a record sits between two scans, and a record with a waiter on another queue costs the next kernel
// about 2.7 us (tools/tune/launch_floor.hip, profiles/r06/round_kernels/launch_floor.log).  What the side stream reads
// before the launch ends -- the row masks (device-scope atomics), the position table and the check slots (stored
// through to memory, sc1), the packed blocks (write-through) -- is at the coherence point once the workgroup's stores
// are acknowledged (s_waitcnt vmcnt(0)), so no workgroup writes its L2 back: an agent-scope release fence per
// workgroup (buffer_wbl2) took the scan from 50 to 99 us per round.
template <bool ON>
struct ScanDone {
  const FusedArgs& a;
  __device__ ~ScanDone() {
    if constexpr (ON) {
      if (a.done == nullptr) return;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores and atomics acknowledged
      __syncthreads();                                   // (every exit of k_scan1f is workgroup-uniform)
      if (threadIdx.x == 0) {
        const uint32_t n = __hip_atomic_fetch_add(&a.done[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (n + 1 == gridDim.x) {
          __hip_atomic_store(&a.done[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(&a.done[1], a.chk_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
  }
};

// The one-rank round's counts, from an earlier launch's slots, one wave: lane i sums slots i, i + 64, ... (loaded by
// tally_load, a launch's first instructions), then a DPP reduction.
__device__ __forceinline__ void tally_load(const uint64_t* src, uint32_t slots, uint32_t* nz, uint32_t* heads) {
  const int lane = threadIdx.x & 63;
  uint32_t z = 0, h = 0;
  for (uint32_t i = lane; i < slots; i += 64) {
    const uint64_t v = src[i];
    z += static_cast<uint32_t>(v);
    h += static_cast<uint32_t>(v >> 32);
  }
  *nz = z;
  *heads = h;
}

// ... reduced over the wave and stored as the completion notice {seq, non-zero blocks, write-set blocks, seq} in ONE
// 16-byte write-through store to host-mapped memory (a host that sees seq in both halves has the counts: each aligned
// 8-byte half lands whole).
__device__ __forceinline__ void publish_tally(uint32_t* dst, uint32_t seq, uint32_t nz, uint32_t heads) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    nz += static_cast<uint32_t>(__shfl_xor(static_cast<int>(nz), d, 64));
    heads += static_cast<uint32_t>(__shfl_xor(static_cast<int>(heads), d, 64));
  }
  if ((threadIdx.x & 63) != 0) return;
  const v4u rec = v4u{seq, nz, nz + heads, seq};
  __builtin_amdgcn_raw_buffer_store_b128(rec, chunk_rsrc(reinterpret_cast<float*>(dst), 16u), 0, 0, kStoreAux);
}

constexpr uint32_t kPackLdsBytes = 128u << 10;  // the waves' stash slots: 8 blocks per wave at B = 256 (16 waves)
constexpr uint32_t kPackGroupRows = 64;         // the position table's row granularity (one wave of row masks)

constexpr uint32_t kDropStore = 0x40000000u;  // voffset past every descriptor range: the store is discarded

// TALLY: at most 96 VGPRs (five waves per SIMD), as the headline form has (92); its tally registers had taken the
// one-rank round's launch to 106 (four waves per SIMD).  Capped: 48.03 / 49.80 us in / out of place against 48.65 /
// 50.14, the headline 47.73 / 49.43 (profiles/r05/timing/vgpr96/tally.log, profiles/r05/plan_v5/tally.log).
template <int VEC, int WAVES, int LOADS = 16, int SKIP = 0, bool PACK = false, bool TALLY = false, bool CHK = false>
__global__ __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(TALLY ? 5 : 1, 8))) void k_scan1f(
    FusedArgs a) {
  constexpr int RB = LOADS / VEC;  // rows per batch (<= 32)
  static_assert(RB >= 1 && RB <= 32 && 32 % RB == 0, "a batch's bits lie inside one 32-bit word");
  [[maybe_unused]] constexpr uint32_t B4 = 64 * VEC;  // 16-byte vectors per block
  __shared__ uint32_t s_wfirst[WAVES], s_wlast[WAVES];
  __shared__ int s_fix;
  __shared__ uint32_t s_carry[64];
  __shared__ uint32_t s_seg_last[64];
  // PACK: dynamic LDS = the segment's non-zero-row bits [ceil(S / 32) words, 16-byte aligned] + the stash slots
  extern __shared__ __attribute__((aligned(16))) uint32_t s_dyn[];
  __shared__ uint32_t s_wcnt[(PACK || TALLY) ? WAVES : 1], s_wpre[PACK ? WAVES : 1];
  __shared__ uint32_t s_base, s_total;
  __shared__ uint32_t s_wnz[CHK ? WAVES : 1];
  [[maybe_unused]] uint32_t nzc = 0;  // CHK: the wave's non-zero blocks (wave-uniform)
  const ScanDone<CHK> scan_done{a};   // (signals at whichever exit the workgroup takes)
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t T = gridDim.x, bid = blockIdx.x;
  // TALLY: workgroup 0 publishes the previous round's counts.  Their loads go out now, ahead of the scan's own (their
  // latency hides behind the first batch), and the store at the end of this workgroup's work, which is in the launch's
  // first wave of workgroups: no part of it waits at the end of the launch.
  [[maybe_unused]] uint32_t pub_nz = 0, pub_heads = 0;
  if constexpr (TALLY) {
    if (bid == 0 && a.pub_src != nullptr && wave == 0) tally_load(a.pub_src, a.pub_slots, &pub_nz, &pub_heads);
  }
  const uint32_t lin = (T % 8 == 0) ? (bid % 8) * (T / 8) + bid / 8 : bid;
  const uint32_t k = lin % a.K, col = lin / a.K + a.part0 * a.lanes;  // col: global (partition, lane) index
  const uint32_t l = col % a.lanes, p = col / a.lanes;
  const uint32_t r0 = k * a.S;                                  // segment's first row within the partition
  const uint64_t row0 = static_cast<uint64_t>(p) * a.rpp + r0;  // its global row
  uint64_t* const masks = a.masks;
  const uint32_t row_bytes = a.lanes * a.block * 4;
  const uint32_t lane_b = l * a.block;
  const uint32_t row_stride = a.lanes * a.block;
  const bool last_seg = (k + 1 == a.K);
  // the wave's rows [lo, hi) of the segment: whole batches, except possibly the last nonempty wave's top one
  const uint32_t rw = ((a.S + WAVES * RB - 1) / (WAVES * RB)) * RB;
  const uint32_t lo = wave * rw < a.S ? wave * rw : a.S;
  const uint32_t hi = lo + rw < a.S ? lo + rw : a.S;
  uint32_t carry = kNone, wlast = kNone;
  // PACK: this segment's shard (the host checked that a segment never straddles two) and whether it is packed
  [[maybe_unused]] uint32_t shard = 0;
  [[maybe_unused]] bool pack = false;
  [[maybe_unused]] uint32_t* const s_bits = s_dyn;
  [[maybe_unused]] const uint32_t bits_words = ((a.S + 31) / 32 + 3) & ~3u;
  [[maybe_unused]] v4f* const stash = reinterpret_cast<v4f*>(s_dyn + bits_words);
  [[maybe_unused]] uint32_t cnt_w = 0, taken = 0;  // the wave's non-zero rows, and how many of them (the highest) it stashed
  [[maybe_unused]] uint32_t head0 = 0;             // TALLY: the column's lane-head block is zero (it is still returned)
  if constexpr (PACK) {
    while (shard + 1 < a.nshards && row0 >= a.bounds[shard + 1]) ++shard;
    pack = static_cast<int32_t>(shard) != a.own_shard;
    if (pack) {
      for (uint32_t i = threadIdx.x; i < bits_words; i += 64 * WAVES) s_bits[i] = 0;
      __syncthreads();
    }
  }
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
    const __amdgpu_buffer_rsrc_t dst = chunk_rsrc(a.out + blk0 * a.block, a.out != nullptr ? nrow * row_bytes : 0u);
    const uint32_t row_step = row_bytes;
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
                                                 dst, (s * row_step + (q * 64 + lane) * 16) | drop, 0, kStoreAux);
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
                                                   dst, (s * row_step + (q * 64 + lane) * 16) | drop, 0, kStoreAux);
        }
      }
    }
    if (static_cast<uint32_t>(lane) < nrow) {
      const uint64_t blk = blk0 + static_cast<uint64_t>(lane) * a.lanes;
      // successor of row rr+lane: next set bit above it in this batch, else the carry (client.cc:19-31)
      const uint32_t above = static_cast<uint32_t>(static_cast<uint64_t>(bits) >> (lane + 1));
      const uint32_t nr = above != 0 ? rr + lane + 1 + static_cast<uint32_t>(__builtin_ctz(above)) : carry;
      if (a.flags != nullptr) a.flags[blk] = static_cast<int32_t>((bits >> lane) & 1u);
      if (nr != kNone) a.next[blk] = static_cast<uint32_t>(row0 + nr) * row_stride + lane_b;
      if (masks != nullptr && ((bits >> lane) & 1u))
        (void)__hip_atomic_fetch_or(&masks[row0 + rr + lane], 1ull << l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if constexpr (PACK) {
      if (pack && bits != 0) {
        cnt_w += static_cast<uint32_t>(__builtin_popcount(bits));
        if (lane == 0) (void)__hip_atomic_fetch_or(&s_bits[rr >> 5], bits << (rr & 31), __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_WORKGROUP);
        // the batch's non-zero blocks into the wave's free slots, highest row first (slot j = j-th from the top)
#pragma unroll
        for (int s = RB - 1; s >= 0; --s) {
          if (((bits >> s) & 1u) && taken < a.wcap) {
            v4f* const slot = stash + (static_cast<uint64_t>(wave) * a.wcap + taken) * B4;
#pragma unroll
            for (int q = 0; q < VEC; ++q) slot[q * 64 + lane] = v[s][q];
            ++taken;
          }
        }
      }
    }
    if constexpr (TALLY) {
      cnt_w += static_cast<uint32_t>(__builtin_popcount(bits));
      if (r0 + rr == 0 && !(bits & 1u)) head0 = 1;
    }
    if constexpr (CHK) nzc += static_cast<uint32_t>(__builtin_popcount(bits));
    if (bits != 0) {
      if (wlast == kNone) wlast = rr + 31 - static_cast<uint32_t>(__builtin_clz(bits));
      carry = rr + static_cast<uint32_t>(__builtin_ctz(bits));
    }
  }
  if (lane == 0) {
    s_wfirst[wave] = carry;  // first non-zero row of the wave's range (kNone: all zero)
    s_wlast[wave] = wlast;   // last one
    if constexpr (TALLY) s_wcnt[wave] = cnt_w | (head0 << 31);
    if constexpr (CHK) s_wnz[wave] = nzc;
  }
  __syncthreads();
  if constexpr (CHK) {  // the round check's slot: one plain store per workgroup (its order against the mask atomics does
                        // not matter: a reader that sees this slot before some of the bits sees too few bits)
    if (threadIdx.x == 0 && a.chk != nullptr) {
      uint32_t t = 0;
      for (uint32_t w2 = 0; w2 < WAVES; ++w2) t += s_wnz[w2];
      // (stored through to memory, sc1: with a completion word the side stream reads it before this launch ends)
      __hip_atomic_store(&a.chk[bid], (static_cast<uint64_t>(a.chk_seq) << 32) | t, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if constexpr (TALLY) {  // the one-rank round's bookkeeping: one slot store per workgroup, no atomic
    if (threadIdx.x == 0) {
      uint32_t nz = 0, heads = 0;
      for (uint32_t w2 = 0; w2 < WAVES; ++w2) {
        nz += s_wcnt[w2] & 0x7fffffffu;
        heads += s_wcnt[w2] >> 31;
      }
      a.tally[bid] = (static_cast<uint64_t>(heads) << 32) | nz;
    }
    if (bid == 0 && a.pub_src != nullptr && wave == 0) publish_tally(a.pub_dst, a.pub_seq, pub_nz, pub_heads);
  }
  // tail rows [wlast or lo, hi): successor = first non-zero row of a later wave, else of a later segment
  uint32_t succ = kNone;
  for (uint32_t w2 = wave + 1; w2 < WAVES; ++w2)
    if (s_wfirst[w2] != kNone) {
      succ = s_wfirst[w2];
      break;
    }
  if (succ != kNone || last_seg) {
    const uint32_t val = succ != kNone ? static_cast<uint32_t>(row0 + succ) * row_stride + lane_b : a.sentinel + lane_b;
    for (uint32_t i = (wlast == kNone ? lo : wlast) + lane; i < hi; i += 64) a.next[(row0 + i) * a.lanes + l] = val;
  }
  if constexpr (PACK) {
    if (pack) {
      if (lane == 0) s_wcnt[wave] = cnt_w;
      __syncthreads();  // (also orders every wave's s_bits updates before the reads below)
      if (threadIdx.x == 0) {  // the segment's place in its shard's stream: one device atomic
        uint32_t t = 0;
        for (uint32_t w2 = 0; w2 < WAVES; ++w2) {
          s_wpre[w2] = t;
          t += s_wcnt[w2];
        }
        s_total = t;
        s_base = t ? __hip_atomic_fetch_add(&a.shard_cnt[shard], t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
      }
      __syncthreads();
      if (s_total != 0) {
        const uint32_t base = s_base;
        // position table: group j's first block = base + the segment's non-zero rows before row 64 j
        const uint64_t seg = static_cast<uint64_t>(p) * a.K + k;
        for (uint32_t j = threadIdx.x; j < a.gps; j += 64 * WAVES) {
          uint32_t c = 0;
          for (uint32_t wd = 0; wd < j * (kPackGroupRows / 32); ++wd) c += static_cast<uint32_t>(__builtin_popcount(s_bits[wd]));
          __hip_atomic_store(&a.pos[(seg * a.gps + j) * a.lanes + l], base + c, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);  // (through to memory: read before the launch ends, as chk)
        }
        // the wave's blocks: its range's non-zero rows take stream places base + s_wpre[wave] + (rank among them)
        float* const sbase = a.send + static_cast<uint64_t>(a.send_row[shard]) * row_stride;
        const uint64_t wb = static_cast<uint64_t>(base) + s_wpre[wave];
        for (uint32_t j = 0; j < taken; ++j) {  // stashed: the j-th from the top has rank cnt_w - 1 - j
          const v4f* const slot = stash + (static_cast<uint64_t>(wave) * a.wcap + j) * B4;
          v4f t[VEC];
#pragma unroll
          for (int q = 0; q < VEC; ++q) t[q] = slot[q * 64 + lane];
          store_block_wt<VEC>(sbase + (wb + cnt_w - 1 - j) * a.block, t, lane);
        }
        // the rest (the wave's lowest cnt_w - taken non-zero rows, in order): re-read, from `out` when the scan wrote
        // 0.0f + x there (the same bits), else from x
        const float* const rsrc = a.out != nullptr ? a.out : a.x;
        uint32_t idx = 0;
        const uint32_t over = cnt_w - taken;
        for (uint32_t wd = lo >> 5; idx < over && wd * 32 < hi; ++wd) {
          uint32_t m = s_bits[wd];
          const uint32_t b0 = wd * 32;
          if (b0 < lo) m &= ~0u << (lo - b0);
          if (hi - b0 < 32) m &= (1u << (hi - b0)) - 1u;
          while (m != 0 && idx < over) {
            const uint32_t r = b0 + static_cast<uint32_t>(__builtin_ctz(m));
            m &= m - 1;
            const v4f* const sp = reinterpret_cast<const v4f*>(rsrc + ((row0 + r) * a.lanes + l) * a.block);
            v4f t[VEC];
#pragma unroll
            for (int q = 0; q < VEC; ++q) t[q] = sp[q * 64 + lane];
            store_block_wt<VEC>(sbase + (wb + idx) * a.block, t, lane);
            ++idx;
          }
        }
      }
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

// ---------------------------------------------------------------- k_scanm: m >= 2 workers on one device
//
// Work unit = the blocks of G consecutive lanes of one row, for every worker (G = 32 lanes: 32 KiB per worker at
// B=256; the whole row when it is narrower).  Units are swept grid-stride, one unit per wave, the workgroup ->
// unit order XCD-contiguous.  Per group of SUB blocks the m workers' blocks are read in rank order (buffer loads,
// nt; SUB*VEC = 32 dwordx4 per lane in flight) and accumulated from +0.0f (server.cc:148-150, :97-98); each block's
// ballot gives the worker's flag bit.  Adding a zero-flagged worker's block (all +-0.0) to an accumulator that
// started at +0.0 never changes it, so summing every worker equals the reference, which only adds the workers
// that sent the block.  The aggregated blocks go out write-through with a static store schedule (a block outside
// the write set is pointed past the row's descriptor and dropped).  Lane w keeps worker w's bits of the unit and
// stores them as the unit's piece of row mask w (a 32-bit store, or the whole 64-bit mask when the unit is the
// row); lane m stores the union's piece.
// The 32-load groups take ~270 VGPRs, i.e. ONE wave per SIMD.  tools/tune_scanm_r02.py (profiles/r02/scanm/):
// at 8 x 256 MiB, with one output per input set as bench.py rotates them, this shape with non-temporal stores
// runs 359 us against 385 us with write-through (sc0 sc1) stores and 439 us for round 1's kernel (a wave per
// 64 KiB row, 16 loads in flight, three waves per SIMD) on the same box.  More waves or more loads in flight per
// CU (a second register set, or forcing 2-3 waves per SIMD) were slower, and staggering the worker buffers'
// offsets (the channel-contention hypothesis) changed nothing.
constexpr int kScanmStoreAux = 2;  // nt: the sums are a separate output stream, not re-read by this launch

template <int VEC, int SUB, int G>
__global__ __launch_bounds__(kWGThreads) void k_scanm(ScanArgs a) {
  constexpr uint32_t B4 = 64 * VEC;  // 16-byte vectors per block
  static_assert(G % SUB == 0 && G <= 64 && SUB <= 32, "a unit is whole SUB-groups of one row");
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // lanes per unit; the host picks SUB <= lanes (launch_scan), so a group never reaches into the next row
  const uint32_t gl = a.lanes < static_cast<uint32_t>(G) ? a.lanes : static_cast<uint32_t>(G);
  const uint32_t upr = a.lanes / gl;  // units per row (1 or 2)
  const uint64_t units = a.rows * upr;
  const uint32_t T = gridDim.x, bid = blockIdx.x;
  const uint32_t lin = (T % 8 == 0) ? (bid % 8) * (T / 8) + bid / 8 : bid;  // XCD-contiguous units
  const uint64_t stride = static_cast<uint64_t>(T) * kWavesPerWG;
  for (uint64_t u = static_cast<uint64_t>(lin) * kWavesPerWG + wave; u < units; u += stride) {
    const uint64_t row = u / upr;
    const uint32_t g0 = static_cast<uint32_t>(u % upr) * gl;
    const bool head = (row % a.rows_per_part) == 0;
    const uint64_t rowbase = row * a.lanes * B4 * 4;  // float offset of the row
    const __amdgpu_buffer_rsrc_t dst = chunk_rsrc(a.out + rowbase, a.out != nullptr ? a.lanes * B4 * 16 : 0u);
    uint64_t lane_wm = 0;  // lane w: worker w's bits of the unit (bit i = lane g0 + i)
    uint64_t um = 0;       // union bits (wave-uniform)
    for (uint32_t l0 = g0; l0 < g0 + gl; l0 += SUB) {
      v4f acc[SUB][VEC];
#pragma unroll
      for (int s = 0; s < SUB; ++s)
#pragma unroll
        for (int q = 0; q < VEC; ++q) acc[s][q] = v4f{0.f, 0.f, 0.f, 0.f};
      uint32_t sub_any = 0;
      const uint64_t goff = rowbase + static_cast<uint64_t>(l0) * B4 * 4;
      for (uint32_t w = 0; w < a.m; ++w) {
        const __amdgpu_buffer_rsrc_t src = chunk_rsrc(a.x.p[w] + goff, SUB * B4 * 16);
        v4f v[SUB][VEC];
#pragma unroll
        for (int s = 0; s < SUB; ++s)
#pragma unroll
          for (int q = 0; q < VEC; ++q)
            v[s][q] = __builtin_bit_cast(
                v4f, __builtin_amdgcn_raw_buffer_load_b128(src, (s * B4 + q * 64 + lane) * 16, 0, kLoadAux));
        __builtin_amdgcn_sched_barrier(0);  // the whole group in flight before the first use
        uint32_t wbits = 0;
#pragma unroll
        for (int s = 0; s < SUB; ++s) {
          uint32_t o = 0;
#pragma unroll
          for (int q = 0; q < VEC; ++q) {
            o |= nz_bits(v[s][q]);
            acc[s][q] = add4(acc[s][q], v[s][q]);  // rank order: worker w after w-1 (server.cc:97-98)
          }
          wbits |= static_cast<uint32_t>(wave_ballot(o != 0) != 0) << s;
        }
        if (lane == static_cast<int>(w)) lane_wm |= static_cast<uint64_t>(wbits) << (l0 - g0);
        sub_any |= wbits;
      }
      um |= static_cast<uint64_t>(sub_any) << (l0 - g0);
#pragma unroll
      for (int s = 0; s < SUB; ++s) {
        const uint32_t drop = (((sub_any >> s) & 1u) || head) ? 0u : kDropStore;
#pragma unroll
        for (int q = 0; q < VEC; ++q)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, acc[s][q]), dst,
                                                 (((l0 + s) * B4 + q * 64 + lane) * 16) | drop, 0, kScanmStoreAux);
      }
    }
    // the unit's piece of row mask `lane` (workers 0..m-1, union at m); lanes >= NB stay zero
    if (lane <= static_cast<int>(a.m)) {
      const uint64_t bits = lane == static_cast<int>(a.m) ? um : lane_wm;
      uint64_t* mrow = a.masks + static_cast<uint64_t>(lane) * a.rows + row;
      if (gl == a.lanes)
        *mrow = bits;
      else  // two 32-lane units per 64-lane row
        reinterpret_cast<uint32_t*>(mrow)[g0 / 32] = static_cast<uint32_t>(bits);
    }
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

constexpr int kScanmUnitLanes = 32;  // G

// ---------------------------------------------------------------- k_next: next-offset chains
//
// next[b] for block b = (row r, lane l) = offset of the first row r' > r of the same partition whose
// mask has bit l, else sentinel + l*B (find_next_nonzero_block(b*B + B*NB), client.cc:19-31).
// Workgroup = one segment of <= 64 rows of one partition and one mask array (blockIdx.y).  A wave holds
// 64 row masks (lane i = row i) and turns them into 64 column masks (lane l = lane-column l, bit i = row i)
// with a 6-stage butterfly bit transpose, so "first non-zero row per lane" is one ctz per thread.
// Wave 0 transposes the segment itself; all four waves then sweep the rows after it, 256 per round, until
// every lane has found its first non-zero row (or the partition ends).
struct NextArgs {
  const uint64_t* masks;
  uint32_t* next;
  uint64_t rows;           // rows per mask array
  uint64_t nb;             // blocks per array (output stride)
  uint32_t rows_per_part;
  uint32_t segs_per_part;
  uint32_t lanes;
  uint32_t block;
  uint32_t sentinel;
};

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
  const uint32_t lo = __shfl_xor(static_cast<uint32_t>(v), m, 64);
  const uint32_t hi = __shfl_xor(static_cast<uint32_t>(v >> 32), m, 64);
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

// 64x64 bit-matrix transpose across a wave: in, lane r holds row r (bit c = element (r, c)); out, lane c
// holds column c (bit r = element (r, c)).  Stage j swaps bit j of the row index with bit j of the column.
__device__ __forceinline__ uint64_t wave_transpose64(uint64_t a, int lane) {
  constexpr uint64_t M[6] = {0x00000000FFFFFFFFull, 0x0000FFFF0000FFFFull, 0x00FF00FF00FF00FFull,
                             0x0F0F0F0F0F0F0F0Full, 0x3333333333333333ull, 0x5555555555555555ull};
#pragma unroll
  for (int s = 0; s < 6; ++s) {
    const int j = 32 >> s;
    const uint64_t m = M[s];
    const uint64_t x = shfl_xor64(a, j);
    a = (lane & j) ? ((a & ~m) | ((x & ~m) >> j)) : ((a & m) | ((x & m) << j));
  }
  return a;
}

// One k_next segment with W waves; mask_of(r) gives row r's mask (one array, or the union of several).
template <int W, typename MaskOf>
__device__ __forceinline__ void next_segment(const NextArgs& a, uint32_t seg_id, const MaskOf& mask_of, uint32_t* next) {
  __shared__ uint64_t s_col[64];
  __shared__ uint32_t s_first[W][64];
  __shared__ uint32_t s_carry_row[64];
  __shared__ int s_done;
  if (threadIdx.x == 0) s_done = 0;
  const uint32_t part = seg_id / a.segs_per_part;
  const uint32_t seg = seg_id % a.segs_per_part;
  const uint64_t part_row0 = static_cast<uint64_t>(part) * a.rows_per_part;
  const uint64_t part_end = part_row0 + a.rows_per_part;
  const uint64_t row0 = part_row0 + static_cast<uint64_t>(seg) * 64;
  const uint64_t seg_end = (row0 + 64 < part_end) ? row0 + 64 : part_end;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const uint32_t row_stride = a.lanes * a.block;  // floats per row

  // the segment's own masks and the first look-ahead rows are loaded together (independent round trips)
  const uint64_t r = row0 + lane;
  const uint64_t seg_mask = (wave == 0 && r < seg_end) ? mask_of(r) : 0ull;
  uint64_t look = seg_end;
  uint64_t rr = look + static_cast<uint64_t>(wave) * 64 + lane;
  uint64_t look_mask = (rr < part_end) ? mask_of(rr) : 0ull;
  if (wave == 0) {
    s_col[lane] = wave_transpose64(seg_mask, lane);
    s_carry_row[lane] = kNone;
  }
  while (look < part_end) {
    const uint64_t col = wave_transpose64(look_mask, lane);
    s_first[wave][lane] = col ? static_cast<uint32_t>(look + wave * 64 + __builtin_ctzll(col)) : kNone;
    __syncthreads();
    if (wave == 0) {
      uint32_t cr = s_carry_row[lane];
#pragma unroll
      for (int w = 0; w < W; ++w)
        if (cr == kNone) cr = s_first[w][lane];
      s_carry_row[lane] = cr;
      const uint64_t open = __ballot(lane < static_cast<int>(a.lanes) && cr == kNone);
      if (lane == 0) s_done = (open == 0);
    }
    __syncthreads();
    if (s_done) break;
    look += 64 * W;
    rr = look + static_cast<uint64_t>(wave) * 64 + lane;
    look_mask = (rr < part_end) ? mask_of(rr) : 0ull;
  }
  __syncthreads();
  const uint32_t nrows = static_cast<uint32_t>(seg_end - row0);
  const uint32_t lshift = static_cast<uint32_t>(__builtin_ctz(a.lanes));  // lanes is a power of two
  const uint32_t total = nrows << lshift;
  for (uint32_t idx = threadIdx.x; idx < total; idx += 64 * W) {
    const uint32_t i = idx >> lshift;
    const uint32_t l = idx & (a.lanes - 1);
    const uint64_t c = (i >= 63) ? 0 : (s_col[l] >> (i + 1));
    uint32_t v;
    if (c != 0) {
      v = static_cast<uint32_t>(row0 + i + 1 + __builtin_ctzll(c)) * row_stride + l * a.block;
    } else {
      const uint32_t cr = s_carry_row[l];
      v = (cr != kNone) ? cr * row_stride + l * a.block : a.sentinel + l * a.block;
    }
    next[(row0 << lshift) + idx] = v;
  }
}

__global__ __launch_bounds__(kWGThreads) void k_next(NextArgs a) {
  const uint64_t* masks = a.masks + static_cast<uint64_t>(blockIdx.y) * a.rows;
  next_segment<kWavesPerWG>(a, blockIdx.x, [&](uint64_t r) { return masks[r]; },
                            a.next + static_cast<uint64_t>(blockIdx.y) * a.nb);
}

// ---------------------------------------------------------------- compaction (mask -> block list)

constexpr int kCompactRows = kWGThreads;  // rows per workgroup

__device__ __forceinline__ uint32_t wg_reduce_sum(uint32_t v, uint32_t* s_tmp) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) s_tmp[wave] = v;
  __syncthreads();
  uint32_t t = 0;
  for (int w = 0; w < kWavesPerWG; ++w) t += s_tmp[w];
  __syncthreads();
  return t;
}

__global__ __launch_bounds__(kWGThreads) void k_compact_count(const uint64_t* masks, uint64_t row_begin,
                                                              uint64_t row_end, uint32_t* chunk_sum) {
  __shared__ uint32_t s_tmp[kWavesPerWG];
  const uint64_t r = row_begin + static_cast<uint64_t>(blockIdx.x) * kCompactRows + threadIdx.x;
  const uint32_t pc = (r < row_end) ? static_cast<uint32_t>(__builtin_popcountll(masks[r])) : 0u;
  const uint32_t t = wg_reduce_sum(pc, s_tmp);
  if (threadIdx.x == 0) chunk_sum[blockIdx.x] = t;
}

__global__ __launch_bounds__(kWGThreads) void k_compact_write(const uint64_t* masks, uint64_t row_begin,
                                                              uint64_t row_end, uint32_t lanes,
                                                              const uint32_t* chunk_sum, uint32_t* list,
                                                              uint32_t* count) {
  __shared__ uint32_t s_tmp[kWavesPerWG];
  __shared__ uint32_t s_wave[kWavesPerWG];
  uint32_t base_part = 0;
  for (uint32_t c = threadIdx.x; c < blockIdx.x; c += kWGThreads) base_part += chunk_sum[c];
  const uint32_t base = wg_reduce_sum(base_part, s_tmp);
  const uint64_t r = row_begin + static_cast<uint64_t>(blockIdx.x) * kCompactRows + threadIdx.x;
  const uint64_t rm = (r < row_end) ? masks[r] : 0;
  const uint32_t pc = static_cast<uint32_t>(__builtin_popcountll(rm));
  // inclusive wave scan
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t inc = pc;
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t t = __shfl_up(inc, off, 64);
    if (lane >= off) inc += t;
  }
  if (lane == 63) s_wave[wave] = inc;
  __syncthreads();
  uint32_t wbase = 0;
  for (int w = 0; w < wave; ++w) wbase += s_wave[w];
  uint32_t pos = base + wbase + inc - pc;
  uint64_t bits = rm;
  while (bits != 0) {
    const uint32_t l = static_cast<uint32_t>(__builtin_ctzll(bits));
    bits &= bits - 1;
    list[pos++] = static_cast<uint32_t>(r * lanes + l);
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == kWGThreads - 1) *count = pos;
}

// ---------------------------------------------------------------- multi-GPU exchange helpers
//
// The N-rank sparse all-reduce (omr/dist.py) moves only non-zero blocks between ranks.  Aggregator s owns a
// contiguous range of rows (the reference shards message slots over aggregators, common.cc:381-383); worker w
// sends it its non-zero blocks of that range in increasing block order.  These kernels derive every block's
// position in such a packed stream from the all-gathered row masks, so no index lists cross the link.

// out[r] = OR over `count` mask arrays of row r; lane-head rows (r % rows_per_part == 0) forced to all lanes
// when heads != 0 (the reference always sends lane heads: client.cc:201-205).
__global__ __launch_bounds__(kWGThreads) void k_mask_union(const uint64_t* masks, uint32_t count, uint64_t rows,
                                                           uint32_t rows_per_part, uint64_t lane_bits, int heads,
                                                           uint64_t* out) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kWGThreads;
  for (uint64_t r = static_cast<uint64_t>(blockIdx.x) * kWGThreads + threadIdx.x; r < rows; r += stride) {
    uint64_t u = 0;
    for (uint32_t w = 0; w < count; ++w) u |= masks[static_cast<uint64_t>(w) * rows + r];
    if (heads && (r % rows_per_part) == 0) u |= lane_bits;
    out[r] = u;
  }
}

// prefix[a][r] = number of set bits of array a in rows [0, r), r = 0..rows (exclusive scan of popcounts).
__global__ __launch_bounds__(kWGThreads) void k_prefix_chunks(const uint64_t* masks, uint64_t rows,
                                                              uint32_t* chunk_sum) {
  __shared__ uint32_t s_tmp[kWavesPerWG];
  const uint64_t* m = masks + static_cast<uint64_t>(blockIdx.y) * rows;
  const uint64_t r = static_cast<uint64_t>(blockIdx.x) * kCompactRows + threadIdx.x;
  const uint32_t pc = (r < rows) ? static_cast<uint32_t>(__builtin_popcountll(m[r])) : 0u;
  const uint32_t t = wg_reduce_sum(pc, s_tmp);
  if (threadIdx.x == 0) chunk_sum[static_cast<uint64_t>(blockIdx.y) * gridDim.x + blockIdx.x] = t;
}

__global__ __launch_bounds__(kWGThreads) void k_prefix_write(const uint64_t* masks, uint64_t rows,
                                                             const uint32_t* chunk_sum, uint32_t* prefix) {
  __shared__ uint32_t s_tmp[kWavesPerWG];
  __shared__ uint32_t s_wave[kWavesPerWG];
  const uint64_t* m = masks + static_cast<uint64_t>(blockIdx.y) * rows;
  const uint32_t* cs = chunk_sum + static_cast<uint64_t>(blockIdx.y) * gridDim.x;
  uint32_t* pre = prefix + static_cast<uint64_t>(blockIdx.y) * (rows + 1);
  uint32_t base_part = 0;
  for (uint32_t c = threadIdx.x; c < blockIdx.x; c += kWGThreads) base_part += cs[c];
  const uint32_t base = wg_reduce_sum(base_part, s_tmp);
  const uint64_t r = static_cast<uint64_t>(blockIdx.x) * kCompactRows + threadIdx.x;
  const uint32_t pc = (r < rows) ? static_cast<uint32_t>(__builtin_popcountll(m[r])) : 0u;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t inc = pc;
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t t = __shfl_up(inc, off, 64);
    if (lane >= off) inc += t;
  }
  if (lane == 63) s_wave[wave] = inc;
  __syncthreads();
  uint32_t wbase = 0;
  for (int w = 0; w < wave; ++w) wbase += s_wave[w];
  if (r < rows) pre[r] = base + wbase + inc - pc;
  if (r == rows - 1) pre[rows] = base + wbase + inc;
}

// Aggregator shard sum over packed worker streams (server.cc:97-98, rank order from a zeroed accumulator):
// for the k-th listed block b = (row r, lane l) of this shard, worker w contributes iff bit l of its mask
// row r is set, and its block sits at position prefix_w[r] - prefix_w[row_begin] + popcount(mask_w[r] below
// bit l) of w's packed stream, which starts at block recv_off[w] of `recv`.
template <int VEC>
__global__ __launch_bounds__(kWGThreads) void k_sparse_sum(const float* recv, const uint64_t* recv_off,
                                                           const uint64_t* masks, uint32_t count, uint64_t rows,
                                                           const uint32_t* prefix, uint64_t row_begin,
                                                           uint32_t lshift, const uint32_t* list, uint32_t num,
                                                           float* out) {
  constexpr int B4 = 64 * VEC;
  const int lane = threadIdx.x & 63;
  const uint32_t nwaves = gridDim.x * kWavesPerWG;
  const v4f* src = reinterpret_cast<const v4f*>(recv);
  for (uint32_t k = blockIdx.x * kWavesPerWG + (threadIdx.x >> 6); k < num; k += nwaves) {
    const uint32_t b = list[k];
    const uint64_t r = b >> lshift;
    const uint32_t l = b & ((1u << lshift) - 1u);
    v4f acc[VEC];
#pragma unroll
    for (int q = 0; q < VEC; ++q) acc[q] = v4f{0.f, 0.f, 0.f, 0.f};
    for (uint32_t w = 0; w < count; ++w) {
      const uint64_t mw = masks[static_cast<uint64_t>(w) * rows + r];
      if ((mw >> l) & 1u) {
        const uint32_t* pw = prefix + static_cast<uint64_t>(w) * (rows + 1);
        const uint64_t idx = recv_off[w] + (pw[r] - pw[row_begin]) +
                             static_cast<uint64_t>(__builtin_popcountll(mw & ((1ull << l) - 1ull)));
#pragma unroll
        for (int q = 0; q < VEC; ++q) acc[q] = add4(acc[q], src[idx * B4 + q * 64 + lane]);
      }
    }
    v4f* dst = reinterpret_cast<v4f*>(out) + static_cast<uint64_t>(k) * B4 + lane;
#pragma unroll
    for (int q = 0; q < VEC; ++q) dst[q * 64] = acc[q];
  }
}

// ---------------------------------------------------------------- block movement / list sum

template <int VEC>
__global__ __launch_bounds__(kWGThreads) void k_gather(const float* src, const uint32_t* list, uint32_t num,
                                                       float* packed) {
  constexpr int B4 = 64 * VEC;
  const int lane = threadIdx.x & 63;
  const uint32_t nwaves = gridDim.x * kWavesPerWG;
  for (uint32_t k = blockIdx.x * kWavesPerWG + (threadIdx.x >> 6); k < num; k += nwaves) {
    const v4f* s = reinterpret_cast<const v4f*>(src) + static_cast<uint64_t>(list[k]) * B4 + lane;
    v4f* d = reinterpret_cast<v4f*>(packed) + static_cast<uint64_t>(k) * B4 + lane;
    v4f v[VEC];
#pragma unroll
    for (int q = 0; q < VEC; ++q) v[q] = s[q * 64];
#pragma unroll
    for (int q = 0; q < VEC; ++q) d[q * 64] = v[q];
  }
}

template <int VEC>
__global__ __launch_bounds__(kWGThreads) void k_scatter(const float* packed, const uint32_t* list,
                                                        uint32_t num, float* dst) {
  constexpr int B4 = 64 * VEC;
  const int lane = threadIdx.x & 63;
  const uint32_t nwaves = gridDim.x * kWavesPerWG;
  for (uint32_t k = blockIdx.x * kWavesPerWG + (threadIdx.x >> 6); k < num; k += nwaves) {
    const v4f* s = reinterpret_cast<const v4f*>(packed) + static_cast<uint64_t>(k) * B4 + lane;
    v4f* d = reinterpret_cast<v4f*>(dst) + static_cast<uint64_t>(list[k]) * B4 + lane;
    v4f v[VEC];
#pragma unroll
    for (int q = 0; q < VEC; ++q) v[q] = s[q * 64];
#pragma unroll
    for (int q = 0; q < VEC; ++q) d[q * 64] = v[q];
  }
}

// Dense rank-order sum of m arrays (the dense stand-in aggregator, omr_dense_sum_f32): four dwordx4 per lane
// per worker in flight, grid-stride.
__global__ __launch_bounds__(kWGThreads) void k_dense_sum(WorkerPtrs in, uint32_t m, uint64_t n4, float* out) {
  constexpr int U = 4;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kWGThreads;
  for (uint64_t i0 = static_cast<uint64_t>(blockIdx.x) * kWGThreads + threadIdx.x; i0 < n4; i0 += stride * U) {
    v4f acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = v4f{0.f, 0.f, 0.f, 0.f};
    for (uint32_t w = 0; w < m; ++w) {
      const v4f* src = reinterpret_cast<const v4f*>(in.p[w]);
      v4f v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = i0 + u * stride < n4 ? src[i0 + u * stride] : v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u] = add4(acc[u], v[u]);
    }
    v4f* dst = reinterpret_cast<v4f*>(out);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i0 + u * stride < n4) dst[i0 + u * stride] = acc[u];
  }
}

template <int VEC>
__global__ __launch_bounds__(kWGThreads) void k_list_sum(WorkerPtrs in, uint32_t m, const uint32_t* list,
                                                         uint32_t num, float* out) {
  constexpr int B4 = 64 * VEC;
  const int lane = threadIdx.x & 63;
  const uint32_t nwaves = gridDim.x * kWavesPerWG;
  for (uint32_t k = blockIdx.x * kWavesPerWG + (threadIdx.x >> 6); k < num; k += nwaves) {
    const uint64_t off = static_cast<uint64_t>(list[k]) * B4 + lane;
    v4f acc[VEC];
#pragma unroll
    for (int q = 0; q < VEC; ++q) acc[q] = v4f{0.f, 0.f, 0.f, 0.f};
    for (uint32_t w = 0; w < m; ++w) {
      const v4f* s = reinterpret_cast<const v4f*>(in.p[w]) + off;
#pragma unroll
      for (int q = 0; q < VEC; ++q) acc[q] = add4(acc[q], s[q * 64]);
    }
    v4f* d = reinterpret_cast<v4f*>(out) + off;
#pragma unroll
    for (int q = 0; q < VEC; ++q) d[q * 64] = acc[q];
  }
}

// ---------------------------------------------------------------- multi-rank round kernels (mask-addressed)
//
// The round's block movement is addressed straight from row masks and their popcount prefixes, with no block
// lists: the k-th set bit of a mask (in block order) is block k of that mask's packed stream.  Work unit = one
// wave per (row, group of `lg` lanes); the unit's SET bits are taken SL at a time, so a batch is SL present
// blocks whatever the density (all loaded before any is stored; a short batch's spare slots are pointed past the
// descriptor range and dropped, keeping the memory-operation count static).  lg is chosen on the host so that
// there are enough units to fill the chip (whole rows when there are many rows).
template <int VEC>
constexpr int move_slots() {  // blocks per batch for a pure move
  return 16 / VEC;
}

__device__ __forceinline__ uint64_t below(uint32_t l) { return l >= 64 ? ~0ull : ((1ull << l) - 1ull); }

// (the builtin returns int: go through uint32_t, or the low half would be sign-extended into the high half)
__device__ __forceinline__ uint64_t readlane64(uint64_t v, uint32_t lane) {
  const uint32_t lo = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(static_cast<uint32_t>(v)), lane));
  const uint32_t hi = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(static_cast<uint32_t>(v >> 32)), lane));
  return static_cast<uint64_t>(lo) | (static_cast<uint64_t>(hi) << 32);
}

// Takes up to SL set bits off `rem` (lowest first): their lane indices, how many, and their mask.
template <int SL>
__device__ __forceinline__ uint32_t take_bits(uint64_t& rem, uint32_t (&lj)[SL], uint64_t& bmask) {
  uint32_t nv = 0;
  bmask = 0;
#pragma unroll
  for (int j = 0; j < SL; ++j) {
    lj[j] = 0;
    if (rem != 0) {
      lj[j] = static_cast<uint32_t>(__builtin_ctzll(rem));
      bmask |= rem & (~rem + 1);
      rem &= rem - 1;
      nv = j + 1;
    }
  }
  return nv;
}

// the pair list's unit: 16 rows x one lane (a quarter of a 64-row group), as k_shard_sum's
constexpr uint32_t kSumUnitRows = 16;
constexpr uint32_t kSumUnitsPerGroup = 64 / kSumUnitRows;
// k_shard_sum's unit rows (a divisor of the 64-row group).  16: 2048 waves at config 4's 8-worker shard, two per
// SIMD, nearly all of them one window (<= 32 pairs); with 32-row units 11 % of the waves needed a second window, a
// round trip after everyone else's (14.16 against 15.35 us, stamped copies, profiles/r04/shard/)
constexpr uint32_t kShardUnitRows = 16;
// a pair record: source block (bits 0-31: in `own` or in `recv`), destination block (32-59), flags
constexpr uint64_t kRecOwn = 1ull << 60, kRecZero = 1ull << 61, kRecFirst = 1ull << 62, kRecLast = 1ull << 63;
// a pair list's unit ends with this word (no real record has every bit set: destinations are < 2^28 blocks), so the
// sum finds its unit's length in the same load as its first records
constexpr uint64_t kRecEnd = ~0ull;

// ---------------------------------------------------------------- the shard sum's pair list, built before the exchange
// (round 3, second session).  The aggregator's shard sum over the fused pack's column streams (k_shard_sum below) spent
// most of its time before its first data load: at an 8-worker shard every wave fetched its unit's index data (one
// round trip), built its (block, contributor) pairs, and only then loaded blocks -- 7.3 of 12 us per wave, the chip's
// 1024 waves in lock step (profiles/r03/round/tune_shard_r03.log).  Everything those pairs depend on is known before
// the exchange: the workers' masks and position tables (all-gathered) and where each worker's stream will land in
// `recv` (a fixed region per worker).  So the pairs are built by extra workgroups of the round's plan launch, hidden
// behind the exchange, and the sum (k_shard_sum_list) starts with one coalesced load of its unit's records.
struct ListArgs {
  const uint64_t* masks;  // worker c's row masks at masks + c * mstride, its position table at word pos_off
  uint64_t mstride, pos_off;
  uint64_t recv_off[OMR_MAX_WORKERS];
  uint64_t rows, r0, r1, all_lanes;
  uint32_t count, me, lanes, rpp, S, gps, cap;
  uint64_t* records;  // unit u's records at records + u * cap, in (block, rank) order
  uint32_t* counts;   // unit u's record count
};

__device__ __forceinline__ uint64_t list_units(const ListArgs& a) {
  return ((a.r1 - a.r0) / a.S) * a.gps * kSumUnitsPerGroup * a.lanes;
}

// Units [u0, units) step ustride, one wave each: unit = kSumUnitRows rows x one lane (a part of a segment's 64-row
// group), as k_shard_sum's column-stream units.  Lane i holds row i of the group: ONE round trip fetches every worker's mask row
// and position-table entry; ballots give each worker's column bits; a wave-wide exclusive scan places each lane's
// pairs; records go straight to global memory.
// Workgroup i of n consecutive ones (the first at grid position base) -> a logical index such that each XCD (the
// hardware deals workgroups to the 8 XCDs round robin by grid position) takes one contiguous range of logical
// indices.  The pair list's neighbouring units read the same mask rows and position-table entries (the 64 lanes of a
// row group, 256 units), so with consecutive units on one XCD each XCD's L2 fetches a group once instead of every
// XCD fetching every group.  n not a multiple of 8: identity.
__device__ __forceinline__ uint32_t xcd_spread(uint32_t i, uint32_t base, uint32_t n) {
  if (n % 8 != 0) return i;
  return ((base + i) % 8) * (n / 8) + i / 8;
}

// W >= count: the workers' mask rows a unit loads (the plan launch's width: at 8 workers half the loads, registers and
// L2 requests of the 16-wide form, whose 2 048 units each fetched every group's rows for 16 workers)
template <int W = OMR_MAX_WORKERS>
__device__ __forceinline__ void build_sum_list(const ListArgs& a, uint64_t u0, uint64_t ustride) {
  const int lane = threadIdx.x & 63;
  const uint64_t units = list_units(a);
  for (uint64_t u = u0; u < units; u += ustride) {
    const uint32_t l = static_cast<uint32_t>(u % a.lanes);
    uint64_t t = u / a.lanes;
    const uint32_t h = static_cast<uint32_t>(t % kSumUnitsPerGroup);
    t /= kSumUnitsPerGroup;
    const uint32_t j = static_cast<uint32_t>(t % a.gps);
    const uint64_t seg = a.r0 / a.S + t / a.gps;
    const uint64_t g0 = seg * a.S + static_cast<uint64_t>(j) * kPackGroupRows;
    const uint32_t nload = a.S - j * kPackGroupRows < kPackGroupRows ? a.S - j * kPackGroupRows : kPackGroupRows;
    const uint32_t h0 = h * kSumUnitRows;
    const uint32_t h1 = nload < h0 + kSumUnitRows ? nload : h0 + kSumUnitRows;
    const uint64_t gidx = seg * a.gps + j;
    if (h0 >= h1) {
      if (lane == 0) {
        a.counts[u] = 0;
        a.records[u * a.cap] = kRecEnd;
      }
      continue;
    }
    const bool rl = static_cast<uint32_t>(lane) < nload;
    const uint64_t r = g0 + (rl ? static_cast<uint32_t>(lane) : 0u);
    uint64_t mk[W];  // (unconditional loads from clamped addresses: one round trip, see plan_rows)
#pragma unroll
    for (uint32_t c = 0; c < W; ++c) {
      const uint64_t v = a.masks[(c < a.count ? c : 0u) * a.mstride + r];
      mk[c] = (c < a.count && rl) ? v : 0ull;
    }
    const bool cl = static_cast<uint32_t>(lane) < a.count;
    const uint32_t base_c =
        cl ? reinterpret_cast<const uint32_t*>(a.masks + lane * a.mstride)[a.pos_off + gidx * a.lanes + l] : 0u;
    uint64_t un = 0;
#pragma unroll
    for (uint32_t c = 0; c < W; ++c) un |= mk[c];
    const uint64_t w = (rl && r % a.rpp == 0) ? (un | a.all_lanes) : un;  // write set: union + lane heads
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
    if (lane == 0) {
      a.counts[u] = total;
      a.records[u * a.cap + total] = kRecEnd;
    }
    if (total == 0) continue;
    uint64_t ccol[W];  // worker c's bits of column l over the group's rows
#pragma unroll
    for (uint32_t c = 0; c < W; ++c) ccol[c] = c < a.count ? __ballot((mk[c] >> l) & 1ull) : 0ull;
    if (np != 0) {
      uint64_t* const rec = a.records + u * a.cap;
      uint32_t k = inc - np;
      const uint32_t first = k, last = inc - 1;
      const uint64_t hdr = (r * a.lanes + l) << 32;  // the block's dense index (the sum converts it when packing)
      if (cb == 0) {
        rec[k] = hdr | kRecZero | kRecFirst | kRecLast;
      } else {
#pragma unroll
        for (uint32_t c = 0; c < W; ++c) {
          if (!((cb >> c) & 1u)) continue;
          uint64_t v;
          if (c == a.me) {
            v = (r * a.lanes + l) | kRecOwn;
          } else {
            const uint32_t bc = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(base_c), c));
            const uint64_t pos = static_cast<uint64_t>(bc) +
                                 static_cast<uint64_t>(__builtin_popcountll(ccol[c] & below(static_cast<uint32_t>(lane))));
            v = (a.recv_off[c] + pos) & 0xFFFFFFFFull;
          }
          v |= hdr | (k == first ? kRecFirst : 0ull) | (k == last ? kRecLast : 0ull);
          rec[k++] = v;
        }
      }
    }
  }
}

struct PlanArgs {
  const uint64_t* masks;  // worker c's row masks at masks + c * mstride
  uint32_t count, rpp, lanes, nbounds;
  uint64_t rows, mstride;
  uint32_t* zero_cnt;     // [zero_cnt_n] cleared (the next round's pack counters), or null
  uint32_t zero_cnt_n;
  const uint64_t* bounds;
  uint64_t* write_set;
  uint64_t* union_masks;  // or null
  uint32_t* prefix;
  uint64_t* counts;       // (seq << 32) | prefix at a bound; device or host-mapped memory (stored at system scope)
  uint64_t* zero_masks;   // or null
  uint64_t* ws;           // [0] ticket counter (zero between launches), [1 + chunk * (W + 1) + a] chunk totals
                          //   (packed at the launch's W: a chunk's lower chunks' totals are consecutive words)
  uint32_t seq;           // this launch's tag (differs from the previous launch's on the workspace)
  uint32_t nchunks, tiles;  // chunks of tiles * 256 rows
  NextArgs chain;       // union_next: the aggregator chain over the union, by workgroups after the chunks' (chain.next
  uint32_t chain_wgs;   //   null: none)
  uint32_t list_wgs;    // the shard sum's pair list, by the workgroups after the chain's (0: none)
  ListArgs list;
  // the round check (omr_round_plan_check), by one workgroup after the list's: worker c's scan slots (k_scan1f CHK) at
  // masks + c * mstride + chk_off; chk_status null: no check
  uint64_t chk_off;
  uint32_t chk_slots;
  uint64_t* chk_status;
};

// Inclusive prefix sum over the 64 lanes of a wave in six DPP steps (no LDS): row_shr 1, 2, 4, 8 inside each 16-lane
// row, then row_bcast:15 (rows 1 and 3 add the last lane of the row before) and row_bcast:31 (rows 2 and 3 add lane 31).
// Lanes whose source is out of the row keep `old` = 0.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x111, 0xf, 0xf, false));
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x112, 0xf, 0xf, false));
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x114, 0xf, 0xf, false));
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x118, 0xf, 0xf, false));
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x142, 0xa, 0xf, false));
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x143, 0xc, 0xf, false));
  return v;
}

// The round's bookkeeping (server.cc:83-96) over row chunks (round 5).  Every mask is read once, by the chunk that owns
// its row, and the chunks run side by side: a single workgroup doing everything measured 32.6 us at config 4's shapes,
// 11 of it per 2048-row tile issuing its prefix stores from one CU (profiles/r05/plan_probe/), and round 3/4's
// workgroup per mask array (the write-set one re-reading every worker's masks) 11.6 us at 1.95-1.99 x the algorithmic
// HBM bytes.  A chunk workgroup (256 threads, one row per thread and tile):
//   1. takes a ticket (its chunk: every lower chunk belongs to a workgroup that has started, so the wait in 3 ends);
//   2. reads its rows of every worker's masks (range-checked buffer loads: a row past the end or a worker past `count`
//      reads 0, no branch), forms union = OR of the workers (the aggregator's min_next domain) and write set = union |
//      lane heads (every lane head is sent and returned, client.cc:201-205), and each array's popcount total;
//   3. publishes its totals tagged with `seq` and adds the lower chunks' totals as they appear (no chain: every chunk
//      publishes before it waits, so the waits overlap);
//   4. lays out its rows' prefixes (DPP wave scans, one LDS exchange of the wave totals) and stores them with the write
//      set, the union and the cleared own masks; a row at a shard bound stores counts[a][s] = (seq << 32) | prefix.
// The host reads the counts when every one it needs carries `seq`: no completion notice, no arrival counter, no wait for
// the stores' acknowledgements inside the kernel.  The last chunk re-arms the ticket and stores the totals.
constexpr uint32_t kPlanThreads = 256;
constexpr uint32_t kPlanWaves = kPlanThreads / 64;
constexpr uint32_t kPlanChunksMax = 64;
constexpr uint32_t kPlanArrays = OMR_MAX_WORKERS + 1;
// ... then the round check's findings (plan_check): per worker the sum of its scan's slots or a stale flag, tagged with
// seq, which the last chunk compares with its totals
constexpr uint64_t kPlanCheckWords = 1 + static_cast<uint64_t>(kPlanChunksMax) * kPlanArrays;
constexpr uint64_t kPlanWorkspaceWords = kPlanCheckWords + OMR_MAX_WORKERS + 1;
constexpr uint32_t kCheckStale = 0x100u, kCheckCount = 0x200u;

template <int W>
__device__ __forceinline__ void plan_chunk(const PlanArgs& a) {
  constexpr uint32_t NA = W + 1;  // arrays unrolled: W workers, then the write set
  __shared__ uint32_t s_wtot[kPlanWaves][NA];
  __shared__ uint32_t s_base[NA];
  __shared__ uint32_t s_chunk;
  __shared__ uint64_t s_bounds[OMR_MAX_WORKERS + 2];
  const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const uint32_t cnt = a.count;
  const uint64_t all_lanes = a.lanes >= 64 ? ~0ull : ((1ull << a.lanes) - 1ull);
  const uint64_t tag = static_cast<uint64_t>(a.seq) << 32;
  if (t == 0) s_chunk = static_cast<uint32_t>(__hip_atomic_fetch_add(&a.ws[0], 1ull, __ATOMIC_RELAXED,
                                                                    __HIP_MEMORY_SCOPE_AGENT));
  if (t < a.nbounds) s_bounds[t] = a.bounds[t];
  if (t < NA) s_base[t] = 0;
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
    load_row(r, mk);
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
    __hip_atomic_store(&a.ws[1 + static_cast<uint64_t>(c) * NA + t], tag | sum, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  for (uint32_t j = t; j < c * NA; j += kPlanThreads) {
    const uint32_t i = j / NA, k = j - i * NA;
    uint64_t v;
    while (((v = __hip_atomic_load(&a.ws[1 + static_cast<uint64_t>(i) * NA + k], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT)) >> 32) != a.seq)
      __builtin_amdgcn_s_sleep(1);
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
  // the round check's verdict (the last chunk: it holds every worker's mask total), from the check workgroup's findings
  if (c + 1 == a.nchunks && a.chk_status != nullptr) {
    __shared__ uint32_t s_bad, s_stale;
    if (t == 0) s_bad = OMR_MAX_WORKERS;
    __syncthreads();
    if (t == 0) s_stale = OMR_MAX_WORKERS;
    __syncthreads();
    if (t < cnt) {  // worker t's check word: its slots' sum, or the top bit for a slot of another round
      uint64_t v;
      while (((v = __hip_atomic_load(&a.ws[kPlanCheckWords + t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 32) !=
             a.seq)
        __builtin_amdgcn_s_sleep(2);
      uint32_t total = 0;
#pragma unroll
      for (uint32_t k = 0; k < static_cast<uint32_t>(W); ++k) total = k == t ? carry[k] : total;
      if (static_cast<uint32_t>(v) & 0x80000000u) (void)atomicMin(&s_stale, t);
      else if (static_cast<uint32_t>(v) != total) (void)atomicMin(&s_bad, t);
    }
    __syncthreads();
    if (t == 0) {
      const uint32_t code = s_stale < OMR_MAX_WORKERS ? (kCheckStale | s_stale)
                                                      : (s_bad < OMR_MAX_WORKERS ? (kCheckCount | s_bad) : 0u);
      __hip_atomic_store(a.chk_status, tag | code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// The round check (round 6): is every worker's all-gathered mask array the one its scan of THIS round
// wrote?  Each of the worker's scan workgroups left a slot (seq << 32) | its non-zero blocks in the array.  One more
// workgroup per worker in the plan launch (plan_check) reads that worker's slots and publishes, tagged with seq, their
// sum, or a flag when one carries another round's number; the last chunk, which holds every worker's mask popcount
// total, compares them (plan_chunk's end) and stores the status beside the counts: (seq << 32) | 0, | 0x100 + worker for a stale slot
// (the copy read the worker's buffer before its scan wrote the slot, or another buffer), | 0x200 + worker when the slot
// sum differs from the masks' popcount (a copy that overtook its producer: a mask array only gains bits between the plan
// that zeroes it and the scan that refills it, so it reads too few).  The round's host fails the round on it, by name,
// instead of relying on the exchange's size check.  (The first form had one check workgroup wait for the chunks' totals
// and add the slots with a shared-memory atomic each: 6 us more than the plan; one workgroup reading every worker's
// slots, 3 us more; profiles/r06/INDEX.md.)
template <int W>
__device__ __forceinline__ void plan_check(const PlanArgs& a, uint32_t c) {
  // worker c's slots, a few per thread, all in flight at once (512 at config 4: two per thread); a slot of another
  // round sets the published word's top bit, else it carries the slots' sum (< 2^28 blocks)
  __shared__ uint32_t s_sum[kPlanWaves], s_stale;
  const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
  if (t == 0) s_stale = 0;
  const uint32_t ns = a.chk_slots;
  const uint64_t* const slots = a.masks + static_cast<uint64_t>(c) * a.mstride + a.chk_off;
  constexpr uint32_t U = 8;  // loads in flight per thread
  uint32_t sum = 0, stale = 0;
  for (uint32_t base = 0; base < ns; base += kPlanThreads * U) {
    uint64_t v[U];
#pragma unroll
    for (uint32_t i = 0; i < U; ++i) {  // (unconditional loads from clamped indices)
      const uint32_t idx = base + i * kPlanThreads + t;
      v[i] = slots[idx < ns ? idx : 0u];
    }
#pragma unroll
    for (uint32_t i = 0; i < U; ++i) {
      if (base + i * kPlanThreads + t >= ns) continue;
      stale |= static_cast<uint32_t>(v[i] >> 32) != a.seq ? 1u : 0u;
      sum += static_cast<uint32_t>(v[i]);
    }
  }
  const uint32_t inc = wave_incl_scan(sum);
  if (lane == 63) s_sum[wave] = inc;
  __syncthreads();  // (s_stale initialised, s_sum filled)
  if (stale) s_stale = 1;
  __syncthreads();
  if (t == 0) {
    uint32_t total = 0;
#pragma unroll
    for (uint32_t w = 0; w < kPlanWaves; ++w) total += s_sum[w];
    const uint64_t word = (static_cast<uint64_t>(a.seq) << 32) | (s_stale ? 0x80000000u : (total & 0x7FFFFFFFu));
    __hip_atomic_store(&a.ws[kPlanCheckWords + c], word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// One launch: the chunks (plan_chunk), then the aggregator chain (server.cc:86-96 min_next over the union, one k_next
// segment each), then the shard sum's pair list (one unit per wave), then the round check (one workgroup, if asked).
// W >= count (2, 4, 8, 16).
template <int W>
__global__ __launch_bounds__(kPlanThreads) void k_round_plan(PlanArgs a) {
  if (blockIdx.x < a.nchunks) {
    plan_chunk<W>(a);
    return;
  }
  const uint32_t b = blockIdx.x - a.nchunks;
  if (a.chk_status != nullptr && b >= a.chain_wgs + a.list_wgs) {  // the round check, one workgroup per worker
    plan_check<W>(a, b - a.chain_wgs - a.list_wgs);
    return;
  }
  if (b >= a.chain_wgs) {  // the shard sum's pair list, one unit per wave
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t li = xcd_spread(b - a.chain_wgs, a.nchunks + a.chain_wgs, a.list_wgs);
    build_sum_list<W>(a.list, static_cast<uint64_t>(li) * kPlanWaves + w, static_cast<uint64_t>(a.list_wgs) * kPlanWaves);
    return;
  }
  const uint64_t* m = a.masks;  // the aggregator chain over the union, one segment each
  const uint32_t cnt = a.count;
  const uint64_t ms = a.mstride;
  next_segment<kPlanWaves>(a.chain, b, [&](uint64_t r) {
    uint64_t u = 0;
    for (uint32_t c = 0; c < cnt; ++c) u |= m[static_cast<uint64_t>(c) * ms + r];
    return u;
  }, a.chain.next);
}

// Dense <-> packed block movement over the set bits of one mask array (dir 0: pack, the worker's gather of
// common.cc:405-407; dir 1: unpack, the worker's in-place result copy of client.cc:89).  Rows [skip_b, skip_e)
// are skipped and do not occupy the packed stream.
struct MoveArgs {
  const float* src;
  float* dst;
  const uint64_t* masks;
  const uint32_t* prefix;  // exclusive popcount prefix of `masks`, rows + 1 entries
  uint64_t rows, skip_b, skip_e;
  uint32_t lanes, block, dir, lg;
};

template <int VEC>
__global__ __launch_bounds__(kWGThreads) void k_move(MoveArgs a) {
  constexpr int SL = move_slots<VEC>();
  const int lane = threadIdx.x & 63;
  const uint32_t groups = a.lanes / a.lg;
  const uint32_t bbytes = a.block * 4;
  const uint64_t units = a.rows * groups;
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * kWavesPerWG;
  const uint32_t skip_cnt = a.prefix[a.skip_e] - a.prefix[a.skip_b];
  for (uint64_t u = static_cast<uint64_t>(blockIdx.x) * kWavesPerWG + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
       u < units; u += nw) {
    const uint64_t r = u / groups;
    const uint32_t g0 = static_cast<uint32_t>(u % groups) * a.lg;
    if (r >= a.skip_b && r < a.skip_e) continue;
    const uint64_t m = a.masks[r];
    const uint32_t pr = a.prefix[r];  // issued with the mask load: one round trip before the data
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
                                                 (off + (q * 64 + lane) * 16) | drop, 0, kStoreAux);
      }
      k += nv;
    }
  }
}

// Aggregator shard sum over rows [r0, r1) of the write set (server.cc:83-99 with the RDMA hop replaced by the
// transport): for every write-set block, ((0.0f + x_a0) + x_a1) + ... over the workers whose mask has it, in rank
// order (a write-set block no worker has, a lane head: +0.0f).  Worker `me`'s contribution is read in place from its
// dense tensor `own`; worker a's from its received stream at recv + recv_off[a] blocks, which is either
//   row-ordered (pos_off == kRowStreams): its blocks of these rows in block order, position from the prefix arrays; or
//   column-ordered (k_scan1f's fused pack): segment by segment, position from its position table.
// Output dense (block position, in place) or packed (write-set order of the shard, for the sums' return trip).
//
// Work unit = UR rows x one lane column (column streams: a part of a segment's 64-row group).  Lane i holds row i
// of the rows it loads: ONE round trip fetches the unit's index data (write-set row, every worker's mask row and
// stream prefix or position).  Ballots over the lanes give each worker's column bits, so every (block, contributor)
// pair's stream position is computed in registers; a wave-wide exclusive scan lays the pairs out in LDS in
// (block, rank) order.  The pairs are then streamed P at a time: all P loads in flight (P * VEC dwordx4 per lane),
// then the segmented sum in rank order, then the stores of the blocks the window completed (a block's last pair).  So
// a unit costs one index round trip plus one per P pairs, whatever the number of contributors (the round-2 kernel
// paid a round trip per contributor per batch of blocks behind a prefix round trip: 2.9 TB/s at an 8-worker shard).
struct SumArgs {
  const float* own;
  const float* recv;
  uint64_t recv_off[OMR_MAX_WORKERS];
  const uint64_t* masks;   // worker c's row masks at masks + c * mstride
  uint64_t mstride;
  const uint32_t* prefix;  // [count + 1][rows + 1]: the workers' row-stream prefixes, then the write set's
  const uint64_t* write_set;
  float* out;
  uint64_t rows, r0, r1;
  uint32_t count, me, lanes, block, packed_out;
  uint32_t units, lane_shift;  // set by the launch (a unit's coordinates are 32-bit shifts)
};


// W >= count: the contributor loops are unrolled W times (the launch picks 2, 4, 8 or 16), so an 8-worker shard does
// half the per-row work of a 16-way unroll.  UR: rows per unit.
template <int VEC, int W, uint32_t UR = kShardUnitRows>
__global__ __launch_bounds__(kWGThreads) void k_shard_sum(SumArgs a) {
  constexpr int P = 32 / VEC;  // pair slots per window
  constexpr int kSlotGroup = P < 8 ? P : 8;
  constexpr uint32_t kRecCap = UR * W;
  __shared__ uint64_t s_rec[kWavesPerWG][kRecCap];
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nw = gridDim.x * kWavesPerWG;
  const uint32_t* const pws = a.prefix + static_cast<uint64_t>(a.count) * (a.rows + 1);
  const uint32_t wpre0 = a.packed_out ? pws[a.r0] : 0u;
  const uint32_t bbytes = a.block * 4;
  for (uint32_t u = blockIdx.x * kWavesPerWG + wave; u < a.units; u += nw) {
    const uint32_t l = u & (a.lanes - 1);
    // the unit: rows [g0, g0 + nload) of lane l (lane i of the wave: row g0 + i)
    const uint64_t g0 = a.r0 + static_cast<uint64_t>(u >> a.lane_shift) * UR;
    const uint32_t nload = a.r1 - g0 < UR ? static_cast<uint32_t>(a.r1 - g0) : UR;
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
      pre[c] = (c < a.count && rl) ? a.prefix[c * (a.rows + 1) + r] : 0u;
    }
    // lane c < count: worker c's stream prefix at r0 (its stream of this shard starts there)
    const uint32_t base_c =
        static_cast<uint32_t>(lane) < a.count ? a.prefix[static_cast<uint64_t>(lane) * (a.rows + 1) + a.r0] : 0u;
    // ---- (block, contributor) pairs of the unit's write-set blocks, rank order within a block
    const bool wb = rl && ((w >> l) & 1ull);
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
            const uint64_t pos = static_cast<uint64_t>(pre[c] - bc) +
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

// The shard sum over a pair list (build_sum_list): per unit, ONE coalesced load of its count and first 64 records,
// then the records' blocks streamed P at a time (every load of a window in flight) into the segmented rank-order sum
// of k_shard_sum.  Packed output: a record's dense block index becomes its write-set position (the write set's row
// prefix and row, loaded beside the window's blocks).
struct ListSumArgs {
  const float* own;
  const float* recv;
  const uint64_t* records;
  const uint32_t* counts;
  const uint64_t* write_set;  // packed output: the write set's rows and row prefix (omr_round_plan's prefix[count])
  const uint32_t* wprefix;
  float* out;
  uint32_t units;
  uint64_t r0;
  uint32_t cap, lanes, block, packed_out;
};

template <int VEC>
__global__ __launch_bounds__(kWGThreads) void k_shard_sum_list(ListSumArgs a) {
  // pair slots per window: 32 at B = 256, so a unit at config 4's density (13 pairs on average, 16 rows x 8 workers at
  // most 128) nearly always fits one window; each window is loads, then every add, then the stores (as k_shard_sum)
  constexpr int P = 2 * kSumUnitRows / VEC;
  static_assert(64 % P == 0, "a window lies inside one 64-record chunk");
  constexpr int kSlotGroup = 8;
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nw = gridDim.x * kWavesPerWG;
  const uint32_t bbytes = a.block * 4;
  const uint32_t wpre0 = a.packed_out ? a.wprefix[a.r0] : 0u;
  for (uint32_t u = blockIdx.x * kWavesPerWG + wave; u < a.units; u += nw) {
    // ONE load: the unit's first 32 words (2 of the 4 lines of a 64-word chunk: a 16-row unit nearly always has fewer
    // records); its length is the first terminator's lane.  Past 31 records the whole first 64 are loaded, past 63
    // the next chunks (lanes >= 32 of the first load hold terminators, so the ballot's low half decides)
    const uint64_t* const rec = a.records + static_cast<uint64_t>(u) * a.cap;
    uint64_t chunk = static_cast<uint32_t>(lane) < (a.cap < 32u ? a.cap : 32u) ? rec[lane] : kRecEnd;
    uint64_t e0 = __ballot(chunk == kRecEnd);
    if ((e0 & 0xFFFFFFFFull) == 0) {
      chunk = static_cast<uint32_t>(lane) < a.cap ? rec[lane] : kRecEnd;
      e0 = __ballot(chunk == kRecEnd);
    }
    uint32_t total = 0;
    for (uint64_t e = e0;; ) {
      if (e != 0) {
        total += static_cast<uint32_t>(__builtin_ctzll(e));
        break;
      }
      total += 64;
      const uint64_t nx = total + lane < a.cap ? rec[total + lane] : kRecEnd;
      e = __ballot(nx == kRecEnd);
    }
    if (total == 0) continue;
    uint64_t pdst = 0;  // packed output: chunk record `lane`'s write-set position
    v4f acc[VEC];
#pragma unroll
    for (int q = 0; q < VEC; ++q) acc[q] = v4f{0.f, 0.f, 0.f, 0.f};
    for (uint32_t wbase = 0; wbase < total; wbase += P) {
      const uint32_t cb = wbase & 63u;  // the window's first record in the chunk (P divides 64)
      if (cb == 0) {
        if (wbase != 0) chunk = wbase + lane < a.cap ? rec[wbase + lane] : 0ull;
        if (a.packed_out && wbase + lane < total) {
          const uint64_t d = (chunk >> 32) & 0x0FFFFFFFull;
          const uint64_t r = d / a.lanes;
          const uint32_t l = static_cast<uint32_t>(d - r * a.lanes);
          pdst = static_cast<uint64_t>(a.wprefix[r] - wpre0) +
                 static_cast<uint64_t>(__builtin_popcountll(a.write_set[r] & below(l)));
        }
      }
      const uint32_t nv = total - wbase < static_cast<uint32_t>(P) ? total - wbase : static_cast<uint32_t>(P);
      v4f v[P][VEC];
#pragma unroll
      for (int g = 0; g < P; g += kSlotGroup) {
        if (static_cast<uint32_t>(g) < nv) {  // (wave-uniform: a sparse unit issues only what it needs)
#pragma unroll
          for (int j = g; j < g + kSlotGroup; ++j) {
            const uint64_t rc = readlane64(chunk, cb + j);
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
      // the segmented rank-order sums (a block's first pair restarts from +0.0f), every slot's running sum kept in
      // its registers; slots past the window's last pair are consumed and discarded, so no slot's load can still be
      // pending at the stores below (the compiler would wait for it there, and so for the stores before it)
#pragma unroll
      for (int j = 0; j < P; ++j) {
        const uint64_t rc = readlane64(chunk, cb + j);
        const bool use = static_cast<uint32_t>(j) < nv;
#pragma unroll
        for (int q = 0; q < VEC; ++q) {
          const v4f sum = add4((rc & kRecFirst) ? v4f{0.f, 0.f, 0.f, 0.f} : acc[q], v[j][q]);
          acc[q] = use ? sum : acc[q];
          v[j][q] = acc[q];
        }
      }
#pragma unroll
      for (int j = 0; j < P; ++j)
#pragma unroll
        for (int q = 0; q < VEC; ++q) asm volatile("" : "+v"(v[j][q]));  // (every add above every store)
#pragma unroll
      for (int j = 0; j < P; ++j) {
        if (static_cast<uint32_t>(j) < nv) {
          const uint64_t rc = readlane64(chunk, cb + j);
          if (rc & kRecLast) {
            const uint64_t dst = a.packed_out ? readlane64(pdst, cb + j) : ((rc >> 32) & 0x0FFFFFFFull);
            store_block_wt<VEC>(a.out + dst * a.block, v[j], lane);
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------- synthetic fill (client.cc:401-419)

__device__ __forceinline__ float hash_uniform(uint64_t idx, uint32_t seed) {
  uint64_t z = idx + 0x9E3779B97F4A7C15ull * (static_cast<uint64_t>(seed) + 1ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  const int32_t u = static_cast<int32_t>(z >> 40) - (1 << 23);  // [-2^23, 2^23)
  return static_cast<float>(u) * (1.0f / 8388608.0f);           // exact, [-1, 1)
}

__global__ __launch_bounds__(kWGThreads) void k_fill(const int32_t* bitmap, uint64_t n4, uint32_t block4,
                                                     int mode, uint32_t seed, float* buf) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kWGThreads;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * kWGThreads + threadIdx.x; i < n4; i += stride) {
    const bool on = bitmap[i / block4] == 1;
    v4f v = v4f{0.f, 0.f, 0.f, 0.f};
    if (on) {
      if (mode == 0) {
        v = v4f{0.01f, 0.01f, 0.01f, 0.01f};
      } else {
        v.x = hash_uniform(i * 4 + 0, seed);
        v.y = hash_uniform(i * 4 + 1, seed);
        v.z = hash_uniform(i * 4 + 2, seed);
        v.w = hash_uniform(i * 4 + 3, seed);
      }
    }
    reinterpret_cast<v4f*>(buf)[i] = v;
  }
}

// ---------------------------------------------------------------- host-side validation

struct Layout {
  uint64_t n, nb, rows;
  uint32_t block, lanes, parts, rows_per_part, vec;
};

int make_layout(uint64_t n, uint32_t block, uint32_t lanes, uint32_t parts, Layout* L) {
  if (block != 256 && block != 512 && block != 1024)
    return fail("block_size %u unsupported (256, 512, 1024)", block);
  if (lanes < 8 || lanes > 64 || (lanes & (lanes - 1)) != 0)
    return fail("num_lanes %u unsupported (a power of two in 8..64)", lanes);
  if (lanes % (block == 256 ? 16u : 8u) != 0) return fail("num_lanes %u too small for block_size %u", lanes, block);
  if (parts == 0) return fail("num_parts must be >= 1");
  const uint64_t row_floats = static_cast<uint64_t>(lanes) * block;
  if (n == 0 || n % (row_floats * parts) != 0)
    return fail("n=%llu is not a multiple of num_parts*num_lanes*block_size=%llu",
                static_cast<unsigned long long>(n), static_cast<unsigned long long>(row_floats * parts));
  if (n > omr_sentinel(block, lanes))
    return fail("n=%llu exceeds the uint32 offset space (sentinel %u, client.cc:24)",
                static_cast<unsigned long long>(n), omr_sentinel(block, lanes));
  L->n = n;
  L->block = block;
  L->lanes = lanes;
  L->parts = parts;
  L->nb = n / block;
  L->rows = L->nb / lanes;
  L->rows_per_part = static_cast<uint32_t>(L->rows / parts);
  L->vec = block / 256;
  return 0;
}

hipStream_t S(omr_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

unsigned grid_for(uint64_t work_items_per_wave_units) {
  uint64_t g = (work_items_per_wave_units + kWavesPerWG - 1) / kWavesPerWG;
  if (g > kMaxGrid) g = kMaxGrid;
  if (g == 0) g = 1;
  return static_cast<unsigned>(g);
}

// Lanes per work unit of the mask-addressed movers: whole rows when there are enough of them, otherwise rows split
// into groups (>= 4 lanes), for at least `min_units` units.  tools/tune_round_r02.py
// (profiles/r02/round/tune_round_r02*.log): 4096 units pack an 8-worker round's blocks 20 % faster than 8192 (whole
// rows: 10.8 vs 13.5 us) and sum an 8-worker shard 20 % faster (8-lane units: 16.9 vs 21.1 us); a one-contributor
// sum (world 1) is a plain move of few blocks per lane group and keeps 8192 (16.9 vs 18.9 us).
uint32_t unit_lanes(uint64_t rows, uint32_t lanes, uint64_t min_units = 4096) {
  uint32_t lg = lanes;
  while (lg > 4 && rows * (lanes / lg) < min_units) lg /= 2;
  return lg;
}

int launch_next(const Layout& L, const uint64_t* masks, uint32_t count, uint32_t* next, hipStream_t st) {
  NextArgs na;
  na.masks = masks;
  na.next = next;
  na.rows = L.rows;
  na.nb = L.nb;
  na.rows_per_part = L.rows_per_part;
  na.segs_per_part = (L.rows_per_part + 63) / 64;
  na.lanes = L.lanes;
  na.block = L.block;
  na.sentinel = omr_sentinel(L.block, L.lanes);
  dim3 grid(L.parts * na.segs_per_part, count);
  k_next<<<grid, kWGThreads, 0, st>>>(na);
  return launch_status("k_next");
}

// Column split of the single-pass kernel: K segments per (partition, lane) column, at least one 16-wave
// workgroup per CU (>= 256: tools/tune_fused.py measured K = 1 at 512 columns (B=256) and K = 2 at 128 columns
// (B=1024) best, profiles/r01/tune_fused_*.log), segments of at least 64 rows, K <= 64 (the fix-up's LDS).
constexpr int kFusedWaves = 16;
constexpr int kFusedLoads = 16;
struct FusedShape {
  uint32_t K = 0, S = 0;
};

FusedShape fused_shape(const Layout& L) {
  FusedShape f;
  const uint64_t cols = static_cast<uint64_t>(L.parts) * L.lanes;
  uint32_t K = 1;
  while (cols * K < 256 && L.rows_per_part % (2 * K) == 0 && L.rows_per_part / (2 * K) >= 64 && 2 * K <= 64) K *= 2;
  f.K = K;
  f.S = L.rows_per_part / K;
  return f;
}

size_t fused_workspace_bytes(const Layout& L, const FusedShape& f) {
  if (f.K <= 1) return 0;
  const uint64_t cols = static_cast<uint64_t>(L.parts) * L.lanes;
  return cols * sizeof(uint32_t) + cols * f.K * sizeof(uint64_t) + 16;
}

// The fused pack of the multi-rank worker scan (k_scan1f<..., PACK>): where the other shards' blocks go.
struct PackSpec {
  float* send;
  uint32_t* shard_cnt;
  uint32_t* pos;
  const uint64_t* bounds;  // host, nshards + 1
  uint32_t nshards;
  int32_t own_shard;
};

uint32_t pack_groups(const FusedShape& f) { return (f.S + kPackGroupRows - 1) / kPackGroupRows; }

uint64_t pack_table_entries(const Layout& L, const FusedShape& f) {
  return static_cast<uint64_t>(L.parts) * f.K * pack_groups(f) * L.lanes;
}

// a fused pack needs every shard to be whole column segments (a segment's blocks go to one shard's stream)
int pack_check(const Layout& L, const FusedShape& f, const uint64_t* bounds, uint32_t nshards) {
  if (nshards == 0 || nshards > OMR_MAX_WORKERS) return fail("pack: %u shards (1..%d)", nshards, OMR_MAX_WORKERS);
  if (bounds == nullptr) return fail("pack: NULL shard bounds");
  if (bounds[0] != 0 || bounds[nshards] != L.rows) return fail("pack: shard bounds must cover rows [0, %llu)",
                                                                static_cast<unsigned long long>(L.rows));
  for (uint32_t s = 0; s < nshards; ++s) {
    if (bounds[s] > bounds[s + 1]) return fail("pack: shard bounds must not decrease");
    if (bounds[s] % f.S != 0)
      return fail("pack: shard bound %llu is not a multiple of the scan's %u-row column segments (a ragged shard: "
                  "pack with omr_move_blocks_f32 instead)", static_cast<unsigned long long>(bounds[s]), f.S);
  }
  return 0;
}

constexpr int kPackWaves = 8;  // the fused pack's workgroups (two per CU)

// First row of shard s's stream in the send buffer, and the buffer's rows (*total_rows): the streams in shard order,
// own_shard's left out (the pack never writes it, so a co-located rank's send buffer is (N - 1) / N of the tensor).
uint64_t pack_send_row(const uint64_t* bounds, uint32_t nshards, int32_t own_shard, uint32_t s, uint64_t* total_rows) {
  const uint64_t own_rows = (own_shard >= 0 && static_cast<uint32_t>(own_shard) < nshards)
                                ? bounds[own_shard + 1] - bounds[own_shard] : 0;
  if (total_rows) *total_rows = bounds[nshards] - own_rows;
  return bounds[s] - ((own_shard >= 0 && s > static_cast<uint32_t>(own_shard)) ? own_rows : 0);
}

template <int VEC, int SKIP, int WAVES = kPackWaves>
int launch_fused_pack(const FusedArgs& a, const Layout& L, const FusedShape& f, unsigned grid, hipStream_t st) {
  const uint32_t bits_words = ((f.S + 31) / 32 + 3) & ~3u;
  const size_t lds = bits_words * sizeof(uint32_t) + static_cast<size_t>(WAVES) * a.wcap * L.block * 4;
  auto* fn = &k_scan1f<VEC, WAVES, kFusedLoads, SKIP, true, false, true>;
  // dynamic LDS beyond 64 KiB is opted into per instantiation, raised when a layout needs more (S sizes the bits)
  static std::atomic<size_t> attr{0};
  if (lds > attr.load()) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    if (e != hipSuccess) {
      (void)hipGetLastError();
      return fail("k_scan1f pack: cannot reserve %zu bytes of LDS: %s", lds, hipGetErrorString(e));
    }
    size_t cur = attr.load();
    while (lds > cur && !attr.compare_exchange_weak(cur, lds)) {
    }
  }
  fn<<<grid, 64 * WAVES, lds, st>>>(a);
  return launch_status("k_scan1f (pack)");
}

// The one-rank round's tally (omr_worker_scan_tally_f32).
struct TallySpec {
  uint64_t* tally;
  const uint64_t* pub_src;  // or null: nothing to publish
  uint32_t* pub_dst;
  uint32_t pub_seq;
};

int launch_fused(const Layout& L, const FusedShape& f, const float* x, float* out, int32_t* flags, uint32_t* next,
                 void* ws, hipStream_t st, uint64_t* masks = nullptr, uint32_t part_begin = 0,
                 uint32_t part_count = 0, const PackSpec* pk = nullptr, const TallySpec* tl = nullptr,
                 uint64_t* chk = nullptr, uint32_t chk_seq = 0, uint32_t* done = nullptr) {
  if (part_count == 0) part_count = L.parts - part_begin;
  FusedArgs a{};
  a.chk = chk;
  a.chk_seq = chk_seq;
  a.done = done;
  a.part0 = part_begin;
  a.x = x;
  a.out = out;
  a.flags = flags;
  a.next = next;
  const uint64_t cols = static_cast<uint64_t>(L.parts) * L.lanes;
  a.cnt = static_cast<uint32_t*>(ws);
  a.summary = ws ? reinterpret_cast<uint64_t*>(static_cast<char*>(ws) + ((cols * sizeof(uint32_t) + 15) / 16) * 16)
                 : nullptr;
  a.lanes = L.lanes;
  a.rpp = L.rows_per_part;
  a.K = f.K;
  a.S = f.S;
  a.block = L.block;
  a.sentinel = omr_sentinel(L.block, L.lanes);
  a.masks = masks;
  const unsigned grid = static_cast<unsigned>(static_cast<uint64_t>(part_count) * L.lanes * f.K);
  constexpr int T = 64 * kFusedWaves;
  if (tl != nullptr) {
    // the one-rank round: the single-GPU step's shape (one 16-wave workgroup per column segment) with its tally
    a.tally = tl->tally;
    a.pub_src = tl->pub_src;
    a.pub_dst = tl->pub_dst;
    a.pub_seq = tl->pub_seq;
    a.pub_slots = grid;  // (the earlier launch had the same shape)
    const unsigned g = grid;
    switch (L.vec) {
      case 1: k_scan1f<1, kFusedWaves, kFusedLoads, 0, false, true><<<g, T, 0, st>>>(a); break;
      case 2: k_scan1f<2, kFusedWaves, kFusedLoads, 0, false, true><<<g, T, 0, st>>>(a); break;
      default: k_scan1f<4, kFusedWaves, kFusedLoads, 1, false, true><<<g, T, 0, st>>>(a); break;
    }
    return launch_status("k_scan1f (tally)");
  }
  if (pk != nullptr) {
    a.send = pk->send;
    a.shard_cnt = pk->shard_cnt;
    a.pos = pk->pos;
    for (uint32_t s = 0; s <= pk->nshards; ++s) a.bounds[s] = static_cast<uint32_t>(pk->bounds[s]);
    for (uint32_t s = 0; s < pk->nshards; ++s)
      a.send_row[s] = static_cast<uint32_t>(pack_send_row(pk->bounds, pk->nshards, pk->own_shard, s, nullptr));
    a.nshards = pk->nshards;
    a.own_shard = pk->own_shard;
    a.gps = pack_groups(f);
    // 8-wave workgroups with half the stash (64 KiB each), so two share a CU: one streams while the other takes its
    // stream place and writes its blocks out.  At config 4's shapes 50.3 us against 52.8 us for one 16-wave workgroup
    // per CU (tools/tune_round_r03.py, profiles/r03/round/tune_round_r03_list.log).
    a.wcap = (kPackLdsBytes / 2) / (kPackWaves * L.block * 4);
    switch (L.vec) {
      case 1: return launch_fused_pack<1, 0>(a, L, f, grid, st);
      case 2: return launch_fused_pack<2, 0>(a, L, f, grid, st);
      default: return launch_fused_pack<4, 1>(a, L, f, grid, st);
    }
  }
  // The multi-rank round's worker scan (it writes row masks) runs 8-wave workgroups, two per CU, as the fused pack's
  // does: beside the round's plan and copy kernels on the other streams a plan workgroup then displaces half a CU's
  // scan instead of all of it.  The world-1 round took 55.8-57.0 us so against 57.6-58.4 with one 16-wave workgroup
  // per CU (54.4-55.7 in a second set of runs), its scan 0.68-0.71 of spec against 0.66; the single-GPU step keeps 16
  // waves (47.8 against 49.6 us alone; profiles/r04/scan_waves/).
  if (masks != nullptr) {
    switch (L.vec) {
      case 1: k_scan1f<1, 8, kFusedLoads, 0, false, false, true><<<grid, 512, 0, st>>>(a); break;
      case 2: k_scan1f<2, 8, kFusedLoads, 0, false, false, true><<<grid, 512, 0, st>>>(a); break;
      default: k_scan1f<4, 8, kFusedLoads, 1, false, false, true><<<grid, 512, 0, st>>>(a); break;
    }
    return launch_status("k_scan1f (8 waves)");
  }
  // Short segments (small tensors: config 1's 4 MiB has 8 rows per partition): one wave holds a whole segment, and
  // 16-wave workgroups would leave 15 idle while taking a CU each (512 of them run in two turns on 256 CUs).
  // Workgroups of one wave per 16-row batch instead.
  const uint32_t rb = static_cast<uint32_t>(kFusedLoads) / L.vec;  // rows per batch
  if (f.S <= 4 * rb) {
    const int w = f.S <= rb ? 1 : (f.S <= 2 * rb ? 2 : 4);
    switch (L.vec * 8 + w) {
      case 9: k_scan1f<1, 1, kFusedLoads><<<grid, 64, 0, st>>>(a); break;
      case 10: k_scan1f<1, 2, kFusedLoads><<<grid, 128, 0, st>>>(a); break;
      case 12: k_scan1f<1, 4, kFusedLoads><<<grid, 256, 0, st>>>(a); break;
      case 17: k_scan1f<2, 1, kFusedLoads><<<grid, 64, 0, st>>>(a); break;
      case 18: k_scan1f<2, 2, kFusedLoads><<<grid, 128, 0, st>>>(a); break;
      case 20: k_scan1f<2, 4, kFusedLoads><<<grid, 256, 0, st>>>(a); break;
      case 33: k_scan1f<4, 1, kFusedLoads, 1><<<grid, 64, 0, st>>>(a); break;
      case 34: k_scan1f<4, 2, kFusedLoads, 1><<<grid, 128, 0, st>>>(a); break;
      default: k_scan1f<4, 4, kFusedLoads, 1><<<grid, 256, 0, st>>>(a); break;
    }
    return launch_status("k_scan1f (short segments)");
  }
  switch (L.vec) {
    case 1: k_scan1f<1, kFusedWaves, kFusedLoads><<<grid, T, 0, st>>>(a); break;
    case 2: k_scan1f<2, kFusedWaves, kFusedLoads><<<grid, T, 0, st>>>(a); break;
    // B = 1024 (1 % non-zero at config 3): a batch of 4 rows rarely has a block to write, and skipping its
    // dropped-store issue altogether measured 1-2 % faster (profiles/r02/fused/tune_c3_skip*.log); at B = 256 the
    // static schedule is faster (most 16-row batches write something)
    default: k_scan1f<4, kFusedWaves, kFusedLoads, 1><<<grid, T, 0, st>>>(a); break;
  }
  return launch_status("k_scan1f");
}

unsigned scan_grid(uint64_t chunks) {
  uint64_t g = (chunks + kScanWaves - 1) / kScanWaves;
  if (g > kMaxGrid) g = kMaxGrid;
  return static_cast<unsigned>(g ? g : 1);
}

int launch_scan(const Layout& L, const ScanArgs& a, hipStream_t st) {
  const unsigned g = grid_for(L.rows);
  if (a.m == 1) {
    constexpr int T = 64 * kScanWaves;
    const uint64_t nbr = static_cast<uint64_t>(a.row_end - a.row_begin) * L.lanes;  // blocks in the range
    switch (L.vec) {
      case 1: k_scan1<1><<<scan_grid(nbr / scan_chunk_blocks<1>()), T, 0, st>>>(a); break;
      case 2: k_scan1<2><<<scan_grid(nbr / scan_chunk_blocks<2>()), T, 0, st>>>(a); break;
      default: k_scan1<4><<<scan_grid(nbr / scan_chunk_blocks<4>()), T, 0, st>>>(a); break;
    }
    return launch_status("k_scan1");
  }
  // one unit per wave: rows x (lanes / G) units, kWavesPerWG per workgroup, no cap (the workgroups run one
  // after another at one wave per SIMD)
  const uint64_t gl = L.lanes < kScanmUnitLanes ? L.lanes : kScanmUnitLanes;
  const uint64_t units = L.rows * (L.lanes / gl);
  const unsigned gm = static_cast<unsigned>((units + kWavesPerWG - 1) / kWavesPerWG);
  (void)g;
  // a group of SUB blocks must lie inside one row: rows narrower than the default group (B=256 with 16 lanes, B=512
  // with 8) take the half-width group (make_layout admits them)
  const bool narrow = L.lanes < static_cast<uint32_t>(32 / L.vec);
  switch (L.vec) {
    case 1:
      if (narrow) k_scanm<1, 16, kScanmUnitLanes><<<gm, kWGThreads, 0, st>>>(a);
      else k_scanm<1, 32, kScanmUnitLanes><<<gm, kWGThreads, 0, st>>>(a);
      break;
    case 2:
      if (narrow) k_scanm<2, 8, kScanmUnitLanes><<<gm, kWGThreads, 0, st>>>(a);
      else k_scanm<2, 16, kScanmUnitLanes><<<gm, kWGThreads, 0, st>>>(a);
      break;
    default: k_scanm<4, 8, kScanmUnitLanes><<<gm, kWGThreads, 0, st>>>(a); break;
  }
  return launch_status("k_scanm");
}


// the pair list's arguments for the layout's column streams (shard rows [row_begin, row_end), whole segments)
int make_list_args(const Layout& L, const uint64_t* masks, uint32_t count, uint64_t mstride, const omr_sum_list* sl,
                   ListArgs* a) {
  const FusedShape f = fused_shape(L);
  if (sl == nullptr || sl->records == nullptr || sl->counts == nullptr || masks == nullptr)
    return fail("sum_list: NULL pointer");
  if (count == 0 || count > OMR_MAX_WORKERS) return fail("sum_list: count %u out of range", count);
  if (sl->me > count) return fail("sum_list: me %u > count %u", sl->me, count);
  if (sl->row_begin > sl->row_end || sl->row_end > L.rows || sl->row_begin % f.S != 0 || sl->row_end % f.S != 0)
    return fail("sum_list: rows [%llu, %llu) are not whole %u-row column segments",
                static_cast<unsigned long long>(sl->row_begin), static_cast<unsigned long long>(sl->row_end), f.S);
  if (mstride < L.rows || sl->pos_offset < L.rows * 2 || sl->pos_offset + pack_table_entries(L, f) > mstride * 2)
    return fail("sum_list: position table outside the mask arrays (stride %llu, offset %llu)",
                static_cast<unsigned long long>(mstride), static_cast<unsigned long long>(sl->pos_offset));
  if (L.nb > (1ull << 28)) return fail("sum_list: more than 2^28 blocks");
  ListArgs& g = *a;
  g = ListArgs{};
  g.masks = masks;
  g.mstride = mstride;
  g.pos_off = sl->pos_offset;
  for (uint32_t c = 0; c < OMR_MAX_WORKERS; ++c) {
    g.recv_off[c] = c < count ? sl->recv_offsets[c] : 0;
    if (c < count && c != sl->me && g.recv_off[c] > 0xFFFFFFFFull) return fail("sum_list: recv offset beyond 2^32");
  }
  g.rows = L.rows;
  g.r0 = sl->row_begin;
  g.r1 = sl->row_end;
  g.all_lanes = L.lanes >= 64 ? ~0ull : ((1ull << L.lanes) - 1ull);
  g.count = count;
  g.me = sl->me;
  g.lanes = L.lanes;
  g.rpp = L.rows_per_part;
  g.S = f.S;
  g.gps = pack_groups(f);
  g.cap = kSumUnitRows * count + 1;  // + the terminator
  g.records = sl->records;
  g.counts = sl->counts;
  return 0;
}

__global__ __launch_bounds__(64) void k_publish_tally(const uint64_t* tally, uint32_t slots, uint32_t* dst, uint32_t seq) {
  uint32_t nz = 0, heads = 0;
  tally_load(tally, slots, &nz, &heads);
  publish_tally(dst, seq, nz, heads);
}

uint64_t list_units_host(const ListArgs& a) { return ((a.r1 - a.r0) / a.S) * a.gps * kSumUnitsPerGroup * a.lanes; }

__global__ __launch_bounds__(kWGThreads) void k_sum_list(ListArgs a) {
  build_sum_list(a, static_cast<uint64_t>(xcd_spread(blockIdx.x, 0, gridDim.x)) * kWavesPerWG +
                        __builtin_amdgcn_readfirstlane(threadIdx.x >> 6),
                 static_cast<uint64_t>(gridDim.x) * kWavesPerWG);
}
}  // namespace

// internal, not in omr.h: the other translation units of libomr.so report through omr_last_error() with this
namespace omr_detail {
int set_error(int code, const char* msg) {
  snprintf(g_err, sizeof(g_err), "%s", msg);
  return code;
}
}  // namespace omr_detail

// ================================================================ C ABI
#ifndef OMR_NO_CAPI

extern "C" {

int omr_abi_version(void) { return OMR_ABI_VERSION; }

const char* omr_last_error(void) { return g_err; }

uint32_t omr_num_lanes(uint32_t block_size) {
  if (block_size == 0 || (OMR_NUM_SLOTS * OMR_MESSAGE_SIZE) % block_size != 0) return 0;
  return OMR_NUM_SLOTS * OMR_MESSAGE_SIZE / block_size;
}

uint32_t omr_sentinel(uint32_t block_size, uint32_t num_lanes) {
  if (block_size == 0 || num_lanes == 0) return 0;
  // (UINT32_MAX/BLOCK_SIZE/NUM_BLOCKS-1)*NUM_BLOCKS*BLOCK_SIZE, uint32 arithmetic (client.cc:24)
  return (UINT32_MAX / block_size / num_lanes - 1u) * num_lanes * block_size;
}

int omr_layout_check(uint64_t n, uint32_t block_size, uint32_t num_lanes, uint32_t num_parts) {
  Layout L;
  return make_layout(n, block_size, num_lanes, num_parts, &L);
}

int omr_gen_bitmap(uint32_t worker_id, double density_ratio, uint64_t num_blocks, int32_t* bitmap,
                   uint64_t* nonzero_count) {
  if (bitmap == nullptr && num_blocks != 0) return fail("bitmap is NULL");
  // glibc srandom_r/random_r TYPE_3 (x**31 + x**3 + 1): r[0] = seed, r[i] = 16807*r[i-1] mod (2^31-1)
  // for i < 31 (Schrage's method, as glibc), r[i] = r[i-31] for 31 <= i < 34, then r[i] = r[i-31] + r[i-3]
  // (mod 2^32); the k-th rand() is r[k+344] >> 1.
  uint32_t seed = worker_id + 1u;  // srand(res.myId+1), client.cc:396
  if (seed == 0) seed = 1;
  uint32_t r[34];
  r[0] = seed;
  for (int i = 1; i < 31; ++i) {
    const int32_t prev = static_cast<int32_t>(r[i - 1]);
    const int32_t hi = prev / 127773, lo = prev % 127773;
    int32_t word = 16807 * lo - 2836 * hi;
    if (word < 0) word += 2147483647;
    r[i] = static_cast<uint32_t>(word);
  }
  for (int i = 31; i < 34; ++i) r[i] = r[i - 31];
  // ring of the last 34 values; index k holds r[k mod 34]
  uint64_t idx = 34;
  auto step = [&]() -> uint32_t {
    const uint32_t v = r[(idx - 31) % 34] + r[(idx - 3) % 34];
    r[idx % 34] = v;
    ++idx;
    return v;
  };
  for (int i = 34; i < 344; ++i) step();
  uint64_t count = 0;
  for (uint64_t i = 0; i < num_blocks; ++i) {
    const int rv = static_cast<int>(step() >> 1);
    const double rnum = rv % 100 / static_cast<double>(101);  // client.cc:407
    const bool on = rnum < density_ratio;                      // client.cc:408 (myId != -1 always)
    bitmap[i] = on ? 1 : 0;
    count += on;
  }
  if (nonzero_count != nullptr) *nonzero_count = count;
  return 0;
}

int omr_fill_blocks_f32(const int32_t* bitmap, uint64_t num_blocks, uint32_t block_size, int mode,
                        uint32_t seed, float* buf, omr_stream_t stream) {
  if (block_size == 0 || block_size % 4 != 0) return fail("block_size %u must be a multiple of 4", block_size);
  if (mode != 0 && mode != 1) return fail("fill mode %d unknown", mode);
  if (num_blocks == 0) return 0;
  if (bitmap == nullptr || buf == nullptr) return fail("fill: NULL pointer");
  const uint64_t n4 = num_blocks * block_size / 4;
  uint64_t g = (n4 + kWGThreads - 1) / kWGThreads;
  if (g > 8192) g = 8192;
  k_fill<<<static_cast<unsigned>(g), kWGThreads, 0, S(stream)>>>(bitmap, n4, block_size / 4, mode, seed, buf);
  return launch_status("k_fill");
}

int omr_scan_sum_f32(const float* const* bufs, uint32_t m, uint64_t n, uint32_t block_size,
                     uint32_t num_lanes, uint32_t num_parts, int32_t* flags, uint64_t* row_masks,
                     uint32_t* next_offsets, float* out, omr_stream_t stream) {
  Layout L;
  if (int rc = make_layout(n, block_size, num_lanes, num_parts, &L)) return rc;
  if (m == 0 || m > OMR_MAX_WORKERS) return fail("m=%u out of range (1..%d)", m, OMR_MAX_WORKERS);
  if (bufs == nullptr) return fail("bufs is NULL");
  if (row_masks == nullptr) return fail("row_masks is NULL");
  ScanArgs a;
  memset(&a, 0, sizeof(a));
  for (uint32_t w = 0; w < m; ++w) {
    if (bufs[w] == nullptr) return fail("bufs[%u] is NULL", w);
    if (reinterpret_cast<uintptr_t>(bufs[w]) % 16 != 0) return fail("bufs[%u] not 16-byte aligned", w);
    a.x.p[w] = bufs[w];
  }
  if (out != nullptr && reinterpret_cast<uintptr_t>(out) % 16 != 0) return fail("out not 16-byte aligned");
  a.m = m;
  a.lanes = L.lanes;
  a.rows_per_part = L.rows_per_part;
  a.row_begin = 0;
  a.row_end = static_cast<uint32_t>(L.rows);
  a.rows = L.rows;
  a.nb = L.nb;
  a.flags = flags;
  a.masks = row_masks;
  a.out = out;
  hipStream_t st = S(stream);
  if (int rc = launch_scan(L, a, st)) return rc;
  if (next_offsets != nullptr) {
    const uint32_t count = (m == 1) ? 1u : m + 1u;
    if (int rc = launch_next(L, row_masks, count, next_offsets, st)) return rc;
  }
  return 0;
}

int omr_scan_sum_rows_f32(const float* buf, uint64_t n, uint32_t block_size, uint32_t num_lanes,
                          uint32_t num_parts, uint64_t row_begin, uint64_t row_end, int32_t* flags,
                          uint64_t* row_masks, float* out, omr_stream_t stream) {
  Layout L;
  if (int rc = make_layout(n, block_size, num_lanes, num_parts, &L)) return rc;
  if (buf == nullptr || row_masks == nullptr) return fail("scan_sum_rows: NULL pointer");
  if (row_begin > row_end || row_end > L.rows) return fail("scan_sum_rows: bad row range");
  if (row_begin == row_end) return 0;
  if (reinterpret_cast<uintptr_t>(buf) % 16 != 0 || reinterpret_cast<uintptr_t>(out) % 16 != 0)
    return fail("scan_sum_rows: buffers must be 16-byte aligned");
  ScanArgs a;
  memset(&a, 0, sizeof(a));
  a.x.p[0] = buf;
  a.m = 1;
  a.lanes = L.lanes;
  a.rows_per_part = L.rows_per_part;
  a.row_begin = static_cast<uint32_t>(row_begin);
  a.row_end = static_cast<uint32_t>(row_end);
  a.rows = L.rows;
  a.nb = L.nb;
  a.flags = flags;
  a.masks = row_masks;
  a.out = out;
  return launch_scan(L, a, S(stream));
}

size_t omr_scan_workspace_bytes(uint64_t n, uint32_t block_size, uint32_t num_lanes, uint32_t num_parts) {
  Layout L;
  if (make_layout(n, block_size, num_lanes, num_parts, &L)) return 0;
  return fused_workspace_bytes(L, fused_shape(L));
}

int omr_scan_sum_fused_f32(const float* buf, uint64_t n, uint32_t block_size, uint32_t num_lanes,
                           uint32_t num_parts, int32_t* flags, uint32_t* next_offsets, float* out, void* workspace,
                           size_t workspace_bytes, omr_stream_t stream) {
  Layout L;
  if (int rc = make_layout(n, block_size, num_lanes, num_parts, &L)) return rc;
  if (buf == nullptr || next_offsets == nullptr) return fail("scan_sum_fused: buf and next_offsets are required");
  if (reinterpret_cast<uintptr_t>(buf) % 16 != 0 || reinterpret_cast<uintptr_t>(out) % 16 != 0)
    return fail("scan_sum_fused: buffers must be 16-byte aligned");
  const FusedShape f = fused_shape(L);
  if (f.K == 0) return fail("scan_sum_fused: rows_per_part=%u has no supported column split", L.rows_per_part);
  const size_t need = fused_workspace_bytes(L, f);
  if (need > 0 && (workspace == nullptr || workspace_bytes < need))
    return fail("scan_sum_fused: needs a zero-initialised workspace of %zu bytes", need);
  return launch_fused(L, f, buf, out, flags, next_offsets, need ? workspace : nullptr, S(stream));
}

int omr_scan_partition_f32(const float* buf, uint64_t n, uint32_t block_size, uint32_t num_lanes, uint32_t num_parts,
                           uint32_t part, int32_t* flags, uint32_t* next_offsets, float* out, void* workspace,
                           size_t workspace_bytes, omr_stream_t stream) {
  Layout L;
  if (int rc = make_layout(n, block_size, num_lanes, num_parts, &L)) return rc;
  if (part >= L.parts) return fail("scan_partition: part %u out of range (num_parts %u)", part, L.parts);
  if (buf == nullptr || next_offsets == nullptr) return fail("scan_partition: buf and next_offsets are required");
  if (reinterpret_cast<uintptr_t>(buf) % 16 != 0 || reinterpret_cast<uintptr_t>(out) % 16 != 0)
    return fail("scan_partition: buffers must be 16-byte aligned");
  const FusedShape f = fused_shape(L);
  const size_t need = fused_workspace_bytes(L, f);
  if (need > 0 && (workspace == nullptr || workspace_bytes < need))
    return fail("scan_partition: needs a zero-initialised workspace of %zu bytes", need);
  return launch_fused(L, f, buf, out, flags, next_offsets, need ? workspace : nullptr, S(stream), nullptr, part, 1);
}

int omr_scan_f32(const float* buf, uint64_t n, uint32_t block_size, uint32_t num_lanes, uint32_t num_parts,
                 int32_t* flags, uint64_t* row_masks, uint32_t* next_offsets, omr_stream_t stream) {
  const float* bufs[1] = {buf};
  return omr_scan_sum_f32(bufs, 1, n, block_size, num_lanes, num_parts, flags, row_masks, next_offsets,
                          nullptr, stream);
}

int omr_next_offsets(const uint64_t* row_masks, uint32_t count, uint64_t n, uint32_t block_size,
                     uint32_t num_lanes, uint32_t num_parts, uint32_t* next_offsets, omr_stream_t stream) {
  Layout L;
  if (int rc = make_layout(n, block_size, num_lanes, num_parts, &L)) return rc;
  if (count == 0) return 0;
  if (row_masks == nullptr || next_offsets == nullptr) return fail("next_offsets: NULL pointer");
  return launch_next(L, row_masks, count, next_offsets, S(stream));
}

int omr_dense_sum_f32(const float* const* inputs, uint32_t m, uint64_t n, float* out, omr_stream_t stream) {
  if (m == 0 || m > OMR_MAX_WORKERS) return fail("dense_sum: m=%u out of range (1..%d)", m, OMR_MAX_WORKERS);
  if (n % 4 != 0) return fail("dense_sum: n=%llu is not a multiple of 4", static_cast<unsigned long long>(n));
  if (n == 0) return 0;
  if (inputs == nullptr || out == nullptr) return fail("dense_sum: NULL pointer");
  if (reinterpret_cast<uintptr_t>(out) % 16 != 0) return fail("dense_sum: out not 16-byte aligned");
  WorkerPtrs in;
  memset(&in, 0, sizeof(in));
  for (uint32_t w = 0; w < m; ++w) {
    if (inputs[w] == nullptr || reinterpret_cast<uintptr_t>(inputs[w]) % 16 != 0)
      return fail("dense_sum: inputs[%u] NULL or not 16-byte aligned", w);
    in.p[w] = inputs[w];
  }
  const uint64_t n4 = n / 4;
  uint64_t g = (n4 + kWGThreads * 4 - 1) / (kWGThreads * 4);
  if (g > kMaxGrid) g = kMaxGrid;
  k_dense_sum<<<static_cast<unsigned>(g), kWGThreads, 0, S(stream)>>>(in, m, n4, out);
  return launch_status("k_dense_sum");
}

int omr_block_sum_f32(const float* const* inputs, uint32_t m, const uint32_t* block_list, uint32_t num_list,
                      uint32_t block_size, float* out, omr_stream_t stream) {
  if (block_size != 256 && block_size != 512 && block_size != 1024)
    return fail("block_size %u unsupported (256, 512, 1024)", block_size);
  if (m == 0 || m > OMR_MAX_WORKERS) return fail("m=%u out of range (1..%d)", m, OMR_MAX_WORKERS);
  if (num_list == 0) return 0;
  if (inputs == nullptr || block_list == nullptr || out == nullptr) return fail("block_sum: NULL pointer");
  WorkerPtrs in;
  memset(&in, 0, sizeof(in));
  for (uint32_t w = 0; w < m; ++w) {
    if (inputs[w] == nullptr) return fail("inputs[%u] is NULL", w);
    in.p[w] = inputs[w];
  }
  const unsigned g = grid_for(num_list);
  hipStream_t st = S(stream);
  switch (block_size / 256) {
    case 1: k_list_sum<1><<<g, kWGThreads, 0, st>>>(in, m, block_list, num_list, out); break;
    case 2: k_list_sum<2><<<g, kWGThreads, 0, st>>>(in, m, block_list, num_list, out); break;
    default: k_list_sum<4><<<g, kWGThreads, 0, st>>>(in, m, block_list, num_list, out); break;
  }
  return launch_status("k_list_sum");
}

size_t omr_compact_workspace_bytes(uint64_t rows) {
  return static_cast<size_t>((rows + kCompactRows - 1) / kCompactRows + 1) * sizeof(uint32_t);
}

int omr_compact(const uint64_t* row_masks, uint64_t row_begin, uint64_t row_end, uint32_t num_lanes,
                uint32_t* block_list, uint32_t* count, void* workspace, size_t workspace_bytes,
                omr_stream_t stream) {
  if (row_end < row_begin) return fail("compact: row_end < row_begin");
  if (num_lanes == 0 || num_lanes > 64) return fail("num_lanes %u out of range", num_lanes);
  if (count == nullptr) return fail("compact: count is NULL");
  hipStream_t st = S(stream);
  const uint64_t rows = row_end - row_begin;
  if (rows == 0) {
    const hipError_t e = hipMemsetAsync(count, 0, sizeof(uint32_t), st);
    if (e != hipSuccess) {
      snprintf(g_err, sizeof(g_err), "compact memset: %s", hipGetErrorString(e));
      return static_cast<int>(e);
    }
    return 0;
  }
  if (row_masks == nullptr || block_list == nullptr || workspace == nullptr)
    return fail("compact: NULL pointer");
  if (workspace_bytes < omr_compact_workspace_bytes(rows)) return fail("compact: workspace too small");
  const uint64_t chunks = (rows + kCompactRows - 1) / kCompactRows;
  if (chunks > 0x7fffffffull) return fail("compact: too many rows");
  uint32_t* chunk_sum = static_cast<uint32_t*>(workspace);
  k_compact_count<<<static_cast<unsigned>(chunks), kWGThreads, 0, st>>>(row_masks, row_begin, row_end,
                                                                        chunk_sum);
  if (int rc = launch_status("k_compact_count")) return rc;
  k_compact_write<<<static_cast<unsigned>(chunks), kWGThreads, 0, st>>>(row_masks, row_begin, row_end,
                                                                        num_lanes, chunk_sum, block_list,
                                                                        count);
  return launch_status("k_compact_write");
}

size_t omr_prefix_workspace_bytes(uint64_t rows, uint32_t count) {
  return static_cast<size_t>((rows + kCompactRows - 1) / kCompactRows) * count * sizeof(uint32_t) + 16;
}

int omr_mask_union(const uint64_t* row_masks, uint32_t count, uint64_t rows, uint32_t rows_per_part,
                   uint32_t num_lanes, int heads, uint64_t* out, omr_stream_t stream) {
  if (rows == 0) return 0;
  if (row_masks == nullptr || out == nullptr) return fail("mask_union: NULL pointer");
  if (num_lanes == 0 || num_lanes > 64) return fail("num_lanes %u out of range", num_lanes);
  if (heads && rows_per_part == 0) return fail("mask_union: rows_per_part must be > 0 with heads");
  const uint64_t lane_bits = (num_lanes == 64) ? ~0ull : ((1ull << num_lanes) - 1);
  uint64_t g = (rows + kWGThreads - 1) / kWGThreads;
  if (g > 4096) g = 4096;
  k_mask_union<<<static_cast<unsigned>(g), kWGThreads, 0, S(stream)>>>(row_masks, count, rows, rows_per_part,
                                                                       lane_bits, heads, out);
  return launch_status("k_mask_union");
}

int omr_row_prefix(const uint64_t* row_masks, uint32_t count, uint64_t rows, uint32_t* prefix, void* workspace,
                   size_t workspace_bytes, omr_stream_t stream) {
  if (rows == 0 || count == 0) return 0;
  if (row_masks == nullptr || prefix == nullptr || workspace == nullptr) return fail("row_prefix: NULL pointer");
  if (workspace_bytes < omr_prefix_workspace_bytes(rows, count)) return fail("row_prefix: workspace too small");
  const uint64_t chunks = (rows + kCompactRows - 1) / kCompactRows;
  if (chunks > 65535u * 16u) return fail("row_prefix: too many rows");
  dim3 grid(static_cast<unsigned>(chunks), count);
  hipStream_t st = S(stream);
  uint32_t* cs = static_cast<uint32_t*>(workspace);
  k_prefix_chunks<<<grid, kWGThreads, 0, st>>>(row_masks, rows, cs);
  if (int rc = launch_status("k_prefix_chunks")) return rc;
  k_prefix_write<<<grid, kWGThreads, 0, st>>>(row_masks, rows, cs, prefix);
  return launch_status("k_prefix_write");
}

int omr_sparse_block_sum_f32(const float* recv, const uint64_t* recv_offsets, const uint64_t* row_masks,
                             uint32_t count, uint64_t rows, const uint32_t* prefix, uint64_t row_begin,
                             uint32_t num_lanes, const uint32_t* block_list, uint32_t num_list,
                             uint32_t block_size, float* out, omr_stream_t stream) {
  if (block_size != 256 && block_size != 512 && block_size != 1024)
    return fail("block_size %u unsupported (256, 512, 1024)", block_size);
  if (num_lanes < 1 || num_lanes > 64 || (num_lanes & (num_lanes - 1)) != 0)
    return fail("num_lanes %u must be a power of two <= 64", num_lanes);
  if (count == 0 || count > OMR_MAX_WORKERS) return fail("count=%u out of range", count);
  if (num_list == 0) return 0;
  if (recv_offsets == nullptr || row_masks == nullptr || prefix == nullptr || block_list == nullptr ||
      out == nullptr)
    return fail("sparse_block_sum: NULL pointer");
  const uint32_t lshift = static_cast<uint32_t>(__builtin_ctz(num_lanes));
  const unsigned g = grid_for(num_list);
  hipStream_t st = S(stream);
  switch (block_size / 256) {
    case 1: k_sparse_sum<1><<<g, kWGThreads, 0, st>>>(recv, recv_offsets, row_masks, count, rows, prefix, row_begin, lshift, block_list, num_list, out); break;
    case 2: k_sparse_sum<2><<<g, kWGThreads, 0, st>>>(recv, recv_offsets, row_masks, count, rows, prefix, row_begin, lshift, block_list, num_list, out); break;
    default: k_sparse_sum<4><<<g, kWGThreads, 0, st>>>(recv, recv_offsets, row_masks, count, rows, prefix, row_begin, lshift, block_list, num_list, out); break;
  }
  return launch_status("k_sparse_sum");
}

int omr_gather_blocks_f32(const float* src, const uint32_t* block_list, uint32_t num_list,
                          uint32_t block_size, float* packed, omr_stream_t stream) {
  if (block_size != 256 && block_size != 512 && block_size != 1024)
    return fail("block_size %u unsupported (256, 512, 1024)", block_size);
  if (num_list == 0) return 0;
  if (src == nullptr || block_list == nullptr || packed == nullptr) return fail("gather: NULL pointer");
  const unsigned g = grid_for(num_list);
  hipStream_t st = S(stream);
  switch (block_size / 256) {
    case 1: k_gather<1><<<g, kWGThreads, 0, st>>>(src, block_list, num_list, packed); break;
    case 2: k_gather<2><<<g, kWGThreads, 0, st>>>(src, block_list, num_list, packed); break;
    default: k_gather<4><<<g, kWGThreads, 0, st>>>(src, block_list, num_list, packed); break;
  }
  return launch_status("k_gather");
}

int omr_scatter_blocks_f32(const float* packed, const uint32_t* block_list, uint32_t num_list,
                           uint32_t block_size, float* dst, omr_stream_t stream) {
  if (block_size != 256 && block_size != 512 && block_size != 1024)
    return fail("block_size %u unsupported (256, 512, 1024)", block_size);
  if (num_list == 0) return 0;
  if (packed == nullptr || block_list == nullptr || dst == nullptr) return fail("scatter: NULL pointer");
  const unsigned g = grid_for(num_list);
  hipStream_t st = S(stream);
  switch (block_size / 256) {
    case 1: k_scatter<1><<<g, kWGThreads, 0, st>>>(packed, block_list, num_list, dst); break;
    case 2: k_scatter<2><<<g, kWGThreads, 0, st>>>(packed, block_list, num_list, dst); break;
    default: k_scatter<4><<<g, kWGThreads, 0, st>>>(packed, block_list, num_list, dst); break;
  }
  return launch_status("k_scatter");
}

// ---------------------------------------------------------------- multi-rank round (mask-addressed)

int omr_worker_scan_f32(const float* buf, uint64_t n, uint32_t block_size, uint32_t num_lanes, uint32_t num_parts,
                        int32_t* flags, uint32_t* next_offsets, uint64_t* row_masks, float* out, void* workspace,
                        size_t workspace_bytes, omr_stream_t stream) {
  return omr_worker_scan_check_f32(buf, n, block_size, num_lanes, num_parts, flags, next_offsets, row_masks, out,
                                   workspace, workspace_bytes, nullptr, 0, nullptr, stream);
}

uint32_t omr_round_check_slots(uint64_t n, uint32_t block_size, uint32_t num_lanes, uint32_t num_parts) {
  Layout L;
  if (make_layout(n, block_size, num_lanes, num_parts, &L)) return 0;
  return static_cast<uint32_t>(static_cast<uint64_t>(L.parts) * L.lanes * fused_shape(L).K);
}

int omr_worker_scan_check_f32(const float* buf, uint64_t n, uint32_t block_size, uint32_t num_lanes, uint32_t num_parts,
                              int32_t* flags, uint32_t* next_offsets, uint64_t* row_masks, float* out, void* workspace,
                              size_t workspace_bytes, uint64_t* check_slots, uint32_t check_seq, uint32_t* done,
                              omr_stream_t stream) {
  Layout L;
  if (int rc = make_layout(n, block_size, num_lanes, num_parts, &L)) return rc;
  if (buf == nullptr || next_offsets == nullptr || row_masks == nullptr)
    return fail("worker_scan: buf, next_offsets and row_masks are required");
  if (reinterpret_cast<uintptr_t>(buf) % 16 != 0 || reinterpret_cast<uintptr_t>(out) % 16 != 0)
    return fail("worker_scan: buffers must be 16-byte aligned");
  const FusedShape f = fused_shape(L);
  const size_t need = fused_workspace_bytes(L, f);
  if (need > 0 && (workspace == nullptr || workspace_bytes < need))
    return fail("worker_scan: needs a zero-initialised workspace of %zu bytes", need);
  if (done != nullptr && check_seq == 0) return fail("worker_scan: a completion word needs a nonzero seq");
  return launch_fused(L, f, buf, out, flags, next_offsets, need ? workspace : nullptr, S(stream), row_masks, 0, 0,
                      nullptr, nullptr, check_slots, check_seq, done);
}

int omr_worker_scan_pack_f32(const float* buf, uint64_t n, uint32_t block_size, uint32_t num_lanes, uint32_t num_parts,
                             int32_t* flags, uint32_t* next_offsets, uint64_t* row_masks, float* out,
                             const uint64_t* shard_bounds, uint32_t num_shards, int32_t own_shard, float* send,
                             uint32_t* shard_counters, uint32_t* pos_table, void* workspace, size_t workspace_bytes,
                             omr_stream_t stream) {
  return omr_worker_scan_pack_check_f32(buf, n, block_size, num_lanes, num_parts, flags, next_offsets, row_masks, out,
                                        shard_bounds, num_shards, own_shard, send, shard_counters, pos_table, workspace,
                                        workspace_bytes, nullptr, 0, nullptr, stream);
}

int omr_worker_scan_pack_check_f32(const float* buf, uint64_t n, uint32_t block_size, uint32_t num_lanes,
                                   uint32_t num_parts, int32_t* flags, uint32_t* next_offsets, uint64_t* row_masks,
                                   float* out, const uint64_t* shard_bounds, uint32_t num_shards, int32_t own_shard,
                                   float* send, uint32_t* shard_counters, uint32_t* pos_table, void* workspace,
                                   size_t workspace_bytes, uint64_t* check_slots, uint32_t check_seq,
                                   uint32_t* done, omr_stream_t stream) {
  Layout L;
  if (int rc = make_layout(n, block_size, num_lanes, num_parts, &L)) return rc;
  if (buf == nullptr || next_offsets == nullptr || row_masks == nullptr || send == nullptr ||
      shard_counters == nullptr || pos_table == nullptr)
    return fail("worker_scan_pack: buf, next_offsets, row_masks, send, shard_counters and pos_table are required");
  if (reinterpret_cast<uintptr_t>(buf) % 16 != 0 || reinterpret_cast<uintptr_t>(out) % 16 != 0 ||
      reinterpret_cast<uintptr_t>(send) % 16 != 0)
    return fail("worker_scan_pack: buffers must be 16-byte aligned");
  const FusedShape f = fused_shape(L);
  if (int rc = pack_check(L, f, shard_bounds, num_shards)) return rc;
  if (own_shard < -1 || own_shard >= static_cast<int32_t>(num_shards))
    return fail("worker_scan_pack: own_shard %d out of range", own_shard);
  const size_t need = fused_workspace_bytes(L, f);
  if (need > 0 && (workspace == nullptr || workspace_bytes < need))
    return fail("worker_scan_pack: needs a zero-initialised workspace of %zu bytes", need);
  const PackSpec pk{send, shard_counters, pos_table, shard_bounds, num_shards, own_shard};
  if (done != nullptr && check_seq == 0) return fail("worker_scan_pack: a completion word needs a nonzero seq");
  return launch_fused(L, f, buf, out, flags, next_offsets, need ? workspace : nullptr, S(stream), row_masks, 0, 0, &pk,
                      nullptr, check_slots, check_seq, done);
}

uint32_t omr_tally_slots(uint64_t n, uint32_t block_size, uint32_t num_lanes, uint32_t num_parts) {
  Layout L;
  if (make_layout(n, block_size, num_lanes, num_parts, &L)) return 0;
  return static_cast<uint32_t>(static_cast<uint64_t>(L.parts) * L.lanes * fused_shape(L).K);
}

int omr_worker_scan_tally_f32(const float* buf, uint64_t n, uint32_t block_size, uint32_t num_lanes, uint32_t num_parts,
                              int32_t* flags, uint32_t* next_offsets, float* out, uint64_t* tally,
                              const uint64_t* publish_src, uint32_t* publish_dst, uint32_t publish_seq, void* workspace,
                              size_t workspace_bytes, omr_stream_t stream) {
  Layout L;
  if (int rc = make_layout(n, block_size, num_lanes, num_parts, &L)) return rc;
  if (buf == nullptr || next_offsets == nullptr || tally == nullptr)
    return fail("worker_scan_tally: buf, next_offsets and tally are required");
  if ((publish_src == nullptr) != (publish_dst == nullptr)) return fail("worker_scan_tally: publish_src and _dst go together");
  if (reinterpret_cast<uintptr_t>(buf) % 16 != 0 || reinterpret_cast<uintptr_t>(out) % 16 != 0 ||
      reinterpret_cast<uintptr_t>(publish_dst) % 16 != 0)
    return fail("worker_scan_tally: buffers must be 16-byte aligned");
  const FusedShape f = fused_shape(L);
  const size_t need = fused_workspace_bytes(L, f);
  if (need > 0 && (workspace == nullptr || workspace_bytes < need))
    return fail("worker_scan_tally: needs a zero-initialised workspace of %zu bytes", need);
  const TallySpec tl{tally, publish_src, publish_dst, publish_seq};
  return launch_fused(L, f, buf, out, flags, next_offsets, need ? workspace : nullptr, S(stream), nullptr, 0, 0, nullptr,
                      &tl);
}

int omr_tally_publish(const uint64_t* tally, uint32_t slots, uint32_t* dst, uint32_t seq, omr_stream_t stream) {
  if (tally == nullptr || dst == nullptr || reinterpret_cast<uintptr_t>(dst) % 16 != 0)
    return fail("tally_publish: NULL or unaligned pointer");
  k_publish_tally<<<1, 64, 0, S(stream)>>>(tally, slots, dst, seq);
  return launch_status("k_publish_tally");
}

int omr_pack_geometry(uint64_t n, uint32_t block_size, uint32_t num_lanes, uint32_t num_parts, uint32_t* seg_rows,
                      uint32_t* groups_per_seg, uint64_t* table_entries) {
  Layout L;
  if (int rc = make_layout(n, block_size, num_lanes, num_parts, &L)) return rc;
  const FusedShape f = fused_shape(L);
  if (seg_rows) *seg_rows = f.S;
  if (groups_per_seg) *groups_per_seg = pack_groups(f);
  if (table_entries) *table_entries = pack_table_entries(L, f);
  return 0;
}

int omr_pack_supported(uint64_t n, uint32_t block_size, uint32_t num_lanes, uint32_t num_parts,
                       const uint64_t* shard_bounds, uint32_t num_shards) {
  Layout L;
  if (int rc = make_layout(n, block_size, num_lanes, num_parts, &L)) return rc;
  return pack_check(L, fused_shape(L), shard_bounds, num_shards);
}

uint64_t omr_pack_send_offset(const uint64_t* shard_bounds, uint32_t num_shards, int32_t own_shard, uint32_t s,
                              uint32_t num_lanes, uint32_t block_size, uint64_t* total) {
  uint64_t rows = 0;
  const uint64_t r = pack_send_row(shard_bounds, num_shards, own_shard, s, &rows);
  const uint64_t row_floats = static_cast<uint64_t>(num_lanes) * block_size;
  if (total) *total = rows * row_floats;
  return r * row_floats;
}

uint64_t omr_round_plan_workspace_words(void) { return kPlanWorkspaceWords; }

int omr_round_plan_check(const uint64_t* row_masks, uint32_t count, uint64_t mask_stride, uint64_t rows,
                         uint32_t rows_per_part, uint32_t num_lanes, const uint64_t* bounds, uint32_t num_bounds,
                         uint64_t* write_set, uint64_t* union_masks, uint32_t* prefix, uint64_t* counts,
                         uint64_t* zero_masks, uint32_t* zero_counters, uint32_t num_zero_counters,
                         uint64_t* workspace, uint32_t seq, uint32_t* union_next, uint32_t block_size,
                         const omr_sum_list* list, uint64_t check_offset, uint32_t check_slots,
                         uint64_t* check_status, omr_stream_t stream) {
  if (mask_stride < rows) return fail("round_plan: mask_stride %llu < rows", static_cast<unsigned long long>(mask_stride));
  if (check_status != nullptr && (check_slots == 0 || check_offset < rows || check_offset + check_slots > mask_stride))
    return fail("round_plan: check slots [%llu, +%u) outside the mask arrays (rows %llu, stride %llu)",
                static_cast<unsigned long long>(check_offset), check_slots, static_cast<unsigned long long>(rows),
                static_cast<unsigned long long>(mask_stride));
  if (num_zero_counters > kPlanThreads || (num_zero_counters > 0 && zero_counters == nullptr))
    return fail("round_plan: zero_counters");
  if (count == 0 || count > OMR_MAX_WORKERS) return fail("round_plan: count %u out of range", count);
  if (rows == 0 || rows_per_part == 0 || rows % rows_per_part != 0) return fail("round_plan: bad rows");
  if (num_lanes == 0 || num_lanes > 64) return fail("round_plan: num_lanes %u out of range", num_lanes);
  if (row_masks == nullptr || write_set == nullptr || prefix == nullptr || workspace == nullptr ||
      (num_bounds > 0 && (bounds == nullptr || counts == nullptr)))
    return fail("round_plan: NULL pointer");
  if (seq == 0) return fail("round_plan: seq 0 (a zero-filled workspace or counts word carries it)");
  if (rows > 0xFFFFFFFFull / 64) return fail("round_plan: too many rows");
  if (num_bounds > OMR_MAX_WORKERS + 2) return fail("round_plan: %u bounds > %d", num_bounds, OMR_MAX_WORKERS + 2);
  PlanArgs a;
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
  // Chunks: about one 256-row tile per workgroup while that keeps them <= 64 (config 4: 1024 rows, 4 chunks).
  const uint64_t tiles_all = (rows + kPlanThreads - 1) / kPlanThreads;
  a.tiles = static_cast<uint32_t>((tiles_all + kPlanChunksMax - 1) / kPlanChunksMax);
  a.nchunks = static_cast<uint32_t>((tiles_all + a.tiles - 1) / a.tiles);
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
    const uint64_t wgs = (units + kPlanWaves - 1) / kPlanWaves;
    // (a multiple of 8 from 8 up, so xcd_spread gives each XCD whole row groups; spare workgroups find no unit)
    a.list_wgs = static_cast<uint32_t>(wgs < 512 ? (wgs >= 8 ? (wgs + 7) / 8 * 8 : wgs) : 512);
  }
  a.chk_off = check_offset;
  a.chk_slots = check_slots;
  a.chk_status = check_status;
  const unsigned grid = a.nchunks + chain_wgs + a.list_wgs + (check_status != nullptr ? count : 0u);
  hipStream_t st = S(stream);
  if (count <= 2) k_round_plan<2><<<grid, kPlanThreads, 0, st>>>(a);
  else if (count <= 4) k_round_plan<4><<<grid, kPlanThreads, 0, st>>>(a);
  else if (count <= 8) k_round_plan<8><<<grid, kPlanThreads, 0, st>>>(a);
  else k_round_plan<OMR_MAX_WORKERS><<<grid, kPlanThreads, 0, st>>>(a);
  return launch_status("k_round_plan");
}

int omr_round_plan_list(const uint64_t* row_masks, uint32_t count, uint64_t mask_stride, uint64_t rows,
                        uint32_t rows_per_part, uint32_t num_lanes, const uint64_t* bounds, uint32_t num_bounds,
                        uint64_t* write_set, uint64_t* union_masks, uint32_t* prefix, uint64_t* counts,
                        uint64_t* zero_masks, uint32_t* zero_counters, uint32_t num_zero_counters,
                        uint64_t* workspace, uint32_t seq, uint32_t* union_next, uint32_t block_size,
                        const omr_sum_list* list, omr_stream_t stream) {
  return omr_round_plan_check(row_masks, count, mask_stride, rows, rows_per_part, num_lanes, bounds, num_bounds,
                              write_set, union_masks, prefix, counts, zero_masks, zero_counters, num_zero_counters,
                              workspace, seq, union_next, block_size, list, 0, 0, nullptr, stream);
}

int omr_round_plan(const uint64_t* row_masks, uint32_t count, uint64_t rows, uint32_t rows_per_part,
                   uint32_t num_lanes, const uint64_t* bounds, uint32_t num_bounds, uint64_t* write_set,
                   uint64_t* union_masks, uint32_t* prefix, uint64_t* counts, uint64_t* zero_masks,
                   uint64_t* workspace, uint32_t seq, omr_stream_t stream) {
  return omr_round_plan_list(row_masks, count, rows, rows, rows_per_part, num_lanes, bounds, num_bounds, write_set,
                             union_masks, prefix, counts, zero_masks, nullptr, 0, workspace, seq, nullptr, 0, nullptr,
                             stream);
}

int omr_move_blocks_f32(const float* src, float* dst, int dir, const uint64_t* row_masks, const uint32_t* prefix,
                        uint64_t rows, uint32_t num_lanes, uint32_t block_size, uint64_t skip_begin,
                        uint64_t skip_end, omr_stream_t stream) {
  if (dir != 0 && dir != 1) return fail("move_blocks: dir must be 0 (pack) or 1 (unpack)");
  if (block_size != 256 && block_size != 512 && block_size != 1024)
    return fail("move_blocks: block_size %u unsupported", block_size);
  const uint32_t vec = block_size / 256;
  if (num_lanes == 0 || num_lanes > 64 || (num_lanes & (num_lanes - 1)) != 0)
    return fail("move_blocks: num_lanes %u", num_lanes);
  if (skip_begin > skip_end || skip_end > rows) return fail("move_blocks: bad skip range");
  if (rows == 0) return 0;
  if (src == nullptr || dst == nullptr || row_masks == nullptr || prefix == nullptr)
    return fail("move_blocks: NULL pointer");
  if (reinterpret_cast<uintptr_t>(src) % 16 != 0 || reinterpret_cast<uintptr_t>(dst) % 16 != 0)
    return fail("move_blocks: buffers must be 16-byte aligned");
  MoveArgs a;
  a.src = src;
  a.dst = dst;
  a.masks = row_masks;
  a.prefix = prefix;
  a.rows = rows;
  a.skip_b = skip_begin;
  a.skip_e = skip_end;
  a.lanes = num_lanes;
  a.block = block_size;
  a.dir = static_cast<uint32_t>(dir);
  a.lg = unit_lanes(rows, num_lanes);
  const unsigned g = grid_for(rows * (num_lanes / a.lg));
  hipStream_t st = S(stream);
  switch (vec) {
    case 1: k_move<1><<<g, kWGThreads, 0, st>>>(a); break;
    case 2: k_move<2><<<g, kWGThreads, 0, st>>>(a); break;
    default: k_move<4><<<g, kWGThreads, 0, st>>>(a); break;
  }
  return launch_status("k_move");
}

}  // extern "C"

namespace {
template <int W>
void launch_shard_sum_w(const SumArgs& a, unsigned g, hipStream_t st) {
  switch (a.block / 256) {
    case 1: k_shard_sum<1, W><<<g, kWGThreads, 0, st>>>(a); break;
    case 2: k_shard_sum<2, W><<<g, kWGThreads, 0, st>>>(a); break;
    default: k_shard_sum<4, W><<<g, kWGThreads, 0, st>>>(a); break;
  }
}

int launch_shard_sum(const SumArgs& a0, const uint64_t* recv_offsets, hipStream_t st) {
  SumArgs a = a0;
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
  const uint64_t units = ((srows + kShardUnitRows - 1) / kShardUnitRows) * a.lanes;
  if (units > 0xFFFFFFFFull) return fail("shard_sum: %llu units", static_cast<unsigned long long>(units));
  a.units = static_cast<uint32_t>(units);
  a.lane_shift = static_cast<uint32_t>(__builtin_ctz(a.lanes));
  const unsigned g = grid_for(units);
  if (a.count <= 2) launch_shard_sum_w<2>(a, g, st);
  else if (a.count <= 4) launch_shard_sum_w<4>(a, g, st);
  else if (a.count <= 8) launch_shard_sum_w<8>(a, g, st);
  else launch_shard_sum_w<OMR_MAX_WORKERS>(a, g, st);
  return launch_status("k_shard_sum");
}
}  // namespace

extern "C" {

int omr_shard_sum_f32(const float* own, uint32_t me, const float* recv, const uint64_t* recv_offsets,
                      const uint64_t* row_masks, uint32_t count, const uint32_t* prefix, const uint64_t* write_set,
                      uint64_t rows, uint64_t row_begin, uint64_t row_end, uint32_t num_lanes, uint32_t block_size,
                      int packed_out, float* out, omr_stream_t stream) {
  return omr_shard_sum_stride_f32(own, me, recv, recv_offsets, row_masks, rows, count, prefix, write_set, rows,
                                  row_begin, row_end, num_lanes, block_size, packed_out, out, stream);
}

int omr_shard_sum_stride_f32(const float* own, uint32_t me, const float* recv, const uint64_t* recv_offsets,
                             const uint64_t* row_masks, uint64_t mask_stride, uint32_t count, const uint32_t* prefix,
                             const uint64_t* write_set, uint64_t rows, uint64_t row_begin, uint64_t row_end,
                             uint32_t num_lanes, uint32_t block_size, int packed_out, float* out, omr_stream_t stream) {
  if (mask_stride < rows) return fail("shard_sum: mask_stride %llu < rows", static_cast<unsigned long long>(mask_stride));
  SumArgs a{};
  a.own = own;
  a.recv = recv;
  a.masks = row_masks;
  a.mstride = mask_stride;
  a.prefix = prefix;
  a.write_set = write_set;
  a.out = out;
  a.rows = rows;
  a.r0 = row_begin;
  a.r1 = row_end;
  a.count = count;
  a.me = me;
  a.lanes = num_lanes;
  a.block = block_size;
  a.packed_out = packed_out ? 1u : 0u;
  return launch_shard_sum(a, recv_offsets, S(stream));
}

int omr_sum_list_geometry(uint64_t n, uint32_t block_size, uint32_t num_lanes, uint32_t num_parts, uint64_t row_begin,
                          uint64_t row_end, uint32_t count, uint64_t* units, uint32_t* capacity) {
  Layout L;
  if (int rc = make_layout(n, block_size, num_lanes, num_parts, &L)) return rc;
  const FusedShape f = fused_shape(L);
  if (count == 0 || count > OMR_MAX_WORKERS) return fail("sum_list: count %u out of range", count);
  if (row_begin > row_end || row_end > L.rows || row_begin % f.S != 0 || row_end % f.S != 0)
    return fail("sum_list: rows [%llu, %llu) are not whole %u-row column segments",
                static_cast<unsigned long long>(row_begin), static_cast<unsigned long long>(row_end), f.S);
  if (units) *units = ((row_end - row_begin) / f.S) * pack_groups(f) * kSumUnitsPerGroup * L.lanes;
  if (capacity) *capacity = kSumUnitRows * count + 1;  // + the terminator
  return 0;
}

int omr_sum_list_build(const uint64_t* row_masks, uint32_t count, uint64_t mask_stride, uint64_t n,
                       uint32_t block_size, uint32_t num_lanes, uint32_t num_parts, const omr_sum_list* list,
                       omr_stream_t stream) {
  Layout L;
  if (int rc = make_layout(n, block_size, num_lanes, num_parts, &L)) return rc;
  ListArgs a;
  if (int rc = make_list_args(L, row_masks, count, mask_stride, list, &a)) return rc;
  const uint64_t units = list_units_host(a);
  if (units == 0) return 0;
  k_sum_list<<<grid_for(units), kWGThreads, 0, S(stream)>>>(a);
  return launch_status("k_sum_list");
}

int omr_shard_sum_list_f32(const float* own, const float* recv, const omr_sum_list* list, uint32_t count, uint64_t n,
                           uint32_t block_size, uint32_t num_lanes, uint32_t num_parts, const uint64_t* write_set,
                           const uint32_t* write_prefix, int packed_out, float* out, omr_stream_t stream) {
  uint64_t units = 0;
  uint32_t cap = 0;
  if (list == nullptr) return fail("shard_sum_list: NULL list");
  if (int rc = omr_sum_list_geometry(n, block_size, num_lanes, num_parts, list->row_begin, list->row_end, count,
                                     &units, &cap))
    return rc;
  if (units == 0) return 0;
  if (list->records == nullptr || list->counts == nullptr || out == nullptr || (list->me < count && own == nullptr) ||
      (count > 1 && recv == nullptr) || (packed_out && (write_set == nullptr || write_prefix == nullptr)))
    return fail("shard_sum_list: NULL pointer");
  if (reinterpret_cast<uintptr_t>(out) % 16 != 0 || reinterpret_cast<uintptr_t>(own) % 16 != 0 ||
      reinterpret_cast<uintptr_t>(recv) % 16 != 0)
    return fail("shard_sum_list: buffers must be 16-byte aligned");
  ListSumArgs a{};
  a.own = own;
  a.recv = recv;
  a.records = list->records;
  a.counts = list->counts;
  a.write_set = write_set;
  a.wprefix = write_prefix;
  a.out = out;
  if (units > 0xFFFFFFFFull) return fail("shard_sum_list: %llu units", static_cast<unsigned long long>(units));
  a.units = static_cast<uint32_t>(units);
  a.r0 = list->row_begin;
  a.cap = cap;
  a.lanes = num_lanes;
  a.block = block_size;
  a.packed_out = packed_out ? 1u : 0u;
  const unsigned g = grid_for(units);
  switch (block_size / 256) {
    case 1: k_shard_sum_list<1><<<g, kWGThreads, 0, S(stream)>>>(a); break;
    case 2: k_shard_sum_list<2><<<g, kWGThreads, 0, S(stream)>>>(a); break;
    default: k_shard_sum_list<4><<<g, kWGThreads, 0, S(stream)>>>(a); break;
  }
  return launch_status("k_shard_sum_list");
}

}  // extern "C"
#endif  // OMR_NO_CAPI

