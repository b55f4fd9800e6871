// omr_msg.hip — the message-level OmniReduce round in the reference's wire format.
//
// The bulk path (omr_scan_sum_*, the multi-rank round) computes the round's RESULT; this file reproduces the
// round's MESSAGES: every worker message and aggregator reply the reference's per-slot state machines
// exchange, byte for byte, in the layout of common.h / common.cc:
//   message   `len` blocks of B floats, then `len` uint32 next offsets, in a 2*MESSAGE_SIZE-float slot
//             (common.cc:399-408, :424); imm = (len << 16) | global slot (common.cc:443, :542)
//   worker    client.cc:180-205 first burst (the slot's lane heads) and client.cc:32-152 handle_recv
//   aggregator server.cc:13-199 handle_recv: min_next completion (:84-96), accumulate (:97-98), reply in
//             completion order (:143-147), lane advance / reset (:173-186)
// with the workers' messages of a protocol round arriving in rank order.
//
// The state machines are not stepped message by message.  Their schedule has a closed form:
// in protocol round r a slot's lane l carries the r-th block of its UNION chain (its head at r = 0, then the
// union's non-zero blocks: server.cc:86-96 makes min_next the union's next); worker w sends it iff r = 0 or w
// flags it; the lane completes on the message of the highest-ranked sender, so the reply lists the active lanes
// in the previous reply's order, stably sorted by that rank (round 0: lane order).  k_msg_schedule walks that
// per slot (one thread per slot, four lanes); everything else is parallel over (slot, round):
//   k_msg_pack       worker w's message of every (slot, round): gather its blocks + its next offsets
//   k_msg_aggregate  every reply: decode the workers' messages (lane from the next-offset meta, server.cc:82-85),
//                    rank-order sums from +0.0f, reply blocks in completion order + the union next offsets
//   k_msg_unpack     a worker applies every reply: block k -> buf[current_offset[lane]] (client.cc:87-90)
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <vector>

#include "omr.h"

namespace omr_detail {
int set_error(int code, const char* msg);
}

namespace {

constexpr uint32_t kMsg = OMR_MESSAGE_SIZE;   // MESSAGE_SIZE floats (common.h:31)
constexpr uint32_t kSlots = OMR_NUM_SLOTS;    // NUM_SLOTS (common.h:34)
constexpr uint32_t kSlotW = 2 * kMsg;         // floats per message slot (common.cc:405, :438)
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr int kWaves = 4;

typedef float v4f __attribute__((ext_vector_type(4)));

int mfail(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
int mfail(const char* fmt, ...) {
  char buf[256];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  return omr_detail::set_error(OMR_EINVAL, buf);
}

int mlaunch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e == hipSuccess) return 0;
  char buf[256];
  snprintf(buf, sizeof(buf), "%s: %s", what, hipGetErrorString(e));
  return omr_detail::set_error(static_cast<int>(e), buf);
}

// One protocol round of one slot: the block each lane carries (kNone: lane finished), the order the workers'
// messages list the lanes in (the previous reply's order; round 0: lane order) and the reply's order, as 4-bit
// lane indices, first position in the low nibble.
struct Sched {
  uint32_t blk[4];
  uint32_t ord_msg, ord_reply, nact, pad;
};

__device__ __forceinline__ uint32_t nib(uint32_t packed, uint32_t p) { return (packed >> (4 * p)) & 0xFu; }

struct SchedArgs {
  const uint64_t* masks;  // [m][rows] the workers' row masks (bit l of row r: block r*NB + l is non-zero)
  const uint32_t* unext;  // [nb] next offsets over the workers' union (the aggregator's min_next chain)
  uint64_t rows;
  uint32_t m, B, NB, rpp, parts, rcap, sentinel;
  Sched* sch;             // [G][rcap]
  uint32_t* rounds;       // [G]
  uint32_t* maxr;         // [1], atomic max (rcap + 1 when a slot overflows)
};

__global__ __launch_bounds__(64) void k_msg_schedule(SchedArgs a) {
  const uint32_t G = a.parts * kSlots;
  const uint32_t gs = blockIdx.x * blockDim.x + threadIdx.x;
  if (gs >= G) return;
  const uint32_t t = gs / kSlots, s = gs % kSlots, bpm = kMsg / a.B;
  uint32_t cur[4] = {kNone, kNone, kNone, kNone};
  for (uint32_t j = 0; j < bpm; ++j) cur[j] = t * a.rpp * a.NB + s * bpm + j;  // lane heads (client.cc:201-204)
  uint32_t ord = 0, nact = bpm;
  for (uint32_t j = 0; j < bpm; ++j) ord |= j << (4 * j);
  for (uint32_t r = 0;; ++r) {
    if (r >= a.rcap) {
      a.rounds[gs] = kNone;
      atomicMax(a.maxr, a.rcap + 1);
      return;
    }
    // completion rank of each active lane: the last sender in rank order (round 0: every worker sends heads)
    uint32_t key[4] = {0, 0, 0, 0};
    for (uint32_t p = 0; p < nact; ++p) {
      const uint32_t j = nib(ord, p);
      uint32_t k = a.m - 1;
      if (r > 0)
        while (k > 0 && ((a.masks[static_cast<uint64_t>(k) * a.rows + cur[j] / a.NB] >> (cur[j] % a.NB)) & 1u) == 0)
          --k;
      key[j] = k;
    }
    // reply order: the message order stably sorted by completion rank (server.cc:92-96 appends on completion)
    uint32_t rep = 0, nrep = 0;
    for (uint32_t k = 0; k < a.m && nrep < nact; ++k)
      for (uint32_t p = 0; p < nact; ++p) {
        const uint32_t j = nib(ord, p);
        if (key[j] == k) rep |= j << (4 * nrep++);
      }
    Sched rec;
    for (uint32_t j = 0; j < 4; ++j) rec.blk[j] = kNone;
    for (uint32_t p = 0; p < nact; ++p) rec.blk[nib(ord, p)] = cur[nib(ord, p)];
    rec.ord_msg = ord;
    rec.ord_reply = rep;
    rec.nact = nact;
    rec.pad = 0;
    a.sch[static_cast<uint64_t>(gs) * a.rcap + r] = rec;
    // advance along the union chain in reply order; lanes reaching the sentinel finish (server.cc:173-186)
    uint32_t nord = 0, nn = 0;
    for (uint32_t p = 0; p < nact; ++p) {
      const uint32_t j = nib(rep, p);
      const uint32_t nx = a.unext[cur[j]];
      if (nx < a.sentinel) {
        cur[j] = nx / a.B;
        nord |= j << (4 * nn++);
      }
    }
    if (nn == 0) {
      a.rounds[gs] = r + 1;
      atomicMax(a.maxr, r + 1);
      return;
    }
    ord = nord;
    nact = nn;
  }
}

struct PackArgs {
  const float* x;
  const int32_t* flags;  // this worker's [nb]
  const uint32_t* next;  // this worker's next-offset chain [nb] (client.cc:19-31 of block + B*NB)
  const Sched* sch;
  const uint32_t* rounds;
  float* msgs;           // [G][rcap][kSlotW]
  uint32_t* imm;         // [G][rcap]
  uint32_t G, rcap, B;
};

template <int VEC>
__global__ __launch_bounds__(64 * kWaves) void k_msg_pack(PackArgs a) {
  const int lane = threadIdx.x & 63;
  const uint64_t u = static_cast<uint64_t>(blockIdx.x) * kWaves + (threadIdx.x >> 6);
  if (u >= static_cast<uint64_t>(a.G) * a.rcap) return;
  const uint32_t gs = static_cast<uint32_t>(u / a.rcap), r = static_cast<uint32_t>(u % a.rcap);
  if (r >= a.rounds[gs]) return;
  const Sched rec = a.sch[u];
  uint32_t sel[4], len = 0;
  for (uint32_t p = 0; p < rec.nact; ++p) {  // lanes in message order that this worker sends
    const uint32_t b = rec.blk[nib(rec.ord_msg, p)];
    if (r == 0 || a.flags[b] == 1) sel[len++] = b;
  }
  if (lane == 0) a.imm[u] = len ? (len << 16) | gs : 0u;
  float* msg = a.msgs + u * kSlotW;
  for (uint32_t k = 0; k < len; ++k) {  // common.cc:405-407: the blocks, then :408 the next offsets
    const v4f* src = reinterpret_cast<const v4f*>(a.x + static_cast<uint64_t>(sel[k]) * a.B);
    v4f* dst = reinterpret_cast<v4f*>(msg + k * a.B);
#pragma unroll
    for (int q = 0; q < VEC; ++q) dst[q * 64 + lane] = src[q * 64 + lane];
  }
  if (static_cast<uint32_t>(lane) < len)
    reinterpret_cast<uint32_t*>(msg + len * a.B)[lane] = a.next[sel[lane]];
}

struct AggArgs {
  const float* msgs[OMR_MAX_WORKERS];
  const uint32_t* imm[OMR_MAX_WORKERS];
  const Sched* sch;
  const uint32_t* rounds;
  const uint32_t* unext;
  float* reply;    // [G][rcap][kSlotW]
  uint32_t* rimm;  // [G][rcap]
  uint32_t m, G, rcap, B, NB;
  uint32_t naggs, agg;  // this aggregator handles the global slots gs with gs % naggs == agg (common.cc:381-383)
};

template <int VEC>
__global__ __launch_bounds__(64 * kWaves) void k_msg_aggregate(AggArgs a) {
  constexpr int BPM = 4 / VEC;  // lanes per slot (BLOCKS_PER_MESSAGE) for B = 256 * VEC
  const int lane = threadIdx.x & 63;
  const uint64_t u = static_cast<uint64_t>(blockIdx.x) * kWaves + (threadIdx.x >> 6);
  if (u >= static_cast<uint64_t>(a.G) * a.rcap) return;
  const uint32_t gs = static_cast<uint32_t>(u / a.rcap), r = static_cast<uint32_t>(u % a.rcap);
  if (gs % a.naggs != a.agg || r >= a.rounds[gs]) return;
  const Sched rec = a.sch[u];
  const uint32_t lane0 = (gs % kSlots) * BPM;
  v4f acc[BPM][VEC];
#pragma unroll
  for (int j = 0; j < BPM; ++j)
#pragma unroll
    for (int q = 0; q < VEC; ++q) acc[j][q] = v4f{0.f, 0.f, 0.f, 0.f};  // the zeroed set (server.cc:148-150)
  for (uint32_t w = 0; w < a.m; ++w) {  // rank-order arrival
    const uint32_t len = a.imm[w][u] >> 16;
    const float* msg = a.msgs[w] + u * kSlotW;
    const uint32_t* meta = reinterpret_cast<const uint32_t*>(msg + len * a.B);
    for (uint32_t k = 0; k < len; ++k) {
      const uint32_t jb = (meta[k] / a.B) % a.NB - lane0;  // the lane, from the next offset (server.cc:82-85)
      const v4f* src = reinterpret_cast<const v4f*>(msg + k * a.B);
#pragma unroll
      for (int j = 0; j < BPM; ++j)
        if (static_cast<uint32_t>(j) == jb) {
#pragma unroll
          for (int q = 0; q < VEC; ++q) acc[j][q] += src[q * 64 + lane];  // server.cc:97-98
        }
    }
  }
  if (lane == 0) a.rimm[u] = (rec.nact << 16) | gs;
  float* out = a.reply + u * kSlotW;
  for (uint32_t p = 0; p < rec.nact; ++p) {  // completion order: sums then min_next (server.cc:144-147)
    const uint32_t jr = nib(rec.ord_reply, p);
    v4f* dst = reinterpret_cast<v4f*>(out + p * a.B);
#pragma unroll
    for (int j = 0; j < BPM; ++j)
      if (static_cast<uint32_t>(j) == jr) {
#pragma unroll
        for (int q = 0; q < VEC; ++q) dst[q * 64 + lane] = acc[j][q];
      }
  }
  if (static_cast<uint32_t>(lane) < rec.nact)
    reinterpret_cast<uint32_t*>(out + rec.nact * a.B)[lane] = a.unext[rec.blk[nib(rec.ord_reply, lane)]];
}

struct UnpackArgs {
  const float* reply;
  const uint32_t* rimm;
  const Sched* sch;
  const uint32_t* rounds;
  float* buf;
  uint32_t G, rcap, B, NB;
};

template <int VEC>
__global__ __launch_bounds__(64 * kWaves) void k_msg_unpack(UnpackArgs a) {
  const int lane = threadIdx.x & 63;
  const uint64_t u = static_cast<uint64_t>(blockIdx.x) * kWaves + (threadIdx.x >> 6);
  if (u >= static_cast<uint64_t>(a.G) * a.rcap) return;
  const uint32_t gs = static_cast<uint32_t>(u / a.rcap), r = static_cast<uint32_t>(u % a.rcap);
  if (r >= a.rounds[gs]) return;
  const Sched rec = a.sch[u];
  const uint32_t lane0 = (gs % kSlots) * (kMsg / a.B);
  const uint32_t len = a.rimm[u] >> 16;
  const float* msg = a.reply + u * kSlotW;
  const uint32_t* meta = reinterpret_cast<const uint32_t*>(msg + len * a.B);
  for (uint32_t k = 0; k < len; ++k) {  // client.cc:87-90: block k -> buf[current_offset[lane of next]]
    const uint32_t j = (meta[k] / a.B) % a.NB - lane0;
    const v4f* src = reinterpret_cast<const v4f*>(msg + k * a.B);
    v4f* dst = reinterpret_cast<v4f*>(a.buf + static_cast<uint64_t>(rec.blk[j]) * a.B);
#pragma unroll
    for (int q = 0; q < VEC; ++q) dst[q * 64 + lane] = src[q * 64 + lane];
  }
}

unsigned waves_grid(uint64_t units) { return static_cast<unsigned>((units + kWaves - 1) / kWaves); }

}  // namespace

// ---------------------------------------------------------------- host driver

struct omr_msg_plan {
  uint64_t n = 0, nb = 0, rows = 0;
  uint32_t B = 0, NB = 0, parts = 0, rpp = 0, m = 0, G = 0, rcap = 0, vec = 1;
  std::vector<float*> msgs;      // per worker [G][rcap][kSlotW]
  std::vector<uint32_t*> imm;    // per worker [G][rcap]
  int32_t* flags = nullptr;      // [m][nb]
  uint32_t* next = nullptr;      // [m][nb]
  uint64_t* masks = nullptr;     // [m][rows]
  uint64_t* umask = nullptr;     // [rows]
  uint32_t* unext = nullptr;     // [nb]
  float* reply = nullptr;        // [G][rcap][kSlotW]
  uint32_t* rimm = nullptr;      // [G][rcap]
  Sched* sch = nullptr;          // [G][rcap]
  uint32_t* rounds = nullptr;    // [G]
  uint32_t* maxr = nullptr;      // [1] device
  uint32_t* maxr_host = nullptr; // pinned
  void* ws = nullptr;
  size_t ws_bytes = 0;
};

namespace {

int hipc(hipError_t e, const char* what) {
  if (e == hipSuccess) return 0;
  char buf[256];
  snprintf(buf, sizeof(buf), "%s: %s", what, hipGetErrorString(e));
  return omr_detail::set_error(static_cast<int>(e), buf);
}

#define MTRY(x)                     \
  do {                              \
    if (int _rc = (x)) return _rc;  \
  } while (0)

void free_logs(omr_msg_plan* p) {
  for (auto* v : p->msgs) (void)hipFree(v);
  for (auto* v : p->imm) (void)hipFree(v);
  p->msgs.assign(p->m, nullptr);
  p->imm.assign(p->m, nullptr);
  (void)hipFree(p->reply);
  (void)hipFree(p->rimm);
  (void)hipFree(p->sch);
  p->reply = nullptr;
  p->rimm = nullptr;
  p->sch = nullptr;
  p->rcap = 0;
}

int alloc_logs(omr_msg_plan* p, uint32_t rcap) {
  free_logs(p);
  const uint64_t units = static_cast<uint64_t>(p->G) * rcap;
  for (uint32_t w = 0; w < p->m; ++w) {
    MTRY(hipc(hipMalloc(&p->msgs[w], units * kSlotW * sizeof(float)), "hipMalloc messages"));
    MTRY(hipc(hipMalloc(&p->imm[w], units * sizeof(uint32_t)), "hipMalloc imm"));
  }
  MTRY(hipc(hipMalloc(&p->reply, units * kSlotW * sizeof(float)), "hipMalloc replies"));
  MTRY(hipc(hipMalloc(&p->rimm, units * sizeof(uint32_t)), "hipMalloc reply imm"));
  MTRY(hipc(hipMalloc(&p->sch, units * sizeof(Sched)), "hipMalloc schedule"));
  p->rcap = rcap;
  return 0;
}

int run_schedule(const uint64_t* masks, uint32_t m, uint64_t rows, const uint32_t* unext, uint32_t B, uint32_t NB,
                 uint32_t rpp, uint32_t parts, uint32_t rcap, Sched* sch, uint32_t* rounds, uint32_t* maxr,
                 hipStream_t st) {
  MTRY(hipc(hipMemsetAsync(maxr, 0, sizeof(uint32_t), st), "hipMemsetAsync"));
  SchedArgs a;
  a.masks = masks;
  a.unext = unext;
  a.rows = rows;
  a.m = m;
  a.B = B;
  a.NB = NB;
  a.rpp = rpp;
  a.parts = parts;
  a.rcap = rcap;
  a.sentinel = omr_sentinel(B, NB);
  a.sch = sch;
  a.rounds = rounds;
  a.maxr = maxr;
  const uint32_t G = parts * kSlots;
  k_msg_schedule<<<(G + 63) / 64, 64, 0, st>>>(a);
  return mlaunch("k_msg_schedule");
}

int launch_schedule(omr_msg_plan* p, hipStream_t st) {
  MTRY(run_schedule(p->masks, p->m, p->rows, p->unext, p->B, p->NB, p->rpp, p->parts, p->rcap, p->sch, p->rounds,
                    p->maxr, st));
  MTRY(hipc(hipMemcpyAsync(p->maxr_host, p->maxr, sizeof(uint32_t), hipMemcpyDeviceToHost, st), "hipMemcpyAsync"));
  return hipc(hipStreamSynchronize(st), "hipStreamSynchronize");
}

int run_pack(const float* x, const int32_t* flags, const uint32_t* next, const Sched* sch, const uint32_t* rounds,
             uint32_t G, uint32_t rcap, uint32_t B, float* msgs, uint32_t* imm, hipStream_t st) {
  PackArgs a;
  a.x = x;
  a.flags = flags;
  a.next = next;
  a.sch = sch;
  a.rounds = rounds;
  a.msgs = msgs;
  a.imm = imm;
  a.G = G;
  a.rcap = rcap;
  a.B = B;
  const unsigned g = waves_grid(static_cast<uint64_t>(G) * rcap);
  switch (B / 256) {
    case 1: k_msg_pack<1><<<g, 64 * kWaves, 0, st>>>(a); break;
    case 2: k_msg_pack<2><<<g, 64 * kWaves, 0, st>>>(a); break;
    default: k_msg_pack<4><<<g, 64 * kWaves, 0, st>>>(a); break;
  }
  return mlaunch("k_msg_pack");
}

int run_aggregate(const float* const* msgs, const uint32_t* const* imm, uint32_t m, const Sched* sch,
                  const uint32_t* rounds, const uint32_t* unext, uint32_t G, uint32_t rcap, uint32_t B, uint32_t NB,
                  uint32_t naggs, uint32_t agg, float* reply, uint32_t* rimm, hipStream_t st) {
  AggArgs ag;
  for (uint32_t w = 0; w < OMR_MAX_WORKERS; ++w) {
    ag.msgs[w] = w < m ? msgs[w] : nullptr;
    ag.imm[w] = w < m ? imm[w] : nullptr;
  }
  ag.sch = sch;
  ag.rounds = rounds;
  ag.unext = unext;
  ag.reply = reply;
  ag.rimm = rimm;
  ag.m = m;
  ag.G = G;
  ag.rcap = rcap;
  ag.B = B;
  ag.NB = NB;
  ag.naggs = naggs;
  ag.agg = agg;
  const unsigned g = waves_grid(static_cast<uint64_t>(G) * rcap);
  switch (B / 256) {
    case 1: k_msg_aggregate<1><<<g, 64 * kWaves, 0, st>>>(ag); break;
    case 2: k_msg_aggregate<2><<<g, 64 * kWaves, 0, st>>>(ag); break;
    default: k_msg_aggregate<4><<<g, 64 * kWaves, 0, st>>>(ag); break;
  }
  return mlaunch("k_msg_aggregate");
}

int run_unpack(const float* reply, const uint32_t* rimm, const Sched* sch, const uint32_t* rounds, uint32_t G,
               uint32_t rcap, uint32_t B, uint32_t NB, float* buf, hipStream_t st) {
  UnpackArgs u;
  u.reply = reply;
  u.rimm = rimm;
  u.sch = sch;
  u.rounds = rounds;
  u.buf = buf;
  u.G = G;
  u.rcap = rcap;
  u.B = B;
  u.NB = NB;
  const unsigned g = waves_grid(static_cast<uint64_t>(G) * rcap);
  switch (B / 256) {
    case 1: k_msg_unpack<1><<<g, 64 * kWaves, 0, st>>>(u); break;
    case 2: k_msg_unpack<2><<<g, 64 * kWaves, 0, st>>>(u); break;
    default: k_msg_unpack<4><<<g, 64 * kWaves, 0, st>>>(u); break;
  }
  return mlaunch("k_msg_unpack");
}

// the message primitives' shared argument check: a layout the wire format supports
int msg_layout(uint64_t n, uint32_t B, uint32_t NB, uint32_t parts, uint32_t* rpp, uint64_t* rows) {
  if (int rc = omr_layout_check(n, B, NB, parts)) return rc;
  if (NB != kSlots * (kMsg / B)) return mfail("message layout: num_lanes must be NUM_SLOTS*MESSAGE_SIZE/BLOCK_SIZE");
  *rows = n / B / NB;
  *rpp = static_cast<uint32_t>(*rows / parts);
  return 0;
}

}  // namespace

extern "C" {

int omr_msg_plan_destroy(omr_msg_plan* p) {
  if (p == nullptr) return 0;
  free_logs(p);
  void* devs[] = {p->flags, p->next, p->masks, p->umask, p->unext, p->rounds, p->maxr, p->ws};
  for (void* v : devs) (void)hipFree(v);
  (void)hipHostFree(p->maxr_host);
  delete p;
  return 0;
}

int omr_msg_plan_create(uint64_t n, uint32_t block_size, uint32_t num_lanes, uint32_t num_parts, uint32_t m,
                        omr_msg_plan** out) {
  if (out == nullptr) return mfail("msg_plan_create: out is NULL");
  *out = nullptr;
  if (int rc = omr_layout_check(n, block_size, num_lanes, num_parts)) return rc;
  if (m == 0 || m > OMR_MAX_WORKERS) return mfail("msg_plan_create: m=%u out of range (1..%d)", m, OMR_MAX_WORKERS);
  if (num_lanes != kSlots * (kMsg / block_size))
    return mfail("msg_plan_create: num_lanes must be NUM_SLOTS*MESSAGE_SIZE/BLOCK_SIZE = %u",
                 kSlots * (kMsg / block_size));
  auto* p = new omr_msg_plan();
  p->n = n;
  p->B = block_size;
  p->NB = num_lanes;
  p->parts = num_parts;
  p->nb = n / block_size;
  p->rows = p->nb / num_lanes;
  p->rpp = static_cast<uint32_t>(p->rows / num_parts);
  p->m = m;
  p->G = num_parts * kSlots;
  p->vec = block_size / 256;
  p->msgs.assign(m, nullptr);
  p->imm.assign(m, nullptr);
  int rc = 0;
  auto A = [&](int r) {
    if (rc == 0) rc = r;
  };
  A(hipc(hipMalloc(&p->flags, static_cast<size_t>(m) * p->nb * sizeof(int32_t)), "hipMalloc flags"));
  A(hipc(hipMalloc(&p->next, static_cast<size_t>(m) * p->nb * sizeof(uint32_t)), "hipMalloc next"));
  A(hipc(hipMalloc(&p->masks, static_cast<size_t>(m) * p->rows * sizeof(uint64_t)), "hipMalloc masks"));
  A(hipc(hipMalloc(&p->umask, p->rows * sizeof(uint64_t)), "hipMalloc union"));
  A(hipc(hipMalloc(&p->unext, p->nb * sizeof(uint32_t)), "hipMalloc union next"));
  A(hipc(hipMalloc(&p->rounds, p->G * sizeof(uint32_t)), "hipMalloc rounds"));
  A(hipc(hipMalloc(&p->maxr, sizeof(uint32_t)), "hipMalloc max rounds"));
  A(hipc(hipHostMalloc(reinterpret_cast<void**>(&p->maxr_host), sizeof(uint32_t)), "hipHostMalloc"));
  p->ws_bytes = omr_scan_workspace_bytes(n, block_size, num_lanes, num_parts);
  A(hipc(hipMalloc(&p->ws, p->ws_bytes ? p->ws_bytes : 16), "hipMalloc workspace"));
  if (rc == 0 && p->ws_bytes) A(hipc(hipMemset(p->ws, 0, p->ws_bytes), "hipMemset workspace"));
  if (rc == 0) A(alloc_logs(p, 16));
  if (rc != 0) {
    omr_msg_plan_destroy(p);
    return rc;
  }
  *out = p;
  return 0;
}

int omr_msg_round_f32(omr_msg_plan* p, const float* const* bufs, float* const* outs, uint32_t* max_rounds,
                      omr_stream_t stream) {
  if (p == nullptr || bufs == nullptr || outs == nullptr) return mfail("msg_round: NULL argument");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const uint32_t m = p->m;
  for (uint32_t w = 0; w < m; ++w) {
    if (bufs[w] == nullptr || outs[w] == nullptr) return mfail("msg_round: NULL buffer for worker %u", w);
    if (reinterpret_cast<uintptr_t>(bufs[w]) % 16 || reinterpret_cast<uintptr_t>(outs[w]) % 16)
      return mfail("msg_round: buffers must be 16-byte aligned");
  }
  // 1. worker scans: flags, next-offset chains, row masks (client.cc:19-31 for every block)
  MTRY(hipc(hipMemsetAsync(p->masks, 0, static_cast<size_t>(m) * p->rows * sizeof(uint64_t), st), "hipMemsetAsync"));
  for (uint32_t w = 0; w < m; ++w)
    MTRY(omr_worker_scan_f32(bufs[w], p->n, p->B, p->NB, p->parts, p->flags + w * p->nb, p->next + w * p->nb,
                             p->masks + w * p->rows, nullptr, p->ws, p->ws_bytes, stream));
  // 2. the aggregator's min_next chain: next offsets over the union (server.cc:86-96)
  MTRY(omr_mask_union(p->masks, m, p->rows, p->rpp, p->NB, 0, p->umask, stream));
  MTRY(omr_next_offsets(p->umask, 1, p->n, p->B, p->NB, p->parts, p->unext, stream));
  // 3. per-slot schedule; grow the logs and redo it when a slot needs more protocol rounds than they hold
  MTRY(launch_schedule(p, st));
  if (*p->maxr_host > p->rcap) {
    uint32_t cap = p->rcap;
    while (cap < p->rpp + 2) cap *= 2;  // a lane carries at most its head plus rows_per_part - 1 blocks
    MTRY(alloc_logs(p, cap));
    MTRY(launch_schedule(p, st));
    if (*p->maxr_host > p->rcap) return mfail("msg_round: %u protocol rounds exceed %u", *p->maxr_host, p->rcap);
  }
  // 4. every worker's messages (client.cc:180-205 first burst, :113-127 later rounds)
  for (uint32_t w = 0; w < m; ++w)
    MTRY(run_pack(bufs[w], p->flags + w * p->nb, p->next + w * p->nb, p->sch, p->rounds, p->G, p->rcap, p->B,
                  p->msgs[w], p->imm[w], st));
  // 5. the aggregator's replies (server.cc:68-162): one aggregator owns every slot here
  std::vector<const float*> mp(p->msgs.begin(), p->msgs.end());
  std::vector<const uint32_t*> ip(p->imm.begin(), p->imm.end());
  MTRY(run_aggregate(mp.data(), ip.data(), m, p->sch, p->rounds, p->unext, p->G, p->rcap, p->B, p->NB, 1, 0, p->reply,
                     p->rimm, st));
  // 6. every worker applies every reply in place (client.cc:87-90)
  for (uint32_t w = 0; w < m; ++w)
    MTRY(run_unpack(p->reply, p->rimm, p->sch, p->rounds, p->G, p->rcap, p->B, p->NB, outs[w], st));
  if (max_rounds) *max_rounds = *p->maxr_host;
  return 0;
}

size_t omr_msg_sched_bytes(void) { return sizeof(Sched); }

int omr_msg_schedule(const uint64_t* row_masks, uint32_t m, const uint32_t* union_next, uint64_t n, uint32_t block_size,
                     uint32_t num_lanes, uint32_t num_parts, uint32_t round_capacity, void* sched, uint32_t* rounds,
                     uint32_t* max_rounds, omr_stream_t stream) {
  uint32_t rpp = 0;
  uint64_t rows = 0;
  MTRY(msg_layout(n, block_size, num_lanes, num_parts, &rpp, &rows));
  if (m == 0 || m > OMR_MAX_WORKERS) return mfail("msg_schedule: m=%u out of range", m);
  if (row_masks == nullptr || union_next == nullptr || sched == nullptr || rounds == nullptr || max_rounds == nullptr)
    return mfail("msg_schedule: NULL argument");
  if (round_capacity == 0) return mfail("msg_schedule: round_capacity is 0");
  return run_schedule(row_masks, m, rows, union_next, block_size, num_lanes, rpp, num_parts, round_capacity,
                      static_cast<Sched*>(sched), rounds, max_rounds, reinterpret_cast<hipStream_t>(stream));
}

int omr_msg_pack_f32(const float* x, const int32_t* flags, const uint32_t* next_offsets, const void* sched,
                     const uint32_t* rounds, uint32_t num_parts, uint32_t round_capacity, uint32_t block_size,
                     float* messages, uint32_t* imm, omr_stream_t stream) {
  if (block_size != 256 && block_size != 512 && block_size != 1024) return mfail("msg_pack: block_size %u", block_size);
  if (x == nullptr || flags == nullptr || next_offsets == nullptr || sched == nullptr || rounds == nullptr ||
      messages == nullptr || imm == nullptr)
    return mfail("msg_pack: NULL argument");
  return run_pack(x, flags, next_offsets, static_cast<const Sched*>(sched), rounds, num_parts * kSlots, round_capacity,
                  block_size, messages, imm, reinterpret_cast<hipStream_t>(stream));
}

int omr_msg_aggregate_f32(const float* const* messages, const uint32_t* const* imm, uint32_t m, const void* sched,
                          const uint32_t* rounds, const uint32_t* union_next, uint32_t num_parts,
                          uint32_t round_capacity, uint32_t block_size, uint32_t num_lanes, uint32_t num_aggregators,
                          uint32_t aggregator, float* replies, uint32_t* reply_imm, omr_stream_t stream) {
  if (block_size != 256 && block_size != 512 && block_size != 1024)
    return mfail("msg_aggregate: block_size %u", block_size);
  if (m == 0 || m > OMR_MAX_WORKERS) return mfail("msg_aggregate: m=%u out of range", m);
  if (num_aggregators == 0 || aggregator >= num_aggregators) return mfail("msg_aggregate: aggregator out of range");
  if (messages == nullptr || imm == nullptr || sched == nullptr || rounds == nullptr || union_next == nullptr ||
      replies == nullptr || reply_imm == nullptr)
    return mfail("msg_aggregate: NULL argument");
  for (uint32_t w = 0; w < m; ++w)
    if (messages[w] == nullptr || imm[w] == nullptr) return mfail("msg_aggregate: NULL log for worker %u", w);
  return run_aggregate(messages, imm, m, static_cast<const Sched*>(sched), rounds, union_next, num_parts * kSlots,
                       round_capacity, block_size, num_lanes, num_aggregators, aggregator, replies, reply_imm,
                       reinterpret_cast<hipStream_t>(stream));
}

int omr_msg_unpack_f32(const float* replies, const uint32_t* reply_imm, const void* sched, const uint32_t* rounds,
                       uint32_t num_parts, uint32_t round_capacity, uint32_t block_size, uint32_t num_lanes,
                       float* buf, omr_stream_t stream) {
  if (block_size != 256 && block_size != 512 && block_size != 1024) return mfail("msg_unpack: block_size %u", block_size);
  if (replies == nullptr || reply_imm == nullptr || sched == nullptr || rounds == nullptr || buf == nullptr)
    return mfail("msg_unpack: NULL argument");
  return run_unpack(replies, reply_imm, static_cast<const Sched*>(sched), rounds, num_parts * kSlots, round_capacity,
                    block_size, num_lanes, buf, reinterpret_cast<hipStream_t>(stream));
}

int omr_msg_logs(omr_msg_plan* p, uint32_t worker, float** messages, uint32_t** imm, float** replies,
                 uint32_t** reply_imm, uint32_t** rounds, uint32_t* round_capacity) {
  if (p == nullptr || worker >= p->m) return mfail("msg_logs: bad plan or worker");
  if (messages) *messages = p->msgs[worker];
  if (imm) *imm = p->imm[worker];
  if (replies) *replies = p->reply;
  if (reply_imm) *reply_imm = p->rimm;
  if (rounds) *rounds = p->rounds;
  if (round_capacity) *round_capacity = p->rcap;
  return 0;
}

}  // extern "C"
