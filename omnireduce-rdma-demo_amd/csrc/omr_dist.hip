// omr_dist.cpp — C++ host side of the multi-rank sparse all-reduce (include/omr_dist.h).
//
// The round is the one omr/dist.py drives from Python (same shard bounds, same packed-stream layout, same
// kernels from libomr.so); this is the C++ host path the ./omr_client and ./omr_server drivers run, with either
// RCCL over xGMI (one process per GPU) or an in-process loopback transport (threads, device-to-device copies).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <utility>
#include <vector>

#include "omr_dist.h"

namespace {

thread_local char g_derr[512];

int derr(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_derr, sizeof(g_derr), fmt, ap);
  va_end(ap);
  return code;
}

int hip_check(hipError_t e, const char* what) {
  return e == hipSuccess ? 0 : derr(static_cast<int>(e), "%s: %s", what, hipGetErrorString(e));
}

int nccl_check(ncclResult_t r, const char* what) {
  return r == ncclSuccess ? 0 : derr(1000 + static_cast<int>(r), "%s: %s", what, ncclGetErrorString(r));
}

int omr_check(int rc, const char* what) {
  return rc == 0 ? 0 : derr(rc, "%s: %s", what, omr_last_error());
}

#define TRY(x)                       \
  do {                               \
    if (int _rc = (x)) return _rc;   \
  } while (0)

struct Slice {
  void* ptr;
  size_t bytes;
};

}  // namespace

// ---------------------------------------------------------------- transports

struct omr_dist {
  int rank = 0, world = 1;
  virtual ~omr_dist() = default;
  // out[p*bytes .. (p+1)*bytes) = rank p's `in`; `in` may alias out + rank*bytes
  virtual int allgather(const void* in, void* out, size_t bytes, hipStream_t st) = 0;
  // sends[p] to peer p, recvs[p] from peer p (sizes agree pairwise; zero = nothing), p != rank
  virtual int exchange(const std::vector<Slice>& sends, const std::vector<Slice>& recvs, hipStream_t st) = 0;
};

namespace {

struct RcclDist final : omr_dist {
  ncclComm_t comm = nullptr;
  ~RcclDist() override {
    if (comm) (void)ncclCommDestroy(comm);
  }
  int allgather(const void* in, void* out, size_t bytes, hipStream_t st) override {
    return nccl_check(ncclAllGather(in, out, bytes, ncclUint8, comm, st), "ncclAllGather");
  }
  int exchange(const std::vector<Slice>& sends, const std::vector<Slice>& recvs, hipStream_t st) override {
    TRY(nccl_check(ncclGroupStart(), "ncclGroupStart"));
    for (int p = 0; p < world; ++p) {
      if (p == rank) continue;
      if (recvs[p].bytes) TRY(nccl_check(ncclRecv(recvs[p].ptr, recvs[p].bytes, ncclUint8, p, comm, st), "ncclRecv"));
      if (sends[p].bytes) TRY(nccl_check(ncclSend(sends[p].ptr, sends[p].bytes, ncclUint8, p, comm, st), "ncclSend"));
    }
    return nccl_check(ncclGroupEnd(), "ncclGroupEnd");
  }
};

}  // namespace

struct omr_local_board {
  int world;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t generation = 0;
  std::vector<const void*> posted;               // allgather inputs
  std::vector<std::vector<Slice>> posted_sends;  // [rank][peer]
  explicit omr_local_board(int w) : world(w), posted(w), posted_sends(w, std::vector<Slice>(w, Slice{nullptr, 0})) {}
  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    const uint64_t gen = generation;
    if (++arrived == world) {
      arrived = 0;
      ++generation;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return generation != gen; });
    }
  }
};

namespace {

// Loopback transport: ranks are threads of one process; each posts its buffers, waits at a barrier, and pulls
// what its peers posted with device-to-device copies (any pair of devices; UVA peer or staged copies).
struct LocalDist final : omr_dist {
  omr_local_board* b = nullptr;
  int allgather(const void* in, void* out, size_t bytes, hipStream_t st) override {
    TRY(hip_check(hipStreamSynchronize(st), "hipStreamSynchronize"));
    b->posted[rank] = in;
    b->barrier();
    for (int p = 0; p < world; ++p) {
      char* dst = static_cast<char*>(out) + static_cast<size_t>(p) * bytes;
      if (b->posted[p] != dst) TRY(hip_check(hipMemcpy(dst, b->posted[p], bytes, hipMemcpyDefault), "hipMemcpy"));
    }
    b->barrier();
    return 0;
  }
  int exchange(const std::vector<Slice>& sends, const std::vector<Slice>& recvs, hipStream_t st) override {
    TRY(hip_check(hipStreamSynchronize(st), "hipStreamSynchronize"));
    b->posted_sends[rank] = sends;
    b->barrier();
    for (int p = 0; p < world; ++p) {
      if (p == rank || recvs[p].bytes == 0) continue;
      const Slice& s = b->posted_sends[p][rank];
      if (s.bytes != recvs[p].bytes)
        return derr(OMR_EINVAL, "local exchange: rank %d expects %zu bytes from %d, peer posted %zu", rank,
                    recvs[p].bytes, p, s.bytes);
      TRY(hip_check(hipMemcpy(recvs[p].ptr, s.ptr, s.bytes, hipMemcpyDefault), "hipMemcpy"));
    }
    b->barrier();
    return 0;
  }
};

// prefix[a*(rows+1) + bounds[s]] for every array a and bound s -> counts[a*(N+1) + s]
__global__ void k_gather_counts(const uint32_t* prefix, uint64_t rows, const uint64_t* bounds, uint32_t arrays,
                                uint32_t nb, uint32_t* counts) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= arrays * nb) return;
  const uint32_t a = i / nb, s = i % nb;
  counts[i] = prefix[static_cast<uint64_t>(a) * (rows + 1) + bounds[s]];
}

template <typename T>
int dev_alloc(T** p, size_t count) {
  return hip_check(hipMalloc(reinterpret_cast<void**>(p), std::max<size_t>(count, 1) * sizeof(T)), "hipMalloc");
}

}  // namespace

struct omr_ar_plan {
  omr_dist* d = nullptr;
  uint64_t n = 0, nb = 0, rows = 0;
  uint32_t B = 0, lanes = 0, parts = 0, rpp = 0;
  int N = 1, me = 0;
  std::vector<uint64_t> bounds;
  uint64_t shard_nb = 0;
  uint64_t* masks_all = nullptr;  // [(N+1)][rows]: workers, then the write set
  uint64_t* umask = nullptr;      // [rows]
  uint32_t* prefix = nullptr;     // [(N+1)][rows+1]
  uint32_t* my_list = nullptr;
  uint32_t* full_list = nullptr;
  uint32_t* shard_list = nullptr;
  uint32_t* count = nullptr;      // [3]
  float* packed = nullptr;        // own non-zero blocks, block order
  float* recv = nullptr;          // this shard's contributions, worker-major
  uint64_t* recv_off = nullptr;   // [N] block offset of each worker's stream in recv
  float* sums = nullptr;          // this shard's sums
  float* results = nullptr;       // every shard's sums, shard-major
  int32_t* flags_ws = nullptr;
  uint32_t* next_ws = nullptr;
  uint32_t* unext_ws = nullptr;
  uint64_t* bounds_dev = nullptr;
  uint32_t* counts_dev = nullptr;
  uint32_t* counts_host = nullptr;    // pinned
  uint64_t* recv_off_host = nullptr;  // pinned
  void* prefix_ws = nullptr;
  size_t prefix_ws_bytes = 0;
  void* compact_ws = nullptr;
  size_t compact_ws_bytes = 0;
};

extern "C" {

const char* omr_dist_last_error(void) { return g_derr; }

int omr_dist_unique_id(void* id) {
  if (id == nullptr) return derr(OMR_EINVAL, "unique id: NULL");
  static_assert(sizeof(ncclUniqueId) == OMR_UNIQUE_ID_BYTES, "ncclUniqueId size");
  return nccl_check(ncclGetUniqueId(static_cast<ncclUniqueId*>(id)), "ncclGetUniqueId");
}

int omr_dist_create_rccl(const void* id, int rank, int world, omr_dist** out) {
  if (id == nullptr || out == nullptr || world < 1 || rank < 0 || rank >= world)
    return derr(OMR_EINVAL, "create_rccl: bad arguments");
  auto* d = new RcclDist();
  d->rank = rank;
  d->world = world;
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  if (int rc = nccl_check(ncclCommInitRank(&d->comm, world, uid, rank), "ncclCommInitRank")) {
    delete d;
    return rc;
  }
  *out = d;
  return 0;
}

omr_local_board* omr_local_board_create(int world) { return world > 0 ? new omr_local_board(world) : nullptr; }
void omr_local_board_destroy(omr_local_board* board) { delete board; }

int omr_dist_create_local(omr_local_board* board, int rank, omr_dist** out) {
  if (board == nullptr || out == nullptr || rank < 0 || rank >= board->world)
    return derr(OMR_EINVAL, "create_local: bad arguments");
  auto* d = new LocalDist();
  d->b = board;
  d->rank = rank;
  d->world = board->world;
  *out = d;
  return 0;
}

int omr_dist_rank(const omr_dist* d) { return d ? d->rank : -1; }
int omr_dist_world(const omr_dist* d) { return d ? d->world : -1; }

int omr_dist_destroy(omr_dist* d) {
  delete d;
  return 0;
}

int omr_ar_plan_destroy(omr_ar_plan* p) {
  if (p == nullptr) return 0;
  void* devs[] = {p->masks_all, p->umask,    p->prefix,    p->my_list,    p->full_list,  p->shard_list,
                  p->count,     p->packed,   p->recv_off,  p->sums,       p->results,
                  p->flags_ws,  p->next_ws,  p->unext_ws,  p->bounds_dev, p->counts_dev, p->prefix_ws,
                  p->compact_ws};
  for (void* v : devs) (void)hipFree(v);
  (void)hipHostFree(p->counts_host);
  (void)hipHostFree(p->recv_off_host);
  delete p;
  return 0;
}

int omr_ar_plan_create(omr_dist* d, uint64_t n, uint32_t block_size, uint32_t num_lanes, uint32_t num_parts,
                       omr_ar_plan** out) {
  if (d == nullptr || out == nullptr) return derr(OMR_EINVAL, "ar_plan_create: NULL");
  *out = nullptr;
  TRY(omr_check(omr_layout_check(n, block_size, num_lanes, num_parts), "omr_layout_check"));
  auto* p = new omr_ar_plan();
  p->d = d;
  p->n = n;
  p->B = block_size;
  p->lanes = num_lanes;
  p->parts = num_parts;
  p->nb = n / block_size;
  p->rows = p->nb / num_lanes;
  p->rpp = static_cast<uint32_t>(p->rows / num_parts);
  p->N = d->world;
  p->me = d->rank;
  const int N = p->N;
  for (int s = 0; s <= N; ++s) p->bounds.push_back(static_cast<uint64_t>(s) * p->rows / N);
  uint64_t max_rows = 0;
  for (int s = 0; s < N; ++s) max_rows = std::max(max_rows, p->bounds[s + 1] - p->bounds[s]);
  p->shard_nb = max_rows * num_lanes;
  int rc = 0;
  auto A = [&](int r) {
    if (rc == 0) rc = r;
  };
  A(dev_alloc(&p->masks_all, (N + 1) * p->rows));
  A(dev_alloc(&p->umask, p->rows));
  A(dev_alloc(&p->prefix, (N + 1) * (p->rows + 1)));
  A(dev_alloc(&p->my_list, p->nb));
  A(dev_alloc(&p->full_list, p->nb));
  A(dev_alloc(&p->shard_list, p->shard_nb));
  A(dev_alloc(&p->count, 3));
  // one allocation: packed own blocks, then the peers' streams, so the shard sum addresses the rank's own
  // contribution in place (no copy into the receive area)
  A(dev_alloc(&p->packed, n + static_cast<size_t>(N) * p->shard_nb * block_size));
  if (rc == 0) p->recv = p->packed + n;
  A(dev_alloc(&p->recv_off, N));
  A(dev_alloc(&p->sums, p->shard_nb * block_size));
  A(dev_alloc(&p->results, n));
  A(dev_alloc(&p->flags_ws, p->nb));
  A(dev_alloc(&p->next_ws, p->nb));
  A(dev_alloc(&p->unext_ws, p->nb));
  A(dev_alloc(&p->bounds_dev, N + 1));
  A(dev_alloc(&p->counts_dev, (N + 1) * (N + 1)));
  p->prefix_ws_bytes = omr_prefix_workspace_bytes(p->rows, N + 1);
  p->compact_ws_bytes = omr_compact_workspace_bytes(p->rows);
  A(dev_alloc(reinterpret_cast<char**>(&p->prefix_ws), p->prefix_ws_bytes));
  A(dev_alloc(reinterpret_cast<char**>(&p->compact_ws), p->compact_ws_bytes));
  A(hip_check(hipHostMalloc(reinterpret_cast<void**>(&p->counts_host), (N + 1) * (N + 1) * sizeof(uint32_t)),
              "hipHostMalloc"));
  A(hip_check(hipHostMalloc(reinterpret_cast<void**>(&p->recv_off_host), N * sizeof(uint64_t)), "hipHostMalloc"));
  if (rc == 0)
    A(hip_check(hipMemcpy(p->bounds_dev, p->bounds.data(), (N + 1) * sizeof(uint64_t), hipMemcpyHostToDevice),
                "hipMemcpy bounds"));
  if (rc != 0) {
    omr_ar_plan_destroy(p);
    return rc;
  }
  *out = p;
  return 0;
}

int omr_sparse_round_f32(omr_ar_plan* p, const float* x, float* out, int32_t* flags, uint32_t* next_offsets,
                         uint32_t* union_next, int mode, uint64_t* sent_blocks, uint64_t* union_blocks,
                         omr_stream_t stream) {
  if (p == nullptr || x == nullptr || out == nullptr) return derr(OMR_EINVAL, "sparse_round: NULL");
  if (mode != OMR_ROUND_ALLREDUCE && mode != OMR_ROUND_REDUCE_SCATTER)
    return derr(OMR_EINVAL, "sparse_round: unknown mode %d", mode);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int N = p->N, me = p->me;
  const uint64_t rows = p->rows, B = p->B;
  uint64_t* my_masks = p->masks_all + static_cast<uint64_t>(me) * rows;
  int32_t* fl = flags ? flags : p->flags_ws;
  uint32_t* nx = next_offsets ? next_offsets : p->next_ws;
  uint32_t* un = union_next ? union_next : p->unext_ws;
  // 1. worker scan: flags, own row masks straight into this rank's all-gather slot, own next chain
  const float* bufs[1] = {x};
  TRY(omr_check(omr_scan_sum_f32(bufs, 1, p->n, p->B, p->lanes, p->parts, fl, my_masks, nx, nullptr, stream),
                "omr_scan_sum_f32"));
  // 2. every worker's row masks (in place)
  TRY(p->d->allgather(my_masks, p->masks_all, rows * sizeof(uint64_t), st));
  // 3. write set (union + lane heads), union, aggregator chain, prefixes, per-shard counts
  uint64_t* wset = p->masks_all + static_cast<uint64_t>(N) * rows;
  TRY(omr_check(omr_mask_union(p->masks_all, N, rows, p->rpp, p->lanes, 1, wset, stream), "omr_mask_union"));
  TRY(omr_check(omr_mask_union(p->masks_all, N, rows, p->rpp, p->lanes, 0, p->umask, stream), "omr_mask_union"));
  TRY(omr_check(omr_next_offsets(p->umask, 1, p->n, p->B, p->lanes, p->parts, un, stream), "omr_next_offsets"));
  TRY(omr_check(omr_row_prefix(p->masks_all, N + 1, rows, p->prefix, p->prefix_ws, p->prefix_ws_bytes, stream),
                "omr_row_prefix"));
  const uint32_t A = N + 1, NB = N + 1;
  k_gather_counts<<<(A * NB + 255) / 256, 256, 0, st>>>(p->prefix, rows, p->bounds_dev, A, NB, p->counts_dev);
  TRY(hip_check(hipGetLastError(), "k_gather_counts"));
  TRY(hip_check(hipMemcpyAsync(p->counts_host, p->counts_dev, A * NB * sizeof(uint32_t), hipMemcpyDeviceToHost, st),
                "hipMemcpyAsync counts"));
  TRY(hip_check(hipStreamSynchronize(st), "hipStreamSynchronize"));
  auto cnt = [&](int a, int s) -> uint64_t { return p->counts_host[a * NB + s]; };
  auto per = [&](int a, int s) -> uint64_t { return cnt(a, s + 1) - cnt(a, s); };
  // 4. pack own non-zero blocks (block order == shard order) and send each shard's slice to its aggregator
  const uint64_t total_send = cnt(me, N);
  TRY(omr_check(omr_compact(my_masks, 0, rows, p->lanes, p->my_list, p->count, p->compact_ws, p->compact_ws_bytes,
                            stream), "omr_compact"));
  TRY(omr_check(omr_gather_blocks_f32(x, p->my_list, static_cast<uint32_t>(total_send), p->B, p->packed, stream),
                "omr_gather_blocks_f32"));
  // stream offsets (in blocks) from p->packed: peers' streams in the receive area, this rank's own slice
  // where the gather left it
  std::vector<uint64_t> roff(N);
  uint64_t acc = 0;
  for (int w = 0; w < N; ++w) {
    roff[w] = acc;
    if (w != me) acc += per(w, me);
    p->recv_off_host[w] = (w == me) ? cnt(me, me) : p->n / p->B + roff[w];
  }
  std::vector<Slice> sends(N), recvs(N);
  for (int s = 0; s < N; ++s) {
    sends[s] = Slice{p->packed + cnt(me, s) * B, s == me ? 0 : per(me, s) * B * sizeof(float)};
    recvs[s] = Slice{p->recv + roff[s] * B, s == me ? 0 : per(s, me) * B * sizeof(float)};
  }
  TRY(hip_check(hipMemcpyAsync(p->recv_off, p->recv_off_host, N * sizeof(uint64_t), hipMemcpyHostToDevice, st),
                "hipMemcpyAsync recv_off"));
  TRY(p->d->exchange(sends, recvs, st));
  // 5. aggregator: rank-order sums of this shard's write set
  const uint64_t r0 = p->bounds[me], r1 = p->bounds[me + 1];
  const uint64_t nres_me = per(N, me);
  TRY(omr_check(omr_compact(wset, r0, r1, p->lanes, p->shard_list, p->count + 1, p->compact_ws,
                            p->compact_ws_bytes, stream), "omr_compact shard"));
  TRY(omr_check(omr_sparse_block_sum_f32(p->packed, p->recv_off, p->masks_all, N, rows, p->prefix, r0, p->lanes,
                                         p->shard_list, static_cast<uint32_t>(nres_me), p->B, p->sums, stream),
                "omr_sparse_block_sum_f32"));
  if (mode == OMR_ROUND_REDUCE_SCATTER) {  // aggregator keeps its shard: sums written in place into `out`
    TRY(omr_check(omr_scatter_blocks_f32(p->sums, p->shard_list, static_cast<uint32_t>(nres_me), p->B, out, stream),
                  "omr_scatter_blocks_f32 shard"));
    TRY(hip_check(hipStreamSynchronize(st), "hipStreamSynchronize"));
    if (sent_blocks) *sent_blocks = total_send - per(me, me);
    if (union_blocks) *union_blocks = nres_me;
    return 0;
  }
  // 6. sums back to every worker, scattered in place
  std::vector<Slice> rs(N), rr(N);
  for (int s = 0; s < N; ++s) {
    rs[s] = Slice{p->sums, s == me ? 0 : nres_me * B * sizeof(float)};
    rr[s] = Slice{p->results + cnt(N, s) * B, per(N, s) * B * sizeof(float)};
  }
  if (nres_me)
    TRY(hip_check(hipMemcpyAsync(rr[me].ptr, p->sums, nres_me * B * sizeof(float), hipMemcpyDeviceToDevice, st),
                  "hipMemcpyAsync own sums"));
  rr[me].bytes = 0;
  TRY(p->d->exchange(rs, rr, st));
  const uint64_t total_res = cnt(N, N);
  TRY(omr_check(omr_compact(wset, 0, rows, p->lanes, p->full_list, p->count + 2, p->compact_ws, p->compact_ws_bytes,
                            stream), "omr_compact full"));
  TRY(omr_check(omr_scatter_blocks_f32(p->results, p->full_list, static_cast<uint32_t>(total_res), p->B, out, stream),
                "omr_scatter_blocks_f32"));
  TRY(hip_check(hipStreamSynchronize(st), "hipStreamSynchronize"));
  if (sent_blocks) *sent_blocks = total_send - per(me, me);
  if (union_blocks) *union_blocks = total_res;
  return 0;
}

int omr_sparse_allreduce_f32(omr_ar_plan* p, const float* x, float* out, int32_t* flags, uint32_t* next_offsets,
                             uint32_t* union_next, uint64_t* sent_blocks, uint64_t* union_blocks,
                             omr_stream_t stream) {
  return omr_sparse_round_f32(p, x, out, flags, next_offsets, union_next, OMR_ROUND_ALLREDUCE, sent_blocks,
                              union_blocks, stream);
}

}  // extern "C"
