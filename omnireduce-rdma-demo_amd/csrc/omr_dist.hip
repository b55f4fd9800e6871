// omr_dist.hip — C++ host side of the multi-rank sparse all-reduce (include/omr_dist.h).
//
// The product's round driver (same shard bounds and packed-stream layout as the test-only Python twin
// tests/dist_twin.py; kernels from libomr.so), run by ./omr_client, ./omr_server, bench.py and omr/cdist.py over
// RCCL (one process per GPU), HIP IPC (processes sharing GPUs) or an in-process loopback transport (threads).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdlib>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <deque>
#include <memory>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "omr_dist.h"

namespace {

thread_local char g_derr[512];
thread_local int g_destroy_rc = 0;  // a transport's teardown that left device-side state behind (omr_dist_destroy)

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
using Slices = std::vector<Slice>;  // several pieces to or from one peer, matched in order (zero-byte ones skipped)

}  // namespace

// ---------------------------------------------------------------- transports

int64_t default_timeout_ms() {
  const char* e = getenv("OMR_DIST_TIMEOUT_MS");
  const long long v = e ? atoll(e) : 0;
  return v > 0 ? v : 60000;
}

struct omr_dist {
  int rank = 0, world = 1;
  // omr_dist_inject_fault (test hook): the next exchange fails once it has issued `fault_after` non-empty pieces
  int64_t fault_after = -1;
  // called before each non-empty piece of an exchange (k = pieces issued so far) and once after the last (k = their
  // count): fails the armed exchange at its k-th piece
  int fault(int64_t k) {
    if (fault_after < 0 || k < fault_after) return 0;
    fault_after = -1;
    return derr(OMR_EINVAL, "exchange: fault injected after %lld pieces (omr_dist_inject_fault)", static_cast<long long>(k));
  }
  // Failure containment (the reference exits on a failed post, common.cc:450-451; a rank of a collective group must
  // instead make sure its peers do not wait for it forever).  Every host-side wait of a transport or a round is bounded
  // by this deadline; any error of an operation, an expired deadline or omr_dist_abort aborts the transport: RCCL's
  // communicators are aborted (ncclCommAbort cancels the operations queued on them), the loopback and IPC groups
  // raise a flag their peers' waits watch, and every later operation fails at once with OMR_EABORTED.
  int64_t timeout_ms = default_timeout_ms();
  std::atomic<bool> aborted{false};
  std::atomic<bool> abort_started{false};
  char abort_why[256] = {};
  // abort the transport (once) and return rc; the caller's message (g_derr) is kept
  int abort_with(int rc, const char* why) {
    if (!abort_started.exchange(true)) {
      snprintf(abort_why, sizeof(abort_why), "%s", why);
      aborted.store(true, std::memory_order_release);
      abort_group();
    }
    return rc;
  }
  int contain(int rc) { return rc == 0 ? 0 : abort_with(rc, g_derr); }
  int check_open(const char* what) const {
    if (!aborted.load(std::memory_order_acquire)) return 0;
    return derr(OMR_EABORTED, "%s: rank %d's transport was aborted (%s)", what, rank, abort_why);
  }
  // the transport's group-wide failure signals: RCCL's asynchronous errors, a loopback or IPC peer's abort; an error
  // aborts this rank's transport too
  int poll() {
    TRY(check_open("poll"));
    return contain(do_poll());
  }
  // the operations the round uses (every rank of the group calls them in the same order); an error aborts
  bool fault_allgather = false;  // omr_dist_inject_allgather_fault (test hook)
  // omr_dist_test_world1_round (test hook): a one-rank group runs the multi-rank round's code path (all-gather, plan,
  // exchange on the side stream) instead of the one-launch round, and RCCL issues its collectives as RCCL calls
  bool world1_general = false;
  int allgather(const void* in, void* out, size_t bytes, hipStream_t st) {
    TRY(check_open("allgather"));
    if (fault_allgather) {
      fault_allgather = false;
      return contain(derr(OMR_EINVAL, "allgather: fault injected (omr_dist_inject_allgather_fault)"));
    }
    return contain(do_allgather(in, out, bytes, st));
  }
  int exchange(const std::vector<Slices>& sends, const std::vector<Slices>& recvs, hipStream_t st) {
    TRY(check_open("exchange"));
    return contain(do_exchange(sends, recvs, st));
  }
  int reduce_scatter(const float* in, float* out, size_t count, hipStream_t st) {
    TRY(check_open("reduce_scatter"));
    return contain(do_reduce_scatter(in, out, count, st));
  }
  virtual ~omr_dist() = default;
  virtual void abort_group() {}
  virtual int do_poll() { return 0; }
  // out[p*bytes .. (p+1)*bytes) = rank p's `in`; `in` may alias out + rank*bytes
  virtual int do_allgather(const void* in, void* out, size_t bytes, hipStream_t st) = 0;
  // sends[p] to peer p, recvs[p] from peer p, p != rank: the k-th non-empty send piece to a peer pairs with that
  // peer's k-th non-empty receive piece from this rank (equal sizes); every rank calls it, possibly with nothing
  virtual int do_exchange(const std::vector<Slices>& sends, const std::vector<Slices>& recvs, hipStream_t st) = 0;
  // out[0 .. count) = sum over ranks p of in_p[rank*count .. (rank+1)*count)  (dense stand-in)
  virtual int do_reduce_scatter(const float* in, float* out, size_t count, hipStream_t st) = 0;
  // Device memory of the plans that run on this transport goes through it: a transport that exports buffers to
  // other processes (HIP IPC) keeps every exported allocation alive until it is destroyed itself and hands it back
  // to the next alloc of the same size, so an address a peer has mapped is never freed and re-allocated under it.
  virtual int alloc(void** ptr, size_t bytes) { return hip_check(hipMalloc(ptr, bytes), "hipMalloc"); }
  // a plan's default side streams at N > 1 (omr_ar_plan_set_side_streams): two, except where ranks share GPUs (IPC)
  virtual int default_side_streams() const { return 2; }
  // whether a plan checks its side streams' hardware queues against the caller's stream (seat_side_streams): not for
  // the loopback transport, whose ranks are threads sharing one process's queues
  virtual bool queue_check_default() const { return true; }
  virtual void release(void* ptr) { (void)hipFree(ptr); }
};

namespace {

// Two communicators over the same ranks: `comm` carries the mask all-gather, `xcomm` the block exchange, so an
// asynchronous round's exchange (on the plan's communication stream) may run beside the next round's all-gather
// (on the caller's stream) — RCCL forbids concurrent use of ONE communicator from two streams.  Each is used in
// the same order on every rank.
struct RcclDist final : omr_dist {
  // Cross-thread abort (omr_dist_abort may run on another thread while this rank waits): ncclCommAbort
  // frees a communicator, so the handles are atomics that every owner-thread call reads ONCE (live() hands out the
  // snapshot) and the aborting thread clears before aborting, under `cm` (which do_poll holds too).  The
  // owner's calls that can block inside RCCL (a group end waiting on a peer) are not held back by it: the aborter
  // waits for them a short grace (kAbortGraceMs, or the deadline if shorter), then aborts anyway, which is what ends
  // such a wait.
  static constexpr int64_t kAbortGraceMs = 500;
  std::atomic<ncclComm_t> comm{nullptr}, xcomm{nullptr};
  std::mutex cm;
  std::atomic<int> in_rccl{0};  // owner-thread RCCL calls in progress (outside `cm`)
  ~RcclDist() override {
    if (ncclComm_t c = xcomm.load()) (void)ncclCommDestroy(c);
    if (ncclComm_t c = comm.load()) (void)ncclCommDestroy(c);
  }
  // ncclCommAbort on both communicators (the split one first): the operations queued on them are cancelled on the
  // device, so this rank's streams drain; the peers' matching operations are left to their own deadlines
  void abort_group() override {
    const auto t0 = std::chrono::steady_clock::now();
    const int64_t grace = std::min<int64_t>(timeout_ms, kAbortGraceMs);
    while (in_rccl.load(std::memory_order_acquire) != 0 &&
           std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(grace))
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    std::lock_guard<std::mutex> g(cm);
    const ncclComm_t x = xcomm.exchange(nullptr), c = comm.exchange(nullptr);
    if (x) (void)ncclCommAbort(x);
    if (c) (void)ncclCommAbort(c);
  }
  int do_poll() override {
    std::lock_guard<std::mutex> g(cm);
    for (ncclComm_t c : {comm.load(), xcomm.load()}) {
      if (c == nullptr) continue;
      ncclResult_t a = ncclSuccess;
      TRY(nccl_check(ncclCommGetAsyncError(c, &a), "ncclCommGetAsyncError"));
      if (a != ncclSuccess && a != ncclInProgress) return nccl_check(a, "RCCL asynchronous error");
    }
    return 0;
  }
  // an owner-thread RCCL call: counted (an aborter waits for it up to the grace), and refused once aborted
  struct InRccl {
    RcclDist* d;
    explicit InRccl(RcclDist* dd) : d(dd) { d->in_rccl.fetch_add(1, std::memory_order_acq_rel); }
    ~InRccl() { d->in_rccl.fetch_sub(1, std::memory_order_acq_rel); }
  };
  // the communicator for this call (`x`: the exchange's), read once
  int live(const char* what, bool x, ncclComm_t* out) {
    *out = (x ? xcomm : comm).load(std::memory_order_acquire);
    if (*out == nullptr || aborted.load(std::memory_order_acquire))
      return derr(OMR_EABORTED, "%s: rank %d's communicators were aborted", what, rank);
    return 0;
  }
  // A one-rank group's collectives are copies: RCCL queues the same copy kernel for them, after 5-10 us of host-side
  // group set-up per call (the world-1 round's host trace, profiles/r04/round_w1_trace/host_laps.txt), so they are
  // issued as the copy directly (world1_general: as RCCL calls, so the fault tests reach RCCL's group and abort paths).
  int do_allgather(const void* in, void* out, size_t bytes, hipStream_t st) override {
    if (world == 1 && !world1_general)
      return in == out ? 0 : hip_check(hipMemcpyAsync(out, in, bytes, hipMemcpyDeviceToDevice, st), "hipMemcpyAsync");
    InRccl g(this);
    ncclComm_t c = nullptr;
    TRY(live("allgather", false, &c));
    return nccl_check(ncclAllGather(in, out, bytes, ncclUint8, c, st), "ncclAllGather");
  }
  int do_exchange(const std::vector<Slices>& sends, const std::vector<Slices>& recvs, hipStream_t st) override {
    if (world == 1 && !world1_general) return fault(0);  // no peers: nothing to send or receive
    InRccl g(this);
    ncclComm_t xc = nullptr;
    TRY(live("exchange", true, &xc));
    TRY(nccl_check(ncclGroupStart(), "ncclGroupStart"));
    // The group is closed on every path: a group left open would capture every later RCCL call of this thread (the
    // next round's all-gather and exchange would be queued into it and never launched).  After a failed piece the
    // pieces already issued still go out with the group, the first error is returned, and the caller (omr_dist::
    // exchange) then aborts both communicators: the peers' pieces that this rank never posted can no longer match.
    int rc = 0;
    int64_t k = 0;
    for (int p = 0; p < world && rc == 0; ++p) {
      if (p == rank) continue;
      for (const Slice& r : recvs[p])
        if (r.bytes && rc == 0 && (rc = fault(k++)) == 0)
          rc = nccl_check(ncclRecv(r.ptr, r.bytes, ncclUint8, p, xc, st), "ncclRecv");
      for (const Slice& t : sends[p])
        if (t.bytes && rc == 0 && (rc = fault(k++)) == 0)
          rc = nccl_check(ncclSend(t.ptr, t.bytes, ncclUint8, p, xc, st), "ncclSend");
    }
    if (rc == 0) rc = fault(k);
    const int rc_end = nccl_check(ncclGroupEnd(), "ncclGroupEnd");
    return rc ? rc : rc_end;
  }
  int do_reduce_scatter(const float* in, float* out, size_t count, hipStream_t st) override {
    if (world == 1 && !world1_general)
      return in == out ? 0
                       : hip_check(hipMemcpyAsync(out, in, count * sizeof(float), hipMemcpyDeviceToDevice, st),
                                   "hipMemcpyAsync");
    InRccl g(this);
    ncclComm_t xc = nullptr;
    TRY(live("reduce_scatter", true, &xc));
    return nccl_check(ncclReduceScatter(in, out, count, ncclFloat32, ncclSum, xc, st), "ncclReduceScatter");
  }
};

}  // namespace

struct omr_local_board {
  int world;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t generation = 0;
  std::vector<const void*> posted;                // allgather inputs
  std::vector<std::vector<Slices>> posted_sends;  // [rank][peer]
  bool aborted = false;  // a rank aborted its transport: every wait of the group ends with an error
  int aborted_by = -1;
  explicit omr_local_board(int w) : world(w), posted(w), posted_sends(w, std::vector<Slices>(w)) {}
  // every rank's arrival, within the deadline; a rank that waits past it aborts the group (its peers then fail at
  // once instead of each waiting out its own deadline)
  int barrier(int rank, int64_t timeout_ms) {
    std::unique_lock<std::mutex> lk(mu);
    if (aborted) return derr(OMR_EABORTED, "loopback: rank %d aborted the group", aborted_by);
    const uint64_t gen = generation;
    if (++arrived == world) {
      arrived = 0;
      ++generation;
      cv.notify_all();
      return 0;
    }
    const bool done = cv.wait_for(lk, std::chrono::milliseconds(timeout_ms),
                                  [&] { return generation != gen || aborted; });
    if (generation != gen) return 0;
    if (aborted) return derr(OMR_EABORTED, "loopback: rank %d aborted the group", aborted_by);
    (void)done;
    abort_locked(rank);
    return derr(OMR_ETIMEDOUT, "loopback: rank %d waited %lld ms for its peers at a barrier", rank,
                static_cast<long long>(timeout_ms));
  }
  void abort_locked(int rank) {
    if (!aborted) aborted_by = rank;
    aborted = true;
    cv.notify_all();
  }
  void abort(int rank) {
    std::lock_guard<std::mutex> g(mu);
    abort_locked(rank);
  }
  bool is_aborted(int* by) {
    std::lock_guard<std::mutex> g(mu);
    *by = aborted_by;
    return aborted;
  }
};

namespace {

// Loopback transport: ranks are threads of one process; each posts its buffers, waits at a barrier, and pulls
// what its peers posted with device-to-device copies on its own stream (any pair of devices; UVA peer or staged
// copies), synchronised before the closing barrier: a device-to-device hipMemcpy may return before the copy is done,
// and a peer must not touch its buffers again until every reader is through.
struct LocalDist final : omr_dist {
  omr_local_board* b = nullptr;
  bool queue_check_default() const override { return false; }
  // (an error return makes omr_dist abort the group: the peers' barriers then end at once, with an error)
  void abort_group() override { b->abort(rank); }
  int do_poll() override {
    int by = -1;
    if (b->is_aborted(&by)) return derr(OMR_EABORTED, "loopback: rank %d aborted the group", by);
    return 0;
  }
  int barrier() { return b->barrier(rank, timeout_ms); }
  int do_allgather(const void* in, void* out, size_t bytes, hipStream_t st) override {
    TRY(hip_check(hipStreamSynchronize(st), "hipStreamSynchronize"));
    b->posted[rank] = in;
    TRY(barrier());
    int rc = 0;
    for (int p = 0; p < world && rc == 0; ++p) {
      char* dst = static_cast<char*>(out) + static_cast<size_t>(p) * bytes;
      if (b->posted[p] != dst)
        rc = hip_check(hipMemcpyAsync(dst, b->posted[p], bytes, hipMemcpyDefault, st), "hipMemcpyAsync");
    }
    if (rc == 0) rc = hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");
    else (void)hipStreamSynchronize(st);  // copies already queued finish before the peers move on
    TRY(rc);
    return barrier();
  }
  int do_exchange(const std::vector<Slices>& sends, const std::vector<Slices>& recvs, hipStream_t st) override {
    TRY(hip_check(hipStreamSynchronize(st), "hipStreamSynchronize"));
    b->posted_sends[rank] = sends;
    TRY(barrier());
    int rc = 0;
    int64_t pieces = 0;
    for (int p = 0; p < world && rc == 0; ++p) {
      if (p == rank) continue;
      const Slices& from = b->posted_sends[p][rank];
      size_t k = 0;
      for (const Slice& r : recvs[p]) {
        if (r.bytes == 0) continue;
        if ((rc = fault(pieces++)) != 0) break;
        while (k < from.size() && from[k].bytes == 0) ++k;
        if (k == from.size() || from[k].bytes != r.bytes) {
          rc = derr(OMR_EINVAL, "local exchange: rank %d expects %zu bytes from %d, peer posted %zu", rank, r.bytes, p,
                    k < from.size() ? from[k].bytes : size_t{0});
          break;
        }
        rc = hip_check(hipMemcpyAsync(r.ptr, from[k].ptr, r.bytes, hipMemcpyDefault, st), "hipMemcpyAsync");
        if (rc) break;
        ++k;
      }
    }
    if (rc == 0) rc = fault(pieces);
    if (rc == 0) rc = hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");
    else (void)hipStreamSynchronize(st);  // copies already queued finish before the peers move on
    // on an error the group is aborted by the caller instead of met here: the peers' closing barrier ends at once
    TRY(rc);
    return barrier();
  }
  int do_reduce_scatter(const float* in, float* out, size_t count, hipStream_t st) override {
    // every rank's input is addressable here (threads of one process): sum the shard in rank order
    TRY(hip_check(hipStreamSynchronize(st), "hipStreamSynchronize"));
    b->posted[rank] = in;
    TRY(barrier());
    std::vector<const float*> ptrs(world);
    for (int p = 0; p < world; ++p) ptrs[p] = static_cast<const float*>(b->posted[p]) + static_cast<size_t>(rank) * count;
    int rc = omr_check(omr_dense_sum_f32(ptrs.data(), static_cast<uint32_t>(world), count, out,
                                         reinterpret_cast<omr_stream_t>(st)), "omr_dense_sum_f32");
    if (rc == 0) rc = hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");  // peers' inputs read first
    else (void)hipStreamSynchronize(st);
    TRY(rc);
    return barrier();
  }
};

// ---------------------------------------------------------------- cross-process transport (HIP IPC)
//
// Ranks are separate processes on one node, any GPUs (several may share one), the stand-in for the reference's
// separate worker / aggregator machines (README.md:13-22) where RCCL cannot run (two ranks on one GPU).  A
// /dev/shm board holds, per rank: its IPC event handles, and per operation the IPC memory handles + offsets of what
// it offers.  Data moves device-to-device: each receiver pulls from the sender's buffer (mapped once with
// hipIpcOpenMemHandle) on its own stream.  Ordering is on the device, as with RCCL: the sender records a "ready"
// IPC event behind the producing work, the receiver's stream waits on it before copying, then records "done", and
// every rank's stream waits for all peers' "done" before it runs on (so a sender does not overwrite a buffer a peer
// is still reading).  The hosts only exchange sequence numbers (no stream synchronisation).  Two channels, as
// RcclDist's two communicators: 0 carries the all-gather, 1 the exchange and the dense reduce-scatter; every rank
// issues each channel's operations in the same order.
//
// An IPC event fails ("hipStreamWaitEvent: invalid argument") once it has been recorded about 32 times (ROCm 7.2,
// measured: the CLI at -W 10 -R 101 died at round ~32), so the events come in generations: a channel's operations
// [g K, (g+1) K) use generation g's events (each recorded K / kIpcRing times).  A rank creates and posts generation
// g+1 when it enters g and opens its peers' generation g then; generations are retired two back and destroyed in
// batches behind a device sync (a peer's or this rank's stream may still hold a wait on them).
constexpr uint32_t kIpcMagic = 0x4f4d5249;  // "OMRI"
constexpr int kIpcChans = 2, kIpcRing = 2, kIpcMaxRanks = 2 * OMR_MAX_WORKERS, kIpcMaxHandles = 32;
constexpr int kIpcMaxEntries = 4096;
constexpr uint64_t kIpcGenOps = 16;  // operations per event generation
constexpr size_t kIpcReap = 256;     // retired events destroyed (behind a device sync) in batches of this size
constexpr uint32_t kIpcAll = 0xFFFFFFFFu;  // an entry every peer reads (all-gather / reduce-scatter input)

struct IpcEntry {
  uint32_t peer, hidx;  // destination rank (kIpcAll: everyone), index into the post's handle table
  uint64_t off, bytes;  // piece = allocation(hidx) + off, bytes
};
struct IpcPost {
  uint32_t nent, nh;
  hipIpcMemHandle_t h[kIpcMaxHandles];
  uint64_t hid[kIpcMaxHandles];  // the poster's id of each handle's allocation (new after the allocation is forgotten)
  IpcEntry e[kIpcMaxEntries];
};
struct IpcRank {
  std::atomic<uint64_t> posted[kIpcChans], done[kIpcChans];
  std::atomic<uint32_t> joined, left;
  std::atomic<uint32_t> aborted;  // this rank aborted its transport (its peers' waits end with an error)
  std::atomic<uint64_t> evgen[kIpcChans][2];  // 1 + the generation whose handles slot [c][g % 2] holds (0: none)
  std::atomic<uint64_t> gpu;                  // 1 + the rank's GPU (PCI domain, bus, device), set before `joined`
  hipIpcMemHandle_t canary;                   // the rank's canary allocation (IpcDist::check_canaries), before `joined`
  hipIpcEventHandle_t ready[kIpcChans][2][kIpcRing], rdone[kIpcChans][2][kIpcRing];
};
struct IpcBoard {
  std::atomic<uint32_t> magic;
  uint32_t world;
  std::atomic<uint32_t> attached;
  IpcRank rank[kIpcMaxRanks];
  IpcPost post[kIpcChans][kIpcRing][kIpcMaxRanks];
};

std::string ipc_board_name(const void* id) {
  const unsigned char* c = static_cast<const unsigned char*>(id);
  char buf[48] = "/omr_";
  for (int i = 0; i < 12; ++i) snprintf(buf + 5 + 2 * i, 3, "%02x", c[i]);
  return buf;
}

// bounded spin on a host condition (peers are other processes: yield the core); ends early with an error when any
// rank of the board has aborted its transport
template <typename F>
int ipc_spin(F ready, const char* what, int rank, int64_t timeout_ms, const IpcBoard* b = nullptr, int world = 0) {
  const auto t0 = std::chrono::steady_clock::now();
  for (uint64_t i = 0;; ++i) {
    if (ready()) return 0;
    if ((i & 1023) == 1023) {
      for (int p = 0; b != nullptr && p < world; ++p)
        if (b->rank[p].aborted.load(std::memory_order_acquire) != 0)
          return derr(OMR_EABORTED, "ipc transport: rank %d aborted the group (rank %d waiting for %s)", p, rank, what);
      if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms))
        return derr(OMR_ETIMEDOUT, "ipc transport: rank %d waited %lld ms for %s", rank,
                    static_cast<long long>(timeout_ms), what);
      sched_yield();
    }
  }
}

// hipDeviceSynchronize within `ms` (run by a helper thread, left behind blocked if the device stays busy): after an
// abort a stream may wait forever on a gone peer (an IPC event that is never recorded), and the teardown must not
// (ADVICE r04).  true once the device is idle.
bool device_sync_within(int64_t ms) {
  struct Done {
    std::mutex mu;
    std::condition_variable cv;
    bool done = false;
  };
  auto d = std::make_shared<Done>();
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::thread t([d, dev] {
    (void)hipSetDevice(dev);
    (void)hipDeviceSynchronize();
    std::lock_guard<std::mutex> g(d->mu);
    d->done = true;
    d->cv.notify_all();
  });
  std::unique_lock<std::mutex> lk(d->mu);
  const bool ok = d->cv.wait_for(lk, std::chrono::milliseconds(ms), [&] { return d->done; });
  lk.unlock();
  if (ok) t.join();
  else t.detach();
  return ok;
}

struct IpcEvents {
  hipEvent_t ready[kIpcRing] = {}, rdone[kIpcRing] = {};
};

// OMR_IPC_TRACE=<path prefix> (diagnostic, round 6): stamps of the transport's ordering, written to <prefix>.<rank>.txt
// when the transport is destroyed.  Per operation (channel, sequence number): the sender's device clock just before its
// "ready" record (a one-wave kernel on the stream, queued behind the producing work) and the receiver's just after its
// wait on that event (queued before the copy), with the host-side hipEventQuery of the peer's event at the wait.  A
// receiver stamp earlier than its sender's means the device-side wait did not hold.  wall_clock64 is the GPU's
// constant 100 MHz clock, one per device, so stamps of processes on one GPU compare directly.
__global__ void k_ipc_stamp(uint64_t* dst) {
  if (threadIdx.x == 0) __hip_atomic_store(dst, wall_clock64(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// (OMR_IPC_TRACE) popcount of `words` 64-bit words: the all-gather's checksum, by its sender before its ready record
// and by each receiver after its copy
__global__ void k_ipc_popcount(const uint64_t* p, uint64_t words, uint64_t* dst) {
  __shared__ uint64_t part[256];
  uint64_t c = 0;
  for (uint64_t i = threadIdx.x; i < words; i += blockDim.x) c += static_cast<uint64_t>(__popcll(p[i]));
  part[threadIdx.x] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0;
    for (int i = 0; i < 256; ++i) t += part[i];
    __hip_atomic_store(dst, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

std::string hex64(const uint64_t* w) {  // an IPC handle's 64 bytes
  std::string o;
  char b[20];
  for (int i = 0; i < 8; ++i) {
    snprintf(b, sizeof(b), "%016llx", static_cast<unsigned long long>(w[i]));
    o += b;
  }
  return o;
}

struct IpcTrace {
  struct Rec {
    uint32_t chan;
    uint64_t seq;
    int32_t peer;   // -1 / -2: this rank's own ready / done record; p: after its wait for peer p's ready, 100 + p: for
                    // peer p's done; -3 / 200 + p: all-gather checksums (popcounts), of what this rank offers / of
                    // what it copied from peer p
    int32_t query;  // hipEventQuery of the peer's event right before the wait (hipSuccess 0, hipErrorNotReady 600)
    int64_t host_ns;
    uint32_t slot;  // its device stamp
  };
  std::string path;
  uint64_t* host = nullptr;
  uint64_t* dev = nullptr;
  uint32_t cap = 0, used = 0;
  std::vector<Rec> recs;
  std::vector<std::string> notes;  // exported / mapped allocations
  bool on() const { return host != nullptr; }
  void note(const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    notes.emplace_back(buf);
  }
  int open(const char* prefix, int rank) {
    path = std::string(prefix) + "." + std::to_string(rank) + ".txt";
    cap = 1u << 16;
    TRY(hip_check(hipHostMalloc(reinterpret_cast<void**>(&host), cap * sizeof(uint64_t),
                                hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc"));
    memset(host, 0, cap * sizeof(uint64_t));
    return hip_check(hipHostGetDevicePointer(reinterpret_cast<void**>(&dev), host, 0), "hipHostGetDevicePointer");
  }
  // words != 0: the record's value is the popcount of `words` words at `data` instead of a clock
  void stamp(hipStream_t st, uint32_t chan, uint64_t seq, int peer, int query, const void* data = nullptr,
             uint64_t words = 0) {
    if (used == cap) return;
    const uint32_t slot = used++;
    if (words) k_ipc_popcount<<<1, 256, 0, st>>>(static_cast<const uint64_t*>(data), words, dev + slot);
    else k_ipc_stamp<<<1, 64, 0, st>>>(dev + slot);
    recs.push_back(Rec{chan, seq, peer, query,
                       std::chrono::duration_cast<std::chrono::nanoseconds>(
                           std::chrono::steady_clock::now().time_since_epoch()).count(), slot});
  }
  // (after an abort the device is not waited for: stamps still pending read 0)
  void close(bool dead) {
    if (!on()) return;
    if (!dead) (void)hipDeviceSynchronize();
    if (FILE* f = fopen(path.c_str(), "w")) {
      for (const std::string& n : notes) fprintf(f, "# %s\n", n.c_str());
      fprintf(f, "# chan seq peer query host_ns device_clock\n");
      for (const Rec& r : recs)
        fprintf(f, "%u %llu %d %d %lld %llu\n", r.chan, static_cast<unsigned long long>(r.seq), r.peer, r.query,
                static_cast<long long>(r.host_ns), static_cast<unsigned long long>(host[r.slot]));
      fclose(f);
    }
    (void)hipHostFree(host);
    host = dev = nullptr;
  }
};

struct IpcDist final : omr_dist {
  IpcBoard* b = nullptr;
  std::string name;
  IpcEvents mine[kIpcChans][2];                          // this rank's events, generation g in [c][g % 2]
  std::vector<std::array<IpcEvents, kIpcChans * 2>> peer;  // peers' events, opened, [p][c * 2 + g % 2]
  std::vector<hipEvent_t> retired;                         // events of old generations, destroyed in batches
  // A batch of retired events goes to a reaper thread, which destroys it behind a device sync of its own.  Round 4
  // synchronised the device on the round's thread: with several ranks on one GPU that held every rank's host about
  // 140 ms each 128 rounds (4 IPC ranks: 4.2-4.9 ms per round over 50 timed rounds that held one, 1.35-1.43 ms
  // otherwise; profiles/r05/side_streams/).
  // The reaper's state is shared with it (not reached through `this`): after an abort its device sync may never return
  // (a stream waiting on a gone peer's event), and the transport is then destroyed without it.
  struct Reap {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::vector<hipEvent_t>> q;
    bool stop = false, exited = false;
    std::atomic<bool> leak{false};  // the group was aborted: drop batches instead of waiting for the device
  };
  std::shared_ptr<Reap> reap;
  std::thread reaper;
  static void reap_main(std::shared_ptr<Reap> r, int dev) {
    (void)hipSetDevice(dev);
    std::unique_lock<std::mutex> lk(r->mu);
    for (;;) {
      r->cv.wait(lk, [&] { return r->stop || !r->q.empty(); });
      if (r->q.empty()) break;
      std::vector<hipEvent_t> batch = std::move(r->q.front());
      r->q.pop_front();
      lk.unlock();
      // every operation queued before this point (the batch's last records and waits among them) has completed
      if (!r->leak.load(std::memory_order_acquire)) {
        (void)hipDeviceSynchronize();
        for (hipEvent_t e : batch) (void)hipEventDestroy(e);
      }
      lk.lock();
    }
    r->exited = true;
    r->cv.notify_all();
  }
  uint64_t seq[kIpcChans] = {0, 0};
  IpcTrace trace;  // OMR_IPC_TRACE (diagnostic)
  void* canary = nullptr;  // exported at attach, freed once every peer has left
  // the peers' canaries as mapped here, kept open (like every other mapping) until the transport goes: an imported
  // range closed during the group's life comes back from a later hipMalloc, and ROCm then refuses to export that
  // allocation (hipIpcGetMemHandle: invalid argument; 8 IPC ranks, profiles/r06/tests/)
  std::vector<void*> canary_maps;
  // allocation (base, size) -> its handle and this rank's id for it.  The plans' exported allocations are never freed
  // while the transport lives (release() parks them), so an entry never outlives its allocation.  A
  // caller's buffer (an input or output tensor) must stay allocated while the transport lives, as omr_dist.h says.
  struct OwnHandle {
    hipIpcMemHandle_t h;
    uint64_t id;
  };
  std::map<std::pair<uintptr_t, size_t>, OwnHandle> own;
  uint64_t next_id = 1;
  struct Mapping {
    uint64_t id;
    char* base;
  };
  std::map<std::pair<int, std::string>, Mapping> opened;  // (peer, handle bytes) -> the mapping of its current id
  std::map<void*, size_t> sized;                           // live allocations made through alloc(): their sizes
  std::multimap<size_t, void*> parked;                     // released exported allocations, by size

  template <typename F>
  int spin(F ready, const char* what) { return ipc_spin(ready, what, rank, timeout_ms, b, world); }
  // (an error return makes omr_dist abort: the flag ends the peers' waits on this rank at once)
  void abort_group() override {
    if (b != nullptr) b->rank[rank].aborted.store(1, std::memory_order_release);
  }
  int do_poll() override {
    for (int p = 0; b != nullptr && p < world; ++p)
      if (b->rank[p].aborted.load(std::memory_order_acquire) != 0)
        return derr(OMR_EABORTED, "ipc transport: rank %d aborted the group", p);
    return 0;
  }
  // Ranks that share a GPU add up their hardware queues, and HIP keeps a stream's queue for the process once made:
  // as 8 ranks on one GPU the round took 11-13 ms on one side stream and 23-28 ms once each rank had an exchange
  // stream too (bisected to that change; 45 ms on one side stream with the exchange stream's queue still held),
  // while 4 ranks ran faster with two (1.43 against 2.47 ms).  So two up to 4 ranks, one beyond
  // (omr_ar_plan_set_side_streams overrides it; profiles/r05/side_streams/).
  // Counted per GPU: the ranks that share THIS rank's GPU (the board has every rank's PCI address), so IPC
  // ranks spread over separate GPUs keep the exchange stream.
  int share_gpu = 1;
  int default_side_streams() const override { return share_gpu <= 4 ? 2 : 1; }
  // No queue check where ranks share this rank's GPU: the processes' queues together oversubscribe the hardware queue
  // slots, which the scheduler then time-slices, and the other ranks' kernels run in between, so whether the probe's
  // mark lands inside its window says more about the other ranks' load than about this process's queue mapping (and
  // every failed probe costs the window).  One rank per GPU checks, as over RCCL.
  bool queue_check_default() const override { return share_gpu <= 1; }

  static void release(IpcEvents& e, std::vector<hipEvent_t>& to) {
    for (int k = 0; k < kIpcRing; ++k) {
      if (e.ready[k]) to.push_back(e.ready[k]);
      if (e.rdone[k]) to.push_back(e.rdone[k]);
      e.ready[k] = e.rdone[k] = nullptr;
    }
  }

  ~IpcDist() override {
    const bool dead = aborted.load(std::memory_order_acquire);
    trace.close(dead);
    bool idle = true;  // the device is through with this transport's work
    if (reaper.joinable()) {
      bool exited;
      {
        std::unique_lock<std::mutex> lk(reap->mu);
        reap->stop = true;
        if (dead) reap->leak.store(true, std::memory_order_release);
        reap->cv.notify_all();
        // (it destroys what is queued first; after an abort it drops it, and is waited for within the deadline only)
        exited = dead ? reap->cv.wait_for(lk, std::chrono::milliseconds(timeout_ms), [&] { return reap->exited; })
                      : (reap->cv.wait(lk, [&] { return reap->exited; }), true);
      }
      if (exited) reaper.join();
      else reaper.detach();  // blocked in a device sync that waits on a gone peer: left behind with its shared state
      idle = exited;
    }
    if (b != nullptr) {
      // every rank's device work (copies out of its peers' buffers, waits on their events) ends before anyone
      // closes a mapping or an event; after an abort within the deadline, or everything device-side is left as is
      if (!dead) (void)hipDeviceSynchronize();
      else if (idle) idle = device_sync_within(timeout_ms);
      if (!idle) {
        (void)derr(OMR_ETIMEDOUT, "ipc transport: rank %d's streams still busy %lld ms after the abort; its mappings, "
                   "events and exported allocations are left as they are", rank, static_cast<long long>(timeout_ms));
        g_destroy_rc = OMR_ETIMEDOUT;
        b->rank[rank].left.store(1, std::memory_order_release);
        const bool last = b->attached.fetch_sub(1) == 1;
        munmap(b, sizeof(IpcBoard));
        if (last) shm_unlink(name.c_str());
        return;
      }
      b->rank[rank].left.store(1, std::memory_order_release);
      // (an aborted group does not wait: a peer may never leave; the driver keeps an exported allocation's memory
      // alive while a peer still maps it)
      for (int p = 0; p < world; ++p)
        if (ipc_spin([&] { return b->rank[p].left.load(std::memory_order_acquire) != 0; }, "peers to leave", rank,
                     timeout_ms, b, world) != 0)
          break;
      for (auto& kv : opened) (void)hipIpcCloseMemHandle(kv.second.base);
      for (void* m : canary_maps) (void)hipIpcCloseMemHandle(m);
    }
    // every peer has left (closed its mappings of them): the parked allocations can go now
    for (auto& kv : parked) (void)hipFree(kv.second);
    if (canary) (void)hipFree(canary);
    for (auto& v : peer)
      for (IpcEvents& e : v) release(e, retired);
    for (auto& row : mine)
      for (IpcEvents& e : row) release(e, retired);
    for (hipEvent_t e : retired) (void)hipEventDestroy(e);
    if (b != nullptr) {
      const bool last = b->attached.fetch_sub(1) == 1;
      munmap(b, sizeof(IpcBoard));
      if (last) shm_unlink(name.c_str());  // (normally gone already: rank 0 removes the name once all have joined)
    }
  }

  int attach(const void* id) {
    // (the ranks meet here after starting up, which takes a process importing its runtime a minute or more on a cold
    // machine: the rendezvous waits at least two minutes, the transport's own deadline applies afterwards)
    struct Rendezvous {
      int64_t& t;
      int64_t keep;
      ~Rendezvous() { t = keep; }
    } rendezvous{timeout_ms, timeout_ms};
    timeout_ms = std::max<int64_t>(timeout_ms, 120000);
    name = ipc_board_name(id);
    if (const char* t = getenv("OMR_IPC_TRACE")) TRY(trace.open(t, rank));
    const size_t bytes = sizeof(IpcBoard);
    int fd = -1;
    if (rank == 0) {
      shm_unlink(name.c_str());
      fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
      if (fd < 0 || ftruncate(fd, static_cast<off_t>(bytes)) != 0) {
        if (fd >= 0) close(fd);
        return derr(OMR_EINVAL, "ipc transport: cannot create %s: %s", name.c_str(), strerror(errno));
      }
    } else {
      TRY(ipc_spin([&] {
            if (fd < 0) fd = shm_open(name.c_str(), O_RDWR, 0600);
            struct stat stt;
            return fd >= 0 && fstat(fd, &stt) == 0 && static_cast<size_t>(stt.st_size) == bytes;
          }, "the board", rank, timeout_ms));
    }
    void* m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (m == MAP_FAILED) return derr(OMR_EINVAL, "ipc transport: mmap %s: %s", name.c_str(), strerror(errno));
    b = static_cast<IpcBoard*>(m);
    if (rank == 0) {
      b->world = static_cast<uint32_t>(world);  // the rest is zero (a fresh shm object)
      b->magic.store(kIpcMagic, std::memory_order_release);
    }
    TRY(ipc_spin([&] { return b->magic.load(std::memory_order_acquire) == kIpcMagic; }, "the board's owner", rank,
                 timeout_ms));
    if (b->world != static_cast<uint32_t>(world))
      return derr(OMR_EINVAL, "ipc transport: board world %u, this rank says %d", b->world, world);
    b->attached.fetch_add(1);
    IpcRank& me = b->rank[rank];
    TRY(make_canary(me));
    {
      int dev = 0, dom = 0, bus = 0, slot = 0;
      TRY(hip_check(hipGetDevice(&dev), "hipGetDevice"));
      TRY(hip_check(hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, dev), "hipDeviceGetAttribute"));
      TRY(hip_check(hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, dev), "hipDeviceGetAttribute"));
      TRY(hip_check(hipDeviceGetAttribute(&slot, hipDeviceAttributePciDeviceId, dev), "hipDeviceGetAttribute"));
      me.gpu.store(1 + ((static_cast<uint64_t>(static_cast<uint32_t>(dom)) << 32) |
                        (static_cast<uint64_t>(static_cast<uint32_t>(bus)) << 8) | static_cast<uint32_t>(slot)),
                   std::memory_order_relaxed);
    }
    for (int c = 0; c < kIpcChans; ++c) {
      TRY(publish(c, 0));
      TRY(publish(c, 1));
    }
    me.joined.store(1, std::memory_order_release);
    if (rank == 0) {  // the name is only needed until every rank has mapped the board
      for (int p = 0; p < world; ++p)
        TRY(spin([&] { return b->rank[p].joined.load(std::memory_order_acquire) != 0; }, "peers to join"));
      shm_unlink(name.c_str());
    }
    peer.assign(world, {});
    for (int p = 0; p < world; ++p)
      TRY(spin([&] { return b->rank[p].joined.load(std::memory_order_acquire) != 0; }, "peers to join"));
    share_gpu = 0;
    for (int p = 0; p < world; ++p)
      share_gpu += b->rank[p].gpu.load(std::memory_order_relaxed) == me.gpu.load(std::memory_order_relaxed) ? 1 : 0;
    if (int rc = check_canaries()) {  // (the peers' checks fail too: none waits on this rank)
      abort_group();
      return rc;
    }
    for (int c = 0; c < kIpcChans; ++c) TRY(open_gen(c, 0));
    return 0;
  }

  // The IPC memory handles must open at the exporter's address in every process.  They do not between a process that
  // loads the AddressSanitizer runtime and one that does not (round 6): ROCm's runtime then gives
  // every device allocation a 4 KiB leading redzone, and each process opens a handle with ITS OWN convention, so a
  // plain importer of a sanitized exporter's buffer lands 4 KiB before the data and a sanitized importer of a plain
  // one 4 KiB after it (OMR_IPC_TRACE: the exporter's handle names its allocation 0x1000 below the pointer; the
  // importers' pointers differ by 0x1000; profiles/r06/ipc_mix/).  The all-gather then copied the wrong 8 KiB and
  // the ranks' block counts disagreed.  So at attach each rank exports a canary (word i = (0xC0DE0000 | rank) << 32 | i:
  // no word is zero, so a zero-filled redzone never passes for one) and opens
  // every peer's: a peer whose canary does not read back from offset 0 fails the group at creation, with the offset.
  // Only the canary's first kCanaryRead bytes are read back, so a handle that opens up to 48 KiB off either way still
  // reads inside the 64 KiB allocation (a device read outside a mapping faults the GPU).
  static constexpr size_t kCanaryWords = 8192;  // 64 KiB
  static constexpr size_t kCanaryRead = 2048;   // words read back: 16 KiB
  static uint64_t canary_word(int r, size_t i) { return ((0xC0DE0000ull | static_cast<uint64_t>(r)) << 32) | i; }
  int make_canary(IpcRank& me) {
    TRY(hip_check(hipMalloc(&canary, kCanaryWords * 8), "hipMalloc canary"));
    std::vector<uint64_t> h(kCanaryWords);
    for (size_t i = 0; i < kCanaryWords; ++i) h[i] = canary_word(rank, i);
    TRY(hip_check(hipMemcpy(canary, h.data(), kCanaryWords * 8, hipMemcpyHostToDevice), "hipMemcpy canary"));
    return hip_check(hipIpcGetMemHandle(&me.canary, canary), "hipIpcGetMemHandle canary");
  }
  int check_canaries() {
    std::vector<uint64_t> h(kCanaryRead);
    for (int p = 0; p < world; ++p) {
      if (p == rank) continue;
      void* mp = nullptr;
      TRY(hip_check(hipIpcOpenMemHandle(&mp, b->rank[p].canary, hipIpcMemLazyEnablePeerAccess),
                    "hipIpcOpenMemHandle canary"));
      canary_maps.push_back(mp);
      const hipError_t e = hipMemcpy(h.data(), mp, kCanaryRead * 8, hipMemcpyDeviceToHost);
      TRY(hip_check(e, "hipMemcpy canary"));
      bool whole = true;  // every word read back where it was written: the handle opens at the exporter's address
      for (size_t i = 0; i < kCanaryRead && whole; ++i) whole = h[i] == canary_word(p, i);
      if (whole) continue;
      long long off = 0;
      bool found = false;
      const uint64_t j = h[0] & 0xFFFFFFFFu;
      if ((h[0] >> 32) == (canary_word(p, 0) >> 32) && j < kCanaryWords && h[1] == canary_word(p, j + 1)) {
        off = static_cast<long long>(j) * 8;  // opened past the start: this much after it
        found = true;
      } else {
        for (size_t i = 1; i + 1 < kCanaryRead && !found; ++i)
          if (h[i] == canary_word(p, 0) && h[i + 1] == canary_word(p, 1)) {
            off = -static_cast<long long>(i * 8);  // opened before the start
            found = true;
          }
      }
      if (found)
        return derr(OMR_EINVAL, "ipc transport: rank %d's IPC memory handles open %+lld bytes off its buffers in rank "
                    "%d: the two processes' HIP runtimes lay out device allocations differently (a process that loads "
                    "the AddressSanitizer runtime gets a 4 KiB leading redzone per allocation); they cannot share device "
                    "buffers", p, off, rank);
      return derr(OMR_EINVAL, "ipc transport: rank %d's canary buffer reads back wrong in rank %d (word 0 = %016llx)", p,
                  rank, static_cast<unsigned long long>(h[0]));
    }
    return 0;
  }

  // create this rank's events of generation g of channel c and post their handles (slot g % 2; the events it
  // replaces, generation g - 2, are retired)
  int publish(int c, uint64_t g) {
    IpcEvents& e = mine[c][g % 2];
    release(e, retired);
    IpcRank& me = b->rank[rank];
    for (int k = 0; k < kIpcRing; ++k) {
      TRY(hip_check(hipEventCreateWithFlags(&e.ready[k], hipEventDisableTiming | hipEventInterprocess),
                    "hipEventCreate"));
      TRY(hip_check(hipEventCreateWithFlags(&e.rdone[k], hipEventDisableTiming | hipEventInterprocess),
                    "hipEventCreate"));
      TRY(hip_check(hipIpcGetEventHandle(&me.ready[c][g % 2][k], e.ready[k]), "hipIpcGetEventHandle"));
      TRY(hip_check(hipIpcGetEventHandle(&me.rdone[c][g % 2][k], e.rdone[k]), "hipIpcGetEventHandle"));
    }
    me.evgen[c][g % 2].store(g + 1, std::memory_order_release);
    return 0;
  }
  // open every peer's events of generation g of channel c, on entering g.  A peer posts them when it enters g - 1
  // (this rank cannot be in g before every peer has passed g - 1's first operation), and overwrites them when it
  // enters g + 1 (it cannot before this rank has posted g's last operation, i.e. after this call)
  int open_gen(int c, uint64_t g) {
    for (int p = 0; p < world; ++p) {
      if (p == rank) continue;
      const IpcRank& pr = b->rank[p];
      TRY(spin([&] { return pr.evgen[c][g % 2].load(std::memory_order_acquire) == g + 1; }, "a peer's events"));
      IpcEvents& e = peer[p][c * 2 + g % 2];
      release(e, retired);
      for (int k = 0; k < kIpcRing; ++k) {
        TRY(hip_check(hipIpcOpenEventHandle(&e.ready[k], pr.ready[c][g % 2][k]), "hipIpcOpenEventHandle"));
        TRY(hip_check(hipIpcOpenEventHandle(&e.rdone[k], pr.rdone[c][g % 2][k]), "hipIpcOpenEventHandle"));
      }
    }
    if (retired.size() >= kIpcReap) {  // this rank's streams may still hold records of, or waits on, them
      if (!reaper.joinable()) {
        int dev = 0;
        TRY(hip_check(hipGetDevice(&dev), "hipGetDevice"));
        reap = std::make_shared<Reap>();
        reaper = std::thread(&IpcDist::reap_main, reap, dev);
      }
      {
        std::lock_guard<std::mutex> g(reap->mu);
        reap->q.push_back(std::move(retired));
      }
      retired.clear();
      reap->cv.notify_all();
    }
    return 0;
  }
  static uint64_t gen_of(uint64_t s) { return (s - 1) / kIpcGenOps; }
  const IpcEvents& mine_of(int c, uint64_t s) const { return mine[c][gen_of(s) % 2]; }
  const IpcEvents& peer_of(int c, uint64_t s, int p) const { return peer[p][c * 2 + gen_of(s) % 2]; }

  // the IPC handle of the allocation holding `ptr`, its id, and ptr's offset in it
  int handle_of(const void* ptr, hipIpcMemHandle_t* h, uint64_t* id, uint64_t* off) {
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    TRY(hip_check(hipMemGetAddressRange(&base, &size, const_cast<void*>(ptr)), "hipMemGetAddressRange"));
    const auto key = std::make_pair(reinterpret_cast<uintptr_t>(base), size);
    auto it = own.find(key);
    if (it == own.end()) {
      OwnHandle oh;
      const hipError_t e = hipIpcGetMemHandle(&oh.h, base);
      if (e != hipSuccess)
        return derr(static_cast<int>(e), "hipIpcGetMemHandle: %s (pointer %p in allocation %p of %zu bytes)",
                    hipGetErrorString(e), ptr, reinterpret_cast<void*>(base), size);
      oh.id = next_id++;
      it = own.emplace(key, oh).first;
      if (trace.on()) {
        const uint64_t* hw = reinterpret_cast<const uint64_t*>(&oh.h);
        trace.note("export id %llu: ptr %p base %p size %zu handle %s",
                   static_cast<unsigned long long>(oh.id), ptr, reinterpret_cast<void*>(base), size, hex64(hw).c_str());
      }
    }
    *h = it->second.h;
    *id = it->second.id;
    *off = static_cast<uint64_t>(static_cast<const char*>(ptr) - static_cast<const char*>(base));
    return 0;
  }

  // Plans' allocations.  An exported one is parked, not freed, when its plan goes: on ROCm 7 a freed allocation that
  // a peer still maps can come back from hipMalloc at the same address, and hipIpcGetMemHandle then refuses it
  // ("invalid argument"; seen when a plan was destroyed and re-created on the transport).  A parked allocation keeps
  // its handle and id, so the peers' mappings of it stay right when the next plan reuses it.
  // A parked allocation of at least the requested size (and at most twice it) is reused, so re-planning at another
  // size (another bucket size, a regrown message log) reuses what it can instead of only adding device memory.  The
  // pool still holds every exported allocation until the transport is destroyed (omr_dist.h).
  int alloc(void** ptr, size_t bytes) override {
    auto it = parked.lower_bound(bytes);
    size_t have = bytes;
    if (it != parked.end() && it->first <= 2 * bytes) {
      *ptr = it->second;
      have = it->first;
      parked.erase(it);
    } else {
      TRY(hip_check(hipMalloc(ptr, bytes), "hipMalloc"));
    }
    sized[*ptr] = have;
    return 0;
  }
  void release(void* ptr) override {
    if (ptr == nullptr) return;
    auto s = sized.find(ptr);
    const auto o = own.lower_bound(std::make_pair(reinterpret_cast<uintptr_t>(ptr), size_t{0}));
    const bool exported = o != own.end() && o->first.first == reinterpret_cast<uintptr_t>(ptr);
    if (s != sized.end() && exported) {
      parked.emplace(s->second, ptr);
    } else {
      if (exported) own.erase(o);
      (void)hipFree(ptr);
    }
    if (s != sized.end()) sized.erase(s);
  }

  // peer p's piece: its allocation mapped once per id (a new id for the same handle bytes replaces the old mapping,
  // whose allocation the peer has freed)
  int map(int p, const IpcPost& post, const IpcEntry& e, char** out) {
    if (e.hidx >= post.nh) return derr(OMR_EINVAL, "ipc transport: bad handle index");
    const hipIpcMemHandle_t& h = post.h[e.hidx];
    const uint64_t id = post.hid[e.hidx];
    const auto key = std::make_pair(p, std::string(reinterpret_cast<const char*>(&h), sizeof(h)));
    auto it = opened.find(key);
    if (it != opened.end() && it->second.id != id) {
      // the stale mapping's last reads were queued behind this rank's earlier operations: let them finish first
      TRY(hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize"));
      (void)hipIpcCloseMemHandle(it->second.base);
      opened.erase(it);
      it = opened.end();
    }
    if (it == opened.end()) {
      void* mp = nullptr;
      TRY(hip_check(hipIpcOpenMemHandle(&mp, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle"));
      it = opened.emplace(key, Mapping{id, static_cast<char*>(mp)}).first;
      if (trace.on()) {
        hipDeviceptr_t mb = nullptr;
        size_t ms = 0;
        const hipError_t e = hipMemGetAddressRange(&mb, &ms, mp);
        const uint64_t* hw = reinterpret_cast<const uint64_t*>(&h);
        trace.note("map peer %d id %llu: at %p (range %p size %zu, %s) handle %s", p,
                   static_cast<unsigned long long>(id), mp, reinterpret_cast<void*>(mb), ms, hipGetErrorString(e),
                   hex64(hw).c_str());
      }
    }
    *out = it->second.base + e.off;
    return 0;
  }

  // post the pieces this rank offers for operation `s` of channel c, behind everything queued on st; then wait for
  // every peer to post the same operation
  int begin(int c, hipStream_t st, const std::vector<std::pair<uint32_t, Slice>>& items, uint64_t* s_out) {
    const uint64_t s = ++seq[c];
    const int k = static_cast<int>(s % kIpcRing);
    if (s > 1 && (s - 1) % kIpcGenOps == 0) {  // entering generation g: post g + 1, open the peers' g
      TRY(publish(c, gen_of(s) + 1));
      TRY(open_gen(c, gen_of(s)));
    }
    IpcPost& P = b->post[c][k][rank];
    P.nent = P.nh = 0;
    for (const auto& it : items) {
      if (it.second.bytes == 0) continue;
      if (P.nent == kIpcMaxEntries) return derr(OMR_EINVAL, "ipc transport: more than %d pieces", kIpcMaxEntries);
      hipIpcMemHandle_t h;
      uint64_t hid = 0, off = 0;
      TRY(handle_of(it.second.ptr, &h, &hid, &off));
      uint32_t hi = 0;
      while (hi < P.nh && P.hid[hi] != hid) ++hi;
      if (hi == P.nh) {
        if (P.nh == kIpcMaxHandles) return derr(OMR_EINVAL, "ipc transport: more than %d buffers", kIpcMaxHandles);
        P.h[P.nh] = h;
        P.hid[P.nh++] = hid;
      }
      P.e[P.nent++] = IpcEntry{it.first, hi, off, it.second.bytes};
    }
    if (trace.on()) trace.stamp(st, static_cast<uint32_t>(c), s, -1, 0);
    TRY(hip_check(hipEventRecord(mine_of(c, s).ready[k], st), "hipEventRecord"));
    b->rank[rank].posted[c].store(s, std::memory_order_release);
    for (int p = 0; p < world; ++p)
      TRY(spin([&] { return b->rank[p].posted[c].load(std::memory_order_acquire) >= s; }, "a peer's post"));
    *s_out = s;
    return 0;
  }
  // st waits until peer p's offered pieces are ready on the device
  int wait_ready(int c, uint64_t s, int p, hipStream_t st) {
    const hipEvent_t ev = peer_of(c, s, p).ready[s % kIpcRing];
    const int q = trace.on() ? static_cast<int>(hipEventQuery(ev)) : 0;
    TRY(hip_check(hipStreamWaitEvent(st, ev, 0), "hipStreamWaitEvent"));
    if (trace.on()) trace.stamp(st, static_cast<uint32_t>(c), s, p, q);
    return 0;
  }
  // this rank is through reading its peers; st then waits until every peer is through reading this rank
  int end(int c, uint64_t s, hipStream_t st) {
    const int k = static_cast<int>(s % kIpcRing);
    if (trace.on()) trace.stamp(st, static_cast<uint32_t>(c), s, -2, 0);
    TRY(hip_check(hipEventRecord(mine_of(c, s).rdone[k], st), "hipEventRecord"));
    b->rank[rank].done[c].store(s, std::memory_order_release);
    for (int p = 0; p < world; ++p) {
      if (p == rank) continue;
      TRY(spin([&] { return b->rank[p].done[c].load(std::memory_order_acquire) >= s; }, "a peer's copies"));
      const hipEvent_t ev = peer_of(c, s, p).rdone[k];
      const int q = trace.on() ? static_cast<int>(hipEventQuery(ev)) : 0;
      TRY(hip_check(hipStreamWaitEvent(st, ev, 0), "hipStreamWaitEvent"));
      if (trace.on()) trace.stamp(st, static_cast<uint32_t>(c), s, 100 + p, q);
    }
    return 0;
  }
  const IpcPost& post_of(int c, uint64_t s, int p) const { return b->post[c][s % kIpcRing][p]; }

  int do_allgather(const void* in, void* out, size_t bytes, hipStream_t st) override {
    uint64_t s = 0;
    // (trace: the sender's checksum of what it offers, peer -3, before its ready record)
    if (trace.on()) trace.stamp(st, 0, seq[0] + 1, -3, 0, in, bytes / 8);
    TRY(begin(0, st, {{kIpcAll, Slice{const_cast<void*>(in), bytes}}}, &s));
    int rc = 0;
    for (int p = 0; p < world && rc == 0; ++p) {
      char* dst = static_cast<char*>(out) + static_cast<size_t>(p) * bytes;
      if (p == rank) {
        if (dst != in) rc = hip_check(hipMemcpyAsync(dst, in, bytes, hipMemcpyDeviceToDevice, st), "hipMemcpyAsync");
        continue;
      }
      const IpcPost& P = post_of(0, s, p);
      char* src = nullptr;
      if (bytes == 0) continue;
      if (P.nent != 1 || P.e[0].bytes != bytes) {
        rc = derr(OMR_EINVAL, "ipc allgather: rank %d offered %u pieces", p, P.nent);
        break;
      }
      rc = map(p, P, P.e[0], &src);
      if (rc == 0) rc = wait_ready(0, s, p, st);
      if (rc == 0) rc = hip_check(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st), "hipMemcpyAsync");
      if (rc == 0 && trace.on()) trace.stamp(st, 0, s, 200 + p, 0, dst, bytes / 8);  // checksum of the copy
    }
    // (on an error this rank aborts instead of ending the operation: the peers' waits for it end at once)
    TRY(rc);
    return end(0, s, st);
  }

  int do_exchange(const std::vector<Slices>& sends, const std::vector<Slices>& recvs, hipStream_t st) override {
    std::vector<std::pair<uint32_t, Slice>> items;
    for (int p = 0; p < world; ++p)
      if (p != rank)
        for (const Slice& t : sends[p]) items.push_back({static_cast<uint32_t>(p), t});
    uint64_t s = 0;
    TRY(begin(1, st, items, &s));
    int rc = 0;
    int64_t pieces = 0;
    for (int p = 0; p < world && rc == 0; ++p) {
      if (p == rank) continue;
      const IpcPost& P = post_of(1, s, p);
      uint32_t k = 0;
      bool waited = false;
      for (const Slice& r : recvs[p]) {
        if (r.bytes == 0) continue;
        if ((rc = fault(pieces++)) != 0) break;
        while (k < P.nent && P.e[k].peer != static_cast<uint32_t>(rank)) ++k;
        if (k == P.nent || P.e[k].bytes != r.bytes) {
          rc = derr(OMR_EINVAL, "ipc exchange: rank %d expects %zu bytes from %d, peer offered %llu", rank, r.bytes,
                    p, k < P.nent ? static_cast<unsigned long long>(P.e[k].bytes) : 0ull);
          break;
        }
        char* src = nullptr;
        rc = map(p, P, P.e[k], &src);
        if (rc == 0 && !waited) {
          rc = wait_ready(1, s, p, st);
          waited = true;
        }
        if (rc == 0) rc = hip_check(hipMemcpyAsync(r.ptr, src, r.bytes, hipMemcpyDeviceToDevice, st), "hipMemcpyAsync");
        if (rc) break;
        ++k;
      }
    }
    if (rc == 0) rc = fault(pieces);
    TRY(rc);  // (aborted by the caller: see allgather)
    return end(1, s, st);
  }

  int do_reduce_scatter(const float* in, float* out, size_t count, hipStream_t st) override {
    uint64_t s = 0;
    TRY(begin(1, st, {{kIpcAll, Slice{const_cast<float*>(in), count * world * sizeof(float)}}}, &s));
    std::vector<const float*> ptrs(world);
    int rc = 0;
    for (int p = 0; p < world && rc == 0; ++p) {
      if (p == rank) {
        ptrs[p] = in + static_cast<size_t>(rank) * count;
        continue;
      }
      const IpcPost& P = post_of(1, s, p);
      char* src = nullptr;
      if (P.nent != 1) {
        rc = derr(OMR_EINVAL, "ipc reduce_scatter: rank %d offered %u pieces", p, P.nent);
        break;
      }
      rc = map(p, P, P.e[0], &src);
      if (rc == 0) rc = wait_ready(1, s, p, st);
      ptrs[p] = reinterpret_cast<const float*>(src) + static_cast<size_t>(rank) * count;
    }
    // the shard of every rank's input summed in rank order (the loopback stand-in's order, server.cc:97-98)
    if (rc == 0)
      rc = omr_check(omr_dense_sum_f32(ptrs.data(), static_cast<uint32_t>(world), count, out,
                                       reinterpret_cast<omr_stream_t>(st)), "omr_dense_sum_f32");
    TRY(rc);
    return end(1, s, st);
  }
};

// Spin until every one of the plan kernel's `n` counts in pinned memory carries the round's sequence number (each is
// one 64-bit store, (seq << 32) | count): the host learns the block counts about a microsecond after the kernel stores
// them, without an event, a stream sync or a completion notice.  Bails out if the stream drains with a count still
// stale (a failed launch), on the transport's group-wide failure signals (RCCL's asynchronous errors, a peer's abort)
// and after the transport's deadline (a stuck or dead peer: the mask all-gather before the plan never completes); the
// transport is then aborted, so no peer waits on this rank.  out[i] = the counts.
int wait_counts(omr_dist* d, const uint64_t* counts, uint32_t n, uint32_t seq, hipStream_t st, uint32_t* out) {
  const auto t0 = std::chrono::steady_clock::now();
  uint32_t i = 0;
  for (uint64_t spin = 1;; ++spin) {
    for (; i < n; ++i) {
      const uint64_t v = __atomic_load_n(counts + i, __ATOMIC_ACQUIRE);
      if (static_cast<uint32_t>(v >> 32) != seq) break;
      out[i] = static_cast<uint32_t>(v);
    }
    if (i == n) return 0;
    if ((spin & 4095) == 0) {
      const hipError_t q = hipStreamQuery(st);
      if (q != hipSuccess && q != hipErrorNotReady) return d->contain(hip_check(q, "round plan"));
      if (q == hipSuccess && static_cast<uint32_t>(__atomic_load_n(counts + i, __ATOMIC_ACQUIRE) >> 32) != seq)
        return d->contain(derr(OMR_EINVAL, "round plan: stream idle but count %u stale (seq %u)", i, seq));
      TRY(d->poll());
      if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(d->timeout_ms))
        return d->contain(derr(OMR_ETIMEDOUT, "round plan: rank %d had no counts after %lld ms (seq %u): "
                                              "a peer is stuck or gone", d->rank,
                               static_cast<long long>(d->timeout_ms), seq));
    }
    __builtin_ia32_pause();
  }
}

// Wait on the host until `ev` has completed, within the transport's deadline and watching its failure signals (the
// host-side counterpart of a device sync for a rank whose work may wait on its peers); aborts the transport on expiry.
int wait_event_bounded(omr_dist* d, hipEvent_t ev, const char* what) {
  const auto t0 = std::chrono::steady_clock::now();
  for (uint64_t spin = 1;; ++spin) {
    const hipError_t q = hipEventQuery(ev);
    if (q == hipSuccess) return 0;
    if (q != hipErrorNotReady) return d->contain(hip_check(q, what));
    if ((spin & 63) == 0) {
      TRY(d->poll());
      if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(d->timeout_ms))
        return d->contain(derr(OMR_ETIMEDOUT, "%s: rank %d's rounds did not complete within %lld ms: a peer is stuck or "
                                              "gone", what, d->rank, static_cast<long long>(d->timeout_ms)));
    }
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

// OMR_HOST_TRACE=1 (diagnostic): host time of a round's steps, summed per step and printed to stderr when the plan
// is destroyed.  The round is host-bound when a call takes longer than the worker scan it queues.
// OMR_HOST_TRACE=2 also logs every lap's end (CLOCK_MONOTONIC ns, the clock of rocprofv3's kernel trace) to
// $OMR_HOST_TRACE_FILE (default /tmp/omr_host_trace.<rank>.txt), to lay the host calls beside the kernels.
struct HostTrace {
  bool on = false, log = false;
  std::chrono::steady_clock::time_point t;
  std::map<std::string, std::pair<double, uint64_t>> acc;  // label -> (microseconds, laps)
  std::vector<std::pair<const char*, int64_t>> events;
  void start() {
    if (!on) return;
    t = std::chrono::steady_clock::now();
    if (log) events.emplace_back("start", std::chrono::duration_cast<std::chrono::nanoseconds>(t.time_since_epoch()).count());
  }
  void lap(const char* label) {
    if (!on) return;
    const auto n = std::chrono::steady_clock::now();
    auto& a = acc[label];
    a.first += std::chrono::duration<double, std::micro>(n - t).count();
    a.second += 1;
    t = n;
    if (log) events.emplace_back(label, std::chrono::duration_cast<std::chrono::nanoseconds>(n.time_since_epoch()).count());
  }
  void print(int rank) const {
    for (const auto& kv : acc)
      fprintf(stderr, "[omr host trace rank %d] %-14s %9.2f us mean over %llu\n", rank, kv.first.c_str(),
              kv.second.first / static_cast<double>(kv.second.second), static_cast<unsigned long long>(kv.second.second));
    if (!log) return;
    const char* f = getenv("OMR_HOST_TRACE_FILE");
    const std::string path = f ? std::string(f) : "/tmp/omr_host_trace." + std::to_string(rank) + ".txt";
    if (FILE* fp = fopen(path.c_str(), "w")) {
      for (const auto& e : events) fprintf(fp, "%lld %s\n", static_cast<long long>(e.second), e.first);
      fclose(fp);
    }
  }
};

// a plan's device buffer, through its transport (omr_dist::alloc); *total (if given) counts its bytes
template <typename T>
int dev_alloc(omr_dist* d, T** p, size_t count, uint64_t* total = nullptr) {
  const size_t bytes = std::max<size_t>(count, 1) * sizeof(T);
  TRY(d->alloc(reinterpret_cast<void**>(p), bytes));
  if (total) *total += bytes;
  return 0;
}

}  // namespace

struct omr_ar_plan {
  omr_dist* d = nullptr;
  uint64_t n = 0, nb = 0, rows = 0;
  uint32_t B = 0, lanes = 0, parts = 0, rpp = 0;
  int N = 1, me = 0;
  // roles: ranks [0, M) are workers; A aggregator shards.  Co-located (M == N): rank r is worker r AND the
  // aggregator of shard r.  Dedicated (M < N): ranks M..N-1 aggregate shards 0..A-1 (A = N - M) and hold no tensor,
  // the reference's separate ./server processes (README.md:13-22)
  int M = 1, A = 1;
  bool colocated = true;
  int shard = 0;                  // this rank's shard, -1 for a worker that aggregates none
  int agg_rank(int s) const { return colocated ? s : M + s; }
  bool worker() const { return me < M; }
  std::vector<uint64_t> bounds;   // shard s = rows [bounds[s], bounds[s+1])
  uint64_t shard_nb = 0;          // blocks of the largest shard
  // Fused pack (omr_worker_scan_pack_f32): the worker scan writes its blocks of the other shards into their send
  // streams itself (no pack pass).  Needs every shard to be whole column segments of the scan (world 2, 4, 8 of a
  // power-of-two layout); otherwise (ragged shards) the round packs with omr_move_blocks_f32.
  // Each rank's all-gathered array is then its masks followed by its position table: mstride words per rank.
  bool fused_pack = false;
  bool sum_list = false;            // the shard sum's pairs built by the plan launch (fused pack, N > 1, an aggregator;
                                    // the default since round 4)
  uint64_t list_units = 0;
  uint32_t list_cap = 0;
  uint64_t mstride = 0;           // uint64 words per rank in masks_all: masks [, position table], check slots
  // The round check (round 6): each worker's scan leaves one slot per workgroup, (seq << 32) | its non-zero blocks, after
  // its masks (and position table) in the array the round all-gathers; the plan launch checks every worker's
  // (omr_round_plan_check) and stores a status word after the counts, which the host reads with them.
  uint64_t chk_off = 0;           // the slots' word offset in a rank's array
  uint32_t chk_slots = 0;
  // per-round state, kSets sets used in turn: an asynchronous round's bookkeeping and exchange still read their
  // set while the next rounds' scans fill the others.  Four: one more round between a set's plan and the scan that
  // refills it (with three the world-1 round took 58.1-64.1 us, with four 56.9-57.3; profiles/r04/round_sets/).
  static constexpr int kSets = 4;
  static constexpr int nsets = kSets;
  struct Set {
    uint64_t* own = nullptr;        // [mstride] this rank's masks (the scan ORs into them; the plan kernel re-zeroes
                                    // them), then (fused pack) its position table
    uint64_t* masks_all = nullptr;  // [N][mstride] every rank's `own` (all-gather)
    uint32_t* pack_cnt = nullptr;   // fused pack: [A] the scan's per-shard stream counters (the plan re-zeroes them)
    uint64_t* wset = nullptr;       // [rows] write set: union + lane heads
    uint32_t* prefix = nullptr;     // [N+1][rows+1] popcount prefixes: workers, then the write set
    uint64_t* plan_ws = nullptr;    // the plan kernel's workspace (its row chunks' totals; zeroed once, self-resetting)
    uint64_t* list_rec = nullptr;   // sum list: the shard sum's pair records, built by the plan launch
    uint32_t* list_cnt = nullptr;   //   and their count per unit
    hipEvent_t scanned = nullptr;   // async: recorded on the caller's stream after the worker scan
    hipEvent_t ready = nullptr;     // recorded once the set is filled (the side stream for async rounds)
    hipEvent_t done = nullptr;      // recorded on the side stream once the round is through with it
    bool pending = false;           // `done` recorded and not yet waited for by a refill
    bool plan_pending = false;      // `ready` recorded (the plan has consumed and re-zeroed `own`) and not yet waited
                                    // for by a scan
  } set[kSets];
  // Send buffers (a worker's other-shard blocks for the exchange; an all-reduce's returned sums land in the same
  // buffer afterwards), kPackBufs used in turn by the rounds: round k's is read by its exchange, issued kDeferDepth calls
  // later, so round k + kPackBufs's scan (the fused pack writes it) waits for that round's `done` (round 5: three
  // instead of one per set, so a 256 MiB plan at world 8 holds 3.6x the tensor instead of 9x).
  static constexpr int kPackBufs = 3;
  struct PackBuf {
    float* buf = nullptr;   // n floats less this rank's own shard (pack_send_floats)
    int done_set = -1;      // the set whose `done` frees it, once its round's second half is issued
    bool scan_wait = false; // fused pack: that `done` not yet waited for by the scan that refills it (guarded by mu)
  } pk[kPackBufs];
  uint64_t pack_floats = 0;
  uint64_t rounds_total = 0;        // rounds issued so far (round k uses pk[k % kPackBufs])
  float* recv = nullptr;            // this shard's blocks from each peer (recv_slot): one buffer, every round's exchange
                                    // and shard sum run in order on the side stream
  int cur = 0;                      // the set the next round fills
  int last_async = -1;              // set of the last asynchronous round (for join)
  // Asynchronous rounds run their steps after the worker scan on side streams: the plan stream (all-gather, plan) and,
  // at N > 1, the exchange stream (exchange, shard sums [, return trip]); a deferred call issues round k-2's exchange
  // before round k's plan.  At world 1 both are one stream (cs == ps).  The caller's stream runs only the scans.
  hipStream_t ps = nullptr;         // the plan stream
  hipStream_t cs = nullptr;         // the exchange stream in use: xstream, or ps (world 1, omr_ar_plan_set_side_streams)
  hipStream_t xstream = nullptr;    // the dedicated exchange stream (N > 1, or made by omr_ar_plan_set_side_streams)
  hipEvent_t switch_ev = nullptr;   // orders the exchange stream's work across a switch of it
  hipStream_t tail = nullptr;       // the stream of the last asynchronous round's last work (the bucket write-back)
  uint64_t* bounds_dev = nullptr;
  uint64_t* counts_host = nullptr;  // [kSets][M+1][A+1] per set: (seq << 32) | prefix[a][bounds[s]], pinned memory the
                                    // plan kernel writes
  uint64_t* counts_map = nullptr;   // its device-side address
  float* results = nullptr;  // an aggregator's own shard sums, write-set order (all-reduce, dedicated aggregators)
  uint64_t last_sums_blocks = 0;  // a dedicated aggregator: blocks of its last round's shard sums in `results`
  int32_t* flags_ws = nullptr;
  uint32_t* next_ws = nullptr;
  void* scan_ws = nullptr;   // omr_worker_scan_f32 segment workspace (zeroed once, self-resetting)
  size_t scan_ws_bytes = 0;
  uint32_t seq = 0;
  // The one-rank round (world 1, one worker = its own aggregator; omr_worker_scan_tally_f32): the bookkeeping is two
  // counts, tallied by the scan's workgroups and published by the NEXT round's scan (one extra workgroup), so a
  // pipelined world-1 round is one launch on the caller's stream.
  uint64_t* tally = nullptr;        // device [kSets][tally_slots]: a slot per scan workgroup
  uint32_t tally_slots = 0;
  uint32_t* pub_host = nullptr;     // pinned [kSets][4]: {seq, non-zero blocks, write-set blocks, seq}
  uint32_t* pub_map = nullptr;
  int pub_set = -1;                 // the set whose tally no launch has published yet
  uint32_t pub_seq = 0;
  hipStream_t pub_st = nullptr;     // the stream its scan went on
  uint64_t dev_bytes = 0;           // device memory of the plan (omr_ar_plan_device_bytes)
  // OMR_ROUND_TIME_EXCHANGE: events around the last timed round's worker -> aggregator exchange, and its bytes
  hipEvent_t xt0 = nullptr, xt1 = nullptr;  // the last timed exchange's events (owned by its ring record)
  bool xt_recorded = false;
  uint64_t xt_out = 0, xt_in = 0;
  // every OMR_ROUND_TIME_EXCHANGE round also lands in a ring: its worker scan and its exchange, for means over the
  // timed rounds (omr_ar_plan_timings)
  struct Timed {
    // s: worker scan (caller's stream); q: all-gather .. pack (bookkeeping stream); x: exchange, x1 .. a1: shard
    // sums [, sums back, unpack] (communication stream)
    hipEvent_t s0 = nullptr, s1 = nullptr, x0 = nullptr, x1 = nullptr, q0 = nullptr, q1 = nullptr, a1 = nullptr;
    bool scan = false, xchg = false, prep = false, agg = false;
    bool open = false;  // the round's second half has not run yet (deferred): the record is left unread
    uint64_t out = 0, in = 0;
  };
  static constexpr int kTimed = 64;
  std::vector<Timed> timed;
  uint32_t timed_next = 0, timed_first = 0;  // ring [first, next) not yet read
  // OMR_ROUND_DEFER: the rounds whose exchange and aggregation later calls (or join) issue, oldest first.  Call k
  // issues round k - kDeferDepth's: its block counts have been in host memory since about the middle of round k-1's
  // scan, so the host never waits for them, and the caller's stream always has the next scan queued.
  static constexpr int kDeferDepth = 2;  // <= kSets - 1 (a set is refilled kSets calls later), < kPackBufs
  static constexpr int defer_depth = kDeferDepth;
  struct Pending {
    bool active = false;
    int si = 0, mode = 0, pki = 0;
    bool timed = false;
    const float* x = nullptr;
    float* out = nullptr;
    uint32_t seq = 0;
    int tslot = -1;            // its timing record (OMR_ROUND_TIME_EXCHANGE)
    hipStream_t st = nullptr;  // the stream its plan went on (the count wait checks it for a failed launch)
  } pend[kDeferDepth + 1];
  int npend = 0;
  // rounds issued on different streams run in call order: the plan's arrival counter, own-mask buffer and scan
  // workspace are shared by every round
  hipStream_t last_st = nullptr;
  hipEvent_t st_ev = nullptr;
  HostTrace ht;
  // OMR_ROUND_THREAD: a progress thread issues each round's steps after the worker scan, in call order.  The
  // calling thread queues the scan, then a job; it runs at most kSets - 1 rounds ahead of the thread's first halves
  // (a set's `ready` / `scanned` events must have been recorded / waited for before the set is reused).
  struct Job {
    int si = 0, mode = 0, tslot = -1, pki = 0;
    uint32_t seq = 0;  // a one-rank round's sequence number (taken when its scan was issued)
    bool async = false, defer = false, timed = false, flush_first = false;
    bool signal = false;  // the scan signals its completion in scan_done (no `scanned` record)
    const float* x = nullptr;
    float* out = nullptr;
    uint32_t* un = nullptr;
    hipStream_t st = nullptr;
  };
  int device = 0;
  std::thread progress;
  std::mutex mu;
  std::condition_variable cv_job, cv_done;
  std::deque<Job> jobs;
  uint64_t rounds_begun = 0, first_halves = 0;  // rounds whose scan is queued / whose bookkeeping is issued
  uint64_t second_halves = 0;  // rounds whose exchange and aggregation are issued (or abandoned on an error)
  bool busy = false, stop = false;
  int thread_rc = 0;
  std::string thread_err;
  HostTrace ht_thread;
  // omr_sparse_buckets_f32 on a pinned-host gradient: a ring of device staging buckets and two copy streams
  // kStage = kDeferDepth + 2: bucket k+1's H2D goes into the buffer of bucket k-3, whose second half (and
  // write-back) was issued a call earlier than bucket k-2's, so the copy in overlaps the write-back out.  With
  // kDeferDepth + 1 buffers the H2D waited for the second half issued just before it, and the two PCIe directions
  // took turns (tools trace).
  static constexpr int kStage = 4;
  float* stage[kStage] = {};
  hipStream_t s_in = nullptr, s_out = nullptr;
  hipEvent_t ev_in[kStage] = {}, ev_round[kStage] = {}, ev_out[kStage] = {};
  bool out_used[kStage] = {};
  // set by omr_sparse_buckets_f32 for one round: the worker scan reads the gradient from here (the pinned host
  // buffer, over PCIe) and writes its non-zero blocks and lane heads (0.0f + x) into the round's x, the staging
  // buffer the rest of the round reads (a sum of 0.0f + x_w equals a sum of x_w bit for bit)
  const float* scan_from = nullptr;
  bool in_buckets = false;  // omr_sparse_buckets_f32 is issuing the rounds
  // The first error of a round that had started (guarded by mu): the transport was aborted with it, and every later
  // call on the plan fails at once (omr_ar_plan_destroy still releases everything).
  int failed = 0;
  std::string failed_why;
  hipEvent_t wait_done = nullptr;  // omr_ar_plan_wait's event
  hipEvent_t host_done = nullptr;  // omr_sparse_buckets_f32 on a mapped host buffer: its results stored (system scope)
  // omr_ar_plan_host_stats: the calling thread's time blocked on the GPU or on the progress thread inside rounds (the
  // count wait, the set-reuse waits, the drain), so a caller can tell issue time from waiting
  std::atomic<uint64_t> host_wait_ns{0};
  std::atomic<uint64_t> host_waits{0};
  // Side streams on hardware queues of their own (round 6, seat_side_streams): the caller's stream they were last
  // checked against, and the outcome (omr_ar_plan_queue_report)
  bool queue_check = true;
  hipStream_t seated_st = nullptr;
  bool seated = false;
  int q_disjoint = -1, q_probes = 0, q_replaced = 0;
  // the worker scan's completion word (omr_worker_scan_check_f32's `done`): {workgroups out, seq of the last scan
  // that finished}; the side stream waits on it with k_wait_seq where the side streams are checked apart (scan_signal)
  uint32_t* scan_done = nullptr;
  uint32_t* qflags_host = nullptr;  // pinned: {hold running, release, mark}
  uint32_t* qflags_dev = nullptr;
};

namespace {
int32_t me_shard(const omr_ar_plan* p) { return p->shard; }
int flush_pending(omr_ar_plan* p, hipStream_t st, uint64_t* sent_blocks, uint64_t* union_blocks);
int thread_drain(omr_ar_plan* p);
void thread_stop(omr_ar_plan* p);
thread_local bool t_progress = false;  // this thread is a plan's progress thread (OMR_ROUND_THREAD)
HostTrace& ht_of(omr_ar_plan* p) { return t_progress ? p->ht_thread : p->ht; }

// Accumulates the calling thread's blocked time into the plan's host statistics (the progress thread's waits are
// off the caller's path and are not counted).
struct HostWait {
  omr_ar_plan* p;
  std::chrono::steady_clock::time_point t0;
  explicit HostWait(omr_ar_plan* pp);
  ~HostWait();
};

// A round that had started failed: record it (first error wins) and abort the transport, so that no peer waits for
// this rank's part of the round (the reference exits on a failed post, common.cc:450-451).  Returns rc.
int plan_fail(omr_ar_plan* p, int rc) {
  if (rc == 0) return 0;
  const std::string why = g_derr;
  {
    std::lock_guard<std::mutex> g(p->mu);
    if (p->failed == 0) {
      p->failed = rc;
      p->failed_why = why;
    }
  }
  (void)p->d->abort_with(rc, why.c_str());
  snprintf(g_derr, sizeof(g_derr), "%s", why.c_str());  // (the caller's message, whatever abort_with did)
  return rc;
}

HostWait::HostWait(omr_ar_plan* pp) : p(t_progress ? nullptr : pp), t0(std::chrono::steady_clock::now()) {}
HostWait::~HostWait() {
  if (p == nullptr) return;
  const auto dt = std::chrono::steady_clock::now() - t0;
  p->host_wait_ns.fetch_add(static_cast<uint64_t>(std::chrono::duration_cast<std::chrono::nanoseconds>(dt).count()),
                            std::memory_order_relaxed);
  p->host_waits.fetch_add(1, std::memory_order_relaxed);
}

// OMR_EABORTED if an earlier round of the plan failed
int plan_check(omr_ar_plan* p, const char* what) {
  std::lock_guard<std::mutex> g(p->mu);
  if (p->failed == 0) return 0;
  return derr(OMR_EABORTED, "%s: the plan failed in an earlier round (%s)", what, p->failed_why.c_str());
}

// Words of one set's counts in pinned memory: (seq << 32) | count per (array, shard bound), then the round check's status.
size_t count_words(const omr_ar_plan* p) { return static_cast<size_t>(p->M + 1) * (p->A + 1) + 1; }

// The round's block counts (wait_counts) and its round check's status (omr_round_plan_check): a failed check fails the
// round with OMR_ESTALE, naming the worker, before any exchange is sized from the counts.
int wait_round_counts(omr_ar_plan* p, const uint64_t* tagged, uint32_t seq, hipStream_t st, uint32_t* counts) {
  const uint32_t n = static_cast<uint32_t>(count_words(p));
  uint32_t all[(OMR_MAX_WORKERS + 1) * (OMR_MAX_WORKERS + 2) + 1];
  TRY(wait_counts(p->d, tagged, n, seq, st, all));
  memcpy(counts, all, (n - 1) * sizeof(uint32_t));
  const uint32_t status = all[n - 1];
  if (status == 0) return 0;
  const unsigned w = status & 0xFFu;
  if (status & 0x100u)
    return p->d->contain(derr(OMR_ESTALE, "round check (seq %u): worker %u's all-gathered masks carry another round's "
                                          "scan slot: the all-gather read its array before its scan of this round "
                                          "wrote it, or read another buffer (DESIGN.md §5)", seq, w));
  return p->d->contain(derr(OMR_ESTALE, "round check (seq %u): worker %u's all-gathered masks do not hold the blocks its "
                                        "scan of this round counted: the all-gather read them before the scan finished "
                                        "(DESIGN.md §5)", seq, w));
}

// ---------------------------------------------------------------- side streams on hardware queues of their own
//
// HIP maps each stream of a process onto one of the process's hardware queues (GPU_MAX_HW_QUEUES, 4 on the box) when
// the stream is made, and the streams that share a queue run as ONE FIFO: a side-stream step queued between two worker
// scans then holds the next scan until it has run.  Round 5 measured the N > 1 layout at 69.5-75.6 us per round on a
// stream created after the plan against 53.5-54.1 on the null stream, for the same code.  Which streams
// share a queue depends on the order the process made them (tools/queue_probe.hip on the box: the null stream shared
// with the second stream made, the third with the sixth, the fourth with the fifth; profiles/r06/queues/), so the plan
// checks instead of guessing.  A probe: stream a holds its queue with a one-wave kernel that spins on a host-mapped
// flag, stream b stores a mark; if the mark lands while a holds, a and b are on different queues.  The hold ends on its
// own after kHoldTicks (and at the release the host stores once the mark has landed or kMarkWindow has passed).
constexpr uint64_t kHoldTicks = 100ull * 1000 * 100;  // wall clock at 100 MHz: 100 ms at most
constexpr auto kMarkWindow = std::chrono::milliseconds(5);
constexpr int kSeatTries = 6;  // fresh streams tried per side stream before keeping the shared one

__global__ void k_queue_hold(uint32_t* flags, uint64_t max_ticks) {
  if (threadIdx.x != 0) return;
  __hip_atomic_store(&flags[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const uint64_t t0 = wall_clock64();
  while (__hip_atomic_load(&flags[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0u && wall_clock64() - t0 < max_ticks)
    __builtin_amdgcn_s_sleep(8);
}

__global__ void k_queue_mark(uint32_t* flags) {
  if (threadIdx.x == 0) __hip_atomic_store(&flags[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The side stream's wait for a worker scan that signals its completion (omr_worker_scan_check_f32's `done`): one wave
// polls done[1] until it has reached `seq` (as int32: the word only moves forward, and a later scan may already have
// moved it on).  Bounded: after max_ticks of the wall clock it ends anyway and the round goes on, and the round check
// then fails the round on the stale masks (OMR_ESTALE) instead of the GPU hanging on a scan that never runs.
constexpr uint64_t kScanWaitTicks = 2ull * 1000 * 1000 * 100;  // 2 s at 100 MHz
__global__ void k_wait_seq(const uint32_t* done, uint32_t seq, uint64_t max_ticks) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = wall_clock64();
  while (static_cast<int32_t>(__hip_atomic_load(&done[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) - seq) < 0 &&
         wall_clock64() - t0 < max_ticks)
    __builtin_amdgcn_s_sleep(2);
}

// *disjoint = work queued on b runs while a's hardware queue is held (so a and b are on different queues).  Work
// queued on a before the probe finishes first (bounded by the transport's deadline); b should be idle.
int queue_probe(omr_ar_plan* p, hipStream_t a, hipStream_t b, bool* disjoint) {
  uint32_t* const h = p->qflags_host;
  __atomic_store_n(&h[0], 0u, __ATOMIC_RELAXED);
  __atomic_store_n(&h[1], 0u, __ATOMIC_RELAXED);
  __atomic_store_n(&h[2], 0u, __ATOMIC_RELAXED);
  __atomic_thread_fence(__ATOMIC_SEQ_CST);
  k_queue_hold<<<1, 64, 0, a>>>(p->qflags_dev, kHoldTicks);
  TRY(hip_check(hipGetLastError(), "k_queue_hold"));
  const auto t0 = std::chrono::steady_clock::now();
  int rc = 0;
  while (__atomic_load_n(&h[0], __ATOMIC_ACQUIRE) == 0) {
    if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(p->d->timeout_ms)) {
      rc = derr(OMR_ETIMEDOUT, "queue probe: the caller's stream did not reach the probe within %lld ms",
                static_cast<long long>(p->d->timeout_ms));
      break;
    }
    __builtin_ia32_pause();
  }
  bool got = false;
  if (rc == 0) {
    k_queue_mark<<<1, 64, 0, b>>>(p->qflags_dev);
    rc = hip_check(hipGetLastError(), "k_queue_mark");
    const auto t1 = std::chrono::steady_clock::now();
    while (rc == 0 && std::chrono::steady_clock::now() - t1 < kMarkWindow)
      if (__atomic_load_n(&h[2], __ATOMIC_ACQUIRE) != 0) {
        got = true;
        break;
      }
  }
  __atomic_store_n(&h[1], 1u, __ATOMIC_RELEASE);  // the hold ends (it would by itself after kHoldTicks)
  TRY(rc);
  TRY(hip_check(hipStreamSynchronize(b), "hipStreamSynchronize"));
  TRY(hip_check(hipStreamSynchronize(a), "hipStreamSynchronize"));
  ++p->q_probes;
  *disjoint = got;
  return 0;
}

// A fresh stream whose queue differs from avoid1's (and avoid2's, if given), or nullptr when kSeatTries fresh streams all
// shared one (the streams tried are kept until the end, so each one made takes another queue, then destroyed).
int fresh_stream(omr_ar_plan* p, hipStream_t avoid1, hipStream_t avoid2, bool check2, hipStream_t* out) {
  *out = nullptr;
  std::vector<hipStream_t> tried;
  int rc = 0;
  for (int i = 0; i < kSeatTries && rc == 0 && *out == nullptr; ++i) {
    hipStream_t c = nullptr;
    if ((rc = hip_check(hipStreamCreateWithFlags(&c, hipStreamNonBlocking), "hipStreamCreate")) != 0) break;
    bool d1 = false, d2 = true;
    rc = queue_probe(p, avoid1, c, &d1);
    if (rc == 0 && d1 && check2) rc = queue_probe(p, avoid2, c, &d2);
    if (rc == 0 && d1 && d2) *out = c;
    else tried.push_back(c);
  }
  for (hipStream_t s : tried) (void)hipStreamDestroy(s);
  return rc;
}

// Make the plan's side streams run on hardware queues apart from the caller's stream `st` and from each other, before the
// first asynchronous round on `st`: the side streams are drained (every step already issued on them has run; a deferred
// round's second half not issued yet goes on the seated streams later), probed, and each one that shares a queue is
// replaced by a fresh stream that does not (the old one is idle, so nothing needs ordering across the switch).  When no
// fresh stream helps (fewer hardware queues than streams) the shared stream is kept and the report says so.
int seat_side_streams(omr_ar_plan* p, hipStream_t st) {
  p->seated_st = st;
  p->seated = true;
  if (p->switch_ev == nullptr)
    TRY(hip_check(hipEventCreateWithFlags(&p->switch_ev, hipEventDisableTiming | hipEventDisableSystemFence),
                  "hipEventCreate"));
  for (hipStream_t s : {p->ps, p->xstream}) {
    if (s == nullptr) continue;
    TRY(hip_check(hipEventRecord(p->switch_ev, s), "hipEventRecord"));
    TRY(wait_event_bounded(p->d, p->switch_ev, "seat side streams"));
  }
  const bool two = p->cs != p->ps;
  bool ok = true;
  bool d = false;
  TRY(queue_probe(p, st, p->ps, &d));
  if (!d) {
    hipStream_t c = nullptr;
    TRY(fresh_stream(p, st, p->cs, two, &c));
    if (c != nullptr) {
      const hipStream_t old = p->ps;
      p->ps = c;
      if (!two) p->cs = c;
      if (p->tail == old) p->tail = c;
      (void)hipStreamDestroy(old);
      ++p->q_replaced;
    } else {
      ok = false;
    }
  }
  if (two) {
    bool d1 = false, d2 = false;
    TRY(queue_probe(p, st, p->cs, &d1));
    if (d1) TRY(queue_probe(p, p->ps, p->cs, &d2));
    if (!(d1 && d2)) {
      hipStream_t c = nullptr;
      TRY(fresh_stream(p, st, p->ps, true, &c));
      if (c != nullptr) {
        const hipStream_t old = p->xstream;
        p->xstream = p->cs = c;
        if (p->tail == old) p->tail = c;
        (void)hipStreamDestroy(old);
        ++p->q_replaced;
      } else {
        ok = false;
      }
    }
  }
  p->q_disjoint = ok ? 1 : 0;
  return 0;
}
}  // namespace

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
  ncclComm_t c = nullptr, x = nullptr;
  int rc = nccl_check(ncclCommInitRank(&c, world, uid, rank), "ncclCommInitRank");
  d->comm.store(c);
  if (rc == 0) rc = nccl_check(ncclCommSplit(c, 0, rank, &x, nullptr), "ncclCommSplit");
  d->xcomm.store(x);
  if (rc != 0) {
    delete d;
    return rc;
  }
  *out = d;
  return 0;
}

int omr_dist_ipc_unique_id(void* id) {
  if (id == nullptr) return derr(OMR_EINVAL, "ipc unique id: NULL");
  unsigned char* c = static_cast<unsigned char*>(id);
  memset(c, 0, OMR_UNIQUE_ID_BYTES);
  int fd = open("/dev/urandom", O_RDONLY);
  ssize_t got = fd >= 0 ? read(fd, c, 16) : -1;
  if (fd >= 0) close(fd);
  if (got != 16) {  // no urandom: time and pid still make the board name unique on this host
    const uint64_t t = static_cast<uint64_t>(std::chrono::steady_clock::now().time_since_epoch().count());
    const uint32_t pid = static_cast<uint32_t>(getpid());
    memcpy(c, &t, sizeof(t));
    memcpy(c + 8, &pid, sizeof(pid));
  }
  return 0;
}

int omr_dist_create_ipc(const void* id, int rank, int world, omr_dist** out) {
  if (id == nullptr || out == nullptr || world < 1 || world > kIpcMaxRanks || rank < 0 || rank >= world)
    return derr(OMR_EINVAL, "create_ipc: bad arguments (world 1..%d)", kIpcMaxRanks);
  *out = nullptr;
  auto* d = new IpcDist();
  d->rank = rank;
  d->world = world;
  if (int rc = d->attach(id)) {
    const std::string why = g_derr;  // (the teardown's own waits may overwrite the message)
    delete d;
    snprintf(g_derr, sizeof(g_derr), "%s", why.c_str());
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
  g_destroy_rc = 0;
  delete d;
  return g_destroy_rc;
}

int omr_dist_abort(omr_dist* d) {
  if (d == nullptr) return derr(OMR_EINVAL, "dist_abort: NULL");
  (void)d->abort_with(0, "omr_dist_abort");
  return 0;
}

int omr_dist_aborted(const omr_dist* d) { return d != nullptr && d->aborted.load() ? 1 : 0; }

int omr_dist_set_timeout(omr_dist* d, int64_t timeout_ms) {
  if (d == nullptr || timeout_ms <= 0) return derr(OMR_EINVAL, "dist_set_timeout: NULL or a deadline <= 0");
  d->timeout_ms = timeout_ms;
  return 0;
}

int omr_dist_poll(omr_dist* d) {
  if (d == nullptr) return derr(OMR_EINVAL, "dist_poll: NULL");
  return d->poll();
}

int omr_dist_inject_fault(omr_dist* d, int64_t after_pieces) {
  if (d == nullptr) return derr(OMR_EINVAL, "inject_fault: NULL");
  d->fault_after = after_pieces < 0 ? -1 : after_pieces;
  return 0;
}

int omr_dist_test_world1_round(omr_dist* d, int on) {
  if (d == nullptr) return derr(OMR_EINVAL, "test_world1_round: NULL");
  d->world1_general = on != 0;
  return 0;
}

int omr_dist_inject_allgather_fault(omr_dist* d) {
  if (d == nullptr) return derr(OMR_EINVAL, "inject_allgather_fault: NULL");
  d->fault_allgather = true;
  return 0;
}

int omr_dist_allgather(omr_dist* d, const void* in, void* out, size_t bytes, omr_stream_t stream) {
  if (d == nullptr || (bytes > 0 && (in == nullptr || out == nullptr))) return derr(OMR_EINVAL, "allgather: NULL");
  return d->allgather(in, out, bytes, reinterpret_cast<hipStream_t>(stream));
}

int omr_dist_exchange(omr_dist* d, void* const* send, const size_t* send_bytes, void* const* recv,
                      const size_t* recv_bytes, omr_stream_t stream) {
  if (d == nullptr || send == nullptr || send_bytes == nullptr || recv == nullptr || recv_bytes == nullptr)
    return derr(OMR_EINVAL, "exchange: NULL");
  std::vector<Slices> sends(d->world), recvs(d->world);
  for (int p = 0; p < d->world; ++p) {
    if (p == d->rank) continue;
    sends[p] = {Slice{send[p], send_bytes[p]}};
    recvs[p] = {Slice{recv[p], recv_bytes[p]}};
  }
  return d->exchange(sends, recvs, reinterpret_cast<hipStream_t>(stream));
}

int omr_ar_plan_destroy(omr_ar_plan* p) {
  if (p == nullptr) return 0;
  (void)thread_drain(p);
  thread_stop(p);
  if (p->ht.on) p->ht.print(p->me);
  if (p->ht_thread.on && !p->ht_thread.acc.empty()) {
    fprintf(stderr, "[omr host trace rank %d] progress thread:\n", p->me);
    p->ht_thread.print(p->me);
  }
  // deferred rounds still owe their exchanges to the peers: issue them and let them drain (not after a failure: the
  // transport is aborted, and their second halves would only fail)
  if (p->npend > 0 && p->failed == 0 && !p->d->aborted.load()) (void)flush_pending(p, p->cs, nullptr, nullptr);
  p->npend = 0;
  if (p->failed == 0 && !p->d->aborted.load()) {
    (void)hipDeviceSynchronize();
  } else {
    // After a failure the device may hold waits on a peer that will never come (an IPC peer's event, on the plan's
    // streams or the caller's; an aborted RCCL communicator has cancelled its queued operations, the IPC and loopback
    // transports cannot): wait for the device within the deadline only, and if it is still busy leave the plan's
    // device memory allocated rather than free it under queued work (hipFree would wait for the device itself;
    // destroy must not block on a dead peer).
    const bool idle = device_sync_within(p->d->timeout_ms);
    (void)hipGetLastError();
    if (!idle) {
      const int rc = derr(OMR_ETIMEDOUT, "ar_plan_destroy: the plan's streams were still busy %lld ms after its failure; "
                          "its device memory is left allocated", static_cast<long long>(p->d->timeout_ms));
      if (p->ht.on) p->ht.print(p->me);
      delete p;  // (host state only: streams, events and buffers may still be in use on the device)
      return rc;
    }
  }
  // back to the transport, which keeps the exported ones alive for the next plan (omr_dist::alloc)
  void* devs[] = {p->bounds_dev, p->results, p->flags_ws, p->next_ws, p->scan_ws, p->recv, p->tally, p->scan_done};
  for (void* v : devs) p->d->release(v);
  for (auto& b : p->pk) p->d->release(b.buf);
  for (auto& st : p->set) {
    void* sv[] = {st.own, st.masks_all, st.wset, st.prefix, st.plan_ws, st.pack_cnt, st.list_rec, st.list_cnt};
    for (void* v : sv) p->d->release(v);
    for (hipEvent_t e : {st.scanned, st.ready, st.done})
      if (e) (void)hipEventDestroy(e);
  }
  if (p->switch_ev) (void)hipEventDestroy(p->switch_ev);
  if (p->xstream) (void)hipStreamDestroy(p->xstream);
  if (p->ps) (void)hipStreamDestroy(p->ps);
  for (int r = 0; r < omr_ar_plan::kStage; ++r) {
    p->d->release(p->stage[r]);
    for (hipEvent_t e : {p->ev_in[r], p->ev_round[r], p->ev_out[r]})
      if (e) (void)hipEventDestroy(e);
  }
  if (p->s_in) (void)hipStreamDestroy(p->s_in);
  if (p->s_out) (void)hipStreamDestroy(p->s_out);
  if (p->st_ev) (void)hipEventDestroy(p->st_ev);
  if (p->wait_done) (void)hipEventDestroy(p->wait_done);
  if (p->host_done) (void)hipEventDestroy(p->host_done);
  for (auto& t : p->timed)
    for (hipEvent_t e : {t.s0, t.s1, t.x0, t.x1, t.q0, t.q1, t.a1})
      if (e) (void)hipEventDestroy(e);
  (void)hipHostFree(p->counts_host);
  (void)hipHostFree(p->pub_host);
  (void)hipHostFree(p->qflags_host);
  delete p;
  return 0;
}

int omr_ar_plan_create(omr_dist* d, uint64_t n, uint32_t block_size, uint32_t num_lanes, uint32_t num_parts,
                       omr_ar_plan** out) {
  if (d == nullptr) return derr(OMR_EINVAL, "ar_plan_create: NULL");
  return omr_ar_plan_create_roles(d, static_cast<uint32_t>(d->world), n, block_size, num_lanes, num_parts, out);
}

int omr_ar_plan_create_roles(omr_dist* d, uint32_t num_workers, uint64_t n, uint32_t block_size, uint32_t num_lanes,
                             uint32_t num_parts, omr_ar_plan** out) {
  if (d == nullptr || out == nullptr) return derr(OMR_EINVAL, "ar_plan_create: NULL");
  *out = nullptr;
  TRY(omr_check(omr_layout_check(n, block_size, num_lanes, num_parts), "omr_layout_check"));
  if (num_workers == 0 || num_workers > static_cast<uint32_t>(d->world) || num_workers > OMR_MAX_WORKERS)
    return derr(OMR_EINVAL, "ar_plan_create: %u workers in a world of %d (at most %d workers)", num_workers, d->world,
                OMR_MAX_WORKERS);
  const int naggs = num_workers == static_cast<uint32_t>(d->world) ? d->world : d->world - static_cast<int>(num_workers);
  if (naggs > OMR_MAX_WORKERS) return derr(OMR_EINVAL, "ar_plan_create: %d aggregators > %d", naggs, OMR_MAX_WORKERS);
  auto* p = new omr_ar_plan();
  const char* trace = getenv("OMR_HOST_TRACE");
  p->ht.on = trace != nullptr && (trace[0] == '1' || trace[0] == '2');
  p->ht.log = trace != nullptr && trace[0] == '2';
  p->M = static_cast<int>(num_workers);
  p->A = naggs;
  p->colocated = num_workers == static_cast<uint32_t>(d->world);
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
  p->shard = p->colocated ? p->me : (p->me >= p->M ? p->me - p->M : -1);
  const int N = p->N, M = p->M, NA = p->A;
  for (int s = 0; s <= NA; ++s) p->bounds.push_back(static_cast<uint64_t>(s) * p->rows / NA);
  uint64_t max_rows = 0;
  for (int s = 0; s < NA; ++s) max_rows = std::max(max_rows, p->bounds[s + 1] - p->bounds[s]);
  p->shard_nb = max_rows * num_lanes;
  p->mstride = p->rows;
  if (N > 1 && omr_pack_supported(n, block_size, num_lanes, num_parts, p->bounds.data(), static_cast<uint32_t>(NA)) == 0) {
    uint64_t entries = 0;
    TRY(omr_check(omr_pack_geometry(n, block_size, num_lanes, num_parts, nullptr, nullptr, &entries),
                  "omr_pack_geometry"));
    p->fused_pack = true;
    p->mstride = p->rows + (entries + 1) / 2;
    // The plan launch builds the shard sum's pairs (16-row units) and omr_shard_sum_list_f32 sums them with its first
    // load: 9.32 us at config 4's 8-worker shard against 11.83 for round 3's form that built its pairs itself (round 4,
    // profiles/r04/round_kernels/tune_round_list16.log; that form is tools/tune/plan_r04.hip's k_shard_sum_r04 now).
    if (p->shard >= 0) {
      TRY(omr_check(omr_sum_list_geometry(n, block_size, num_lanes, num_parts, p->bounds[p->shard],
                                          p->bounds[p->shard + 1], static_cast<uint32_t>(p->M), &p->list_units,
                                          &p->list_cap), "omr_sum_list_geometry"));
      p->sum_list = p->list_units > 0;
    }
  }
  p->chk_off = p->mstride;
  p->chk_slots = omr_round_check_slots(n, block_size, num_lanes, num_parts);
  p->mstride += p->chk_slots;
  int rc = 0;
  auto A = [&](int r) {
    if (rc == 0) rc = r;
  };
  uint64_t* const DB = &p->dev_bytes;
  // the round's events order work between streams of this device only: no system-scope fence (a record costs
  // its stream 1.2 us instead of 2.8, tools/event_cost.hip); what the host reads goes out as system-scope stores
  const unsigned evflags = hipEventDisableTiming | hipEventDisableSystemFence;
  for (int i = 0; i < p->nsets; ++i) {
    omr_ar_plan::Set& st = p->set[i];
    A(dev_alloc(p->d, &st.own, p->mstride, DB));
    A(dev_alloc(p->d, &st.masks_all, static_cast<size_t>(N) * p->mstride, DB));
    if (p->fused_pack) A(dev_alloc(p->d, &st.pack_cnt, NA, DB));
    A(dev_alloc(p->d, &st.wset, p->rows, DB));
    A(dev_alloc(p->d, &st.prefix, static_cast<size_t>(M + 1) * (p->rows + 1), DB));
    A(dev_alloc(p->d, &st.plan_ws, omr_round_plan_workspace_words(), DB));
    if (p->sum_list) {
      A(dev_alloc(p->d, &st.list_rec, p->list_units * p->list_cap, DB));
      A(dev_alloc(p->d, &st.list_cnt, p->list_units, DB));
    }
    for (hipEvent_t* e : {&st.scanned, &st.ready, &st.done})
      A(hip_check(hipEventCreateWithFlags(e, evflags), "hipEventCreate"));
  }
  // The side streams.  Each stream the process makes takes one of its hardware queues (GPU_MAX_HW_QUEUES, 4 on the box)
  // round robin, and streams that share a queue run one after the other: with two side streams the world-1 round ran
  // 2x slower in the stream orders whose side stream shared the caller's queue (profiles/r04/inproc/).  World 1 has
  // no exchange, so it keeps one side stream (and the one-rank round uses none); at N > 1 the exchange gets its own,
  // so round k-2's exchange runs beside round k's all-gather and plan instead of before them: as 4 IPC ranks on one
  // GPU one side stream took 2.18 ms per round (profiles/r05/ipc_cliff/ipc_w4.json) against 1.36-1.43 with two
  // (round 4).  The multi-rank test hook at world 1 (omr_dist_test_world1_round) takes the N > 1 layout.
  A(hip_check(hipStreamCreateWithFlags(&p->ps, hipStreamNonBlocking), "hipStreamCreate"));
  p->cs = p->ps;
  if ((N > 1 && p->d->default_side_streams() == 2) || p->d->world1_general) {
    A(hip_check(hipStreamCreateWithFlags(&p->xstream, hipStreamNonBlocking), "hipStreamCreate"));
    if (rc == 0) p->cs = p->xstream;
  }
  A(hip_check(hipEventCreateWithFlags(&p->st_ev, evflags), "hipEventCreate"));
  A(dev_alloc(p->d, &p->bounds_dev, NA + 1, DB));
  if (N > 1 && p->worker()) {
    // (N - 1) / N of the tensor on a co-located rank: the own shard is never sent, and the sums of the other shards
    // that an all-reduce returns fit the same space
    p->pack_floats = p->colocated ? n - (p->bounds[p->me + 1] - p->bounds[p->me]) * num_lanes * block_size : n;
    for (auto& b : p->pk) A(dev_alloc(p->d, &b.buf, p->pack_floats, DB));
  }
  if (N > 1 && p->shard >= 0)  // every other worker's stream of this shard, worker w's at recv_slot(w)
    A(dev_alloc(p->d, &p->recv, static_cast<size_t>(p->colocated ? M - 1 : M) * p->shard_nb * block_size, DB));
  if (p->shard >= 0) A(dev_alloc(p->d, &p->results, p->shard_nb * block_size, DB));
  A(dev_alloc(p->d, &p->flags_ws, p->nb, DB));
  A(dev_alloc(p->d, &p->next_ws, p->nb, DB));
  A(dev_alloc(p->d, &p->scan_done, 2, DB));
  p->scan_ws_bytes = omr_scan_workspace_bytes(n, block_size, num_lanes, num_parts);
  A(dev_alloc(p->d, reinterpret_cast<char**>(&p->scan_ws), p->scan_ws_bytes, DB));
  p->tally_slots = omr_tally_slots(n, block_size, num_lanes, num_parts);
  A(dev_alloc(p->d, &p->tally, static_cast<size_t>(p->tally_slots) * omr_ar_plan::kSets, DB));
  constexpr int NSETS = omr_ar_plan::kSets;
  const size_t ncounts = static_cast<size_t>(NSETS) * count_words(p);
  A(hip_check(hipHostMalloc(reinterpret_cast<void**>(&p->counts_host), ncounts * sizeof(uint64_t),
                            hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc"));
  if (rc == 0) {
    for (size_t i = 0; i < ncounts; ++i) p->counts_host[i] = 0;  // (tag 0: no round's)
    A(hip_check(hipHostGetDevicePointer(reinterpret_cast<void**>(&p->counts_map), p->counts_host, 0),
                "hipHostGetDevicePointer"));
  }
  A(hip_check(hipHostMalloc(reinterpret_cast<void**>(&p->pub_host), NSETS * 4 * sizeof(uint32_t),
                            hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc"));
  if (rc == 0) {
    memset(p->pub_host, 0, NSETS * 4 * sizeof(uint32_t));
    A(hip_check(hipHostGetDevicePointer(reinterpret_cast<void**>(&p->pub_map), p->pub_host, 0),
                "hipHostGetDevicePointer"));
  }
  p->queue_check = p->d->queue_check_default();
  A(hip_check(hipHostMalloc(reinterpret_cast<void**>(&p->qflags_host), 64, hipHostMallocMapped | hipHostMallocCoherent),
              "hipHostMalloc"));
  if (rc == 0) {
    memset(p->qflags_host, 0, 64);
    A(hip_check(hipHostGetDevicePointer(reinterpret_cast<void**>(&p->qflags_dev), p->qflags_host, 0),
                "hipHostGetDevicePointer"));
  }
  if (rc == 0) {  // the probe's kernels loaded before any probe times them (a first launch loads the code object)
    p->qflags_host[1] = 1;
    k_queue_hold<<<1, 64, 0, p->ps>>>(p->qflags_dev, 0);
    k_queue_mark<<<1, 64, 0, p->ps>>>(p->qflags_dev);
    A(hip_check(hipGetLastError(), "queue probe warm-up"));
  }
  for (int i = 0; i < p->nsets && rc == 0; ++i) {
    omr_ar_plan::Set& st = p->set[i];
    A(hip_check(hipMemset(st.own, 0, p->mstride * sizeof(uint64_t)), "hipMemset own masks"));
    if (rc == 0)
      A(hip_check(hipMemset(st.plan_ws, 0, omr_round_plan_workspace_words() * sizeof(uint64_t)), "hipMemset plan ws"));
    if (rc == 0 && st.pack_cnt) A(hip_check(hipMemset(st.pack_cnt, 0, NA * sizeof(uint32_t)), "hipMemset pack counters"));
  }
  if (rc == 0 && p->scan_ws_bytes) A(hip_check(hipMemset(p->scan_ws, 0, p->scan_ws_bytes), "hipMemset scan ws"));
  if (rc == 0) A(hip_check(hipMemset(p->scan_done, 0, 2 * sizeof(uint32_t)), "hipMemset scan done"));
  if (rc == 0)
    A(hip_check(hipMemcpy(p->bounds_dev, p->bounds.data(), (NA + 1) * sizeof(uint64_t), hipMemcpyHostToDevice),
                "hipMemcpy bounds"));
  if (rc == 0) A(hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize"));
  if (rc != 0) {
    omr_ar_plan_destroy(p);
    return rc;
  }
  *out = p;
  return 0;
}

}  // extern "C"

namespace {

// The second half of a round (steps 4b-7): wait for the plan's counts, exchange, shard sums [, sums back,
// unpack].  `async`: on the communication stream, behind the set's `ready` event.
// a timed round's ring record: the next slot (events created on first use)
int timed_slot(omr_ar_plan* p, int* slot) {
  if (p->timed.empty()) p->timed.resize(omr_ar_plan::kTimed);
  const int k = static_cast<int>(p->timed_next++ % omr_ar_plan::kTimed);
  if (p->timed_next - p->timed_first > omr_ar_plan::kTimed) p->timed_first = p->timed_next - omr_ar_plan::kTimed;
  omr_ar_plan::Timed& t = p->timed[k];
  // timing-only events without the system-scope fence (as bench.py's own): a fenced record on the caller's stream
  // held the world-1 round's next scan back 6 us (profiles/r05/final/w1_trace/), 1.2 us per round at one timed round
  // in ten
  if (t.s0 == nullptr)
    for (hipEvent_t* e : {&t.s0, &t.s1, &t.x0, &t.x1, &t.q0, &t.q1, &t.a1})
      TRY(hip_check(hipEventCreateWithFlags(e, hipEventDisableSystemFence), "hipEventCreate"));
  t.scan = t.xchg = t.prep = t.agg = false;
  t.open = true;
  *slot = k;
  return 0;
}
// the timed round's exchange was bracketed by its record's x0 / x1; note its bytes
int timed_exchange(omr_ar_plan* p, int slot) {
  omr_ar_plan::Timed& t = p->timed[slot];
  t.xchg = true;
  t.out = p->xt_out;
  t.in = p->xt_in;
  p->xt0 = t.x0;  // the last timed exchange (omr_ar_plan_exchange_time)
  p->xt1 = t.x1;
  return 0;
}

// The next round's sequence number: never 0 (the tag of no round: the plan launch refuses it), so a plan that runs
// past 2^32 rounds wraps to 1.  Every rank of a group issues the same rounds, so their numbers agree.
uint32_t next_seq(omr_ar_plan* p) {
  if (++p->seq == 0) ++p->seq;
  return p->seq;
}

// Worker w's stream of this rank's shard lands at a fixed region of `recv`, so the shard sum's pairs can be addressed
// before the exchange (the plan launch builds them: omr_round_plan_list).  A co-located aggregator reads its own blocks
// in place: its slot is left out.
uint64_t recv_slot(const omr_ar_plan* p, int w) {
  return static_cast<uint64_t>(p->colocated && w > p->me ? w - 1 : w) * p->shard_nb;
}

omr_sum_list list_desc(const omr_ar_plan* p, const omr_ar_plan::Set& S) {
  omr_sum_list l{};
  l.records = S.list_rec;
  l.counts = S.list_cnt;
  l.row_begin = p->bounds[p->shard];
  l.row_end = p->bounds[p->shard + 1];
  l.pos_offset = 2 * p->rows;  // each worker's position table follows its masks (omr_worker_scan_pack_f32)
  l.me = p->colocated ? static_cast<uint32_t>(p->me) : static_cast<uint32_t>(p->M);
  for (int w = 0; w < p->M; ++w) l.recv_offsets[w] = recv_slot(p, w);
  return l;
}

// (internal bits in a round's mode, see sparse_round_issue: a one-rank round whose worker scan wrote the sums itself,
// and one whose worker scan also tallied its bookkeeping, the one-launch round)
constexpr int kModeSolo = 0x10000;
constexpr int kModeTally = 0x20000;

int wait_ev(hipStream_t on, hipEvent_t ev);
int order_after(omr_ar_plan* p, hipStream_t on, hipEvent_t ev, const char* what);

// The one-rank round's counts: {seq, non-zero blocks, write-set blocks, seq} from omr_worker_scan_tally_f32's publishing
// workgroup (or omr_tally_publish).  Bounded as wait_flag; `st` is the stream the publication went on.
int wait_pub(omr_dist* d, const uint32_t* rec, uint32_t seq, hipStream_t st, uint32_t* nz, uint32_t* ws) {
  const auto t0 = std::chrono::steady_clock::now();
  for (uint64_t spin = 1;; ++spin) {
    if (__atomic_load_n(&rec[0], __ATOMIC_ACQUIRE) == seq && __atomic_load_n(&rec[3], __ATOMIC_ACQUIRE) == seq) {
      *nz = __atomic_load_n(&rec[1], __ATOMIC_ACQUIRE);
      *ws = __atomic_load_n(&rec[2], __ATOMIC_ACQUIRE);
      return 0;
    }
    if ((spin & 4095) == 0) {
      const hipError_t q = hipStreamQuery(st);
      if (q != hipSuccess && q != hipErrorNotReady) return d->contain(hip_check(q, "one-rank round"));
      if (q == hipSuccess && !(__atomic_load_n(&rec[0], __ATOMIC_ACQUIRE) == seq &&
                               __atomic_load_n(&rec[3], __ATOMIC_ACQUIRE) == seq))
        return d->contain(derr(OMR_EINVAL, "one-rank round: stream idle but no counts (seq %u)", seq));
      TRY(d->poll());
      if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(d->timeout_ms))
        return d->contain(derr(OMR_ETIMEDOUT, "one-rank round: no counts after %lld ms (seq %u)",
                               static_cast<long long>(d->timeout_ms), seq));
    }
    __builtin_ia32_pause();
  }
}

// The oldest round whose tally no launch has published: publish it now, by a launch of its own (no later scan of the
// plan will, or its second half is wanted before the next scan).
int publish_pending(omr_ar_plan* p) {
  if (p->pub_set < 0) return 0;
  const int si = p->pub_set;
  p->pub_set = -1;
  return omr_check(omr_tally_publish(p->tally + static_cast<size_t>(p->tally_slots) * si, p->tally_slots,
                                     p->pub_map + 4 * si, p->pub_seq, reinterpret_cast<omr_stream_t>(p->pub_st)),
                   "omr_tally_publish");
}

// The second half of a round (steps 4b-7): wait for the plan's counts, exchange, shard sums [, sums back, unpack].
// `async`: on the side stream, behind the round's first half (issued on it earlier: no event needed).
int round_finish(omr_ar_plan* p, int si, int pki, const float* x, float* out, int mode, bool async, bool timed,
                 uint32_t seq, hipStream_t st, uint64_t* sent_blocks, uint64_t* union_blocks, int tslot) {
  const bool solo = (mode & kModeSolo) != 0, tally = (mode & kModeTally) != 0;
  mode &= ~(kModeSolo | kModeTally);
  struct CloseRecord {  // the timing record is complete (or abandoned) once this second half returns
    omr_ar_plan* p;
    int slot;
    ~CloseRecord() {
      if (slot >= 0) p->timed[slot].open = false;
    }
  } close_record{p, timed ? tslot : -1};
  struct CountHalf {  // (a fused-pack scan that refills this round's send buffer waits until this second half is issued)
    omr_ar_plan* p;
    ~CountHalf() {
      {
        std::lock_guard<std::mutex> g(p->mu);
        ++p->second_halves;
      }
      p->cv_done.notify_all();
    }
  } count_half{p};
  omr_ar_plan::Set& S = p->set[si];
  const int N = p->N, M = p->M, NA = p->A, me = p->me, sh = p->shard;
  const uint64_t rows = p->rows, B = p->B;
  ht_of(p).start();
  if (tally) {
    // the one-launch round: its worker scan wrote the sums and tallied the counts; they reach the host through the next
    // round's scan or, if none has been issued, a publication of their own.  A caller that wants neither count waits
    // for nothing: the launch is the whole round (its counts stay with the next scan, which publishes them anyway).
    if (sent_blocks == nullptr && union_blocks == nullptr) return 0;
    if (p->pub_set == si && p->pub_seq == seq) TRY(publish_pending(p));
    uint32_t nz = 0, ws = 0;
    {
      HostWait hw(p);
      TRY(wait_pub(p->d, p->pub_host + 4 * si, seq, st, &nz, &ws));
    }
    ht_of(p).lap("2:wait counts");
    if (sent_blocks) *sent_blocks = 0;
    if (union_blocks) *union_blocks = ws;
    return 0;
  }
  const uint32_t NS = static_cast<uint32_t>(NA + 1);  // count columns per array (shard bounds)
  const uint64_t* const tagged = p->counts_host + static_cast<size_t>(si) * count_words(p);
  uint32_t counts[(OMR_MAX_WORKERS + 1) * (OMR_MAX_WORKERS + 2)];
  // at N > 1 the exchange stream waits for this round's plan on the plan stream (a deferred round's `ready` has
  // normally fired long before: then no wait is queued)
  if (async && p->cs != p->ps) TRY(order_after(p, p->cs, S.ready, "round: its plan"));
  const hipStream_t xs = async ? p->cs : st;
  ht_of(p).lap("2:cs wait ready");
  const omr_stream_t xstream = reinterpret_cast<omr_stream_t>(xs);
  auto cnt = [&](int a, int s) -> uint64_t { return counts[a * NS + s]; };
  auto per = [&](int a, int s) -> uint64_t { return cnt(a, s + 1) - cnt(a, s); };
  auto finish_async = [&](bool used_pack) {
    TRY(hip_check(hipEventRecord(S.done, xs), "hipEventRecord"));
    S.pending = true;
    p->last_async = si;
    p->tail = xs;  // the stream this round's last work is on
    if (used_pack) {
      std::lock_guard<std::mutex> g(p->mu);
      p->pk[pki].done_set = si;
      p->pk[pki].scan_wait = true;
    }
    return 0;
  };
  if (mode == OMR_ROUND_DENSE_REDUCE_SCATTER) {  // co-located only (checked by the caller)
    // the dense stand-in: every element of this rank's shard, reduced over all ranks by the transport
    const uint64_t r0 = p->bounds[me], r1 = p->bounds[me + 1];
    const uint64_t row_floats = static_cast<uint64_t>(p->lanes) * B;
    if (timed) TRY(hip_check(hipEventRecord(p->timed[tslot].x0, xs), "hipEventRecord"));
    TRY(p->d->reduce_scatter(x, out + r0 * row_floats, (r1 - r0) * row_floats, xs));
    if (timed) {
      TRY(hip_check(hipEventRecord(p->timed[tslot].x1, xs), "hipEventRecord"));
      // a ring reduce-scatter sends and receives (N-1)/N of the tensor per rank
      p->xt_out = p->xt_in = static_cast<uint64_t>(N - 1) * (r1 - r0) * row_floats * sizeof(float);
      p->xt_recorded = true;
      TRY(timed_exchange(p, tslot));
    }
    if (async) TRY(finish_async(false));
    if (sent_blocks != nullptr || union_blocks != nullptr) {
      HostWait hw(p);
      TRY(wait_round_counts(p, tagged, seq, st, counts));
    }
    if (sent_blocks) *sent_blocks = (r1 - r0) * p->lanes * static_cast<uint64_t>(N - 1);
    if (union_blocks) *union_blocks = per(M, me);
    return 0;
  }
  {
    HostWait hw(p);
    TRY(wait_round_counts(p, tagged, seq, st, counts));
  }
  ht_of(p).lap("2:wait counts");
  const bool wk = p->worker();
  float* const send = (wk && N > 1) ? p->pk[pki].buf : nullptr;
  // a co-located rank keeps its own shard's blocks out of its send streams (and reads them in place)
  const uint64_t own_shard = (wk && p->colocated) ? per(me, me) : 0;
  const uint64_t total_send = wk ? cnt(me, NA) - own_shard : 0;
  // 4b. workers send each shard's slice to its aggregator (common.cc:449); an aggregator receives its shard's blocks
  //     from every worker but itself
  std::vector<uint64_t> roff(M, 0);
  uint64_t in_blocks = 0;
  if (timed) TRY(hip_check(hipEventRecord(p->timed[tslot].x0, xs), "hipEventRecord"));
  if (N > 1) {
    std::vector<Slices> sends(N), recvs(N);
    if (wk)
      for (int s = 0; s < NA; ++s) {
        const int ar = p->agg_rank(s);
        if (ar == me) continue;
        // the fused pack's stream of shard s starts at the shard's place in the send buffer (the shards in order, the
        // own one left out); the pack pass's streams follow one another in block order without the own shard
        const uint64_t k0 = p->fused_pack ? omr_pack_send_offset(p->bounds.data(), static_cast<uint32_t>(NA),
                                                                 p->colocated ? me : -1, static_cast<uint32_t>(s),
                                                                 p->lanes, p->B, nullptr) / B
                                          : cnt(me, s) - (p->colocated && s > me ? own_shard : 0);
        sends[ar] = {Slice{send + k0 * B, per(me, s) * B * sizeof(float)}};
      }
    if (sh >= 0)
      for (int w = 0; w < M; ++w) {
        if (w == me) continue;
        roff[w] = recv_slot(p, w);
        recvs[w] = {Slice{p->recv + roff[w] * B, per(w, sh) * B * sizeof(float)}};
        in_blocks += per(w, sh);
      }
    TRY(p->d->exchange(sends, recvs, xs));
  }
  ht_of(p).lap("2:exchange");
  if (timed) {
    TRY(hip_check(hipEventRecord(p->timed[tslot].x1, xs), "hipEventRecord"));
    p->xt_out = total_send * B * sizeof(float);
    p->xt_in = in_blocks * B * sizeof(float);
    p->xt_recorded = true;
    TRY(timed_exchange(p, tslot));
  }
  const bool rs_mode = mode == OMR_ROUND_REDUCE_SCATTER;
  // 5. aggregator: rank-order shard sums (server.cc:97-98); a co-located rank reads its own blocks in place.
  //    Co-located reduce-scatter writes them in place (dense); otherwise packed in write-set order into `results`
  float* sums = nullptr;
  const uint32_t* const wprefix = S.prefix + static_cast<uint64_t>(M) * (rows + 1);
  uint64_t r0 = 0, r1 = 0;
  if (sh >= 0 && !solo) {  // (a one-rank round's worker scan wrote its sums: 0.0f + x over the write set)
    r0 = p->bounds[sh];
    r1 = p->bounds[sh + 1];
    const bool dense_out = rs_mode && p->colocated;
    sums = dense_out ? out : p->results;
    const float* own = p->colocated ? x : nullptr;
    const uint32_t own_idx = p->colocated ? static_cast<uint32_t>(me) : static_cast<uint32_t>(M);
    if (p->sum_list) {  // the pairs were built by this round's plan launch
      const omr_sum_list l = list_desc(p, S);
      TRY(omr_check(omr_shard_sum_list_f32(own, p->recv, &l, static_cast<uint32_t>(M), p->n, p->B, p->lanes, p->parts,
                                           S.wset, wprefix, dense_out ? 0 : 1, sums, xstream),
                    "omr_shard_sum_list_f32"));
    } else {  // row-ordered streams (the pack pass of ragged shards)
      TRY(omr_check(omr_shard_sum_stride_f32(own, own_idx, p->recv, roff.data(), S.masks_all, p->mstride,
                                             static_cast<uint32_t>(M), S.prefix, S.wset, rows, r0, r1, p->lanes, p->B,
                                             dense_out ? 0 : 1, sums, xstream),
                    "omr_shard_sum_stride_f32"));
    }
    if (!p->colocated) p->last_sums_blocks = per(M, sh);
  }
  ht_of(p).lap("2:shard sum");
  if (!rs_mode) {
    // 6. sums back to every worker (server.cc:162), into the round's send buffer (its exchange above is through with
    //    it), then scattered in place (client.cc:89).  A co-located rank's own shard comes from `results`.
    auto back_off = [&](int s) -> uint64_t {  // shard s's returned sums in the send buffer (blocks)
      return cnt(M, s) - (p->colocated && s > me ? per(M, me) : 0);
    };
    if (N > 1) {
      std::vector<Slices> ss(N), sr(N);
      if (sh >= 0)
        for (int w = 0; w < M; ++w)
          if (w != me) ss[w] = {Slice{sums, per(M, sh) * B * sizeof(float)}};
      if (wk)
        for (int s = 0; s < NA; ++s) {
          const int ar = p->agg_rank(s);
          if (ar != me) sr[ar] = {Slice{send + back_off(s) * B, per(M, s) * B * sizeof(float)}};
        }
      TRY(p->d->exchange(ss, sr, xs));
    }
    if (wk && out != nullptr && !solo) {
      const bool own_part = p->colocated && sh >= 0;
      if (N > 1 && (!own_part || r1 - r0 < rows))  // the other shards' sums (a co-located rank's own rows skipped)
        TRY(omr_check(omr_move_blocks_f32(send, out, 1, S.wset, wprefix, rows, p->lanes, p->B, own_part ? r0 : 0,
                                          own_part ? r1 : 0, xstream), "omr_move_blocks_f32 unpack"));
      if (own_part && r1 > r0) {  // its own shard's, from `results` (write-set order from row r0)
        const float* rbase = reinterpret_cast<const float*>(reinterpret_cast<uintptr_t>(p->results) -
                                                            cnt(M, sh) * B * sizeof(float));
        TRY(omr_check(omr_move_blocks_f32(rbase, out + r0 * p->lanes * B, 1, S.wset + r0, wprefix + r0, r1 - r0,
                                          p->lanes, p->B, 0, 0, xstream), "omr_move_blocks_f32 unpack own"));
      }
    }
  }
  if (timed && p->timed[tslot].xchg) {
    TRY(hip_check(hipEventRecord(p->timed[tslot].a1, xs), "hipEventRecord"));
    p->timed[tslot].agg = true;
  }
  if (async) TRY(finish_async(send != nullptr));
  ht_of(p).lap("2:rest");
  if (sent_blocks) *sent_blocks = total_send;
  if (union_blocks) *union_blocks = (rs_mode || !wk) ? (sh >= 0 ? per(M, sh) : 0) : cnt(M, NA);
  return 0;
}

// Issue the oldest deferred round's second half.
int issue_oldest(omr_ar_plan* p, uint64_t* sent_blocks, uint64_t* union_blocks) {
  const omr_ar_plan::Pending q = p->pend[0];
  for (int i = 1; i < p->npend; ++i) p->pend[i - 1] = p->pend[i];
  --p->npend;
  return round_finish(p, q.si, q.pki, q.x, q.out, q.mode, true, q.timed, q.seq, q.st, sent_blocks, union_blocks,
                      q.tslot);
}

// Issue every deferred round's second half, oldest first (outputs: the last one's counts; 0 if none).
int flush_pending(omr_ar_plan* p, hipStream_t st, uint64_t* sent_blocks, uint64_t* union_blocks) {
  (void)st;
  if (sent_blocks) *sent_blocks = 0;
  if (union_blocks) *union_blocks = 0;
  while (p->npend > 0) TRY(issue_oldest(p, sent_blocks, union_blocks));
  return 0;
}

// (event waits are skipped when the host already sees the event complete: a stream-wait packet costs the GPU a
// few microseconds of dispatch even when its event has long fired)
int wait_ev(hipStream_t on, hipEvent_t ev) {
  const hipError_t q = hipEventQuery(ev);
  if (q == hipErrorNotReady) return hip_check(hipStreamWaitEvent(on, ev, 0), "hipStreamWaitEvent");
  return hip_check(q, "hipEventQuery");
}

// Order the work issued next on side stream `on` after `ev`.  On the progress thread (OMR_ROUND_THREAD) the thread
// waits on the host until `ev` has completed and queues no wait packet: a side stream that shares a hardware queue
// with the caller's stream then never holds the caller's later scans behind a wait (in FIFO order they were queued
// before the step that waits), which is how a shared queue slows the round.  Elsewhere, and on the
// thread too once the side streams are checked to be on queues apart from the caller's (seat_side_streams: a wait
// packet there holds nothing of the caller's), a device-side wait, so no thread blocks.  Bounded by the transport's
// deadline and failure signals.
int order_after(omr_ar_plan* p, hipStream_t on, hipEvent_t ev, const char* what) {
  if (!t_progress || (p->seated && p->q_disjoint == 1)) return wait_ev(on, ev);
  const auto t0 = std::chrono::steady_clock::now();
  for (uint64_t spin = 1;; ++spin) {
    const hipError_t q = hipEventQuery(ev);
    if (q == hipSuccess) return 0;
    if (q != hipErrorNotReady) return p->d->contain(hip_check(q, what));
    if ((spin & 1023) == 0) {
      TRY(p->d->poll());
      if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(p->d->timeout_ms))
        return p->d->contain(derr(OMR_ETIMEDOUT, "%s: rank %d waited %lld ms: a peer is stuck or gone", what,
                                  p->d->rank, static_cast<long long>(p->d->timeout_ms)));
    }
    __builtin_ia32_pause();
  }
}

// Steps 2-7 of a round whose worker scan (and, when asynchronous, its `scanned` record) is queued: on the calling
// thread, or on the progress thread (OMR_ROUND_THREAD) in call order.
int round_rest(omr_ar_plan* p, const omr_ar_plan::Job& j, uint64_t* sent_blocks, uint64_t* union_blocks) {
  HostTrace& ht = ht_of(p);
  if (t_progress) ht.start();
  const int si = j.si, mode = j.mode, tslot = j.tslot, M = p->M, me = p->me, N = p->N;
  const bool async = j.async, timed = j.timed;
  const bool tally = (mode & kModeTally) != 0;
  const uint64_t rows = p->rows;
  const uint32_t NS = static_cast<uint32_t>(p->A + 1);
  const float* x = j.x;
  omr_ar_plan::Set& S = p->set[si];
  // a threaded round that is not deferred finishes the deferred ones first (rounds complete in call order)
  if (j.flush_first) TRY(flush_pending(p, j.st, nullptr, nullptr));
  // Deferred: the second half of the round kDeferDepth calls back goes first, on the side stream, so its exchange
  // runs beside this round's scan (and, at N > 1, on the exchange stream beside this round's plan) instead of queueing
  // behind this round's wait for it.
  // Its counts have long been in host memory, so the host does not wait either.
  if (j.defer && p->npend >= p->defer_depth) TRY(issue_oldest(p, sent_blocks, union_blocks));
  else if (j.defer) {
    if (sent_blocks) *sent_blocks = 0;
    if (union_blocks) *union_blocks = 0;
  }
  // the round's bookkeeping stream: an asynchronous round runs it on the side stream, so the caller's stream is left
  // with the worker scans alone (round k+1's scan overlaps round k's all-gather and plan, and round k-1's exchange)
  hipStream_t qs = async ? p->ps : j.st;
  const omr_stream_t qstream = reinterpret_cast<omr_stream_t>(qs);
  uint32_t seq = 0;
  if (tally) {
    // the one-launch round: the scan tallied the bookkeeping (omr_worker_scan_tally_f32); nothing runs after it
    seq = j.seq;
  } else {
    if (async && j.signal) {
      k_wait_seq<<<1, 64, 0, qs>>>(p->scan_done, j.seq, kScanWaitTicks);
      TRY(hip_check(hipGetLastError(), "k_wait_seq"));
    } else if (async) {
      TRY(order_after(p, qs, S.scanned, "round: the worker scan"));
    }
    // the rest of the set is refilled from here on: the round kSets calls back must be through with it (on the side
    // stream, in stream order already)
    if (S.pending) {
      if (qs != p->cs) TRY(order_after(p, qs, S.done, "round: the set's last round"));
      S.pending = false;
    }
    // 2. every worker's row masks
    ht.lap("1:refill wait");
    if (timed) TRY(hip_check(hipEventRecord(p->timed[tslot].q0, qs), "hipEventRecord"));
    TRY(p->d->allgather(S.own, S.masks_all, p->mstride * sizeof(uint64_t), qs));
    ht.lap("1:allgather");
    // 3. write set, prefixes, per-shard counts; own mask buffer cleared for its next round (the counts are stored
    //    straight into pinned host memory: no copy-engine hop before the host sees them)
    //    ... and, by extra workgroups of the same launch, the aggregator chain (server.cc:86-96 min_next) over the
    //    union, when asked for, and the shard sum's pair list (sum_list)
    seq = j.seq;  // (taken when its scan was issued: the scan's check slots carry it)
    const omr_sum_list sl = p->sum_list ? list_desc(p, S) : omr_sum_list{};
    uint64_t* const cw = p->counts_map + static_cast<size_t>(si) * count_words(p);
    TRY(omr_check(omr_round_plan_check(S.masks_all, static_cast<uint32_t>(M), p->mstride, rows, p->rpp, p->lanes,
                                       p->bounds_dev, NS, S.wset, nullptr, S.prefix, cw, S.own, S.pack_cnt,
                                       S.pack_cnt ? static_cast<uint32_t>(p->A) : 0u, S.plan_ws, seq, j.un, p->B,
                                       p->sum_list ? &sl : nullptr, p->chk_off, p->chk_slots,
                                       cw + static_cast<size_t>(M + 1) * NS, qstream),
                  "omr_round_plan_check"));
    ht.lap("1:plan");
    // 4a. pack own non-zero blocks of the other shards (block order == shard order, common.cc:405-407) where the scan
    //     could not (ragged shards): addressed by device-side data only, so it is queued before the host learns the
    //     counts.  (Every host API call costs microseconds; a round that spends them on streams and events is
    //     host-bound.)
    if (N > 1 && (mode & ~(kModeSolo | kModeTally)) != OMR_ROUND_DENSE_REDUCE_SCATTER && p->worker() &&
        !p->fused_pack) {
      const uint64_t r0 = p->colocated ? p->bounds[me] : 0, r1 = p->colocated ? p->bounds[me + 1] : 0;
      // the send buffer is free once the round kPackBufs calls back is through with it (its exchange, and an
      // all-reduce's return trip into it, on the exchange stream): this stream waits for that round's `done` unless
      // the two are one stream (the fused-pack scan does the same wait itself)
      if (qs != p->cs) {
        bool w;
        int ds;
        {
          std::lock_guard<std::mutex> g(p->mu);
          w = p->pk[j.pki].scan_wait;
          ds = p->pk[j.pki].done_set;
          p->pk[j.pki].scan_wait = false;
        }
        if (w) TRY(order_after(p, qs, p->set[ds].done, "round: the send buffer's last round"));
      }
      TRY(omr_check(omr_move_blocks_f32(x, p->pk[j.pki].buf, 0, S.masks_all + static_cast<uint64_t>(me) * p->mstride,
                                        S.prefix + static_cast<uint64_t>(me) * (rows + 1), rows, p->lanes, p->B, r0,
                                        r1, qstream), "omr_move_blocks_f32 pack"));
    }
    if (timed) {
      TRY(hip_check(hipEventRecord(p->timed[tslot].q1, qs), "hipEventRecord"));
      p->timed[tslot].prep = true;
    }
    ht.lap("1:pack");
    // the same event tells the scan that refills this set's own masks that the plan has consumed and re-zeroed them
    if (async) {
      TRY(hip_check(hipEventRecord(S.ready, qs), "hipEventRecord"));
      S.plan_pending = true;
    }
  }
  {  // the set's `ready` is recorded and its `scanned` waited for: the caller may reuse it
    std::lock_guard<std::mutex> g(p->mu);
    ++p->first_halves;
  }
  p->cv_done.notify_all();
  ht.lap("1:next+ready");
  (void)NS;
  // (a one-rank round's counts come on the caller's stream: the wait for them watches that stream)
  if (!j.defer)
    return round_finish(p, si, j.pki, x, j.out, mode, async, timed, seq, tally ? j.st : qs, sent_blocks, union_blocks,
                        tslot);
  // deferred: this round's second half waits in the queue (issued kDeferDepth calls later, or by join)
  omr_ar_plan::Pending& q = p->pend[p->npend++];
  q.active = true;
  q.si = si;
  q.pki = j.pki;
  q.mode = mode;
  q.timed = timed;
  q.x = x;
  q.out = j.out;
  q.seq = seq;
  q.tslot = tslot;
  q.st = tally ? j.st : qs;
  return 0;
}

// The progress thread: runs queued rounds' steps 2-7 in call order.  After a failure it records the error and
// skips the remaining jobs (counting them as issued, so no caller waits on them); calls then return the error.
void progress_main(omr_ar_plan* p) {
  t_progress = true;
  (void)hipSetDevice(p->device);
  std::unique_lock<std::mutex> lk(p->mu);
  for (;;) {
    p->cv_job.wait(lk, [&] { return p->stop || !p->jobs.empty(); });
    if (p->jobs.empty()) return;  // stop requested, nothing left
    const omr_ar_plan::Job j = p->jobs.front();
    p->jobs.pop_front();
    p->busy = true;
    const bool failed = p->thread_rc != 0;
    lk.unlock();
    const int rc = failed ? 0 : round_rest(p, j, nullptr, nullptr);
    if (rc != 0) (void)plan_fail(p, rc);  // (takes mu itself)
    if (failed && j.tslot >= 0) p->timed[j.tslot].open = false;  // a skipped round's record is never read
    lk.lock();
    if (rc != 0) {
      p->thread_rc = rc;
      p->thread_err = g_derr;
    }
    if (p->thread_rc != 0) p->first_halves = p->second_halves = p->rounds_begun;
    p->busy = false;
    p->cv_done.notify_all();
  }
}

int thread_start(omr_ar_plan* p) {
  if (p->progress.joinable()) return 0;
  TRY(hip_check(hipGetDevice(&p->device), "hipGetDevice"));
  p->ht_thread.on = p->ht.on;
  try {
    p->progress = std::thread(progress_main, p);
  } catch (const std::exception& e) {
    return derr(OMR_EINVAL, "sparse_round: cannot start the progress thread: %s", e.what());
  }
  return 0;
}

// every queued round issued; returns (and keeps) the progress thread's error, if any
int thread_drain(omr_ar_plan* p) {
  if (!p->progress.joinable()) return 0;
  HostWait hw(p);
  std::unique_lock<std::mutex> lk(p->mu);
  p->cv_done.wait(lk, [&] { return p->jobs.empty() && !p->busy; });
  if (p->thread_rc != 0) return derr(p->thread_rc, "%s", p->thread_err.c_str());
  return 0;
}

void thread_stop(omr_ar_plan* p) {
  if (!p->progress.joinable()) return;
  {
    std::lock_guard<std::mutex> g(p->mu);
    p->stop = true;
  }
  p->cv_job.notify_one();
  p->progress.join();
}

}  // namespace

extern "C" {

// One round: scan -> mask all-gather -> one bookkeeping launch -> block counts to the host (the
// round's single mid-round sync: the transport needs host-side sizes) -> pack -> send/recv -> shard sums
// [-> sums back -> unpack].  Every block movement is addressed by masks and prefixes.
}  // extern "C"

namespace {

// omr_sparse_round_f32 after its argument checks (mode: the base mode; the flags separately)
int sparse_round_issue(omr_ar_plan* p, const float* x, float* out, int32_t* flags, uint32_t* next_offsets,
                       uint32_t* union_next, int mode, bool threaded, bool defer, bool async, bool timed,
                       uint64_t* sent_blocks, uint64_t* union_blocks, omr_stream_t stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // A one-rank group's aggregator sums one worker's blocks: its shard sum is 0.0f + x over the write set (the worker's
  // non-zero blocks and the lane heads), exactly what the worker scan writes when it is given `out` (k_scan1f, as the
  // single-GPU step): so the scan writes the sums (solo).  Its bookkeeping is two counts (the union is the worker's own
  // blocks, min_next its own chain), which the scan tallies too (tally): the round is ONE launch
  // (omr_worker_scan_tally_f32) on the caller's stream, no side stream, no event, and no progress thread (nothing to
  // issue after the scan).  (Not in the staged bucket pipeline, whose scan reads a staging buffer and whose write-back
  // goes beside the next bucket's scan; a one-rank group's mapped buckets do run this way, reading and writing host
  // memory in the one launch.  omr_dist_test_world1_round keeps the bookkeeping on the multi-rank round's path:
  // all-gather and plan on the side stream.)
  const bool solo = p->N == 1 && p->worker() && p->colocated && p->scan_from == nullptr && !p->in_buckets &&
                    mode != OMR_ROUND_DENSE_REDUCE_SCATTER;
  const bool tally = solo && !p->d->world1_general;
  if (tally) threaded = false;
  // before the first asynchronous round on a caller's stream: the side streams on hardware queues apart from its queue
  // (seat_side_streams; a one-launch round uses none)
  if (async && !tally && p->queue_check && (!p->seated || p->seated_st != st)) {
    TRY(thread_drain(p));
    TRY(seat_side_streams(p, st));
  }
  // a threaded round hands its steps after the scan to the progress thread; any other call first lets the thread
  // issue everything queued (the plan's state is then this thread's alone)
  TRY(threaded ? thread_start(p) : thread_drain(p));
  p->ht.start();
  int32_t* fl = flags ? flags : p->flags_ws;
  uint32_t* nx = next_offsets ? next_offsets : p->next_ws;
  // (no union_next: the plan launch skips the aggregator chain, whose only output it is)
  uint32_t* un = union_next;
  // a stream other than the previous round's starts behind it (plan-wide state is shared by every round)
  if (p->last_st != nullptr && p->last_st != st) {
    TRY(hip_check(hipEventRecord(p->st_ev, p->last_st), "hipEventRecord"));
    TRY(hip_check(hipStreamWaitEvent(st, p->st_ev, 0), "hipStreamWaitEvent"));
  }
  p->last_st = st;
  // a round that is not deferred finishes a deferred one first (rounds complete in call order; a threaded round's
  // progress thread does this, it owns the deferred rounds)
  if (!defer && !threaded) TRY(flush_pending(p, st, nullptr, nullptr));
  // a synchronous round after asynchronous ones: its all-gather and exchange go on `stream`, so the side stream must
  // be idle first (one communicator is never driven from two streams at once; the last asynchronous round's `done`
  // follows all of its side-stream work)
  if (!async && p->last_async >= 0) {
    TRY(hip_check(hipStreamWaitEvent(st, p->set[p->last_async].done, 0), "hipStreamWaitEvent"));
    p->last_async = -1;
  }
  const int si = p->cur;
  omr_ar_plan::Set& S = p->set[si];
  p->cur = (p->cur + 1) % p->nsets;
  const int pki = static_cast<int>(p->rounds_total++ % omr_ar_plan::kPackBufs);
  // 1. worker scan (client.cc:19-31): flags, own next chain, own row masks, in one pass (a dedicated aggregator
  //    offers its all-zero mask buffer to the all-gather).  The set's own masks must have been consumed and
  //    re-zeroed by the plan of the round kSets calls back.
  int tslot = -1;
  if (timed) TRY(timed_slot(p, &tslot));
  uint32_t solo_seq = 0;
  bool signal = false;  // (below: the scan signals its completion on the device)
  if (tally) {
    if (timed) TRY(hip_check(hipEventRecord(p->timed[tslot].s0, st), "hipEventRecord"));
    // the previous one-rank round's counts go out with this scan's extra workgroup (on its own stream if it was
    // another one: then by a launch of its own, before this scan)
    if (p->pub_set >= 0 && p->pub_st != st) TRY(publish_pending(p));
    const int ps_i = p->pub_set;
    p->pub_set = -1;
    solo_seq = next_seq(p);
    const size_t TS = p->tally_slots;
    TRY(omr_check(omr_worker_scan_tally_f32(x, p->n, p->B, p->lanes, p->parts, fl, nx, out, p->tally + TS * si,
                                            ps_i >= 0 ? p->tally + TS * ps_i : nullptr,
                                            ps_i >= 0 ? p->pub_map + 4 * ps_i : nullptr, p->pub_seq, p->scan_ws,
                                            p->scan_ws_bytes, stream),
                  "omr_worker_scan_tally_f32"));
    p->pub_set = si;
    p->pub_seq = solo_seq;
    p->pub_st = st;
    // min_next over one worker is the worker's own chain
    if (un != nullptr)
      TRY(hip_check(hipMemcpyAsync(un, nx, p->nb * sizeof(uint32_t), hipMemcpyDeviceToDevice, st), "hipMemcpyAsync"));
    if (timed) {
      TRY(hip_check(hipEventRecord(p->timed[tslot].s1, st), "hipEventRecord"));
      p->timed[tslot].scan = true;
    }
    p->ht.lap("1:scan");
  } else {
    solo_seq = next_seq(p);  // (the round's number, carried by its scan's check slots)
    if (threaded) {  // that plan has been issued (and this set's `scanned` waited for) by the progress thread
      HostWait hw(p);
      std::unique_lock<std::mutex> lk(p->mu);
      const uint64_t need = p->rounds_begun >= static_cast<uint64_t>(p->nsets - 1) ? p->rounds_begun - (p->nsets - 1) : 0;
      p->cv_done.wait(lk, [&] { return p->first_halves >= need || p->thread_rc != 0; });
      if (p->thread_rc != 0) return derr(p->thread_rc, "%s", p->thread_err.c_str());
    }
    if (S.plan_pending) {
      // (threaded, the caller runs up to kSets rounds ahead of the GPU, so that plan has usually not run yet when this
      // scan is issued: a device-side wait would sit between two scans on the caller's stream and hold the next one
      // 3-7 us (profiles/r06/world1_general/trace_signalled/).  The caller waits for it on the host instead, which
      // keeps it two to three rounds ahead, as the deferred caller is.)
      if (threaded) TRY(wait_event_bounded(p->d, S.ready, "round: the set's last plan"));
      else TRY(wait_ev(st, S.ready));
      S.plan_pending = false;
    }
    // A fused-pack scan refills the round's send buffer: the round kPackBufs calls back, which read it (its exchange
    // issued up to kDeferDepth calls later, on the side stream), must be through first.  The progress thread may not
    // have issued it yet: wait until it has (at most one call behind then), then for it on the device.
    // A one-rank group's send buffer is empty (no other shard: the scan packs nothing), so its scan waits for nothing:
    // that wait put the tail of the exchange three rounds back (at world 1 over RCCL, its group's small kernels, run
    // only once the previous scan's workgroups drain) between two scans, 8-10 us per round (profiles/r06/world1_general/
    // trace/), and on the host for the progress thread.
    const bool pack_scan = p->fused_pack && p->worker() && mode != OMR_ROUND_DENSE_REDUCE_SCATTER;
    const bool pack_wait = pack_scan && p->pack_floats > 0;
    if (pack_scan) {
      std::unique_lock<std::mutex> lk(p->mu);
      constexpr uint64_t KP = omr_ar_plan::kPackBufs;
      const uint64_t need = p->rounds_begun >= KP ? p->rounds_begun - (KP - 1) : 0;
      if (threaded && pack_wait) {
        HostWait hw(p);
        p->cv_done.wait(lk, [&] { return p->second_halves >= need || p->thread_rc != 0; });
      }
      if (p->thread_rc != 0) return derr(p->thread_rc, "%s", p->thread_err.c_str());
      const bool w = p->pk[pki].scan_wait;
      const int ds = p->pk[pki].done_set;
      p->pk[pki].scan_wait = false;
      lk.unlock();
      if (w && pack_wait) TRY(wait_ev(st, p->set[ds].done));
    }
    // An asynchronous round's side stream starts behind the scan.  Where the side streams are checked to run on queues
    // apart from the caller's, the scan signals its own completion on the device (scan_done) and the side stream
    // waits for that with a one-wave kernel, so nothing is queued on the caller's stream between two scans; elsewhere
    // (and for a bucket's scan, or a rank with nothing to scan) an event recorded behind the scan.
    signal = async && p->worker() && p->seated && p->seated_st == st && p->q_disjoint == 1 && !p->in_buckets &&
             p->scan_from == nullptr;
    if (p->worker()) {
      if (timed) TRY(hip_check(hipEventRecord(p->timed[tslot].s0, st), "hipEventRecord"));
      const float* src = p->scan_from ? p->scan_from : x;
      // (a one-rank round's scan writes the sums; a bucket's writes the staging buffer's blocks when it reads the
      // pinned host buffer, and the sums come from the round's own shard sum)
      float* sout = p->scan_from ? const_cast<float*>(x) : (solo ? out : nullptr);
      uint64_t* const chk = S.own + p->chk_off;  // (the round check's slots, after the masks [and position table])
      if (pack_scan)  // the scan also writes this worker's blocks of the other shards into their send streams
        TRY(omr_check(omr_worker_scan_pack_check_f32(src, p->n, p->B, p->lanes, p->parts, fl, nx, S.own, sout,
                                                     p->bounds.data(), static_cast<uint32_t>(p->A),
                                                     p->colocated ? me_shard(p) : -1, p->pk[pki].buf, S.pack_cnt,
                                                     reinterpret_cast<uint32_t*>(S.own + p->rows), p->scan_ws,
                                                     p->scan_ws_bytes, chk, solo_seq,
                                                     signal ? p->scan_done : nullptr, stream),
                      "omr_worker_scan_pack_check_f32"));
      else
        TRY(omr_check(omr_worker_scan_check_f32(src, p->n, p->B, p->lanes, p->parts, fl, nx, S.own, sout, p->scan_ws,
                                                p->scan_ws_bytes, chk, solo_seq, signal ? p->scan_done : nullptr,
                                                stream),
                      "omr_worker_scan_check_f32"));
      if (timed) {
        TRY(hip_check(hipEventRecord(p->timed[tslot].s1, st), "hipEventRecord"));
        p->timed[tslot].scan = true;
      }
      p->ht.lap("1:scan");
    }
    // (a dedicated aggregator has nothing to scan: the side stream starts behind whatever the caller queued)
    if (async && !signal) TRY(hip_check(hipEventRecord(S.scanned, st), "hipEventRecord"));
  }
  p->ht.lap("1:scan events");
  omr_ar_plan::Job j;
  j.si = si;
  j.pki = pki;
  j.seq = solo_seq;
  j.signal = signal;
  j.mode = mode | (solo ? kModeSolo : 0) | (tally ? kModeTally : 0);
  j.tslot = tslot;
  j.async = async;
  j.defer = defer;
  j.timed = timed;
  j.flush_first = threaded && !defer;
  j.x = x;
  j.out = out;
  j.un = un;
  j.st = st;
  if (!threaded) {
    {
      std::lock_guard<std::mutex> g(p->mu);
      ++p->rounds_begun;
    }
    const int rc = round_rest(p, j, sent_blocks, union_blocks);
    if (rc != 0) {
      // a failed round counts as issued in both halves (a first-half failure left second_halves behind,
      // and a later fused-pack threaded round waited for it forever), and its timing record is closed unread
      {
        std::lock_guard<std::mutex> g(p->mu);
        p->first_halves = p->rounds_begun;
        p->second_halves = std::max(p->second_halves, p->rounds_begun);
      }
      if (tslot >= 0) p->timed[tslot].open = false;
      p->cv_done.notify_all();
    }
    return rc;
  }
  if (sent_blocks) *sent_blocks = 0;
  if (union_blocks) *union_blocks = 0;
  {
    std::lock_guard<std::mutex> g(p->mu);
    ++p->rounds_begun;
    p->jobs.push_back(j);
  }
  p->cv_job.notify_one();
  return 0;
}

}  // namespace

extern "C" {

int omr_sparse_round_f32(omr_ar_plan* p, const float* x, float* out, int32_t* flags, uint32_t* next_offsets,
                         uint32_t* union_next, int mode, uint64_t* sent_blocks, uint64_t* union_blocks,
                         omr_stream_t stream) {
  if (p == nullptr) return derr(OMR_EINVAL, "sparse_round: NULL plan");
  if (p->worker() && (x == nullptr || out == nullptr)) return derr(OMR_EINVAL, "sparse_round: a worker needs x and out");
  const bool threaded = (mode & OMR_ROUND_THREAD) != 0;
  const bool defer = (mode & OMR_ROUND_DEFER) != 0;
  const bool async = threaded || defer || (mode & OMR_ROUND_ASYNC) != 0;
  const bool timed = (mode & OMR_ROUND_TIME_EXCHANGE) != 0;
  mode &= ~(OMR_ROUND_ASYNC | OMR_ROUND_DEFER | OMR_ROUND_TIME_EXCHANGE | OMR_ROUND_THREAD);
  if (mode != OMR_ROUND_ALLREDUCE && mode != OMR_ROUND_REDUCE_SCATTER && mode != OMR_ROUND_DENSE_REDUCE_SCATTER)
    return derr(OMR_EINVAL, "sparse_round: unknown mode %d", mode);
  if (mode == OMR_ROUND_DENSE_REDUCE_SCATTER && !p->colocated)
    return derr(OMR_EINVAL, "sparse_round: the dense reduce-scatter stand-in needs every rank to be a worker");
  if (mode == OMR_ROUND_DENSE_REDUCE_SCATTER && p->rows % p->N != 0)
    return derr(OMR_EINVAL, "sparse_round: dense reduce-scatter needs equal shards (rows %llu, world %d)",
                static_cast<unsigned long long>(p->rows), p->N);
  TRY(plan_check(p, "sparse_round"));
  TRY(p->d->check_open("sparse_round"));
  // from here on the round has started: any error fails the plan and aborts the transport (plan_fail)
  return plan_fail(p, sparse_round_issue(p, x, out, flags, next_offsets, union_next, mode, threaded, defer, async, timed,
                                         sent_blocks, union_blocks, stream));
}

}  // extern "C"

namespace {

// the device mapping of a pinned host buffer (NULL if it has none)
float* host_mapping(float* buf, const hipPointerAttribute_t& attr) {
  float* const hbuf = static_cast<float*>(attr.hostPointer ? attr.hostPointer : buf);
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, hbuf, 0) == hipSuccess && d != nullptr) return static_cast<float*>(d);
  (void)hipGetLastError();
  return nullptr;
}

// omr_sparse_buckets_f32; *started is set once the first round or copy has been issued (an error after that fails
// the plan and aborts the transport)
int sparse_buckets_issue(omr_ar_plan* p, float* buf, uint64_t total_n, int mode, uint64_t* sent_blocks,
                         uint64_t* union_blocks, omr_stream_t stream, bool* started) {
  TRY(thread_drain(p));
  struct InBuckets {  // (staged rounds keep their shard sum off the scan: see omr_sparse_round_f32)
    omr_ar_plan* p;
    ~InBuckets() { p->in_buckets = false; }
  } in_buckets{p};
  if (total_n == 0 || total_n % p->n != 0)
    return derr(OMR_EINVAL, "sparse_buckets: total_n %llu is not a multiple of the plan's bucket of %llu floats",
                static_cast<unsigned long long>(total_n), static_cast<unsigned long long>(p->n));
  if (mode != OMR_ROUND_ALLREDUCE && mode != OMR_ROUND_REDUCE_SCATTER)
    return derr(OMR_EINVAL, "sparse_buckets: mode %d (OMR_ROUND_ALLREDUCE or OMR_ROUND_REDUCE_SCATTER)", mode);
  hipPointerAttribute_t attr;
  if (hipPointerGetAttributes(&attr, buf) != hipSuccess) {
    (void)hipGetLastError();
    return derr(OMR_EINVAL, "sparse_buckets: buf is neither device memory nor pinned host memory "
                            "(register it: omr_host_register / hipHostRegister)");
  }
  if (attr.type != hipMemoryTypeHost && attr.type != hipMemoryTypeDevice)
    return derr(OMR_EINVAL, "sparse_buckets: buf is neither device memory nor pinned host memory (memory type %d): "
                            "register it (omr_host_register / hipHostRegister)", static_cast<int>(attr.type));
  const bool host = attr.type == hipMemoryTypeHost;
  if (host && !p->worker()) return derr(OMR_EINVAL, "sparse_buckets: a worker's call (this rank aggregates only)");
  *started = true;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const uint64_t K = total_n / p->n, bytes = p->n * sizeof(float);
  const int rmode = mode | OMR_ROUND_DEFER;
  uint64_t sent = 0, uni = 0, s1 = 0, u1 = 0;
  auto acc = [&] {
    sent += s1;
    uni += u1;
  };
  // A pinned buffer with a device mapping needs no staging (the reference's registered res->buf is read and written in
  // place too: common.cc:873-914, client.cc:89).  Each bucket's round runs on the mapped bucket itself: the worker scan
  // reads it over PCIe and (N > 1) packs the other shards' non-zero blocks into the device send buffers, the shard sum
  // reads this rank's own blocks in place and stores the shard's write set back into it, and an all-reduce's returned
  // sums are scattered straight into it -- both link directions at once, as omr_host_scan_sum_zero_copy_f32 does.  A
  // one-rank group's round is one launch that does all of it: at N = 1 this is the default (config 5's shape: 52.5 GB/s
  // against 46.7 staged, round 5).  At N > 1 the rounds' PCIe traffic is split over kernels on two streams (the scan's
  // reads, the shard sum's reads of the rank's own blocks, the unpack's write-back), and as 2 IPC ranks on one GPU it
  // ran at half the staged rate (21.6 against 45.0 GB/s; profiles/r06/c5_ipc/), so there it is
  // opt-in (OMR_BUCKETS_DIRECT=1) and the staging ring stays the default.  OMR_BUCKETS_STAGED=1 (or either staging
  // mode below) stages a one-rank group too.
  float* const hmap = host ? host_mapping(buf, attr) : nullptr;
  const bool direct = host && hmap != nullptr && p->worker() &&
                      (p->N == 1 ? getenv("OMR_BUCKETS_STAGED") == nullptr : getenv("OMR_BUCKETS_DIRECT") != nullptr) &&
                      getenv("OMR_BUCKETS_STAGED_D2H") == nullptr && getenv("OMR_BUCKETS_SCAN_HOST") == nullptr;
  if (!host || direct) {  // device-resident (or mapped): one deferred round per bucket, in place
    float* const base = host ? hmap : buf;
    for (uint64_t k = 0; k < K; ++k) {
      float* b = base + k * p->n;
      TRY(omr_sparse_round_f32(p, b, b, nullptr, nullptr, nullptr, rmode, &s1, &u1, stream));
      acc();
    }
    while (p->npend > 0) {
      TRY(issue_oldest(p, &s1, &u1));
      acc();
    }
    TRY(omr_ar_plan_join(p, stream));
    // (host memory: the call returns once the buffer holds the result, as below: an event with the system-scope release
    // after the last round's last work, whichever stream it is on, then the caller's stream)
    if (host) {
      if (p->host_done == nullptr)
        TRY(hip_check(hipEventCreateWithFlags(&p->host_done, hipEventDisableTiming), "hipEventCreate"));
      TRY(hip_check(hipEventRecord(p->host_done, p->tail != nullptr ? p->tail : st), "hipEventRecord"));
      TRY(hip_check(hipEventSynchronize(p->host_done), "hipEventSynchronize"));
      TRY(hip_check(hipStreamSynchronize(st), "hipStreamSynchronize"));
    }
    if (sent_blocks) *sent_blocks = sent;
    if (union_blocks) *union_blocks = uni;
    return 0;
  }
  p->in_buckets = true;
  // pinned host: H2D(k+1) on s_in || scan(k) on stream || exchange + sums(k-1) on the plan's stream || D2H(k-2)
  constexpr int R = omr_ar_plan::kStage;
  if (p->s_in == nullptr) {
    for (int r = 0; r < R; ++r) {
      TRY(dev_alloc(p->d, &p->stage[r], p->n, &p->dev_bytes));
      TRY(hip_check(hipEventCreateWithFlags(&p->ev_in[r], hipEventDisableTiming), "hipEventCreate"));
      TRY(hip_check(hipEventCreateWithFlags(&p->ev_round[r], hipEventDisableTiming), "hipEventCreate"));
      TRY(hip_check(hipEventCreateWithFlags(&p->ev_out[r], hipEventDisableTiming), "hipEventCreate"));
    }
    TRY(hip_check(hipStreamCreateWithFlags(&p->s_in, hipStreamNonBlocking), "hipStreamCreate"));
    TRY(hip_check(hipStreamCreateWithFlags(&p->s_out, hipStreamNonBlocking), "hipStreamCreate"));
  }
  float* hbuf = static_cast<float*>(attr.hostPointer ? attr.hostPointer : buf);
  // reduce-scatter returns only this rank's shard: only those rows travel back
  const uint64_t row_floats = static_cast<uint64_t>(p->lanes) * p->B;
  const bool rs = mode == OMR_ROUND_REDUCE_SCATTER;
  // Write-back.  When the pinned buffer has a device mapping, each round writes its results straight into it: the
  // unpack (all-reduce) or the shard sum (reduce-scatter) stores only the write-set blocks over PCIe, as the
  // reference's worker copies only the blocks it gets back (client.cc:89), and every other block already holds its
  // (all-zero) input.  Otherwise (or with OMR_BUCKETS_STAGED_D2H set) the bucket, or the rank's shard, is copied
  // back whole from its staging buffer.
  float* const hdev = host_mapping(buf, attr);
  const bool zc = hdev != nullptr && getenv("OMR_BUCKETS_STAGED_D2H") == nullptr;
  // Read-in: each bucket is copied into a staging buffer (H2D on s_in).  With OMR_BUCKETS_SCAN_HOST=1 (and the
  // mapping) the worker scan instead reads the bucket straight from the pinned buffer and leaves its non-zero blocks
  // and lane heads in the staging buffer for the pack and the shard sum, so no copy engine runs.  That measured
  // slower (config 5, N = 1: 38.9 against 49.1 GB/s with the copy), so the copy stays the default.
  const bool zr = zc && getenv("OMR_BUCKETS_SCAN_HOST") != nullptr;
  const bool own_rs = rs && p->shard >= 0;  // co-located: the shard's sums land in place
  const uint64_t back0 = own_rs ? p->bounds[p->shard] * row_floats : 0;
  const uint64_t back_n = rs ? (own_rs ? (p->bounds[p->shard + 1] - p->bounds[p->shard]) * row_floats : 0) : p->n;
  auto h2d = [&](uint64_t k) -> int {
    const int r = static_cast<int>(k % R);
    if (p->out_used[r]) TRY(hip_check(hipStreamWaitEvent(p->s_in, p->ev_out[r], 0), "hipStreamWaitEvent"));
    TRY(hip_check(hipMemcpyAsync(p->stage[r], hbuf + k * p->n, bytes, hipMemcpyHostToDevice, p->s_in),
                  "hipMemcpyAsync H2D"));
    return hip_check(hipEventRecord(p->ev_in[r], p->s_in), "hipEventRecord");
  };
  auto d2h = [&](uint64_t k) -> int {  // after round k's second half, which is queued on the plan's stream
    const int r = static_cast<int>(k % R);
    if (zc) {  // the results are already in host memory: the staging buffer is free once the second half is through
      p->out_used[r] = true;
      return hip_check(hipEventRecord(p->ev_out[r], p->tail ? p->tail : p->cs), "hipEventRecord");
    }
    TRY(hip_check(hipEventRecord(p->ev_round[r], p->tail ? p->tail : p->cs), "hipEventRecord"));
    TRY(hip_check(hipStreamWaitEvent(p->s_out, p->ev_round[r], 0), "hipStreamWaitEvent"));
    if (back_n)
      TRY(hip_check(hipMemcpyAsync(hbuf + k * p->n + back0, p->stage[r] + back0, back_n * sizeof(float),
                                   hipMemcpyDeviceToHost, p->s_out), "hipMemcpyAsync D2H"));
    p->out_used[r] = true;
    return hip_check(hipEventRecord(p->ev_out[r], p->s_out), "hipEventRecord");
  };
  // after call k, the second halves of buckets <= k - kDeferDepth are queued: the write-back of bucket
  // k - kDeferDepth goes behind it, and frees its staging buffer for the H2D of bucket k - kDeferDepth + R
  static_assert(omr_ar_plan::kStage >= omr_ar_plan::kDeferDepth + 1, "staging ring >= deferral depth + 1");
  const uint64_t DD = static_cast<uint64_t>(p->defer_depth);  // <= kStage - 1
  if (!zr) TRY(h2d(0));
  for (uint64_t k = 0; k < K; ++k) {
    const int r = static_cast<int>(k % R);
    if (zr) {  // the scan refills stage[r]: the second half that last read it must be through
      if (p->out_used[r]) TRY(hip_check(hipStreamWaitEvent(st, p->ev_out[r], 0), "hipStreamWaitEvent"));
      p->scan_from = hdev + k * p->n;
    } else {
      TRY(hip_check(hipStreamWaitEvent(st, p->ev_in[r], 0), "hipStreamWaitEvent"));
    }
    const int rc = omr_sparse_round_f32(p, p->stage[r], zc ? hdev + k * p->n : p->stage[r], nullptr, nullptr,
                                        nullptr, rmode, &s1, &u1, stream);
    p->scan_from = nullptr;
    TRY(rc);
    acc();  // (the counts of bucket k - kDeferDepth, whose second half this call issued)
    if (k >= DD) TRY(d2h(k - DD));
    if (!zr && k + 1 < K) TRY(h2d(k + 1));
  }
  while (p->npend > 0) {  // the last buckets' second halves, oldest first, each followed by its D2H
    const uint64_t k = K - static_cast<uint64_t>(p->npend);
    TRY(issue_oldest(p, &s1, &u1));
    acc();
    TRY(d2h(k));
  }
  TRY(hip_check(hipStreamSynchronize(p->s_out), "hipStreamSynchronize"));  // the host buffer holds the result
  TRY(omr_ar_plan_join(p, stream));
  if (zc) {
    // written by the rounds themselves through the buffer's device mapping: wait for the event recorded (with the
    // default system-scope release) after the last bucket's second half on the communication stream, so the host
    // sees every store on return, then for the caller's stream
    TRY(hip_check(hipEventSynchronize(p->ev_out[(K - 1) % R]), "hipEventSynchronize"));
    TRY(hip_check(hipStreamSynchronize(st), "hipStreamSynchronize"));
  }
  if (sent_blocks) *sent_blocks = sent;
  if (union_blocks) *union_blocks = uni;
  return 0;
}

}  // namespace

extern "C" {

int omr_sparse_buckets_f32(omr_ar_plan* p, float* buf, uint64_t total_n, int mode, uint64_t* sent_blocks,
                           uint64_t* union_blocks, omr_stream_t stream) {
  if (p == nullptr || buf == nullptr) return derr(OMR_EINVAL, "sparse_buckets: NULL");
  TRY(plan_check(p, "sparse_buckets"));
  TRY(p->d->check_open("sparse_buckets"));
  bool started = false;
  const int rc = sparse_buckets_issue(p, buf, total_n, mode, sent_blocks, union_blocks, stream, &started);
  return started ? plan_fail(p, rc) : rc;
}

int omr_ar_plan_shard(omr_ar_plan* p, int* shard, uint64_t* row_begin, uint64_t* row_end, const float** sums,
                      uint64_t* num_blocks) {
  if (p == nullptr) return derr(OMR_EINVAL, "ar_plan_shard: NULL");
  TRY(thread_drain(p));
  if (shard) *shard = p->shard;
  if (row_begin) *row_begin = p->shard >= 0 ? p->bounds[p->shard] : 0;
  if (row_end) *row_end = p->shard >= 0 ? p->bounds[p->shard + 1] : 0;
  if (sums) *sums = p->colocated ? nullptr : p->results;
  if (num_blocks) *num_blocks = p->colocated ? 0 : p->last_sums_blocks;
  return 0;
}

int omr_ar_plan_fused_pack(const omr_ar_plan* p) { return p != nullptr && p->fused_pack ? 1 : 0; }

uint64_t omr_ar_plan_device_bytes(const omr_ar_plan* p) { return p != nullptr ? p->dev_bytes : 0; }

int omr_ar_plan_join(omr_ar_plan* p, omr_stream_t stream) {
  if (p == nullptr) return derr(OMR_EINVAL, "ar_plan_join: NULL");
  TRY(plan_check(p, "ar_plan_join"));
  TRY(plan_fail(p, thread_drain(p)));
  TRY(plan_fail(p, flush_pending(p, reinterpret_cast<hipStream_t>(stream), nullptr, nullptr)));
  if (p->last_async < 0) return 0;
  // the side stream runs rounds in issue order: waiting for the last one covers every earlier one
  TRY(hip_check(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), p->set[p->last_async].done, 0),
                "hipStreamWaitEvent"));
  return 0;
}

int omr_ar_plan_set_side_streams(omr_ar_plan* p, int n) {
  if (p == nullptr) return derr(OMR_EINVAL, "ar_plan_set_side_streams: NULL");
  if (n != 1 && n != 2) return derr(OMR_EINVAL, "ar_plan_set_side_streams: %d side streams (1 or 2)", n);
  TRY(plan_check(p, "ar_plan_set_side_streams"));
  if (n == 2 && p->xstream == nullptr)
    TRY(plan_fail(p, hip_check(hipStreamCreateWithFlags(&p->xstream, hipStreamNonBlocking), "hipStreamCreate")));
  hipStream_t want = n == 1 ? p->ps : p->xstream;
  if (want == p->cs) return 0;
  // every queued round's steps are issued first, on the old layout; then the new exchange stream (and the plan stream)
  // start after everything the old exchange stream holds: the set and send-buffer events it recorded are covered
  TRY(plan_fail(p, thread_drain(p)));
  TRY(plan_fail(p, flush_pending(p, p->ps, nullptr, nullptr)));
  if (p->switch_ev == nullptr)
    TRY(plan_fail(p, hip_check(hipEventCreateWithFlags(&p->switch_ev, hipEventDisableTiming |
                                                                             hipEventDisableSystemFence),
                               "hipEventCreate")));
  TRY(plan_fail(p, hip_check(hipEventRecord(p->switch_ev, p->cs), "hipEventRecord")));
  TRY(plan_fail(p, hip_check(hipStreamWaitEvent(want, p->switch_ev, 0), "hipStreamWaitEvent")));
  if (want != p->ps) TRY(plan_fail(p, hip_check(hipStreamWaitEvent(p->ps, p->switch_ev, 0), "hipStreamWaitEvent")));
  const hipStream_t old = p->cs;
  p->cs = want;
  p->seated = false;  // (the next asynchronous round checks the new layout's queues)
  if (p->tail != nullptr) p->tail = want;
  if (n == 1 && old == p->xstream) {
    // the exchange stream goes once it is idle: a stream keeps its hardware queue mapped while it exists, and with
    // several processes on one GPU the queues add up (8 IPC ranks: 45 ms per round on one side stream with the idle
    // exchange stream alive, 13 ms without it; profiles/r05/side_streams/)
    TRY(plan_fail(p, wait_event_bounded(p->d, p->switch_ev, "ar_plan_set_side_streams")));
    TRY(plan_fail(p, hip_check(hipStreamDestroy(p->xstream), "hipStreamDestroy")));
    p->xstream = nullptr;
  }
  return 0;
}

int omr_ar_plan_side_streams(const omr_ar_plan* p) { return p == nullptr ? 0 : (p->cs != p->ps ? 2 : 1); }

int omr_ar_plan_set_queue_check(omr_ar_plan* p, int on) {
  if (p == nullptr) return derr(OMR_EINVAL, "ar_plan_set_queue_check: NULL");
  p->queue_check = on != 0;
  p->seated = false;
  return 0;
}

int omr_ar_plan_queue_report(const omr_ar_plan* p, int* disjoint, int* probes, int* replaced) {
  if (p == nullptr) return derr(OMR_EINVAL, "ar_plan_queue_report: NULL");
  if (disjoint) *disjoint = p->q_disjoint;
  if (probes) *probes = p->q_probes;
  if (replaced) *replaced = p->q_replaced;
  return 0;
}

int omr_ar_plan_wait(omr_ar_plan* p, omr_stream_t stream) {
  if (p == nullptr) return derr(OMR_EINVAL, "ar_plan_wait: NULL");
  TRY(omr_ar_plan_join(p, stream));
  if (p->wait_done == nullptr)
    TRY(hip_check(hipEventCreateWithFlags(&p->wait_done, hipEventDisableTiming), "hipEventCreate"));
  TRY(plan_fail(p, hip_check(hipEventRecord(p->wait_done, reinterpret_cast<hipStream_t>(stream)), "hipEventRecord")));
  return plan_fail(p, wait_event_bounded(p->d, p->wait_done, "ar_plan_wait"));
}

int omr_ar_plan_host_stats(omr_ar_plan* p, double* wait_us, uint64_t* waits, int reset) {
  if (p == nullptr) return derr(OMR_EINVAL, "ar_plan_host_stats: NULL");
  if (wait_us) *wait_us = static_cast<double>(p->host_wait_ns.load()) * 1e-3;
  if (waits) *waits = p->host_waits.load();
  if (reset) {
    p->host_wait_ns.store(0);
    p->host_waits.store(0);
  }
  return 0;
}

int omr_ar_plan_failed(omr_ar_plan* p) {
  if (p == nullptr) return 0;
  std::lock_guard<std::mutex> g(p->mu);
  return p->failed;
}

int omr_ar_plan_exchange_time(omr_ar_plan* p, float* ms, uint64_t* bytes_out, uint64_t* bytes_in) {
  if (p == nullptr || ms == nullptr) return derr(OMR_EINVAL, "ar_plan_exchange_time: NULL");
  TRY(thread_drain(p));
  if (!p->xt_recorded) return derr(OMR_EINVAL, "ar_plan_exchange_time: no OMR_ROUND_TIME_EXCHANGE round issued");
  TRY(hip_check(hipEventSynchronize(p->xt1), "hipEventSynchronize"));
  TRY(hip_check(hipEventElapsedTime(ms, p->xt0, p->xt1), "hipEventElapsedTime"));
  if (bytes_out) *bytes_out = p->xt_out;
  if (bytes_in) *bytes_in = p->xt_in;
  return 0;
}

int omr_ar_plan_stage_timings(omr_ar_plan* p, float* stage_ms, uint64_t* bytes_out, uint64_t* bytes_in,
                              uint32_t* rounds) {
  if (p == nullptr) return derr(OMR_EINVAL, "ar_plan_stage_timings: NULL");
  TRY(thread_drain(p));
  double sum[OMR_ROUND_STAGES] = {0, 0, 0, 0};
  uint32_t cnt[OMR_ROUND_STAGES] = {0, 0, 0, 0};
  uint64_t bo = 0, bi = 0;
  auto add = [&](int k, hipEvent_t a, hipEvent_t b) -> int {
    float ms = 0;
    TRY(hip_check(hipEventSynchronize(b), "hipEventSynchronize"));
    TRY(hip_check(hipEventElapsedTime(&ms, a, b), "hipEventElapsedTime"));
    sum[k] += ms;
    ++cnt[k];
    return 0;
  };
  // (a deferred round whose exchange has not been issued yet stops the read: it and the later records stay unread
  // until a later call, so their stages are never counted without their exchange)
  uint32_t i = p->timed_first;
  for (; i < p->timed_next; ++i) {
    omr_ar_plan::Timed& t = p->timed[i % omr_ar_plan::kTimed];
    if (t.open) break;
    if (t.scan) TRY(add(0, t.s0, t.s1));
    if (t.prep) TRY(add(1, t.q0, t.q1));
    if (t.xchg) {
      TRY(add(2, t.x0, t.x1));
      bo += t.out;
      bi += t.in;
    }
    if (t.agg) TRY(add(3, t.x1, t.a1));
  }
  p->timed_first = i;
  if (stage_ms)
    for (int k = 0; k < OMR_ROUND_STAGES; ++k) stage_ms[k] = cnt[k] ? static_cast<float>(sum[k] / cnt[k]) : 0.f;
  if (bytes_out) *bytes_out = cnt[2] ? bo / cnt[2] : 0;
  if (bytes_in) *bytes_in = cnt[2] ? bi / cnt[2] : 0;
  if (rounds) *rounds = std::max(cnt[0], cnt[2]);
  return 0;
}

int omr_ar_plan_timings(omr_ar_plan* p, float* scan_ms, float* exchange_ms, uint64_t* bytes_out, uint64_t* bytes_in,
                        uint32_t* rounds) {
  float ms[OMR_ROUND_STAGES];
  TRY(omr_ar_plan_stage_timings(p, ms, bytes_out, bytes_in, rounds));
  if (scan_ms) *scan_ms = ms[0];
  if (exchange_ms) *exchange_ms = ms[2];
  return 0;
}

int omr_sparse_allreduce_f32(omr_ar_plan* p, const float* x, float* out, int32_t* flags, uint32_t* next_offsets,
                             uint32_t* union_next, uint64_t* sent_blocks, uint64_t* union_blocks,
                             omr_stream_t stream) {
  return omr_sparse_round_f32(p, x, out, flags, next_offsets, union_next, OMR_ROUND_ALLREDUCE, sent_blocks,
                              union_blocks, stream);
}

}  // extern "C"

// ================================================================ message-level round over a transport
//
// The reference's wire messages (common.cc:374-476 -> server.cc:56-199) between worker and aggregator processes:
// every rank computes the same per-slot schedule from the all-gathered row masks; each worker packs its messages of
// every slot (omr_msg_pack_f32) and sends aggregator j the slots gs with gs % n == j (common.cc:381-383); aggregator
// j builds their replies (omr_msg_aggregate_f32) and sends them to every worker, which applies them in place
// (omr_msg_unpack_f32).  Logs hold one 2*MESSAGE_SIZE-float message per (slot, protocol round); a slot's rounds are
// contiguous, so one transport piece per (slot, peer) carries all of them.
struct omr_msgd_plan {
  omr_dist* d = nullptr;
  int N = 1, M = 1, A = 1, me = 0, agg = -1;  // world, workers, aggregators, rank, this rank's aggregator index
  bool colocated = true;
  uint64_t n = 0, nb = 0, rows = 0;
  uint32_t B = 0, NB = 0, parts = 0, G = 0, rcap = 0;
  uint64_t* own_masks = nullptr;  // [rows]
  uint64_t* masks_all = nullptr;  // [N][rows]
  uint64_t* umask = nullptr;      // [rows]
  uint32_t* unext = nullptr;      // [nb]
  int32_t* flags = nullptr;       // [nb]
  uint32_t* next = nullptr;       // [nb]
  void* scan_ws = nullptr;
  size_t scan_ws_bytes = 0;
  char* sched = nullptr;          // [G][rcap] schedule records
  uint32_t* rounds = nullptr;     // [G]
  uint32_t* maxr = nullptr;       // [1]
  uint32_t* host_r = nullptr;     // pinned [G + 1]: rounds, then the max
  float* msgs = nullptr;          // a worker's own log [G][rcap][2*MESSAGE_SIZE]
  uint32_t* imm = nullptr;        // [G][rcap]
  std::vector<float*> wmsgs;      // an aggregator's copy of every worker's log (its slots filled)
  std::vector<uint32_t*> wimm;
  float* reply = nullptr;         // replies: an aggregator's own slots; a worker: every slot's, received
  uint32_t* rimm = nullptr;
  int agg_rank(uint32_t gs) const { return colocated ? static_cast<int>(gs % A) : M + static_cast<int>(gs % A); }
  bool worker() const { return me < M; }
};

namespace {

constexpr uint32_t kMsgW = 2 * OMR_MESSAGE_SIZE;

void msgd_free_logs(omr_msgd_plan* p) {
  // through the transport, which keeps exported logs alive for reuse (a regrown log may otherwise land at a freed
  // one's addresses while a peer still maps it)
  auto release = [&](void* v) { p->d->release(v); };
  release(p->sched);
  release(p->msgs);
  release(p->imm);
  release(p->reply);
  release(p->rimm);
  for (float* v : p->wmsgs) release(v);
  for (uint32_t* v : p->wimm) release(v);
  p->sched = nullptr;
  p->msgs = nullptr;
  p->imm = nullptr;
  p->reply = nullptr;
  p->rimm = nullptr;
  p->wmsgs.assign(p->wmsgs.size(), nullptr);
  p->wimm.assign(p->wimm.size(), nullptr);
}

int msgd_alloc_logs(omr_msgd_plan* p, uint32_t rcap) {
  msgd_free_logs(p);
  const uint64_t units = static_cast<uint64_t>(p->G) * rcap;
  TRY(dev_alloc(p->d, &p->sched, units * omr_msg_sched_bytes()));
  if (p->worker()) {
    TRY(dev_alloc(p->d, &p->msgs, units * kMsgW));
    TRY(dev_alloc(p->d, &p->imm, units));
  }
  TRY(dev_alloc(p->d, &p->reply, units * kMsgW));
  TRY(dev_alloc(p->d, &p->rimm, units));
  if (p->agg >= 0)
    for (int w = 0; w < p->M; ++w) {
      if (w == p->me) continue;  // a co-located aggregator reads its own worker's log in place
      TRY(dev_alloc(p->d, &p->wmsgs[w], units * kMsgW));
      TRY(dev_alloc(p->d, &p->wimm[w], units));
    }
  p->rcap = rcap;
  return 0;
}

// the schedule, its round counts on the host (one synchronisation: the transport needs the pieces' sizes), and
// the logs grown until they hold the longest slot; identical on every rank (same masks)
int msgd_schedule(omr_msgd_plan* p, hipStream_t st) {
  for (int attempt = 0; attempt < 2; ++attempt) {
    TRY(omr_check(omr_msg_schedule(p->masks_all, static_cast<uint32_t>(p->M), p->unext, p->n, p->B, p->NB, p->parts,
                                   p->rcap, p->sched, p->rounds, p->maxr, reinterpret_cast<omr_stream_t>(st)),
                  "omr_msg_schedule"));
    TRY(hip_check(hipMemcpyAsync(p->host_r, p->rounds, p->G * sizeof(uint32_t), hipMemcpyDeviceToHost, st),
                  "hipMemcpyAsync"));
    TRY(hip_check(hipMemcpyAsync(p->host_r + p->G, p->maxr, sizeof(uint32_t), hipMemcpyDeviceToHost, st),
                  "hipMemcpyAsync"));
    TRY(hip_check(hipStreamSynchronize(st), "hipStreamSynchronize"));
    if (p->host_r[p->G] <= p->rcap) return 0;
    uint32_t cap = p->rcap;
    const uint32_t rpp = static_cast<uint32_t>(p->rows / p->parts);
    while (cap < rpp + 2) cap *= 2;  // a lane carries at most its head plus rows_per_part - 1 blocks
    TRY(hip_check(hipStreamSynchronize(st), "hipStreamSynchronize"));
    TRY(msgd_alloc_logs(p, cap));
  }
  return derr(OMR_EINVAL, "msgd: %u protocol rounds exceed the logs' %u", p->host_r[p->G], p->rcap);
}

}  // namespace

extern "C" {

int omr_msgd_plan_destroy(omr_msgd_plan* p) {
  if (p == nullptr) return 0;
  (void)hipDeviceSynchronize();
  msgd_free_logs(p);
  void* devs[] = {p->own_masks, p->masks_all, p->umask, p->unext, p->flags, p->next, p->scan_ws, p->rounds, p->maxr};
  for (void* v : devs) p->d->release(v);
  (void)hipHostFree(p->host_r);
  delete p;
  return 0;
}

int omr_msgd_plan_create(omr_dist* d, uint32_t num_workers, uint64_t n, uint32_t block_size, uint32_t num_lanes,
                         uint32_t num_parts, omr_msgd_plan** out) {
  if (d == nullptr || out == nullptr) return derr(OMR_EINVAL, "msgd_plan_create: NULL");
  *out = nullptr;
  TRY(omr_check(omr_layout_check(n, block_size, num_lanes, num_parts), "omr_layout_check"));
  if (num_lanes != OMR_NUM_SLOTS * (OMR_MESSAGE_SIZE / block_size))
    return derr(OMR_EINVAL, "msgd_plan_create: num_lanes must be NUM_SLOTS*MESSAGE_SIZE/BLOCK_SIZE");
  if (num_workers == 0 || num_workers > static_cast<uint32_t>(d->world) || num_workers > OMR_MAX_WORKERS)
    return derr(OMR_EINVAL, "msgd_plan_create: %u workers in a world of %d", num_workers, d->world);
  auto* p = new omr_msgd_plan();
  p->d = d;
  p->N = d->world;
  p->M = static_cast<int>(num_workers);
  p->colocated = p->M == p->N;
  p->A = p->colocated ? p->N : p->N - p->M;
  p->me = d->rank;
  p->agg = p->colocated ? p->me : (p->me >= p->M ? p->me - p->M : -1);
  p->n = n;
  p->B = block_size;
  p->NB = num_lanes;
  p->parts = num_parts;
  p->nb = n / block_size;
  p->rows = p->nb / num_lanes;
  p->G = num_parts * OMR_NUM_SLOTS;
  p->wmsgs.assign(p->M, nullptr);
  p->wimm.assign(p->M, nullptr);
  int rc = 0;
  auto A = [&](int r) {
    if (rc == 0) rc = r;
  };
  A(dev_alloc(p->d, &p->own_masks, p->rows));
  A(dev_alloc(p->d, &p->masks_all, static_cast<size_t>(p->N) * p->rows));
  A(dev_alloc(p->d, &p->umask, p->rows));
  A(dev_alloc(p->d, &p->unext, p->nb));
  A(dev_alloc(p->d, &p->flags, p->nb));
  A(dev_alloc(p->d, &p->next, p->nb));
  p->scan_ws_bytes = omr_scan_workspace_bytes(n, block_size, num_lanes, num_parts);
  A(dev_alloc(p->d, reinterpret_cast<char**>(&p->scan_ws), p->scan_ws_bytes));
  A(dev_alloc(p->d, &p->rounds, p->G));
  A(dev_alloc(p->d, &p->maxr, 1));
  A(hip_check(hipHostMalloc(reinterpret_cast<void**>(&p->host_r), (p->G + 1) * sizeof(uint32_t)), "hipHostMalloc"));
  if (rc == 0) A(hip_check(hipMemset(p->own_masks, 0, p->rows * sizeof(uint64_t)), "hipMemset"));
  if (rc == 0 && p->scan_ws_bytes) A(hip_check(hipMemset(p->scan_ws, 0, p->scan_ws_bytes), "hipMemset"));
  if (rc == 0) A(msgd_alloc_logs(p, 16));
  if (rc == 0) A(hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize"));
  if (rc != 0) {
    omr_msgd_plan_destroy(p);
    return rc;
  }
  *out = p;
  return 0;
}

int omr_msgd_round_f32(omr_msgd_plan* p, const float* x, float* out, uint32_t* max_rounds, omr_stream_t stream) {
  if (p == nullptr) return derr(OMR_EINVAL, "msgd_round: NULL plan");
  if (p->worker() && (x == nullptr || out == nullptr)) return derr(OMR_EINVAL, "msgd_round: a worker needs x and out");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const uint64_t rows = p->rows;
  // 1. worker scan: flags, next chain (client.cc:19-31), row masks
  if (p->worker()) {
    TRY(hip_check(hipMemsetAsync(p->own_masks, 0, rows * sizeof(uint64_t), st), "hipMemsetAsync"));
    TRY(omr_check(omr_worker_scan_f32(x, p->n, p->B, p->NB, p->parts, p->flags, p->next, p->own_masks, nullptr,
                                      p->scan_ws, p->scan_ws_bytes, stream), "omr_worker_scan_f32"));
  }
  // 2. every rank learns every worker's masks; 3. the aggregator chain over their union (server.cc:86-96)
  TRY(p->d->allgather(p->own_masks, p->masks_all, rows * sizeof(uint64_t), st));
  TRY(omr_check(omr_mask_union(p->masks_all, static_cast<uint32_t>(p->M), rows, static_cast<uint32_t>(rows / p->parts),
                               p->NB, 0, p->umask, stream), "omr_mask_union"));
  TRY(omr_check(omr_next_offsets(p->umask, 1, p->n, p->B, p->NB, p->parts, p->unext, stream), "omr_next_offsets"));
  // 4. the per-slot schedule (the same on every rank)
  TRY(msgd_schedule(p, st));
  const uint32_t G = p->G, cap = p->rcap;
  const uint32_t* R = p->host_r;
  const size_t mb = static_cast<size_t>(kMsgW) * sizeof(float);
  auto msg_piece = [&](float* log, uint32_t gs) { return Slice{log + static_cast<uint64_t>(gs) * cap * kMsgW, R[gs] * mb}; };
  auto imm_piece = [&](uint32_t* log, uint32_t gs) {
    return Slice{log + static_cast<uint64_t>(gs) * cap, R[gs] * sizeof(uint32_t)};
  };
  // 5. a worker's messages of every slot (client.cc:180-205, :113-127; common.cc:399-408)
  if (p->worker())
    TRY(omr_check(omr_msg_pack_f32(x, p->flags, p->next, p->sched, p->rounds, p->parts, cap, p->B, p->msgs, p->imm,
                                   stream), "omr_msg_pack_f32"));
  // 6. workers -> the aggregator of each slot (common.cc:381-383, :449)
  {
    std::vector<Slices> sends(p->N), recvs(p->N);
    if (p->worker())
      for (uint32_t gs = 0; gs < G; ++gs) {
        const int a = p->agg_rank(gs);
        if (a == p->me) continue;
        sends[a].push_back(msg_piece(p->msgs, gs));
        sends[a].push_back(imm_piece(p->imm, gs));
      }
    if (p->agg >= 0)
      for (int w = 0; w < p->M; ++w) {
        if (w == p->me) continue;
        for (uint32_t gs = static_cast<uint32_t>(p->agg); gs < G; gs += static_cast<uint32_t>(p->A)) {
          recvs[w].push_back(msg_piece(p->wmsgs[w], gs));
          recvs[w].push_back(imm_piece(p->wimm[w], gs));
        }
      }
    TRY(p->d->exchange(sends, recvs, st));
  }
  // 7. the aggregator's replies to its slots (server.cc:68-162)
  if (p->agg >= 0) {
    std::vector<const float*> wm(p->M);
    std::vector<const uint32_t*> wi(p->M);
    for (int w = 0; w < p->M; ++w) {
      wm[w] = w == p->me ? p->msgs : p->wmsgs[w];
      wi[w] = w == p->me ? p->imm : p->wimm[w];
    }
    TRY(omr_check(omr_msg_aggregate_f32(wm.data(), wi.data(), static_cast<uint32_t>(p->M), p->sched, p->rounds,
                                        p->unext, p->parts, cap, p->B, p->NB, static_cast<uint32_t>(p->A),
                                        static_cast<uint32_t>(p->agg), p->reply, p->rimm, stream),
                  "omr_msg_aggregate_f32"));
  }
  // 8. replies -> every worker (server.cc:162, common.cc:548)
  {
    std::vector<Slices> sends(p->N), recvs(p->N);
    if (p->agg >= 0)
      for (int w = 0; w < p->M; ++w) {
        if (w == p->me) continue;
        for (uint32_t gs = static_cast<uint32_t>(p->agg); gs < G; gs += static_cast<uint32_t>(p->A)) {
          sends[w].push_back(msg_piece(p->reply, gs));
          sends[w].push_back(imm_piece(p->rimm, gs));
        }
      }
    if (p->worker())
      for (uint32_t gs = 0; gs < G; ++gs) {
        const int a = p->agg_rank(gs);
        if (a == p->me) continue;
        recvs[a].push_back(msg_piece(p->reply, gs));
        recvs[a].push_back(imm_piece(p->rimm, gs));
      }
    TRY(p->d->exchange(sends, recvs, st));
  }
  // 9. the worker applies every reply in place (client.cc:87-90)
  if (p->worker())
    TRY(omr_check(omr_msg_unpack_f32(p->reply, p->rimm, p->sched, p->rounds, p->parts, cap, p->B, p->NB, out, stream),
                  "omr_msg_unpack_f32"));
  if (max_rounds) *max_rounds = R[G];
  return 0;
}

int omr_msgd_logs(omr_msgd_plan* p, uint32_t worker, float** messages, uint32_t** imm, float** replies,
                  uint32_t** reply_imm, uint32_t** rounds, uint32_t* round_capacity) {
  if (p == nullptr || worker >= static_cast<uint32_t>(p->M)) return derr(OMR_EINVAL, "msgd_logs: bad plan or worker");
  const bool own = static_cast<int>(worker) == p->me;
  if (messages) *messages = own ? p->msgs : p->wmsgs[worker];
  if (imm) *imm = own ? p->imm : p->wimm[worker];
  if (replies) *replies = p->reply;
  if (reply_imm) *reply_imm = p->rimm;
  if (rounds) *rounds = p->rounds;
  if (round_capacity) *round_capacity = p->rcap;
  return 0;
}

}  // extern "C"
