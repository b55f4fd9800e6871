/*
 * omr_dist.h — C ABI of the multi-rank sparse all-reduce (one OmniReduce round across ranks), host side in C++
 * (omnireduce-rdma-demo_amd/csrc/omr_dist.hip, library libomr_dist.so, on top of libomr.so).
 *
 * Replaces the reference's RDMA transport and per-thread protocol loops for the hot path: every rank is worker r
 * and aggregator of shard r (README.md:13-22; common.cc:381-383 shards slots over aggregators).  One call =
 *   worker scan (client.cc:19-31) -> all-gather of row masks -> pack own non-zero blocks (common.cc:405-407) ->
 *   grouped send/recv to the shard aggregators -> rank-order shard sums (server.cc:97-98) -> sums back to every
 *   worker (server.cc:162) -> in-place scatter (client.cc:89).
 *
 * Two transports:
 *   RCCL  — one process per GPU over xGMI; bootstrap with omr_dist_unique_id on one rank, shared out of band
 *           (the ./omr_server rendezvous does this, standing in for the reference's TCP bootstrap common.cc:50-197).
 *   local — `world` ranks as threads of ONE process (any number of GPUs, several ranks may share a GPU) that
 *           exchange through device-to-device copies; the loopback stand-in for testing "multi-node" without a
 *           cluster.
 * Return convention as omr.h: 0 ok, OMR_EINVAL on bad arguments, otherwise a hip/rccl error code; message in
 * omr_dist_last_error().
 */
#ifndef OMR_DIST_H
#define OMR_DIST_H

#include <stddef.h>
#include <stdint.h>

#include "omr.h"

#ifdef __cplusplus
extern "C" {
#endif

#define OMR_UNIQUE_ID_BYTES 128
/* Returned once a transport has been aborted (by an error, a deadline or omr_dist_abort), and by a plan whose
 * earlier round failed. */
#define OMR_EABORTED (-2)
/* A host-side wait of the transport or of a round passed the transport's deadline (omr_dist_set_timeout). */
#define OMR_ETIMEDOUT (-3)
/* The round check failed (round 6): a worker's all-gathered row masks were not the ones its scan of that round wrote
 * (read before the scan wrote or finished them, or from another buffer); the round is failed and the transport aborted
 * before any exchange is sized from them (omr_round_plan_check in omr.h). */
#define OMR_ESTALE (-4)

typedef struct omr_dist omr_dist;               /* a transport endpoint (one rank) */
typedef struct omr_local_board omr_local_board; /* shared state of an in-process group */
typedef struct omr_ar_plan omr_ar_plan;         /* workspaces of one sparse all-reduce shape */

const char* omr_dist_last_error(void);

int omr_dist_unique_id(void* id /* OMR_UNIQUE_ID_BYTES */);
int omr_dist_create_rccl(const void* id, int rank, int world, omr_dist** out);

/* Cross-process transport over HIP IPC: `world` ranks as separate processes of one node (any GPUs; several may
 * share one, which RCCL refuses), the stand-in for the reference's separate worker and aggregator machines.  One
 * rank calls omr_dist_ipc_unique_id and shares the id out of band (the ./omr_server rendezvous does); every rank
 * then calls omr_dist_create_ipc, which returns once all have joined.  Data moves device to device (each receiver
 * copies out of the sender's IPC-mapped buffer); ordering is carried on the device by IPC events, so calls return
 * without synchronising any stream, as with RCCL.  The transport caches IPC handles and peer mappings per allocation.
 * Plans allocate their device buffers through the transport, which keeps every buffer it exported alive until it is
 * destroyed itself and hands it to the next plan whose request it fits (its size up to twice the request; a freed
 * allocation a peer still maps may come back from hipMalloc at the same address, and ROCm then refuses to export it).
 * So device memory only grows while the transport lives: re-planning at larger sizes adds to the pool.  Buffers the
 * caller hands to a round must stay allocated while the transport lives.  Destroy is collective. */
int omr_dist_ipc_unique_id(void* id /* OMR_UNIQUE_ID_BYTES */);
int omr_dist_create_ipc(const void* id, int rank, int world, omr_dist** out);

omr_local_board* omr_local_board_create(int world);
void omr_local_board_destroy(omr_local_board* board);
int omr_dist_create_local(omr_local_board* board, int rank, omr_dist** out);

int omr_dist_rank(const omr_dist* d);
int omr_dist_world(const omr_dist* d);
/* 0; OMR_ETIMEDOUT if, after an abort, the rank's streams were still busy (waiting on a gone peer) past the deadline:
 * the transport's device-side state (mappings, events, exported allocations) is then left allocated */
int omr_dist_destroy(omr_dist* d);

/* The transport's two operations, as the round uses them (every rank of the group calls them in the same order).
 * omr_dist_allgather: out[p*bytes .. (p+1)*bytes) = rank p's `in` (device buffers).  omr_dist_exchange: send[p]
 * (send_bytes[p]) to peer p and recv[p] (recv_bytes[p]) from peer p for every p != rank, entries at p == rank
 * ignored, zero-byte pieces skipped; sizes must match the peer's.  Over RCCL these are ncclAllGather and one group of
 * ncclSend/ncclRecv (the reference's post_send / post_receive loop, common.cc:374-476, on the communication channel).
 * Both return with the transfer enqueued on `stream`. */
int omr_dist_allgather(omr_dist* d, const void* in, void* out, size_t bytes, omr_stream_t stream);
int omr_dist_exchange(omr_dist* d, void* const* send, const size_t* send_bytes, void* const* recv,
                      const size_t* recv_bytes, omr_stream_t stream);
/* Failure containment (the reference exits on a failed post, common.cc:450-451; a rank of a collective group must
 * make sure its peers do not wait for it forever).
 *   - Every host-side wait of a transport or of a round (a loopback barrier, an IPC rendezvous, a round's wait for
 *     its block counts, omr_ar_plan_wait) ends after the transport's deadline: omr_dist_set_timeout (default 60 s, or
 *     the environment's OMR_DIST_TIMEOUT_MS), with OMR_ETIMEDOUT.  The count wait also polls the group's failure
 *     signals: RCCL's asynchronous errors (ncclCommGetAsyncError), a loopback or IPC peer's abort.
 *   - Any error of a transport operation, an expired deadline, a failure signal, or omr_dist_abort ABORTS the
 *     transport: RCCL's two communicators are aborted (ncclCommAbort cancels the operations queued on them, so this
 *     rank's streams drain; peers' matching operations end at their own deadlines), the loopback and IPC groups
 *     raise a flag that ends their peers' waits on this rank at once.  Every later operation fails with
 *     OMR_EABORTED; the transport can only be destroyed (a recovery makes a new group).
 *   - A round that fails after it has started (any error in omr_sparse_round_f32 past its argument checks, in
 *     omr_sparse_buckets_f32, in join or wait) also marks its plan failed: later calls on the plan return
 *     OMR_EABORTED; omr_ar_plan_destroy still releases it without waiting on peers.
 * omr_dist_abort may be called from another thread while this rank waits.  omr_dist_poll returns the group's
 * failure signals (0 while healthy). */
int omr_dist_abort(omr_dist* d);
int omr_dist_aborted(const omr_dist* d); /* 1 once aborted */
int omr_dist_set_timeout(omr_dist* d, int64_t timeout_ms);
int omr_dist_poll(omr_dist* d);
/* Test hooks.  omr_dist_inject_fault: the next exchange on `d` (omr_dist_exchange or a round's) fails with OMR_EINVAL
 * once it has issued `after_pieces` non-empty pieces (0: before the first; a negative value disarms): the RCCL group
 * is closed (the pieces already issued still run, so no group is left open to capture later calls) and the
 * transport is then aborted as above, standing in for a rank that stops issuing its part of an exchange.
 * omr_dist_inject_allgather_fault: the next all-gather fails before it moves anything (a round failing in its first
 * half). */
int omr_dist_inject_fault(omr_dist* d, int64_t after_pieces);
int omr_dist_inject_allgather_fault(omr_dist* d);
/* Test hook (on: 1): a one-rank group runs the multi-rank round's code path -- worker scan, mask all-gather and plan on
 * the plan stream, exchange on the exchange stream -- instead of the one-launch round, and an RCCL transport issues its
 * all-gather, exchange and reduce-scatter as RCCL calls instead of as copies.  Plans made after the call also take
 * the N > 1 round's two side streams.  So the fault tests reach RCCL's group and ncclCommAbort paths, and the N > 1
 * round's stream layout can be timed, on a one-GPU box. */
int omr_dist_test_world1_round(omr_dist* d, int on);

/* Workspaces for tensors of n floats on the layout (block_size, num_lanes, num_parts); allocated on the current
 * HIP device, which must be the device the rank's tensors live on. */
int omr_ar_plan_create(omr_dist* d, uint64_t n, uint32_t block_size, uint32_t num_lanes, uint32_t num_parts,
                       omr_ar_plan** out);
int omr_ar_plan_destroy(omr_ar_plan* plan); /* before its transport (omr_dist_destroy) */
/* The same with roles (the reference's m workers and n aggregators, README.md:13-22): ranks [0, num_workers) are
 * workers; if num_workers < world the other ranks are dedicated aggregators — the ./omr_server processes, holding no
 * tensor — aggregator j = rank num_workers + j owning row shard j of n = world - num_workers (rows [j*rows/n,
 * (j+1)*rows/n)); num_workers == world is omr_ar_plan_create (every rank a worker and the aggregator of its own
 * shard).  A dedicated aggregator calls omr_sparse_round_f32 with x = out = NULL in the same sequence of modes as the
 * workers; in all-reduce mode its sums go back to every worker, in reduce-scatter mode they stay with it
 * (omr_ar_plan_shard).  The dense stand-in needs every rank to be a worker. */
int omr_ar_plan_create_roles(omr_dist* d, uint32_t num_workers, uint64_t n, uint32_t block_size, uint32_t num_lanes,
                             uint32_t num_parts, omr_ar_plan** out);
/* This rank's aggregator shard: *shard (-1: none), its rows [*row_begin, *row_end), and for a dedicated aggregator the
 * last round's sums (device, write-set order of the shard rows: union blocks and lane heads in block order, as the
 * reply of server.cc:143-147) and their count; NULL / 0 for a co-located rank (its sums are written in place). */
int omr_ar_plan_shard(omr_ar_plan* plan, int* shard, uint64_t* row_begin, uint64_t* row_end, const float** sums,
                      uint64_t* num_blocks);

/* One round on this rank.  x: the rank's gradient (device, n floats).  out: receives the all-reduced tensor
 * (rank-order sums over the union of non-zero blocks plus lane heads); may equal x for the reference's in-place
 * result, otherwise it must already hold x's values outside that set.  flags / next_offsets / union_next (device,
 * nb entries each, may be NULL) receive the worker's flags, its next-offset chain and the aggregator chain.
 * *sent_blocks / *union_blocks (host, may be NULL) receive this rank's off-rank sent blocks and the write-set size.
 * Waits once mid-round for the block counts (the transport needs host-side sizes; the bookkeeping kernel stores
 * them straight into pinned host memory) and returns with the rest of the round enqueued on `stream`:
 * synchronise `stream` before reading out / flags / next_offsets / union_next.  (A one-rank group's round is one
 * launch; with both count pointers NULL it does not wait at all.) */
int omr_sparse_allreduce_f32(omr_ar_plan* plan, const float* x, float* out, int32_t* flags,
                             uint32_t* next_offsets, uint32_t* union_next, uint64_t* sent_blocks,
                             uint64_t* union_blocks, omr_stream_t stream);

/* The round with a choice of how far it goes:
 *   OMR_ROUND_ALLREDUCE       as omr_sparse_allreduce_f32 (workers get every shard's sums back);
 *   OMR_ROUND_REDUCE_SCATTER  stops at the aggregators: `out` receives only this rank's shard sums (its part of
 *                             the write set, in place) — the worker -> aggregator "reduce" of BASELINE config 4;
 *                             *union_blocks = this shard's write-set size. */
#define OMR_ROUND_ALLREDUCE 0
#define OMR_ROUND_REDUCE_SCATTER 1
/*   OMR_ROUND_DENSE_REDUCE_SCATTER  the dense stand-in: the worker scan and the aggregator chain as
 *                             usual, then the WHOLE tensor reduce-scattered (RCCL ncclReduceScatter, ncclSum;
 *                             loopback: omr_dense_sum_f32 in rank order): `out` receives this rank's shard of the
 *                             elementwise sum, every block, zero or not; other rows untouched.  RCCL's summation order
 *                             is its own (results within fp32 reassociation error of the rank-order sum).  Shards
 *                             must be equal: rows % world == 0.  Moves 7/8*S per rank at N=8 whatever the density. */
#define OMR_ROUND_DENSE_REDUCE_SCATTER 2
/* OR-ed into `mode`: only the worker scan runs on `stream`.  The round's bookkeeping (mask all-gather, plan, pack,
 * aggregator chain) goes on the plan's own plan stream, and its exchange and aggregation (send/recv, shard sums
 * [, sums back, unpack]) on its communication stream, so the next call's worker scan overlaps this round's
 * bookkeeping and its transfer over xGMI (the bucket pipeline of a training step).  flags / next_offsets are ready
 * in `stream` order as usual; union_next and `out` are ready once omr_ar_plan_join() has made a stream wait for the
 * round (or after a device-wide synchronise).  Rounds use three plan buffer sets in turn; a round waits for the one
 * three calls back before reusing its set.  x and out must stay untouched (and must not be a later round's input)
 * until the round is joined. */
#define OMR_ROUND_ASYNC 0x100
/* OR-ed into `mode`: bracket this round's worker -> aggregator exchange (the grouped send/recv; the dense
 * stand-in's reduce-scatter) with timing events on the stream it runs on; read them with
 * omr_ar_plan_exchange_time().  Measurement only: the events cost host time, so time a sample of rounds. */
#define OMR_ROUND_TIME_EXCHANGE 0x200
/* OR-ed into `mode` (implies OMR_ROUND_ASYNC): a deeper pipeline.  The call queues this round's first half (worker
 * scan on `stream`; mask all-gather, plan, pack, aggregator chain on the plan stream) and only then issues the
 * exchange and aggregation of the deferred round TWO calls back on the communication stream; this round's follow two
 * deferred calls later, at a call without this flag, or at omr_ar_plan_join().  The host therefore never waits for
 * block counts: that round's counts have been in host memory since the middle of the previous round's scan, and
 * the caller's stream always has the next scan queued.  *sent_blocks / *union_blocks receive the values of the
 * round whose exchange this call issued (0 if none).  Every rank must use the same sequence of modes; join (or a non-deferred call) before
 * reading `out` or destroying the plan (destroy issues a pending exchange and synchronises the device). */
#define OMR_ROUND_DEFER 0x400
/* OR-ed into `mode` (implies OMR_ROUND_ASYNC; combines with OMR_ROUND_DEFER): the call only queues the worker scan
 * on `stream`.  A progress thread of the plan then issues everything else (steps 2-7 above, every host API call and
 * transport call of the round) in call order, so the host cost of a round is split over two cores.  The round's
 * stream order, results and buffer rules are those of OMR_ROUND_ASYNC / OMR_ROUND_DEFER.  *sent_blocks /
 * *union_blocks receive 0: the counts are not known when the call returns.  A call runs at most two rounds
 * ahead of the thread.  An error in the thread is returned by the next call on the plan (and by omr_ar_plan_join).
 * Calls without this flag, omr_ar_plan_join, the timing reads and omr_ar_plan_shard first wait until the thread
 * has issued every queued round.  Transports are driven from the thread: RCCL, the IPC and the loopback
 * transports all allow it. */
#define OMR_ROUND_THREAD 0x800
int omr_sparse_round_f32(omr_ar_plan* plan, const float* x, float* out, int32_t* flags, uint32_t* next_offsets,
                         uint32_t* union_next, int mode, uint64_t* sent_blocks, uint64_t* union_blocks,
                         omr_stream_t stream);
/* Duration of the last OMR_ROUND_TIME_EXCHANGE round's exchange (waits for it), with the bytes this rank sent
 * to and received from its peers in it (bytes_out / bytes_in may be NULL).  OMR_EINVAL if no round was timed. */
int omr_ar_plan_exchange_time(omr_ar_plan* plan, float* ms, uint64_t* bytes_out, uint64_t* bytes_in);
/* A whole gradient of total_n floats (a multiple of the plan's n: one bucket), reduced in place bucket by bucket,
 * one round per bucket with the next bucket's worker scan queued before the previous bucket's exchange
 * (OMR_ROUND_DEFER).  mode: OMR_ROUND_ALLREDUCE or OMR_ROUND_REDUCE_SCATTER (the rank's shard of every bucket).
 * buf is device memory, or PINNED HOST memory (the reference's registered region res->buf, common.cc:873-914, that
 * the worker fills and gets the results back in: client.cc:89, :401-421): then buckets come in through a ring of
 * four device buffers (H2D of bucket k+1 beside bucket k's scan and the earlier buckets' exchanges), each round
 * stores its write set (union + lane heads; the shard's, for reduce-scatter) straight into the pinned buffer
 * through its device mapping, and the call returns once the host buffer holds the result (a buffer without a
 * mapping, or OMR_BUCKETS_STAGED_D2H set: each bucket, or the rank's shard, is copied back whole instead).  A
 * one-rank group with a mapped buffer stages nothing: each bucket's round is one launch that reads the bucket from
 * host memory and stores its write set back into it.  Device memory: returns with the work enqueued on `stream`
 * (joined).  *sent_blocks / *union_blocks: sums over the buckets. */
int omr_sparse_buckets_f32(omr_ar_plan* plan, float* buf, uint64_t total_n, int mode, uint64_t* sent_blocks,
                           uint64_t* union_blocks, omr_stream_t stream);
/* Means over the OMR_ROUND_TIME_EXCHANGE rounds issued since the last call (at most the last 64): the worker scan
 * kernel (events on the round's stream around omr_worker_scan_f32), the worker -> aggregator exchange and its bytes
 * per rank; *rounds = how many rounds were timed.  Waits for those rounds' events. */
int omr_ar_plan_timings(omr_ar_plan* plan, float* scan_ms, float* exchange_ms, uint64_t* bytes_out, uint64_t* bytes_in,
                        uint32_t* rounds);
/* As omr_ar_plan_timings, per stage of the timed rounds: stage_ms[OMR_ROUND_STAGES] = the means of
 *   [0] the worker scan (the caller's stream),
 *   [1] the bookkeeping: mask all-gather, plan (+ aggregator chain), pack (the plan stream when asynchronous),
 *   [2] the worker -> aggregator exchange,
 *   [3] the aggregation after it: shard sums [, sums back to the workers, unpack] (the communication stream),
 * each from HIP events on the stream it runs on (a stage's time includes what that stream does meanwhile, e.g. a
 * transport's waits). */
#define OMR_ROUND_STAGES 4
int omr_ar_plan_stage_timings(omr_ar_plan* plan, float* stage_ms, uint64_t* bytes_out, uint64_t* bytes_in,
                              uint32_t* rounds);
/* 1 if the plan's worker scan packs the blocks for the exchange itself (omr_worker_scan_pack_f32: every shard is
 * whole column segments of the scan, world > 1), 0 if a separate pack pass does
 * (omr_move_blocks_f32). */
int omr_ar_plan_fused_pack(const omr_ar_plan* plan);
/* Device memory the plan holds (bytes), through its transport: per round set the masks, write set, prefixes and pair
 * list; three send buffers of the tensor less this rank's own shard (the exchange's streams, then an all-reduce's
 * returned sums); one receive buffer for this shard's blocks from the other workers; this shard's sums; the scan's
 * flags / next offsets when the caller passes none; and, once omr_sparse_buckets_f32 has staged a host gradient, its
 * four staging buckets.  A 256 MiB plan at world 8 holds about 3.6 x the tensor (round 5; 9 x before). */
uint64_t omr_ar_plan_device_bytes(const omr_ar_plan* plan);
/* Make `stream` wait for every OMR_ROUND_ASYNC round issued so far on this plan (no-op if none). */
int omr_ar_plan_join(omr_ar_plan* plan, omr_stream_t stream);
/* The asynchronous rounds' side streams: 2 (the default at world > 1, except over IPC where more than 4 ranks share this
 * rank's GPU and their hardware queues add up) = a plan stream for the mask all-gather and the
 * plan, an exchange stream for the exchange, the shard sums and the return trip, so round k-2's exchange runs beside
 * round k's plan; 1 (the default at world 1) = everything after the scan on one stream, in issue order.  Which is
 * faster depends on how the process's streams share its hardware queues: bench.py's N>1 lines measure
 * both on the node.  Issues every queued round's remaining steps first; rounds after the call use the new layout.
 * Returns OMR_EINVAL for n other than 1 or 2. */
int omr_ar_plan_set_side_streams(omr_ar_plan* plan, int n);
int omr_ar_plan_side_streams(const omr_ar_plan* plan);
/* Side streams on hardware queues of their own (round 6).  HIP maps each stream onto one of the process's hardware
 * queues when it is made, and streams that share one run as one FIFO: a side-stream step queued between two worker
 * scans then holds the next scan.  So before the first asynchronous round on a caller's stream (again
 * whenever the caller's stream changes, or after omr_ar_plan_set_side_streams) the plan drains its side streams and
 * probes them: a one-wave kernel holds one stream's queue while a mark is queued on the other; a side stream whose mark
 * cannot run while the caller's queue (or the other side stream's) is held is replaced by a fresh stream that passes
 * (up to six tried).  About a millisecond once per caller stream.  On by default, except for the loopback transport
 * (threads sharing one process's queues) and IPC ranks that share their GPU with other ranks (their processes' queues
 * oversubscribe the hardware's, so a probe would time the other ranks' load); omr_ar_plan_set_queue_check(plan, 0|1)
 * overrides it.
 * omr_ar_plan_queue_report: *disjoint = 1 when the last check left every side stream on a queue of its own, 0 when
 * some stream still shares one, -1 before any check; *probes / *replaced count the probes run and the side streams
 * replaced so far (any pointer may be NULL). */
int omr_ar_plan_set_queue_check(omr_ar_plan* plan, int on);
int omr_ar_plan_queue_report(const omr_ar_plan* plan, int* disjoint, int* probes, int* replaced);
/* Join, then wait on the host until `stream` has run every round issued so far: the bounded counterpart of a stream
 * synchronise for a rank whose rounds wait on its peers.  Past the transport's deadline (or on a failure signal) the
 * transport is aborted and OMR_ETIMEDOUT / the error is returned, instead of blocking on a peer that is gone. */
int omr_ar_plan_wait(omr_ar_plan* plan, omr_stream_t stream);
/* The plan's first failure (0: none); see failure containment above. */
int omr_ar_plan_failed(omr_ar_plan* plan);
/* The calling thread's time blocked inside this plan's calls since the last reset, in microseconds (the wait for a
 * round's block counts, the set-reuse and drain waits on the progress thread), and how many waits: a round's host
 * ISSUE time is its call time minus this.  reset != 0 zeroes them after reading. */
int omr_ar_plan_host_stats(omr_ar_plan* plan, double* wait_us, uint64_t* waits, int reset);

/* ---------------------------------------------------------------- the round as wire messages between processes
 *
 * The reference's message protocol between separate worker and aggregator processes: each
 * worker packs its messages of every global slot gs (client.cc:180-205, :113-127; wire format common.cc:399-443)
 * and sends them to aggregator gs % n (common.cc:381-383); aggregator j replies to its slots (server.cc:56-199,
 * rank-order sums from +0.0f) and sends the replies to every worker, which applies them in place (client.cc:87-90).
 * Roles as omr_ar_plan_create_roles (num_workers == world: every rank also aggregates; n = world; otherwise ranks
 * >= num_workers are the n = world - num_workers aggregators).  num_lanes must be NUM_SLOTS*MESSAGE_SIZE/block_size.
 * Logs: one 2*MESSAGE_SIZE-float message per (slot, protocol round), grown to the longest slot (about num_parts*16 *
 * rows_per_part * 8 KiB per worker log at worst: a fidelity path for small tensors).  omr_msgd_round_f32
 * synchronises `stream` once (the schedule's round counts size the transfers); an aggregator passes x = out = NULL.
 * omr_msgd_logs: a worker's own log (worker == its rank) or, on an aggregator, the log it received from `worker`;
 * the replies it holds (a worker: every slot's; an aggregator: its own slots'). */
typedef struct omr_msgd_plan omr_msgd_plan;
int omr_msgd_plan_create(omr_dist* d, uint32_t num_workers, uint64_t n, uint32_t block_size, uint32_t num_lanes,
                         uint32_t num_parts, omr_msgd_plan** out);
int omr_msgd_plan_destroy(omr_msgd_plan* plan);
int omr_msgd_round_f32(omr_msgd_plan* plan, const float* x, float* out, uint32_t* max_rounds, omr_stream_t stream);
int omr_msgd_logs(omr_msgd_plan* plan, uint32_t worker, float** messages, uint32_t** imm, float** replies,
                  uint32_t** reply_imm, uint32_t** rounds, uint32_t* round_capacity);

#ifdef __cplusplus
}
#endif
#endif /* OMR_DIST_H */
