/*
 * omr.h — C ABI of the MI355X-native OmniReduce sparse-block hot path.
 *
 * This is the drop-in boundary for the two hot loops of Phlix1/OmniReduce-RDMA-Demo:
 *   - the worker-side non-zero-block scan   (reference client.cc:19-31, driven from client.cc:87-102, :191-205)
 *   - the aggregator-side per-block fp32 sum (reference server.cc:83-99, the add at server.cc:97-98)
 * on the block/lane/partition layout fixed by reference common.h:27-42.
 *
 * The reference has no plugin/FFI API of its own: its seams are internal C++ calls on `struct resources*`
 * (common.h:79-105, :106-128).  Each entry point below names the reference function/loop it replaces.
 *
 * Conventions:
 *   - plain C types only; every buffer is caller-owned; device pointers unless a parameter says "host";
 *   - `omr_stream_t` is a hipStream_t (NULL = the default stream); every launch is asynchronous on it and
 *     performs no allocation and no host synchronisation, so a caller may capture calls into a hipGraph;
 *   - return 0 on success, OMR_EINVAL (<0) on a bad argument (message in omr_last_error()), or a positive
 *     hipError_t code if a launch failed;
 *   - calls on disjoint buffers/streams are safe to issue concurrently (the reference runs one pthread per
 *     partition on disjoint ranges, client.cc:384-392).
 *
 * Layout vocabulary (reference common.h:27-42):
 *   n            floats in the gradient tensor (DATA_SIZE, common.h:40)
 *   block_size   floats per block (BLOCK_SIZE, common.h:32); supported: 256, 512, 1024
 *   num_lanes    NUM_BLOCKS = NUM_SLOTS*MESSAGE_SIZE/BLOCK_SIZE (common.h:36-37): 64 at B=256, 16 at B=1024
 *   num_parts    NUM_THREADS partitions of n/num_parts floats each (common.h:35, :38)
 *   block b      floats [b*B, (b+1)*B); lane bid = b % num_lanes (client.cc:23, server.cc:85)
 *   row          num_lanes consecutive blocks (one block per lane); a partition is rows_per_part rows
 *   offset       uint32 float-element index of a block's first element (client.cc:19, common.cc:407)
 *   sentinel     omr_sentinel(B, num_lanes) + bid*B marks "no further non-zero block in this lane"
 *                (client.cc:24, :42; server.cc:16)
 *   row mask     uint64 per row, bit l set iff block (row, lane l) is non-zero  (this build's compact flag form)
 */
#ifndef OMR_H
#define OMR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OMR_ABI_VERSION 2
#define OMR_EINVAL (-1)
#define OMR_MAX_WORKERS 16 /* reference caps peers at 10: common.h:59 peer_names[10] */

/* Reference layout constants (common.h:31, :36). */
#define OMR_MESSAGE_SIZE 1024u
#define OMR_NUM_SLOTS 16u
#define OMR_NUM_THREADS 8u

typedef void* omr_stream_t; /* hipStream_t */

/* ---------------------------------------------------------------- layout helpers (common.h:27-42) */

int omr_abi_version(void);
const char* omr_last_error(void);

/* NUM_BLOCKS for a block size: NUM_SLOTS*MESSAGE_SIZE/BLOCK_SIZE (common.h:33, :36-37). */
uint32_t omr_num_lanes(uint32_t block_size);

/* Sentinel base (UINT32_MAX/B/NB-1)*NB*B = 4294934528 for every supported B (client.cc:24, server.cc:16). */
uint32_t omr_sentinel(uint32_t block_size, uint32_t num_lanes);

/* 0 iff (n, B, NB, parts) is a layout this library runs: B in {256,512,1024}, NB*B a multiple of 256,
 * NB <= 64, n a multiple of parts*NB*B, n <= sentinel base (uint32 offsets, client.cc:24). */
int omr_layout_check(uint64_t n, uint32_t block_size, uint32_t num_lanes, uint32_t num_parts);

/* ---------------------------------------------------------------- synthetic input (client.cc:396-421) */

/* Reference generator: srand(worker_id+1); for every block i in order,
 * bitmap[i] = (rand()%100/(double)101 < density_ratio) (client.cc:396, :406-414).
 * glibc rand() is restated (TYPE_3 additive feedback) so the library does not touch the process-global
 * libc generator.  `bitmap` is HOST memory.  *nonzero_count (may be NULL) gets the count (client.cc:410). */
int omr_gen_bitmap(uint32_t worker_id, double density_ratio, uint64_t num_blocks, int32_t* bitmap,
                   uint64_t* nonzero_count);

/* Fill `buf` (n = num_blocks*block_size floats, device) from a device bitmap:
 * mode 0: the reference fill, 0.01f in flagged blocks and 0 elsewhere (client.cc:401-404, :415-419);
 * mode 1: flagged blocks get uniform [-1,1) values from a counter hash of (seed, element index), others 0
 *         (the random-valued tolerance variant of SURVEY.md §8d). */
int omr_fill_blocks_f32(const int32_t* bitmap, uint64_t num_blocks, uint32_t block_size, int mode,
                        uint32_t seed, float* buf, omr_stream_t stream);

/* ---------------------------------------------------------------- ★1 worker scan (client.cc:19-31) */

/* Worker-side non-zero-block scan of one fp32 gradient (replaces find_next_nonzero_block, client.cc:19-31,
 * and its drivers client.cc:87-102 / :191-205, with the flag derived from the data as north_star requires
 * instead of the generator's precomputed bitmap, client.cc:26):
 *   flags[b]        (int32, may be NULL)   1 iff some element of block b is != 0.0f (-0.0 counts as zero,
 *                                          NaN as non-zero); the reference's `int *bitmap` (common.h:98)
 *   row_masks[r]    (uint64, required)     bit l = flags[r*NB + l]
 *   next_offsets[b] (uint32, may be NULL)  find_next_nonzero_block(b*B + B*NB): offset of the first non-zero
 *                                          block after b in the same lane and partition, else sentinel+bid*B
 */
int omr_scan_f32(const float* buf, uint64_t n, uint32_t block_size, uint32_t num_lanes, uint32_t num_parts,
                 int32_t* flags, uint64_t* row_masks, uint32_t* next_offsets, omr_stream_t stream);

/* ---------------------------------------------------------------- ★1+★3 fused scan + aggregation */

/* m worker scans plus the aggregator sum in one HBM pass over the m tensors (server.cc:83-99):
 *   bufs            HOST array of m device pointers (worker rank order), 1 <= m <= OMR_MAX_WORKERS
 *   flags           [m][nb] int32 per-worker flags, or NULL
 *   row_masks       [m][rows] per-worker row masks, then (m > 1 only) [rows] union masks at index m
 *   next_offsets    [m][nb] per-worker chains, then (m > 1 only) [nb] aggregator chain = next over the union
 *                   (server.cc:86-96: min over workers of their next offsets), or NULL
 *   out             dense fp32[n] or NULL: for every block that is non-zero in some worker, and for every
 *                   lane-head block (row 0 of a partition, always sent: client.cc:201-205), out block =
 *                   ((0.0f + x_0) + x_1) + ... + x_{m-1} (rank order, accumulator zeroed first as at
 *                   server.cc:148-150); other blocks of `out` are not written (pass a worker's own buffer
 *                   for the reference's in-place result, client.cc:89). out may alias bufs[i].
 */
int omr_scan_sum_f32(const float* const* bufs, uint32_t m, uint64_t n, uint32_t block_size,
                     uint32_t num_lanes, uint32_t num_parts, int32_t* flags, uint64_t* row_masks,
                     uint32_t* next_offsets, float* out, omr_stream_t stream);

/* Single-pass m = 1 worker step (one launch): flags, next offsets AND the aggregated blocks, computed per
 * (partition, lane) column so that every find_next_nonzero_block chain (client.cc:19-31) is resolved inside one
 * workgroup.  Same outputs as omr_scan_sum_f32 with m = 1 (row masks are not produced).  When the layout has too
 * few columns to fill the chip (e.g. B = 1024), columns are split into segments that meet through device
 * atomics in `workspace`: omr_scan_workspace_bytes() bytes (0 = none needed), zero-filled once by the caller
 * (e.g. hipMemset), left zeroed by every call; one workspace per concurrently running call. */
size_t omr_scan_workspace_bytes(uint64_t n, uint32_t block_size, uint32_t num_lanes, uint32_t num_parts);
int omr_scan_sum_fused_f32(const float* buf, uint64_t n, uint32_t block_size, uint32_t num_lanes,
                           uint32_t num_parts, int32_t* flags, uint32_t* next_offsets, float* out, void* workspace,
                           size_t workspace_bytes, omr_stream_t stream);

/* The single-pass worker step for ONE partition `part` (< num_parts) of the tensor: the per-thread seam of the
 * reference, where worker thread `res->threadId` walks only its own DATA_SIZE_PER_THREAD slice (client.cc:22-29,
 * :168-223; threads started at client.cc:384-392).  Writes flags / next_offsets / out for that partition's blocks
 * only (global block indexing, global float offsets in next_offsets); other partitions are untouched.  Calls on
 * different partitions may run concurrently on different streams and may share one workspace (each partition uses
 * its own counters in it): omr_scan_workspace_bytes(n, ...) bytes, zero-filled once, left zeroed. */
int omr_scan_partition_f32(const float* buf, uint64_t n, uint32_t block_size, uint32_t num_lanes, uint32_t num_parts,
                           uint32_t part, int32_t* flags, uint32_t* next_offsets, float* out, void* workspace,
                           size_t workspace_bytes, omr_stream_t stream);

/* The m = 1 fused scan + aggregate over rows [row_begin, row_end) only (a pipelined piece of the tensor, e.g.
 * the part that has landed from host memory); `buf`, `out`, `flags`, `row_masks` are whole-tensor arrays indexed
 * by global block/row.  Next offsets need every row: run omr_next_offsets once all pieces are scanned. */
int omr_scan_sum_rows_f32(const float* buf, uint64_t n, uint32_t block_size, uint32_t num_lanes,
                          uint32_t num_parts, uint64_t row_begin, uint64_t row_end, int32_t* flags,
                          uint64_t* row_masks, float* out, omr_stream_t stream);

/* Next-offset chains from row masks (client.cc:19-31 for one worker; for a union mask, the aggregator's
 * min_next chain server.cc:86-96).  `count` mask arrays of `rows` each, stride `rows`; output stride nb. */
int omr_next_offsets(const uint64_t* row_masks, uint32_t count, uint64_t n, uint32_t block_size,
                     uint32_t num_lanes, uint32_t num_parts, uint32_t* next_offsets, omr_stream_t stream);

/* ---------------------------------------------------------------- ★3 aggregator sum over a block list */

/* For each listed global block index b: out[b*B + j] = ((0.0f + in_0) + in_1) + ... for j < B
 * (server.cc:97-98 in rank order; the accumulator zeroing of server.cc:148-150 is the 0.0f start).
 * `inputs` is a HOST array of m device pointers, dense layout. */
int omr_block_sum_f32(const float* const* inputs, uint32_t m, const uint32_t* block_list, uint32_t num_list,
                      uint32_t block_size, float* out, omr_stream_t stream);

/* The dense stand-in aggregator: out[i] = ((0.0f + in_0[i]) + in_1[i]) + ... for every i < n (all blocks, zero
 * or not; rank order as server.cc:97-98).  `inputs` is a HOST array of m device pointers; n a multiple of 4,
 * pointers 16-byte aligned; out may alias an input. */
int omr_dense_sum_f32(const float* const* inputs, uint32_t m, uint64_t n, float* out, omr_stream_t stream);

/* ---------------------------------------------------------------- compaction and block movement */

/* Bytes of device workspace omr_compact needs for `rows` rows. */
size_t omr_compact_workspace_bytes(uint64_t rows);

/* List the set bits of row masks in increasing block order: block_list[k] = global block index
 * (row*NB + lane) of the k-th non-zero block; *count (device uint32) = total.  Rows [row_begin, row_end). */
int omr_compact(const uint64_t* row_masks, uint64_t row_begin, uint64_t row_end, uint32_t num_lanes,
                uint32_t* block_list, uint32_t* count, void* workspace, size_t workspace_bytes,
                omr_stream_t stream);

/* Pack listed blocks contiguously (the worker-side gather of common.cc:405-407) / scatter them back in
 * place (the worker-side result copy of client.cc:89). */
int omr_gather_blocks_f32(const float* src, const uint32_t* block_list, uint32_t num_list,
                          uint32_t block_size, float* packed, omr_stream_t stream);
int omr_scatter_blocks_f32(const float* packed, const uint32_t* block_list, uint32_t num_list,
                           uint32_t block_size, float* dst, omr_stream_t stream);

/* ---------------------------------------------------------------- multi-GPU sparse exchange helpers */

/* out[r] = OR of `count` mask arrays (stride `rows`) — the union the aggregator's min_next chain runs over
 * (server.cc:86-96); with heads != 0 every lane-head row (r % rows_per_part == 0) is forced to all lanes,
 * giving the set of blocks the aggregator returns (lane heads are always sent: client.cc:201-205). */
int omr_mask_union(const uint64_t* row_masks, uint32_t count, uint64_t rows, uint32_t rows_per_part,
                   uint32_t num_lanes, int heads, uint64_t* out, omr_stream_t stream);

/* Exclusive prefix of per-row popcounts: prefix[a*(rows+1) + r] = set bits of array a in rows [0, r). */
size_t omr_prefix_workspace_bytes(uint64_t rows, uint32_t count);
int omr_row_prefix(const uint64_t* row_masks, uint32_t count, uint64_t rows, uint32_t* prefix, void* workspace,
                   size_t workspace_bytes, omr_stream_t stream);

/* Aggregator shard sum over packed worker streams (server.cc:83-99 with the RDMA hop replaced by RCCL):
 * worker w's stream holds its non-zero blocks of rows [row_begin, ...) in increasing order, starting at block
 * recv_offsets[w] (device uint64[count]) of `recv`.  For the k-th listed global block b:
 * out[k*B + j] = ((0.0f + x_w0[b][j]) + x_w1[b][j]) + ... over the workers whose mask has b, in rank order. */
int omr_sparse_block_sum_f32(const float* recv, const uint64_t* recv_offsets, const uint64_t* row_masks,
                             uint32_t count, uint64_t rows, const uint32_t* prefix, uint64_t row_begin,
                             uint32_t num_lanes, const uint32_t* block_list, uint32_t num_list,
                             uint32_t block_size, float* out, omr_stream_t stream);

/* ---------------------------------------------------------------- multi-rank round, mask-addressed */

/* Single-pass worker scan for a multi-rank round (client.cc:19-31 + :87-102 over the whole tensor): as
 * omr_scan_sum_fused_f32 (flags, next offsets, and out if non-NULL), plus row masks: the bit of every non-zero
 * block is OR-ed into row_masks (device uint64[rows], all zero on entry). */
int omr_worker_scan_f32(const float* buf, uint64_t n, uint32_t block_size, uint32_t num_lanes, uint32_t num_parts,
                        int32_t* flags, uint32_t* next_offsets, uint64_t* row_masks, float* out, void* workspace,
                        size_t workspace_bytes, omr_stream_t stream);

/* The round's worker scan with the worker's pack fused in (the multi-rank round's form; common.cc:399-407): as
 * omr_worker_scan_f32, and every non-zero block of a row of shard s != own_shard is also written to `send`, so no
 * separate pass re-reads the blocks to pack them.  Shards: rows [shard_bounds[s], shard_bounds[s+1]) (HOST uint64,
 * num_shards + 1 entries, 0 .. rows), each made of whole column segments of the scan (omr_pack_supported says
 * whether a set of bounds is; a ragged shard packs with omr_move_blocks_f32 instead).  The streams follow one another
 * in shard order without own_shard's: shard s's starts at send + (shard_bounds[s] - (s > own_shard ? own_shard's rows :
 * 0)) * num_lanes * block_size floats (send: device, n floats less own_shard's rows; omr_pack_send_offset gives the
 * offset), and holds its non-zero blocks segment by segment (column segments of omr_pack_geometry's seg_rows rows),
 * each segment's in row order; segments
 * take their places in completion order through shard_counters (device uint32[num_shards], zero on entry: after the
 * call counter s = the stream's block count).  pos_table (device uint32[table_entries]) receives for each
 * (segment, 64-row group g, lane l) the stream position of the first block of lane l at or after row 64 g of the
 * segment: the aggregator's address of block (row r, lane l) is pos + the lane's set bits in the group below r
 * (the pair list of omr_sum_list_build / omr_round_plan_list).  Entries of segments with no non-zero block, and of
 * own_shard's, are not written.
 * own_shard: -1 packs every shard (a worker that aggregates none). */
int omr_worker_scan_pack_f32(const float* buf, uint64_t n, uint32_t block_size, uint32_t num_lanes, uint32_t num_parts,
                             int32_t* flags, uint32_t* next_offsets, uint64_t* row_masks, float* out,
                             const uint64_t* shard_bounds, uint32_t num_shards, int32_t own_shard, float* send,
                             uint32_t* shard_counters, uint32_t* pos_table, void* workspace, size_t workspace_bytes,
                             omr_stream_t stream);
/* The round check (round 6).  The two worker scans above with check_slots (device
 * uint64[omr_round_check_slots()], or NULL: none): workgroup b also stores check_slots[b] = (check_seq << 32) | the
 * non-zero blocks it found, i.e. the number of row-mask bits it set.  Put in the array the round all-gathers (after
 * the masks and position table), they let the plan launch check on the device that each worker's gathered array is
 * the one its scan of THIS round wrote (omr_round_plan_check).
 * done (device uint32[2], or NULL): the launch's completion, signalled on the device.  done[0] must be zero before the
 * first launch (each launch leaves it zero); the launch's last workgroup to finish stores check_seq (nonzero) into
 * done[1] after every workgroup's stores are visible at device scope, so work on another stream may wait for the word
 * (e.g. a kernel polling done[1] - seq >= 0 as int32) instead of for an event recorded behind the scan. */
uint32_t omr_round_check_slots(uint64_t n, uint32_t block_size, uint32_t num_lanes, uint32_t num_parts);
int omr_worker_scan_check_f32(const float* buf, uint64_t n, uint32_t block_size, uint32_t num_lanes, uint32_t num_parts,
                              int32_t* flags, uint32_t* next_offsets, uint64_t* row_masks, float* out, void* workspace,
                              size_t workspace_bytes, uint64_t* check_slots, uint32_t check_seq, uint32_t* done,
                              omr_stream_t stream);
int omr_worker_scan_pack_check_f32(const float* buf, uint64_t n, uint32_t block_size, uint32_t num_lanes,
                                   uint32_t num_parts, int32_t* flags, uint32_t* next_offsets, uint64_t* row_masks,
                                   float* out, const uint64_t* shard_bounds, uint32_t num_shards, int32_t own_shard,
                                   float* send, uint32_t* shard_counters, uint32_t* pos_table, void* workspace,
                                   size_t workspace_bytes, uint64_t* check_slots, uint32_t check_seq, uint32_t* done,
                                   omr_stream_t stream);
/* The one-rank round's worker scan (a world-1 group: one worker, one aggregator; server.cc:83-96 with one worker:
 * the union is the worker's own blocks and min_next its own chain, so the aggregator's bookkeeping is two counts).
 * As omr_scan_sum_fused_f32 (flags, next offsets, out = 0.0f + x over the write set if non-NULL), plus
 *   tally (device uint64[omr_tally_slots()]): workgroup b stores {non-zero blocks, zero lane-head blocks} of its part
 *   as (heads << 32) | non-zero (one slot per workgroup, overwritten by every launch);
 *   publish_src / publish_dst (both or neither): workgroup 0 of the same launch sums an EARLIER launch's slots (same
 *   layout) and stores {publish_seq, non-zero blocks, write-set blocks = non-zero + zero lane heads (client.cc:201-205),
 *   publish_seq} (one 16-byte system-scope store) into publish_dst (host-mapped, 16-byte aligned).  A host that reads
 *   publish_seq in both halves has the counts.
 * So a pipelined one-rank round is ONE launch on the caller's stream (no event, no side stream). */
uint32_t omr_tally_slots(uint64_t n, uint32_t block_size, uint32_t num_lanes, uint32_t num_parts);
int omr_worker_scan_tally_f32(const float* buf, uint64_t n, uint32_t block_size, uint32_t num_lanes, uint32_t num_parts,
                              int32_t* flags, uint32_t* next_offsets, float* out, uint64_t* tally,
                              const uint64_t* publish_src, uint32_t* publish_dst, uint32_t publish_seq, void* workspace,
                              size_t workspace_bytes, omr_stream_t stream);
/* The same publication as a launch of its own (one wave): for a round no later scan follows. */
int omr_tally_publish(const uint64_t* tally, uint32_t slots, uint32_t* dst, uint32_t seq, omr_stream_t stream);
/* The fused pack's geometry on this layout: rows per column segment, 64-row groups per segment, position-table
 * entries (num_parts * segments per partition * groups * num_lanes); and whether shard bounds (HOST) are whole
 * segments (0, else OMR_EINVAL with the reason). */
int omr_pack_geometry(uint64_t n, uint32_t block_size, uint32_t num_lanes, uint32_t num_parts, uint32_t* seg_rows,
                      uint32_t* groups_per_seg, uint64_t* table_entries);
int omr_pack_supported(uint64_t n, uint32_t block_size, uint32_t num_lanes, uint32_t num_parts,
                       const uint64_t* shard_bounds, uint32_t num_shards);
/* Where shard s's stream starts in omr_worker_scan_pack_f32's `send` (floats), and the floats `send` needs (*total;
 * NULL: not asked), for shard bounds in rows (HOST, num_shards + 1 entries) and own_shard (-1: none). */
uint64_t omr_pack_send_offset(const uint64_t* shard_bounds, uint32_t num_shards, int32_t own_shard, uint32_t s,
                              uint32_t num_lanes, uint32_t block_size, uint64_t* total);

/* The aggregator bookkeeping of a round in ONE launch (server.cc:83-96, for the whole tensor at once), from
 * `count` workers' row masks (device, stride rows):
 *   union_masks[r] = OR of the workers' masks (the domain of the min_next chain, server.cc:86-96);
 *   write_set[r]   = union_masks[r], with every lane of a lane-head row (r % rows_per_part == 0) set: the blocks
 *                    the aggregators return (lane heads are always sent: client.cc:201-205);
 *   prefix[a*(rows+1) + r] = set bits of array a in rows [0, r), for a < count (workers) and a == count (the
 *                    write set); r = rows gives the total;
 *   counts[a*num_bounds + s] = (seq << 32) | prefix[a][bounds[s]] (bounds: device uint64[num_bounds], each <= rows),
 *                    stored at system scope: counts may be pinned host memory (mapped), and a host that polls them
 *                    until every one it needs carries `seq` has them without synchronising the stream (the
 *                    multi-rank round does);
 *   zero_masks (device uint64[rows] or NULL) is cleared (the next round's omr_worker_scan_f32 target);
 *   union_masks may be NULL (not stored).
 * workspace: device uint64[omr_round_plan_workspace_words()], zero-filled before its first launch and left to the
 * plan between launches (the kernel re-arms it); launches sharing a workspace run in stream order.  seq != 0 and must
 * not repeat the seq of ANY earlier launch on the same workspace and counts (a strictly increasing counter, as the
 * multi-rank round's, skipping 0 when it wraps): chunk totals are tagged, never cleared, so a launch with an earlier
 * launch's seq could take that launch's stale totals for chunks it has more of.  Row chunks of the launch
 * run side by side and hand each other their popcount totals through the workspace (ABI 2; ABI 1 took an arrival
 * counter); the round check (omr_round_plan_check) hands the last chunk its findings there too (1106 words since
 * round 6). */
uint64_t omr_round_plan_workspace_words(void);
int omr_round_plan(const uint64_t* row_masks, uint32_t count, uint64_t rows, uint32_t rows_per_part,
                   uint32_t num_lanes, const uint64_t* bounds, uint32_t num_bounds, uint64_t* write_set,
                   uint64_t* union_masks, uint32_t* prefix, uint64_t* counts, uint64_t* zero_masks,
                   uint64_t* workspace, uint32_t seq, omr_stream_t stream);
struct omr_sum_list;
/* omr_round_plan with worker c's masks at row_masks + c * mask_stride (mask_stride >= rows: the all-gathered arrays
 * of the fused pack carry each worker's position table after its masks), plus, in the same launch:
 *   zero_counters (device uint32[num_zero_counters <= 256], or NULL) cleared: the next round's pack counters;
 *   union_next (device uint32[rows * num_lanes], or NULL): the aggregator chain (server.cc:86-96: min_next over
 *     the workers = next offsets over the union, the omr_next_offsets layout of the union masks), computed by
 *     extra workgroups from the workers' masks directly;
 *   list (or NULL): an aggregator's shard-sum pair list (omr_sum_list below) over the layout (rows * num_lanes *
 *     block_size floats, rows / rows_per_part partitions). */
int omr_round_plan_list(const uint64_t* row_masks, uint32_t count, uint64_t mask_stride, uint64_t rows,
                        uint32_t rows_per_part, uint32_t num_lanes, const uint64_t* bounds, uint32_t num_bounds,
                        uint64_t* write_set, uint64_t* union_masks, uint32_t* prefix, uint64_t* counts,
                        uint64_t* zero_masks, uint32_t* zero_counters, uint32_t num_zero_counters,
                        uint64_t* workspace, uint32_t seq, uint32_t* union_next, uint32_t block_size,
                        const struct omr_sum_list* list, omr_stream_t stream);
/* omr_round_plan_list plus the round check, by one more workgroup of the launch (check_status NULL: none): worker c's
 * check slots are words [check_offset, check_offset + check_slots) of its array (row_masks + c * mask_stride); the
 * check stores *check_status = (seq << 32) | code at system scope (it may be pinned host memory, polled as the
 * counts): 0 when every slot carries `seq` and each worker's slots add up to its masks' popcount; 0x100 + c when a
 * slot of worker c carries another round's seq (its array was read before its scan wrote it, or another buffer was
 * read); 0x200 + c when worker c's masks hold fewer (or other) bits than its scan counted (the array was read before
 * the scan finished: an array only gains bits between the plan that clears it and the scan that refills it). */
int omr_round_plan_check(const uint64_t* row_masks, uint32_t count, uint64_t mask_stride, uint64_t rows,
                         uint32_t rows_per_part, uint32_t num_lanes, const uint64_t* bounds, uint32_t num_bounds,
                         uint64_t* write_set, uint64_t* union_masks, uint32_t* prefix, uint64_t* counts,
                         uint64_t* zero_masks, uint32_t* zero_counters, uint32_t num_zero_counters,
                         uint64_t* workspace, uint32_t seq, uint32_t* union_next, uint32_t block_size,
                         const struct omr_sum_list* list, uint64_t check_offset, uint32_t check_slots,
                         uint64_t* check_status, omr_stream_t stream);

/* Block movement addressed by a row mask and its prefix (no block list): the k-th set bit of `row_masks` over
 * rows [0, rows) minus [skip_begin, skip_end) is block k of the packed stream.
 *   dir 0 (pack, the worker's gather of common.cc:405-407): dst packed <- src dense;
 *   dir 1 (unpack, the worker's in-place result copy of client.cc:89): dst dense <- src packed. */
int omr_move_blocks_f32(const float* src, float* dst, int dir, const uint64_t* row_masks, const uint32_t* prefix,
                        uint64_t rows, uint32_t num_lanes, uint32_t block_size, uint64_t skip_begin,
                        uint64_t skip_end, omr_stream_t stream);

/* Aggregator shard sum (server.cc:83-99 with the RDMA hop replaced by the transport) over rows
 * [row_begin, row_end) of write_set: every write-set block gets ((0.0f + x_a0) + x_a1) + ... over the workers a
 * whose mask has it, in rank order (lane-head blocks no worker has: +0.0f).  Worker `me`'s blocks are read in
 * place from its dense tensor `own`; worker a != me's from recv + recv_offsets[a] blocks (HOST uint64[count]):
 * its non-zero blocks of these rows in block order.  `prefix` as omr_round_plan.  packed_out 0: out is dense
 * (blocks written at their own positions; may alias own); 1: out is packed in write-set order of the rows. */
int omr_shard_sum_f32(const float* own, uint32_t me, const float* recv, const uint64_t* recv_offsets,
                      const uint64_t* row_masks, uint32_t count, const uint32_t* prefix, const uint64_t* write_set,
                      uint64_t rows, uint64_t row_begin, uint64_t row_end, uint32_t num_lanes, uint32_t block_size,
                      int packed_out, float* out, omr_stream_t stream);
/* The same with worker c's masks at row_masks + c * mask_stride (mask_stride >= rows: the round's all-gathered arrays,
 * which carry the round check's slots after the masks). */
int omr_shard_sum_stride_f32(const float* own, uint32_t me, const float* recv, const uint64_t* recv_offsets,
                             const uint64_t* row_masks, uint64_t mask_stride, uint32_t count, const uint32_t* prefix,
                             const uint64_t* write_set, uint64_t rows, uint64_t row_begin, uint64_t row_end,
                             uint32_t num_lanes, uint32_t block_size, int packed_out, float* out, omr_stream_t stream);

/* The shard sum over the fused pack's column-ordered streams (omr_worker_scan_pack_f32; the multi-rank round's form),
 * in two steps: its (block, contributor) pair list, which depends only on the all-gathered masks and position tables
 * and on where each worker's stream will land in `recv`, is built before the exchange (by the plan launch:
 * omr_round_plan_list); the sum then streams the pairs' blocks (server.cc:97-98, rank order from +0.0f: the same sums,
 * bit for bit, as omr_shard_sum_f32 over row-ordered streams).
 *   records  device uint64[units * capacity] (omr_sum_list_geometry: a unit's records end with a terminator word),
 *   counts   device uint32[units] (each unit's record count);
 *   rows [row_begin, row_end): the shard, whole column segments of the layout;
 *   pos_offset: word offset of each worker's position table in its array (2 * rows in the round);
 *   me: the worker whose blocks are read in place from `own` (< count), or count (none: a dedicated aggregator);
 *   recv_offsets[a]: worker a's stream of these rows starts at recv + recv_offsets[a] blocks (< 2^32). */
typedef struct omr_sum_list {
  uint64_t* records;
  uint32_t* counts;
  uint64_t row_begin, row_end;
  uint64_t pos_offset;
  uint32_t me;
  uint64_t recv_offsets[OMR_MAX_WORKERS];
} omr_sum_list;
int omr_sum_list_geometry(uint64_t n, uint32_t block_size, uint32_t num_lanes, uint32_t num_parts, uint64_t row_begin,
                          uint64_t row_end, uint32_t count, uint64_t* units, uint32_t* capacity);
/* Build the list in a launch of its own (worker c's array at row_masks + c * mask_stride, as omr_round_plan_list). */
int omr_sum_list_build(const uint64_t* row_masks, uint32_t count, uint64_t mask_stride, uint64_t n,
                       uint32_t block_size, uint32_t num_lanes, uint32_t num_parts, const omr_sum_list* list,
                       omr_stream_t stream);
/* The sum over a built list.  packed_out 0: out dense (may alias own); 1: out packed in write-set order of the shard's
 * rows, from write_set and its row prefix write_prefix (omr_round_plan's prefix + count * (rows + 1)). */
int omr_shard_sum_list_f32(const float* own, const float* recv, const omr_sum_list* list, uint32_t count, uint64_t n,
                           uint32_t block_size, uint32_t num_lanes, uint32_t num_parts, const uint64_t* write_set,
                           const uint32_t* write_prefix, int packed_out, float* out, omr_stream_t stream);

/* ---------------------------------------------------------------- message-level round (wire format) */

/* The round as the reference's messages, byte for byte, for m workers on one device
 * (the loopback stand-in for m machines): every worker message and aggregator reply of the per-slot state
 * machines (client.cc:32-205, server.cc:13-199), with a protocol round's worker messages arriving in rank order.
 * Wire format (common.cc:399-408, :424, :443, :542): a message occupies a slot of 2*MESSAGE_SIZE floats:
 * `len` blocks of block_size floats, then `len` uint32 next offsets; imm = (len << 16) | global slot (gs = slot +
 * NUM_SLOTS*partition).  Logs (device, valid for round r < rounds[gs]):
 *   messages[(gs*cap + r)*2*MESSAGE_SIZE ...], imm[gs*cap + r]   worker `worker`'s message (imm 0: none sent)
 *   replies [(gs*cap + r)*2*MESSAGE_SIZE ...], reply_imm[...]     the aggregator's reply (the same to every worker)
 * outs[w] (device, may equal bufs[w]) receives worker w's buffer after the round: every reply block written at
 * the worker's current offset of its lane (client.cc:87-90).  num_lanes must be NUM_SLOTS*MESSAGE_SIZE/block_size.
 * omr_msg_round_f32 synchronises `stream` once (the schedule's round count sizes the logs). */
typedef struct omr_msg_plan omr_msg_plan;
int omr_msg_plan_create(uint64_t n, uint32_t block_size, uint32_t num_lanes, uint32_t num_parts, uint32_t m,
                        omr_msg_plan** plan);
int omr_msg_plan_destroy(omr_msg_plan* plan);
int omr_msg_round_f32(omr_msg_plan* plan, const float* const* bufs, float* const* outs, uint32_t* max_rounds,
                      omr_stream_t stream);
int omr_msg_logs(omr_msg_plan* plan, uint32_t worker, float** messages, uint32_t** imm, float** replies,
                 uint32_t** reply_imm, uint32_t** rounds, uint32_t* round_capacity);

/* The same round split into its message primitives, for workers and aggregators in different processes (the
 * reference's separate ./client and ./server machines, common.cc:374-476 -> server.cc:56-199), all on device
 * buffers; a transport moves the logs (omr_dist.h: omr_msgd_*).  Log layout as above: message (gs, r) at
 * [(gs*round_capacity + r) * 2*MESSAGE_SIZE] floats, imm at [gs*round_capacity + r]; gs < num_parts*NUM_SLOTS.
 *   omr_msg_schedule  per slot, the protocol rounds' blocks, message and reply orders (sched: omr_msg_sched_bytes()
 *                     per (slot, round)), rounds[gs], and *max_rounds (device uint32; > round_capacity means the logs
 *                     are too small: redo with a larger capacity), from the m workers' row masks (device [m][rows])
 *                     and the union's next offsets (the aggregator's min_next chain, server.cc:86-96);
 *   omr_msg_pack_f32  one worker's messages of every slot (client.cc:180-205, :113-127; common.cc:399-408);
 *   omr_msg_aggregate_f32  the replies of the slots one aggregator owns: gs % num_aggregators == aggregator
 *                     (common.cc:381-383), from the m workers' logs (HOST arrays of device pointers, rank order):
 *                     rank-order sums from +0.0f (server.cc:97-98, :148-150), completion order, min_next
 *                     (server.cc:143-147);
 *   omr_msg_unpack_f32  a worker applies every reply in place (client.cc:87-90). */
size_t omr_msg_sched_bytes(void);
int omr_msg_schedule(const uint64_t* row_masks, uint32_t m, const uint32_t* union_next, uint64_t n, uint32_t block_size,
                     uint32_t num_lanes, uint32_t num_parts, uint32_t round_capacity, void* sched, uint32_t* rounds,
                     uint32_t* max_rounds, omr_stream_t stream);
int omr_msg_pack_f32(const float* x, const int32_t* flags, const uint32_t* next_offsets, const void* sched,
                     const uint32_t* rounds, uint32_t num_parts, uint32_t round_capacity, uint32_t block_size,
                     float* messages, uint32_t* imm, omr_stream_t stream);
int omr_msg_aggregate_f32(const float* const* messages, const uint32_t* const* imm, uint32_t m, const void* sched,
                          const uint32_t* rounds, const uint32_t* union_next, uint32_t num_parts,
                          uint32_t round_capacity, uint32_t block_size, uint32_t num_lanes, uint32_t num_aggregators,
                          uint32_t aggregator, float* replies, uint32_t* reply_imm, omr_stream_t stream);
int omr_msg_unpack_f32(const float* replies, const uint32_t* reply_imm, const void* sched, const uint32_t* rounds,
                       uint32_t num_parts, uint32_t round_capacity, uint32_t block_size, uint32_t num_lanes,
                       float* buf, omr_stream_t stream);

/* ---------------------------------------------------------------- host-resident end-to-end path */

/* The gradient lives in host memory (the reference's registered region, common.cc:873-914): H2D in row chunks,
 * scan + aggregate of each landed chunk, whose aggregated blocks (non-zero blocks + lane heads, client.cc:89) the
 * kernel stores straight into the pinned buffer through its device mapping while the next chunk comes in (without
 * a mapping, or with OMR_HOST_STAGED_D2H set, each chunk is copied back whole); then the next-offset chains.
 * host_buf should be pinned (omr_host_register or hipHostMalloc).
 * host_flags / host_next (may be NULL) receive the int32 flags / uint32 next offsets.  *seconds = wall time. */
typedef struct omr_host_plan omr_host_plan;
const char* omr_host_last_error(void);
int omr_host_register(void* ptr, size_t bytes);
int omr_host_unregister(void* ptr);
int omr_host_plan_create(uint64_t n, uint32_t block_size, uint32_t num_lanes, uint32_t num_parts,
                         uint64_t chunk_rows, omr_host_plan** plan);
int omr_host_plan_destroy(omr_host_plan* plan);
int omr_host_scan_sum_f32(omr_host_plan* plan, float* host_buf, int32_t* host_flags, uint32_t* host_next,
                          double* seconds);
/* The same round without staging copies: the single-pass kernel (omr_scan_sum_fused_f32) reads the pinned host
 * buffer over PCIe and writes the aggregated blocks (non-zero blocks + lane heads) straight back into it, in place
 * (client.cc:89); only the flag / next arrays travel as copies.  The link carries S one way and the written blocks
 * the other, at once.  host_buf must be pinned (omr_host_register or hipHostMalloc), else OMR_EINVAL. */
int omr_host_scan_sum_zero_copy_f32(omr_host_plan* plan, float* host_buf, int32_t* host_flags, uint32_t* host_next,
                                    double* seconds);

#ifdef __cplusplus
}
#endif
#endif /* OMR_H */
