/*
 * omr_oracle.c — CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library, and only as
 * the checker (or the timed CPU baseline) — never as the product path.  The product is the HIP library
 * behind include/omr.h.
 *
 * Every function restates a piece of Phlix1/OmniReduce-RDMA-Demo (read-only at /root/reference) and cites
 * it.  Parity pinning: the reference cannot be built here — common.h:22 includes
 * <infiniband/verbs.h> and the Makefile links -libverbs (Makefile:8), neither of which this image has — and
 * it holds no tests, fixtures or golden vectors.  The oracle is therefore pinned by
 *   (1) the reference's own generator: glibc srand/rand are called directly, exactly as client.cc:396-414
 *       does, so the bitmaps ARE the reference's bitmaps;
 *   (2) the reference's own known-answer check (client.cc:449-465): after the round every worker's buffer
 *       equals the elementwise MPI_SUM of all workers' inputs, compared with `!=` (bit-exact);
 *   (3) the closed-form next-offset semantics of client.cc:19-31 and server.cc:83-96.
 * Next-offset vectors beyond (3) are "parity unpinned" in the strict sense: no reference-produced vectors
 * exist to compare against.
 */
#define _GNU_SOURCE
#include "omr_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <sched.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------ layout (common.h:27-42) */

uint32_t orc_sentinel(uint32_t B, uint32_t NB) {
  /* max_index base: (UINT32_MAX/BLOCK_SIZE/NUM_BLOCKS-1)*NUM_BLOCKS*BLOCK_SIZE (client.cc:24, :42) */
  return (uint32_t)((UINT32_MAX / B / NB - 1u) * NB * B);
}

/* ------------------------------------------------------------------ generator (client.cc:396-421) */

uint64_t orc_gen_bitmap(uint32_t worker_id, double density, uint64_t nb, int32_t* bitmap) {
  uint64_t count = 0;
  srand(worker_id + 1); /* client.cc:396 srand(res.myId+1) */
  for (uint64_t i = 0; i < nb; i++) {
    double rnum = rand() % 100 / (double)101; /* client.cc:407 */
    if (rnum < density) {                     /* client.cc:408 (res.myId != -1 always holds) */
      bitmap[i] = 1;
      count++;
    } else {
      bitmap[i] = 0;
    }
  }
  return count;
}

/* Uniform [-1,1) from a counter hash (the random-valued variant), restated independently of
 * the HIP fill kernel: splitmix64 finaliser of idx + golden*(seed+1), top 24 bits, centred, scaled. */
static float orc_hash_uniform(uint64_t idx, uint32_t seed) {
  uint64_t z = idx + 0x9E3779B97F4A7C15ull * ((uint64_t)seed + 1ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  int32_t u = (int32_t)(z >> 40) - (1 << 23);
  return (float)u / 8388608.0f;
}

void orc_fill(const int32_t* bitmap, uint64_t nb, uint32_t B, int mode, uint32_t seed, float* buf) {
  for (uint64_t i = 0; i < nb; i++) {
    for (uint32_t j = 0; j < B; j++) {
      uint64_t e = i * B + j;
      if (bitmap[i] == 1) /* client.cc:415-419: flagged blocks hold 0.01 (a double literal stored as float) */
        buf[e] = mode == 0 ? (float)0.01 : orc_hash_uniform(e, seed);
      else
        buf[e] = 0.0f; /* client.cc:401-404 */
    }
  }
}

/* ------------------------------------------------------------------ flags */

/* Data-derived flag (north_star): block non-zero iff some element != 0.0f.  -0.0 == 0.0f is zero, NaN is
 * non-zero.  On reference inputs (0.01f vs 0) this equals the generator bitmap (client.cc:406-414). */
void orc_flags_from_data(const float* buf, uint64_t nb, uint32_t B, int32_t* flags) {
  for (uint64_t i = 0; i < nb; i++) {
    int f = 0;
    const float* p = buf + i * B;
    for (uint32_t j = 0; j < B; j++)
      if (p[j] != 0.0f) {
        f = 1;
        break;
      }
    flags[i] = f;
  }
}

void orc_row_masks(const int32_t* flags, uint64_t nb, uint32_t NB, uint64_t* masks) {
  uint64_t rows = nb / NB;
  for (uint64_t r = 0; r < rows; r++) {
    uint64_t m = 0;
    for (uint32_t l = 0; l < NB; l++)
      if (flags[r * NB + l] == 1) m |= 1ull << l;
    masks[r] = m;
  }
}

void orc_union_flags(const int32_t* flags, uint32_t m, uint64_t nb, int32_t* out) {
  for (uint64_t i = 0; i < nb; i++) {
    int32_t f = 0;
    for (uint32_t w = 0; w < m; w++) f |= flags[(uint64_t)w * nb + i];
    out[i] = f;
  }
}

/* ------------------------------------------------------------------ scan (client.cc:19-31) */

/* find_next_nonzero_block restated on a flag array: from `off`, step B*NB floats (same lane) while still
 * inside partition `tid` ([tid*P, (tid+1)*P), uint32 arithmetic as client.cc:25); return the first offset
 * whose block flag is 1, else the lane sentinel SENT + bid*B (client.cc:23-24). */
uint32_t orc_find_next_nonzero_block(const int32_t* flags, uint32_t P, uint32_t B, uint32_t NB, uint32_t tid,
                                     uint32_t next_offset) {
  uint32_t off = next_offset;
  uint32_t start = P * tid;
  uint32_t bid = (off / B) % NB;
  uint32_t max_index = orc_sentinel(B, NB) + bid * B;
  while (off - start < P) {
    if (flags[off / B] == 1) return off;
    off += B * NB;
  }
  return max_index;
}

/* next[b] = find_next_nonzero_block(b*B + B*NB) for every block b: the value the worker attaches to block b
 * when it sends it (client.cc:94, :203) and, on a union flag array, the aggregator's min_next for it
 * (server.cc:86-96).  Partition of block b = b*B / P (the thread that owns it, client.cc:22). */
void orc_next_offsets(const int32_t* flags, uint64_t n, uint32_t B, uint32_t NB, uint32_t parts,
                      uint32_t* next) {
  uint64_t nb = n / B;
  uint32_t P = (uint32_t)(n / parts);
  for (uint64_t b = 0; b < nb; b++) {
    uint32_t off = (uint32_t)(b * B);
    uint32_t tid = off / P;
    next[b] = orc_find_next_nonzero_block(flags, P, B, NB, tid, off + B * NB);
  }
}

/* ------------------------------------------------------------------ aggregation (server.cc:83-99) */

/* Aggregator sum: for every block the workers send — every union-non-zero block, plus every lane head
 * (row 0 of a partition, sent unconditionally by client.cc:201-205) — the accumulator is zeroed
 * (server.cc:148-150) and each worker's block added (server.cc:97-98).  Workers are added in rank order
 * (the reference adds in arrival order; for the reference generator all addends are equal, so the order
 * does not change the result).  Blocks that no worker sends are left untouched in `out` (the worker keeps
 * its own values: client.cc:89 only overwrites returned blocks). */
void orc_block_sum(const float* const* bufs, uint32_t m, uint64_t n, uint32_t B, uint32_t NB, uint32_t parts,
                   const int32_t* uflags, float* out) {
  uint64_t nb = n / B;
  uint64_t rows_per_part = nb / NB / parts;
  for (uint64_t b = 0; b < nb; b++) {
    uint64_t row = b / NB;
    int head = (row % rows_per_part) == 0;
    if (!(uflags[b] == 1 || head)) continue;
    for (uint32_t j = 0; j < B; j++) {
      float acc = 0.0f;
      for (uint32_t w = 0; w < m; w++) acc += bufs[w][b * B + j];
      out[b * B + j] = acc;
    }
  }
}

/* ------------------------------------------------------------------ message-level streams (Appendix A.3/4) */

/* Worker w's send stream for one lane of one partition (client.cc:201-205 first burst, then :87-102):
 * the head block h = tid*P + bid*B with next(h), then each own non-zero block c > h with next(c).
 * Writes pairs (current, next) and returns how many. */
uint32_t orc_lane_stream(const int32_t* flags, uint64_t n, uint32_t B, uint32_t NB, uint32_t parts, uint32_t tid,
                         uint32_t bid, uint32_t* cur_out, uint32_t* next_out, uint32_t cap) {
  uint32_t P = (uint32_t)(n / parts);
  uint32_t sent = orc_sentinel(B, NB);
  uint32_t c = P * tid + bid * B;
  uint32_t k = 0;
  for (;;) {
    uint32_t nx = orc_find_next_nonzero_block(flags, P, B, NB, tid, c + B * NB);
    if (k < cap) {
      cur_out[k] = c;
      next_out[k] = nx;
    }
    k++;
    if (nx >= sent) break; /* client.cc:91 current_offset < max_index[0] */
    c = nx;
  }
  return k;
}

/* ------------------------------------------------------------------ CPU baseline (timed on the GPU box) */

typedef struct {
  const float* x;
  const int32_t* bitmap;
  int32_t* flags;
  uint32_t* next;
  float* out;
  uint64_t n;
  uint32_t B, NB, parts, tid, variant;
} orc_job;

/* One partition of one round, as one reference thread does it (client.cc:168-223 + server.cc:83-99).
 * variant 0, reference-faithful: walk each lane's chain with find_next_nonzero_block over the generator's
 *   precomputed bitmap (client.cc:26) and aggregate the visited blocks (0.0f + x: server.cc:148-150, :97-98);
 *   zero blocks are never read.
 * variant 1, data-derived: compute every block's flag from the fp32 data (reads the whole partition), then
 *   the next offsets from those flags, then aggregate the non-zero blocks and lane heads — the work the GPU
 *   kernel does. */
static void orc_partition(const orc_job* j) {
  uint32_t P = (uint32_t)(j->n / j->parts);
  uint64_t b0 = (uint64_t)j->tid * P / j->B, b1 = b0 + P / j->B;
  uint32_t sent = orc_sentinel(j->B, j->NB);
  if (j->variant == 0) {
    for (uint32_t bid = 0; bid < j->NB; bid++) {
      uint32_t c = P * j->tid + bid * j->B;
      for (;;) {
        uint32_t nx = orc_find_next_nonzero_block(j->bitmap, P, j->B, j->NB, j->tid, c + j->B * j->NB);
        j->next[c / j->B] = nx;
        const float* s = j->x + c;
        float* d = j->out + c;
        for (uint32_t e = 0; e < j->B; e++) d[e] = 0.0f + s[e];
        if (nx >= sent) break;
        c = nx;
      }
    }
    return;
  }
  for (uint64_t b = b0; b < b1; b++) {
    const float* p = j->x + b * j->B;
    int f = 0;
    for (uint32_t e = 0; e < j->B; e++) f |= (p[e] != 0.0f);
    j->flags[b] = f;
  }
  uint64_t rows = (b1 - b0) / j->NB;
  for (uint32_t l = 0; l < j->NB; l++) {
    uint32_t nx = sent + l * j->B;
    for (uint64_t r = rows; r-- > 0;) {
      uint64_t b = b0 + r * j->NB + l;
      j->next[b] = nx;
      if (j->flags[b] == 1 || r == 0) {
        const float* s = j->x + b * j->B;
        float* d = j->out + b * j->B;
        for (uint32_t e = 0; e < j->B; e++) d[e] = 0.0f + s[e];
      }
      if (j->flags[b] == 1) nx = (uint32_t)(b * j->B);
    }
  }
}

typedef struct {
  orc_job job;
  pthread_barrier_t* start;
  pthread_barrier_t* done;
  int rounds;
  int cpu; /* core this thread pins itself to (-1: none) */
} orc_worker;

/* Cores the last orc_cpu_baseline run pinned its threads to (the reference pins its per-partition threads,
 * client.cc:384-392; here the threads are spread evenly over distinct physical cores of the package the caller
 * runs on (orc_pick_cores), so they stay inside its cgroup, near its memory, and use every CCD's memory link). */
static int g_cores[256];
static int g_ncores = 0;

int orc_cpu_baseline_cores(int* out, int cap) {
  int k = 0;
  for (; k < g_ncores && k < cap; k++) out[k] = g_cores[k];
  return k;
}

/* sysfs topology value of a CPU (-1 if unreadable). */
static int cpu_topo(int cpu, const char* what) {
  char path[128];
  snprintf(path, sizeof(path), "/sys/devices/system/cpu/cpu%d/topology/%s", cpu, what);
  FILE* f = fopen(path, "r");
  if (f == NULL) return -1;
  int v = -1;
  if (fscanf(f, "%d", &v) != 1) v = -1;
  fclose(f);
  return v;
}

/* The cores the baseline's threads may use, in the order they are handed out: CPUs this process may run on, in
 * the package of the CPU it runs on now (where its pages were first touched), one logical CPU per physical core
 * (no SMT sibling pairs).  Falls back to every allowed CPU when the topology is unreadable. */
static int orc_pick_cores(int* out, int cap) {
  cpu_set_t allowed;
  int n = 0;
  if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return 0;
  const int here = sched_getcpu();
  const int pkg = here >= 0 ? cpu_topo(here, "physical_package_id") : -1;
  int seen_core[1024], nseen = 0;
  for (int c = 0; c < CPU_SETSIZE && n < cap; c++) {
    if (!CPU_ISSET(c, &allowed)) continue;
    const int cp = cpu_topo(c, "physical_package_id"), core = cpu_topo(c, "core_id");
    if (pkg >= 0 && cp != pkg) continue;
    int dup = 0;
    for (int i = 0; i < nseen && core >= 0; i++) dup |= (seen_core[i] == core);
    if (dup) continue;
    if (core >= 0 && nseen < 1024) seen_core[nseen++] = core;
    out[n++] = c;
  }
  if (n == 0)
    for (int c = 0; c < CPU_SETSIZE && n < cap; c++)
      if (CPU_ISSET(c, &allowed)) out[n++] = c;
  return n;
}

static void* orc_thread(void* arg) {
  orc_worker* w = (orc_worker*)arg;
  if (w->cpu >= 0) {
    cpu_set_t set;
    CPU_ZERO(&set);
    CPU_SET(w->cpu, &set);
    (void)pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
  }
  for (int r = 0; r < w->rounds; r++) {
    pthread_barrier_wait(w->start);
    orc_partition(&w->job);
    pthread_barrier_wait(w->done);
  }
  return NULL;
}

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

/* Runs warmups + rounds of the m=1 scan+aggregate with `nthreads` persistent pthreads (the reference's
 * NUM_THREADS partitions are split over them round-robin; nthreads == parts reproduces client.cc:384-392).
 * Returns the mean seconds per timed round, or a negative value on error. */
double orc_cpu_baseline(const float* x, const int32_t* bitmap, uint64_t n, uint32_t B, uint32_t NB,
                        uint32_t parts, uint32_t nthreads, uint32_t variant, int warmups, int rounds,
                        int32_t* flags, uint32_t* next, float* out) {
  if (nthreads == 0 || parts % nthreads != 0) return -1.0;
  int total = warmups + rounds;
  pthread_barrier_t start, done;
  pthread_barrier_init(&start, NULL, nthreads + 1);
  pthread_barrier_init(&done, NULL, nthreads + 1);
  orc_worker* ws = (orc_worker*)calloc(nthreads, sizeof(orc_worker));
  pthread_t* th = (pthread_t*)calloc(nthreads, sizeof(pthread_t));
  uint32_t per = parts / nthreads;
  int avail[256];
  const int navail = orc_pick_cores(avail, 256);
  g_ncores = 0;
  /* each worker thread handles `per` consecutive partitions: fold them into one job per partition loop */
  for (uint32_t t = 0; t < nthreads; t++) {
    /* spread over the allowed cores (every CCD's memory link in use), not packed onto the first ones */
    ws[t].cpu = (per == 1 && navail > 0) ? avail[((uint64_t)t * navail / nthreads) % navail] : -1;
    if (ws[t].cpu >= 0 && g_ncores < 256) g_cores[g_ncores++] = ws[t].cpu;
    ws[t].job.x = x;
    ws[t].job.bitmap = bitmap;
    ws[t].job.flags = flags;
    ws[t].job.next = next;
    ws[t].job.out = out;
    ws[t].job.n = n;
    ws[t].job.B = B;
    ws[t].job.NB = NB;
    ws[t].job.parts = parts;
    ws[t].job.tid = t; /* per == 1 case; larger `per` handled below */
    ws[t].job.variant = variant;
    ws[t].start = &start;
    ws[t].done = &done;
    ws[t].rounds = (per == 1) ? total : 0;
  }
  double t0 = 0.0, acc = 0.0;
  if (per == 1) {
    for (uint32_t t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, orc_thread, &ws[t]);
    for (int r = 0; r < total; r++) {
      t0 = now_s();
      pthread_barrier_wait(&start);
      pthread_barrier_wait(&done);
      if (r >= warmups) acc += now_s() - t0;
    }
    for (uint32_t t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  } else {
    /* fewer threads than partitions (e.g. the 1-thread figure): run partitions sequentially per round */
    for (int r = 0; r < total; r++) {
      t0 = now_s();
      for (uint32_t p = 0; p < parts; p++) {
        orc_job j = ws[0].job;
        j.tid = p;
        orc_partition(&j);
      }
      if (r >= warmups) acc += now_s() - t0;
    }
  }
  pthread_barrier_destroy(&start);
  pthread_barrier_destroy(&done);
  free(ws);
  free(th);
  return rounds > 0 ? acc / rounds : 0.0;
}

/* ------------------------------------------------------------------ message-level protocol (one round)
 *
 * A literal restatement of the two per-slot state machines, one message at a time, with the workers' messages
 * of a protocol round arriving in RANK order (one admissible arrival order; the reference's order is whatever
 * the NIC delivers):
 *   worker      client.cc:180-205 (first burst: the slot's lane heads, each with find_next_nonzero_block of
 *               head + B*NB) and client.cc:32-152 handle_recv (per reply block: copy the sum to
 *               buf[current_offset[bid]] (:89), current = the reply's next (:90), queue it when below the
 *               sentinel and own bitmap == 1 (:91-96), else reset the lane and count it finished (:98-101);
 *               send the queue if the slot is not finished (:113-127));
 *   aggregator  server.cc:13-199 handle_recv (per received block: block_next_offset[bid][w] = next (:84-86),
 *               min over every worker (:87-91), complete when current_offset < min_next (:92-96), add into the
 *               slot's accumulator set (:97-98); reply when completed >= BLOCKS_PER_MESSAGE - finished
 *               (:143): sums of the completed lanes in completion order + their min_next (:144-147), zero the
 *               other accumulator set (:148-150); advance / reset lanes (:173-186); flip the set (:193)).
 * Wire format (common.cc:399-407, :424, :443, :503, :522, :542): a message is `len` blocks of B floats then `len`
 * uint32 next offsets, in a 2*MESSAGE_SIZE-float slot; imm = (len << 16) | global slot.
 * Logs: wmsg[w][gs][r] / wimm[w][gs][r] = worker w's message of protocol round r of global slot gs (imm 0 = it
 * sent none), rmsg[gs][r] / rimm[gs][r] = the aggregator's reply; outs[w] = worker w's buffer after the round
 * (callers pass copies of the inputs: results are written in place, client.cc:89).  rounds[gs] = replies in
 * slot gs.  Returns the largest round count, or -1 if rcap is too small / the state machines disagree. */

#define ORC_MSG 1024u  /* MESSAGE_SIZE (common.h:31) */
#define ORC_SLOTS 16u  /* NUM_SLOTS (common.h:34) */
#define ORC_MAXW 16u

int orc_msg_simulate(const float* const* bufs, const int32_t* const* flags, uint32_t m, uint64_t n, uint32_t B,
                     uint32_t NB, uint32_t parts, uint32_t rcap, float* wmsg, uint32_t* wimm, float* rmsg,
                     uint32_t* rimm, float* const* outs, uint32_t* rounds) {
  const uint32_t BPM = ORC_MSG / B;                 /* BLOCKS_PER_MESSAGE (common.h:33) */
  const uint32_t SLOTW = 2 * ORC_MSG;               /* floats per message slot */
  const uint32_t P = (uint32_t)(n / parts);         /* DATA_SIZE_PER_THREAD */
  const uint32_t sent = orc_sentinel(B, NB);        /* max_index base (client.cc:42, server.cc:16) */
  const uint64_t G = (uint64_t)parts * ORC_SLOTS;   /* global slots */
  if (m == 0 || m > ORC_MAXW || BPM == 0 || BPM > 4 || NB != ORC_SLOTS * BPM) return -1;
  int maxr = 0;
  for (uint32_t t = 0; t < parts; t++) {
    const uint32_t start = P * t;
    for (uint32_t s = 0; s < ORC_SLOTS; s++) {
      const uint64_t gs = (uint64_t)t * ORC_SLOTS + s;
      /* worker state (client.cc:35-48) and pending message */
      uint32_t wcur[ORC_MAXW][4], wfin[ORC_MAXW], qlen[ORC_MAXW], qcur[ORC_MAXW][4], qnext[ORC_MAXW][4];
      /* aggregator state (server.cc:14-48) */
      uint32_t acur[4], bno[4][ORC_MAXW], minn[4], ccur[4], cnext[4], ncomp = 0, afin = 0, set = 0;
      float acc[2][4][1024], rsum[4][1024];
      memset(acc, 0, sizeof(acc));
      for (uint32_t j = 0; j < BPM; j++) {
        acur[j] = start + (s * BPM + j) * B;
        for (uint32_t w = 0; w < m; w++) bno[j][w] = 0;
      }
      for (uint32_t w = 0; w < m; w++) {
        wfin[w] = 0;
        qlen[w] = BPM; /* first burst (client.cc:198-205): the slot's lane heads, unconditionally */
        for (uint32_t j = 0; j < BPM; j++) {
          wcur[w][j] = start + (s * BPM + j) * B;
          qcur[w][j] = start + s * ORC_MSG + j * B;
          qnext[w][j] = orc_find_next_nonzero_block(flags[w], P, B, NB, t, qcur[w][j] + B * NB);
        }
      }
      uint32_t r = 0;
      int done = 0;
      while (!done) {
        if (r >= rcap) return -1;
        int replied = 0;
        uint32_t rcur[4], rnext[4], nrep = 0; /* the round's reply, applied by the workers after the round */
        for (uint32_t w = 0; w < m; w++) { /* rank-order arrival of the messages pending at the round start */
          const uint32_t len = qlen[w];
          uint32_t* imm = wimm ? wimm + ((uint64_t)w * G + gs) * rcap + r : NULL;
          if (imm) *imm = 0;
          if (len == 0) continue;
          if (replied) return -1; /* a message after the round's reply: the state machines disagree */
          float* msg = wmsg ? wmsg + (((uint64_t)w * G + gs) * rcap + r) * SLOTW : NULL;
          for (uint32_t k = 0; k < len; k++) { /* worker pack: common.cc:405-407 blocks, :408 next offsets */
            const float* src = bufs[w] + qcur[w][k];
            if (msg) memcpy(msg + k * B, src, B * sizeof(float));
          }
          if (msg) memcpy(msg + len * B, qnext[w], len * sizeof(uint32_t));
          if (imm) *imm = (len << 16) | (uint32_t)gs; /* common.cc:443 */
          /* aggregator receive (server.cc:68-99) */
          for (uint32_t k = 0; k < len; k++) {
            const uint32_t bo = qnext[w][k];
            const uint32_t lane = (bo / B) % NB, j = lane - s * BPM;
            bno[j][w] = bo;
            uint32_t mn = bno[j][0];
            for (uint32_t v = 1; v < m; v++)
              if (mn > bno[j][v]) mn = bno[j][v];
            minn[j] = mn;
            if (acur[j] < minn[j]) {
              ccur[ncomp] = acur[j];
              cnext[ncomp] = minn[j];
              ncomp++;
            }
            const float* src = bufs[w] + qcur[w][k];
            for (uint32_t e = 0; e < B; e++) acc[set][j][e] += src[e];
          }
          if (ncomp >= BPM - afin) { /* server.cc:143: reply */
            float* rm = rmsg ? rmsg + (gs * rcap + r) * SLOTW : NULL;
            for (uint32_t k = 0; k < ncomp; k++) {
              const uint32_t j = (ccur[k] / B) % NB - s * BPM;
              if (rm) memcpy(rm + k * B, acc[set][j], B * sizeof(float));
            }
            if (rm) memcpy(rm + ncomp * B, cnext, ncomp * sizeof(uint32_t));
            if (rimm) rimm[gs * rcap + r] = (ncomp << 16) | (uint32_t)gs;
            for (uint32_t k = 0; k < ncomp; k++) { /* the reply as sent: completed sums + min_next */
              const uint32_t j = (ccur[k] / B) % NB - s * BPM;
              rcur[k] = ccur[k];
              rnext[k] = cnext[k];
              memcpy(rsum[k], acc[set][j], B * sizeof(float));
            }
            nrep = ncomp;
            memset(acc[set ^ 1u], 0, sizeof(acc[0])); /* server.cc:148-150 */
            /* aggregator lane advance (server.cc:173-186) */
            for (uint32_t k = 0; k < ncomp; k++) {
              const uint32_t lane = (cnext[k] / B) % NB, j = lane - s * BPM;
              acur[j] = cnext[k];
              if (cnext[k] >= sent) {
                acur[j] = start + lane * B;
                for (uint32_t v = 0; v < m; v++) bno[j][v] = 0;
                afin++;
              }
            }
            ncomp = 0;
            if (afin == BPM) done = 1; /* server.cc:187-192 */
            set ^= 1u;                 /* server.cc:193 */
            replied = 1;
          }
        }
        if (!replied) return -1; /* every worker idle but the slot unfinished */
        /* every worker receives the reply (client.cc:67-127) */
        for (uint32_t v = 0; v < m; v++) {
          uint32_t nq = 0;
          for (uint32_t k = 0; k < nrep; k++) {
            const uint32_t lane = (rnext[k] / B) % NB, j = lane - s * BPM;
            memcpy(outs[v] + wcur[v][j], rsum[k], B * sizeof(float)); /* client.cc:89 */
            wcur[v][j] = rnext[k];
            if (wcur[v][j] < sent) {
              if (flags[v][wcur[v][j] / B] == 1) {
                qcur[v][nq] = wcur[v][j];
                qnext[v][nq] = orc_find_next_nonzero_block(flags[v], P, B, NB, t, wcur[v][j] + B * NB);
                nq++;
              }
            } else {
              wcur[v][j] = start + lane * B;
              wfin[v]++;
            }
          }
          qlen[v] = wfin[v] < BPM ? nq : 0;
        }
        (void)rcur;
        r++;
      }
      if (rounds) rounds[gs] = r;
      if ((int)r > maxr) maxr = (int)r;
    }
  }
  return maxr;
}
