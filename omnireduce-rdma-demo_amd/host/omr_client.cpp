// omr_client.cpp — ./omr_client: the worker with the reference CLI and benchmark loop (client.cc:240-491).
//
//   ./omr_client [-p port] [-d ib-dev] [-i ib-port] [-g gid-idx] [-s service-level] [-r density] agg_ip[,agg_ip...]
//
// MI355X-build extensions:  -n floats (DATA_SIZE, default common.h:40 = 128 Mi)   -b BLOCK_SIZE (256)
//   -W warm-ups (10)  -R rounds (101) (client.cc:368-369)  -G gpu (default $LOCAL_RANK or 0)
//   -c  check the result against the rank-order sum of every worker's input (the working CHECK of
//       client.cc:449-465)    -I  in place (the reference writes results into res->buf, so rounds after the first
//       start from the previous round's output)    -L k  run k workers as threads of this process over the
//       loopback transport (no server needed)    -H  the tensor in pinned host memory, as the reference's registered
//       res->buf: each round reads it and returns its results into it (omr_sparse_buckets_f32 with one bucket; a
//       one-rank group reads and writes it in one launch, more ranks stage it through device buffers)
//   -M  (with -L k) message mode: the k workers share one GPU and the round runs as the reference's messages
//       (omr_msg_round_f32: every worker message and aggregator reply of the per-slot state machines, in the
//       wire format of common.cc:399-443)    -T file  (with -M) write the last round's wire trace: per message
//       a {src, dst, imm, len} record of four uint32 (workers 0..k-1, aggregator 100) then its payload, the
//       (B*len + len)*4 bytes an ibv_post_send would carry (common.cc:424), slot by slot, round by round
//
// With an aggregator list agg[:port][,agg[:port]...] the worker connects to every ./omr_server in list order, as the
// reference's sock_connect does (common.cc:71-97): each server gives it its ID (the position of its IP in the
// server's worker list, common.cc:123-133) and the servers are the round's aggregator ranks, aggregator j owning the
// j-th shard (-M: the global slots gs with gs % n == j, common.cc:381-383).  -X rccl (default; one process per GPU,
// RCCL over xGMI) or -X ipc (processes sharing GPUs, HIP IPC: one host, no RCCL)  -C the workers aggregate their own
// shards instead (the servers only meet them)  -l k orders workers that share an IP and a GPU (default
// $LOCAL_RANK).  Output lines are the reference's: per round
// "data size: ... time: ... us; alg bw: ... GB/s" (client.cc:447), the average (client.cc:473), and
// "test result is N" (client.cc:486).  alg bw keeps the reference formula DATA_SIZE*4/2^30/s (client.cc:445).
#include <getopt.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <thread>
#include <vector>

#include "omr.h"
#include "omr_dist.h"
#include "omr_net.hpp"

namespace {

struct Opts {
  int port = 19875, ib_port = 1, gid = -1, sl = 0;  // client.cc:9-18
  const char* dev = nullptr;
  double density = 1.0;  // client.cc:253
  uint64_t n = 128ull << 20;
  uint32_t block = 256;
  int warmups = 10, rounds = 101;  // client.cc:368-369
  int gpu = -1, local = 0;
  bool check = false, inplace = false, messages = false, colocated = false;
  bool host = false;  // -H: the tensor in pinned host memory, as the reference's registered res->buf
  int transport = omrnet::kRccl, local_id = -1;
  const char* trace = nullptr;
};

void usage(const char* argv0) {  // common.cc:1441-1457 (default port and -r text corrected: SURVEY.md §5)
  fprintf(stdout, "Usage:\n %s <host> connect to server at <host>\n\n", argv0);
  fprintf(stdout, "Options:\n");
  fprintf(stdout, " -p, --port <port> listen on/connect to port <port> (default 19875)\n");
  fprintf(stdout, " -d, --ib-dev <dev> accepted for compatibility (no verbs device is used)\n");
  fprintf(stdout, " -i, --ib-port <port> accepted for compatibility\n");
  fprintf(stdout, " -g, --gid_idx <git index> accepted for compatibility\n");
  fprintf(stdout, " -s, --service-level <sl> accepted for compatibility\n");
  fprintf(stdout, " -r, --density-ratio <r> fraction of non-zero blocks, as rand()%%100/101 < r (default 1.0)\n");
  fprintf(stdout, " -n <floats> -b <block size> -W <warm-ups> -R <rounds> -G <gpu> -c (check) -I (in place)\n");
  fprintf(stdout, " -L <k> run k workers in this process over the loopback transport\n");
  fprintf(stdout, " -M message mode: the round as the reference's wire messages; -T <file> trace them\n");
  fprintf(stdout, " -H the tensor in pinned host memory (the reference's registered buffer): each round reads it and\n"
                  "    returns its results into it (omr_sparse_buckets_f32, one bucket)\n");
  fprintf(stdout, " -X rccl|ipc transport to the servers (default rccl)  -C co-located aggregation  -l <k> local id\n");
  fprintf(stdout, " -h, --help show this help message\n");
}

#define HIPOK(x)                                                                 \
  do {                                                                           \
    hipError_t _e = (x);                                                         \
    if (_e != hipSuccess) {                                                      \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(_e));             \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

// the worker's tensor: the reference generator (client.cc:396-421) on the device
int make_input(uint32_t worker_id, const Opts& o, float* d_x, int32_t* d_bitmap) {
  const uint64_t nb = o.n / o.block;
  std::vector<int32_t> bm(nb);
  uint64_t nz = 0;
  if (omr_gen_bitmap(worker_id, o.density, nb, bm.data(), &nz)) return 1;
  HIPOK(hipMemcpy(d_bitmap, bm.data(), nb * sizeof(int32_t), hipMemcpyHostToDevice));
  if (omr_fill_blocks_f32(d_bitmap, nb, o.block, 0, 0, d_x, nullptr)) return 1;
  HIPOK(hipDeviceSynchronize());
  return 0;
}

// The CHECK of client.cc:449-465, done right and without the GPU: the expected result is the rank-order sum of every
// worker's input (the reference's MPI_Allreduce SUM).  Every input is the generator's (client.cc:396-421): a non-zero
// block holds 0.01f in every element, so block b of the sum is the k-fold sequential fp32 sum of 0.01f from +0.0f,
// k = the number of workers whose bitmap flags b (+0.0 when none does).  The bitmaps are regenerated on the host
// (omr_gen_bitmap: glibc's rand() restated); no kernel of this library computes the expectation.
// Returns 0 (check OK), 1 (mismatch, the reference's "error: " line printed) or -1 (could not check).
int host_check(const Opts& o, int workers, const float* d_result) {
  const uint64_t nb = o.n / o.block;
  std::vector<uint8_t> cnt(nb, 0);
  std::vector<int32_t> bm(nb);
  for (int w = 0; w < workers; ++w) {
    uint64_t nz = 0;
    if (omr_gen_bitmap(static_cast<uint32_t>(w), o.density, nb, bm.data(), &nz)) return -1;
    for (uint64_t b = 0; b < nb; ++b) cnt[b] = static_cast<uint8_t>(cnt[b] + (bm[b] != 0 ? 1 : 0));
  }
  std::vector<float> ka(static_cast<size_t>(workers) + 1);
  volatile float acc = 0.0f;  // one fp32 rounding per add, as server.cc:97-98 accumulates
  ka[0] = acc;
  for (int k = 1; k <= workers; ++k) {
    acc = acc + 0.01f;
    ka[k] = acc;
  }
  std::vector<float> got(o.n);
  if (hipMemcpy(got.data(), d_result, o.n * sizeof(float), hipMemcpyDefault) != hipSuccess) return -1;
  for (uint64_t b = 0; b < nb; ++b) {
    const float e = ka[cnt[b]];
    for (uint64_t i = b * o.block; i < (b + 1) * o.block; ++i)
      if (memcmp(&got[i], &e, sizeof(float)) != 0) {
        std::cout << "error: " << e << "<---->" << got[i] << std::endl;  // client.cc:453-456
        return 1;
      }
  }
  return 0;
}

int run_worker(omr_dist* d, const Opts& o, int gpu, bool printer, int num_workers = 0) {
  HIPOK(hipSetDevice(gpu));
  const int rank = omr_dist_rank(d);
  const int world = num_workers > 0 ? num_workers : omr_dist_world(d);  // the workers (the rest aggregate)
  const uint32_t lanes = omr_num_lanes(o.block);
  const uint64_t nb = o.n / o.block;
  if (omr_layout_check(o.n, o.block, lanes, OMR_NUM_THREADS)) {
    fprintf(stderr, "bad layout: %s\n", omr_last_error());
    return 1;
  }
  float *d_x = nullptr, *d_out = nullptr;
  int32_t* d_bitmap = nullptr;
  HIPOK(hipMalloc(&d_x, o.n * sizeof(float)));
  HIPOK(hipMalloc(&d_out, o.n * sizeof(float)));
  HIPOK(hipMalloc(&d_bitmap, nb * sizeof(int32_t)));
  if (make_input(static_cast<uint32_t>(rank), o, d_x, d_bitmap)) return 1;  // srand(res.myId+1)
  HIPOK(hipMemcpy(d_out, d_x, o.n * sizeof(float), hipMemcpyDeviceToDevice));
  omr_ar_plan* plan = nullptr;
  if (omr_ar_plan_create_roles(d, static_cast<uint32_t>(world), o.n, o.block, lanes, OMR_NUM_THREADS, &plan)) {
    fprintf(stderr, "omr_ar_plan_create: %s\n", omr_dist_last_error());
    return 1;
  }
  hipStream_t st;
  HIPOK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  // -c with -I: every round starts from the generator's input, as the reference's CHECK restores res.buf = input
  // after each checked round (client.cc:463-464); without it the in-place rounds would compound
  const bool restore = o.check && (o.inplace || o.host);
  float* d_in = nullptr;
  if (restore) {
    HIPOK(hipMalloc(&d_in, o.n * sizeof(float)));
    HIPOK(hipMemcpyAsync(d_in, d_x, o.n * sizeof(float), hipMemcpyDeviceToDevice, st));
    HIPOK(hipStreamSynchronize(st));
  }
  // -H: the round's tensor lives in pinned host memory with a device mapping (the reference's res->buf, registered
  // for RDMA: common.cc:873-914); each round reads it and stores its results back into it (client.cc:89)
  float* h_x = nullptr;
  if (o.host) {
    HIPOK(hipHostMalloc(reinterpret_cast<void**>(&h_x), o.n * sizeof(float), hipHostMallocMapped));
    HIPOK(hipMemcpy(h_x, d_x, o.n * sizeof(float), hipMemcpyDeviceToHost));
  }
  if (printer) std::cout << "density: " << o.density << std::endl;  // client.cc:405
  const double gib = o.n * sizeof(float) / (1024.0 * 1024.0 * 1024.0);
  double avg_bw = 0.0;
  unsigned long avg_time_usec = 0;
  int print_count = 0;
  auto start = std::chrono::steady_clock::now();
  for (int round = 0; round < o.warmups + o.rounds; ++round) {
    float* out = o.inplace ? d_x : d_out;
    // (no counts asked for: the reference's round reports none, and a one-rank round then never waits mid-round;
    // -H: the call returns once the host buffer holds the results)
    if (o.host ? omr_sparse_buckets_f32(plan, h_x, o.n, OMR_ROUND_ALLREDUCE, nullptr, nullptr, st)
               : omr_sparse_allreduce_f32(plan, d_x, out, nullptr, nullptr, nullptr, nullptr, nullptr, st)) {
      fprintf(stderr, "failed to run the round: %s\n", omr_dist_last_error());  // client.cc:131-135
      return 1;
    }
    HIPOK(hipStreamSynchronize(st));  // a round ends when its results are in place (client.cc:220 wait())
    if (round >= o.warmups) {  // client.cc:439-448, print_freq 1
      if (round - o.warmups > 0) {
        const auto now = std::chrono::steady_clock::now();
        const unsigned long us =
            static_cast<unsigned long>(std::chrono::duration_cast<std::chrono::microseconds>(now - start).count());
        const double bw = gib / (us / 1e6);
        ++print_count;
        avg_time_usec += us;
        avg_bw += bw;
        if (printer)
          fprintf(stdout, "data size: %lu Bytes; time: %lu us; alg bw: %f GB/s\n",
                  static_cast<unsigned long>(o.n * sizeof(float)), us, bw);
      }
      start = std::chrono::steady_clock::now();
    }
    if (restore && round + 1 < o.warmups + o.rounds) {  // res.buf = input (client.cc:463-464), outside the timing
      HIPOK(hipMemcpyAsync(o.host ? h_x : d_x, d_in, o.n * sizeof(float), hipMemcpyDefault, st));
      HIPOK(hipStreamSynchronize(st));
      start = std::chrono::steady_clock::now();
    }
  }
  (void)hipFree(d_in);
  int rc = 0;
  struct FreeHost {  // (after the check, which reads it)
    float* h;
    ~FreeHost() { (void)hipHostFree(h); }
  } free_host{h_x};
  if (o.check) {  // the CHECK of client.cc:449-465, done right: expected = rank-order sum of every input
    HIPOK(hipDeviceSynchronize());
    const int c = host_check(o, world, o.host ? h_x : (o.inplace ? d_x : d_out));
    if (c == 0) std::cout << "check OK" << std::endl;  // every worker reports its own check (client.cc:460)
    if (c < 0) fprintf(stderr, "check skipped: %s\n", omr_last_error());
    if (c == 1) rc = 1;
  }
  if (printer && print_count > 0)  // client.cc:473
    fprintf(stdout, "data size: %lu Bytes; average time: %lu us; average alg bw: %f GB/s\n",
            static_cast<unsigned long>(o.n * sizeof(float)), avg_time_usec / print_count, avg_bw / print_count);
  omr_ar_plan_destroy(plan);
  (void)hipStreamDestroy(st);
  (void)hipFree(d_x);
  (void)hipFree(d_out);
  (void)hipFree(d_bitmap);
  return rc;
}

// -M: k workers on one GPU, the round as the reference's messages (omr_msg_round_f32)
int run_messages(const Opts& o, int gpu) {
  HIPOK(hipSetDevice(gpu));
  const int k = o.local;
  const uint32_t lanes = omr_num_lanes(o.block);
  const uint64_t nb = o.n / o.block;
  if (omr_layout_check(o.n, o.block, lanes, OMR_NUM_THREADS)) {
    fprintf(stderr, "bad layout: %s\n", omr_last_error());
    return 1;
  }
  std::vector<float*> x(k), out(k);
  int32_t* d_bitmap = nullptr;
  HIPOK(hipMalloc(&d_bitmap, nb * sizeof(int32_t)));
  for (int w = 0; w < k; ++w) {
    HIPOK(hipMalloc(&x[w], o.n * sizeof(float)));
    HIPOK(hipMalloc(&out[w], o.n * sizeof(float)));
    if (make_input(static_cast<uint32_t>(w), o, x[w], d_bitmap)) return 1;  // srand(myId+1) per worker
    HIPOK(hipMemcpy(out[w], x[w], o.n * sizeof(float), hipMemcpyDeviceToDevice));
  }
  omr_msg_plan* plan = nullptr;
  if (omr_msg_plan_create(o.n, o.block, lanes, OMR_NUM_THREADS, static_cast<uint32_t>(k), &plan)) {
    fprintf(stderr, "omr_msg_plan_create: %s\n", omr_last_error());
    return 1;
  }
  hipStream_t st;
  HIPOK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  std::cout << "density: " << o.density << std::endl;  // client.cc:405
  const double gib = o.n * sizeof(float) / (1024.0 * 1024.0 * 1024.0);
  double avg_bw = 0.0;
  unsigned long avg_time_usec = 0;
  int print_count = 0;
  uint32_t maxr = 0;
  std::vector<const float*> in(x.begin(), x.end());
  const bool restore = o.check && o.inplace;  // client.cc:463-464, as in run_worker
  std::vector<float*> pristine(k, nullptr);
  if (restore)
    for (int w = 0; w < k; ++w) {
      HIPOK(hipMalloc(&pristine[w], o.n * sizeof(float)));
      HIPOK(hipMemcpyAsync(pristine[w], x[w], o.n * sizeof(float), hipMemcpyDeviceToDevice, st));
    }
  HIPOK(hipStreamSynchronize(st));
  auto start = std::chrono::steady_clock::now();
  for (int round = 0; round < o.warmups + o.rounds; ++round) {
    if (restore && round > 0) {  // res.buf = input before every round after the first (client.cc:463-464)
      for (int w = 0; w < k; ++w)
        HIPOK(hipMemcpyAsync(x[w], pristine[w], o.n * sizeof(float), hipMemcpyDeviceToDevice, st));
      HIPOK(hipStreamSynchronize(st));
      start = std::chrono::steady_clock::now();
    }
    std::vector<float*> dst = o.inplace ? x : out;
    if (omr_msg_round_f32(plan, in.data(), dst.data(), &maxr, st)) {
      fprintf(stderr, "failed to run the round: %s\n", omr_last_error());
      return 1;
    }
    HIPOK(hipStreamSynchronize(st));
    if (round >= o.warmups) {
      if (round - o.warmups > 0) {
        const auto now = std::chrono::steady_clock::now();
        const unsigned long us =
            static_cast<unsigned long>(std::chrono::duration_cast<std::chrono::microseconds>(now - start).count());
        const double bw = gib / (us / 1e6);
        ++print_count;
        avg_time_usec += us;
        avg_bw += bw;
        fprintf(stdout, "data size: %lu Bytes; time: %lu us; alg bw: %f GB/s\n",
                static_cast<unsigned long>(o.n * sizeof(float)), us, bw);
      }
      start = std::chrono::steady_clock::now();
    }
  }
  for (float* b : pristine) (void)hipFree(b);
  std::cout << "protocol rounds (largest slot): " << maxr << std::endl;
  int rc = 0;
  if (o.trace) {  // the last round's wire traffic, SURVEY.md Appendix B.6 record layout
    FILE* f = fopen(o.trace, "wb");
    if (!f) {
      fprintf(stderr, "cannot open %s\n", o.trace);
      return 1;
    }
    const uint32_t G = OMR_NUM_THREADS * OMR_NUM_SLOTS, W = 2 * OMR_MESSAGE_SIZE;
    float *dm = nullptr, *drep = nullptr;
    uint32_t *dimm = nullptr, *drimm = nullptr, *drounds = nullptr, cap = 0;
    std::vector<std::vector<float>> msg(k);
    std::vector<std::vector<uint32_t>> imm(k);
    std::vector<float> rep;
    std::vector<uint32_t> rimm, rounds(G);
    for (int w = 0; w < k; ++w) {
      omr_msg_logs(plan, static_cast<uint32_t>(w), &dm, &dimm, &drep, &drimm, &drounds, &cap);
      msg[w].resize(static_cast<size_t>(G) * cap * W);
      imm[w].resize(static_cast<size_t>(G) * cap);
      HIPOK(hipMemcpy(msg[w].data(), dm, msg[w].size() * sizeof(float), hipMemcpyDeviceToHost));
      HIPOK(hipMemcpy(imm[w].data(), dimm, imm[w].size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
    }
    rep.resize(static_cast<size_t>(G) * cap * W);
    rimm.resize(static_cast<size_t>(G) * cap);
    HIPOK(hipMemcpy(rep.data(), drep, rep.size() * sizeof(float), hipMemcpyDeviceToHost));
    HIPOK(hipMemcpy(rimm.data(), drimm, rimm.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
    HIPOK(hipMemcpy(rounds.data(), drounds, G * sizeof(uint32_t), hipMemcpyDeviceToHost));
    uint64_t records = 0;
    auto put = [&](uint32_t src, uint32_t dst, uint32_t word, const float* payload) {
      const uint32_t len = word >> 16;
      const uint32_t rec[4] = {src, dst, word, len};
      fwrite(rec, sizeof(rec), 1, f);
      fwrite(payload, sizeof(float), static_cast<size_t>(o.block) * len + len, f);  // common.cc:424
      ++records;
    };
    for (uint32_t gs = 0; gs < G; ++gs)
      for (uint32_t r = 0; r < rounds[gs]; ++r) {
        const size_t u = static_cast<size_t>(gs) * cap + r;
        for (int w = 0; w < k; ++w)
          if (imm[w][u]) put(static_cast<uint32_t>(w), 100, imm[w][u], &msg[w][u * W]);
        for (int w = 0; w < k; ++w) put(100, static_cast<uint32_t>(w), rimm[u], &rep[u * W]);
      }
    fclose(f);
    std::cout << "trace: " << records << " messages -> " << o.trace << std::endl;
  }
  if (o.check) {  // every worker must hold the rank-order sum of every input (client.cc:449-465, done right)
    HIPOK(hipDeviceSynchronize());
    for (int w = 0; w < k && rc == 0; ++w) {
      const int c = host_check(o, k, o.inplace ? x[w] : out[w]);
      if (c < 0) {
        fprintf(stderr, "check skipped: %s\n", omr_last_error());
        break;
      }
      rc = c;
    }
    if (rc == 0) std::cout << "check OK" << std::endl;
  }
  if (print_count > 0)  // client.cc:473
    fprintf(stdout, "data size: %lu Bytes; average time: %lu us; average alg bw: %f GB/s\n",
            static_cast<unsigned long>(o.n * sizeof(float)), avg_time_usec / print_count, avg_bw / print_count);
  omr_msg_plan_destroy(plan);
  (void)hipStreamDestroy(st);
  for (int w = 0; w < k; ++w) {
    (void)hipFree(x[w]);
    (void)hipFree(out[w]);
  }
  (void)hipFree(d_bitmap);
  return rc;
}

// One trace record per message: {src, dst, imm, len} then the (B*len + len)*4 payload
// bytes an ibv_post_send carries (common.cc:424); workers are 0..m-1, aggregator j is 100 + j.
struct TraceWriter {
  FILE* f = nullptr;
  uint32_t block = 256;
  uint64_t records = 0;
  void put(uint32_t src, uint32_t dst, uint32_t word, const float* payload) {
    const uint32_t len = word >> 16;
    const uint32_t rec[4] = {src, dst, word, len};
    fwrite(rec, sizeof(rec), 1, f);
    fwrite(payload, sizeof(float), static_cast<size_t>(block) * len + len, f);
    ++records;
  }
};

// -M with aggregator processes: this worker's rounds as the reference's messages over the transport (omr_msgd_*);
// -T writes the messages it sent and the replies it got, slot by slot, round by round
int run_msg_worker(omr_dist* d, const Opts& o, int gpu, int num_workers, int num_aggs) {
  HIPOK(hipSetDevice(gpu));
  const int rank = omr_dist_rank(d);
  const uint32_t lanes = omr_num_lanes(o.block);
  const uint64_t nb = o.n / o.block;
  float *d_x = nullptr, *d_out = nullptr;
  int32_t* d_bitmap = nullptr;
  HIPOK(hipMalloc(&d_x, o.n * sizeof(float)));
  HIPOK(hipMalloc(&d_out, o.n * sizeof(float)));
  HIPOK(hipMalloc(&d_bitmap, nb * sizeof(int32_t)));
  if (make_input(static_cast<uint32_t>(rank), o, d_x, d_bitmap)) return 1;
  omr_msgd_plan* plan = nullptr;
  if (omr_msgd_plan_create(d, static_cast<uint32_t>(num_workers), o.n, o.block, lanes, OMR_NUM_THREADS, &plan)) {
    fprintf(stderr, "omr_msgd_plan_create: %s\n", omr_dist_last_error());
    return 1;
  }
  hipStream_t st;
  HIPOK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const bool printer = rank == 0;
  if (printer) std::cout << "density: " << o.density << std::endl;  // client.cc:405
  const double gib = o.n * sizeof(float) / (1024.0 * 1024.0 * 1024.0);
  double avg_bw = 0.0;
  unsigned long avg_time_usec = 0;
  int print_count = 0;
  uint32_t maxr = 0;
  auto start = std::chrono::steady_clock::now();
  for (int round = 0; round < o.warmups + o.rounds; ++round) {
    float* out = o.inplace ? d_x : d_out;
    if (!o.inplace) HIPOK(hipMemcpyAsync(d_out, d_x, o.n * sizeof(float), hipMemcpyDeviceToDevice, st));
    if (omr_msgd_round_f32(plan, d_x, out, &maxr, st)) {
      fprintf(stderr, "failed to run the round: %s\n", omr_dist_last_error());
      return 1;
    }
    HIPOK(hipStreamSynchronize(st));
    if (round >= o.warmups) {
      if (round - o.warmups > 0) {
        const auto now = std::chrono::steady_clock::now();
        const unsigned long us =
            static_cast<unsigned long>(std::chrono::duration_cast<std::chrono::microseconds>(now - start).count());
        const double bw = gib / (us / 1e6);
        ++print_count;
        avg_time_usec += us;
        avg_bw += bw;
        if (printer)
          fprintf(stdout, "data size: %lu Bytes; time: %lu us; alg bw: %f GB/s\n",
                  static_cast<unsigned long>(o.n * sizeof(float)), us, bw);
      }
      start = std::chrono::steady_clock::now();
    }
    if (o.inplace && o.check && round + 1 < o.warmups + o.rounds) {  // res.buf = input (client.cc:463-464)
      if (make_input(static_cast<uint32_t>(rank), o, d_x, d_bitmap)) return 1;
      start = std::chrono::steady_clock::now();
    }
  }
  if (printer) std::cout << "protocol rounds (largest slot): " << maxr << std::endl;
  int rc = 0;
  if (o.trace) {
    const uint32_t G = OMR_NUM_THREADS * OMR_NUM_SLOTS, W = 2 * OMR_MESSAGE_SIZE;
    float *dm = nullptr, *drep = nullptr;
    uint32_t *dimm = nullptr, *drimm = nullptr, *drounds = nullptr, cap = 0;
    omr_msgd_logs(plan, static_cast<uint32_t>(rank), &dm, &dimm, &drep, &drimm, &drounds, &cap);
    std::vector<float> msg(static_cast<size_t>(G) * cap * W), rep(msg.size());
    std::vector<uint32_t> imm(static_cast<size_t>(G) * cap), rimm(imm.size()), rounds(G);
    HIPOK(hipMemcpy(msg.data(), dm, msg.size() * sizeof(float), hipMemcpyDeviceToHost));
    HIPOK(hipMemcpy(imm.data(), dimm, imm.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
    HIPOK(hipMemcpy(rep.data(), drep, rep.size() * sizeof(float), hipMemcpyDeviceToHost));
    HIPOK(hipMemcpy(rimm.data(), drimm, rimm.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
    HIPOK(hipMemcpy(rounds.data(), drounds, G * sizeof(uint32_t), hipMemcpyDeviceToHost));
    TraceWriter tw;
    tw.f = fopen(o.trace, "wb");
    tw.block = o.block;
    if (!tw.f) {
      fprintf(stderr, "cannot open %s\n", o.trace);
      return 1;
    }
    const uint32_t A = static_cast<uint32_t>(num_aggs);
    for (uint32_t gs = 0; gs < G; ++gs)
      for (uint32_t r = 0; r < rounds[gs]; ++r) {
        const size_t u = static_cast<size_t>(gs) * cap + r;
        if (imm[u]) tw.put(static_cast<uint32_t>(rank), 100 + gs % A, imm[u], &msg[u * W]);
        tw.put(100 + gs % A, static_cast<uint32_t>(rank), rimm[u], &rep[u * W]);
      }
    fclose(tw.f);
    std::cout << "trace: " << tw.records << " messages -> " << o.trace << std::endl;
  }
  if (o.check) {  // the CHECK of client.cc:449-465, done right: the rank-order sum of every worker's input
    HIPOK(hipDeviceSynchronize());
    const int c = host_check(o, num_workers, o.inplace ? d_x : d_out);
    if (c == 0) std::cout << "check OK" << std::endl;
    if (c < 0) fprintf(stderr, "check skipped: %s\n", omr_last_error());
    if (c == 1) rc = 1;
  }
  if (printer && print_count > 0)  // client.cc:473
    fprintf(stdout, "data size: %lu Bytes; average time: %lu us; average alg bw: %f GB/s\n",
            static_cast<unsigned long>(o.n * sizeof(float)), avg_time_usec / print_count, avg_bw / print_count);
  omr_msgd_plan_destroy(plan);
  (void)hipStreamDestroy(st);
  (void)hipFree(d_x);
  (void)hipFree(d_out);
  (void)hipFree(d_bitmap);
  return rc;
}

}  // namespace

int main(int argc, char* argv[]) {
  Opts o;
  static option longopts[] = {{"port", 1, nullptr, 'p'},          {"ib-dev", 1, nullptr, 'd'},
                              {"ib-port", 1, nullptr, 'i'},       {"gid-idx", 1, nullptr, 'g'},
                              {"service-level", 1, nullptr, 's'}, {"density-ratio", 1, nullptr, 'r'},
                              {"help", 0, nullptr, 'h'},          {nullptr, 0, nullptr, 0}};
  while (true) {
    int c = getopt_long(argc, argv, "p:d:i:g:s:r:n:b:W:R:G:L:T:X:l:cIMCHh", longopts, nullptr);
    if (c == -1) break;
    switch (c) {
      case 'p': o.port = static_cast<int>(strtoul(optarg, nullptr, 0)); break;
      case 'd': o.dev = optarg; break;
      case 'i': o.ib_port = static_cast<int>(strtoul(optarg, nullptr, 0)); break;
      case 'g': o.gid = static_cast<int>(strtoul(optarg, nullptr, 0)); break;
      case 's': o.sl = static_cast<int>(strtoul(optarg, nullptr, 0)); break;
      case 'r':
        o.density = strtod(optarg, nullptr);
        if (o.density < 0) o.density = 1.0;  // client.cc:302-308
        break;
      case 'n': o.n = strtoull(optarg, nullptr, 0); break;
      case 'b': o.block = static_cast<uint32_t>(strtoul(optarg, nullptr, 0)); break;
      case 'W': o.warmups = atoi(optarg); break;
      case 'R': o.rounds = atoi(optarg); break;
      case 'G': o.gpu = atoi(optarg); break;
      case 'L': o.local = atoi(optarg); break;
      case 'c': o.check = true; break;
      case 'I': o.inplace = true; break;
      case 'M': o.messages = true; break;
      case 'T': o.trace = optarg; break;
      case 'X':
        if (strcmp(optarg, "ipc") == 0) o.transport = omrnet::kIpc;
        else if (strcmp(optarg, "rccl") == 0) o.transport = omrnet::kRccl;
        else {
          usage(argv[0]);
          return 1;
        }
        break;
      case 'l': o.local_id = atoi(optarg); break;
      case 'C': o.colocated = true; break;
      case 'H': o.host = true; break;
      default: usage(argv[0]); return 1;
    }
  }
  if (o.host && o.messages) {  // (the message round runs on device tensors only)
    fprintf(stderr, "-H and -M cannot be combined\n");
    usage(argv[0]);
    return 1;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    fprintf(stderr, "no HIP device\n");
    fprintf(stdout, "\ntest result is 1\n");
    return 1;
  }
  std::vector<std::string> aggs = omrnet::split_list(optind == argc - 1 ? argv[optind] : nullptr);
  omrnet::print_config(false, aggs, o.port, o.dev, o.ib_port, o.gid, o.sl);
  int rc = 0;
  if (o.messages && o.local > 0) {  // message mode, k workers on one GPU: the round as the reference's wire messages
    if (o.local <= 0 || o.local > OMR_MAX_WORKERS) {
      fprintf(stderr, "-M needs -L k with 1 <= k <= %d\n", OMR_MAX_WORKERS);
      return 1;
    }
    std::cout << "Number of aggregators: 1; Number of workers is " << o.local << " (message mode, one GPU)"
              << std::endl;
    printf("Connected.\n");
    rc = run_messages(o, o.gpu >= 0 ? o.gpu : 0);
    fprintf(stdout, "\ntest result is %d\n", rc);
    return rc;
  }
  if (o.local > 0) {  // loopback: k workers as threads, GPUs round-robin
    omr_local_board* board = omr_local_board_create(o.local);
    std::vector<int> rcs(o.local, 0);
    std::vector<std::thread> th;
    std::cout << "Number of aggregators: " << o.local << "; Number of workers is " << o.local
              << "; My ID is 0 (loopback, " << ndev << " GPU(s))" << std::endl;
    printf("Connected.\n");
    for (int t = 0; t < o.local; ++t)
      th.emplace_back([&, t] {
        if (hipSetDevice(t % ndev) != hipSuccess) {
          rcs[t] = 1;
          return;
        }
        omr_dist* d = nullptr;
        if (omr_dist_create_local(board, t, &d)) {
          rcs[t] = 1;
          return;
        }
        rcs[t] = run_worker(d, o, t % ndev, t == 0);
        omr_dist_destroy(d);
      });
    for (auto& t : th) t.join();
    omr_local_board_destroy(board);
    for (int r : rcs) rc |= r;
    fprintf(stdout, "\ntest result is %d\n", rc);
    return rc;
  }
  if (aggs.empty()) {
    usage(argv[0]);
    return 1;
  }
  const char* lr = getenv("LOCAL_RANK");
  const int gpu = o.gpu >= 0 ? o.gpu : (lr ? atoi(lr) : 0) % ndev;
  const int local_id = o.local_id >= 0 ? o.local_id : (lr ? atoi(lr) : 0);
  const int naggs = static_cast<int>(aggs.size());
  auto fail = [&](const char* what) {
    fprintf(stderr, "%s\n", what);
    fprintf(stdout, "\ntest result is 1\n");
    return 1;
  };
  fprintf(stdout, "start connected\n");  // client.cc:348
  // connect to every aggregator in list order (common.cc:71-97) and learn this worker's ID from each
  std::vector<int> fds(naggs, -1);
  int rank = -1, num_workers = 0;
  for (int j = 0; j < naggs; ++j) {
    fds[j] = omrnet::connect_to(omrnet::host_of(aggs[j]).c_str(), omrnet::port_of(aggs[j], o.port));
    if (fds[j] < 0) return fail("failed to connect to an aggregator");
    omrnet::Hello2 h{omrnet::kMagic2, gpu, local_id, j, naggs, o.transport, o.messages ? 1 : 0, o.colocated ? 1 : 0,
                     o.warmups, o.rounds, o.block, o.n};
    omrnet::Assign2 a{};
    if (!omrnet::send_all(fds[j], &h, sizeof(h)) || !omrnet::recv_all(fds[j], &a, sizeof(a)) ||
        a.magic != omrnet::kMagic2)
      return fail("rendezvous failed");
    if (j == 0) {
      rank = a.rank;
      num_workers = a.num_workers;
    } else if (a.rank != rank || a.num_workers != num_workers) {
      return fail("machine ID or number error");  // common.cc:1225-1230
    }
  }
  if (hipSetDevice(gpu) != hipSuccess) return fail("hipSetDevice failed");
  // the transport: workers 0..m-1 (+ the n aggregators m..m+n-1 unless -C); worker 0 makes its id, aggregator 0
  // relays it to the other workers
  char uid[omrnet::kIdBytes];
  if (rank == 0) {
    const int rc0 = o.transport == omrnet::kIpc ? omr_dist_ipc_unique_id(uid) : omr_dist_unique_id(uid);
    if (rc0) return fail(omr_dist_last_error());
    for (int j = 0; j < naggs; ++j)
      if (!omrnet::send_all(fds[j], uid, sizeof(uid))) return fail("failed to send the transport id");
  } else if (!omrnet::recv_all(fds[0], uid, sizeof(uid))) {
    return fail("failed to receive the transport id");
  }
  const int world = o.colocated ? num_workers : num_workers + naggs;
  omr_dist* d = nullptr;
  const int crc = o.transport == omrnet::kIpc ? omr_dist_create_ipc(uid, rank, world, &d)
                                              : omr_dist_create_rccl(uid, rank, world, &d);
  if (crc) return fail(omr_dist_last_error());
  std::cout << "Number of aggregators: " << (o.colocated ? num_workers : naggs) << "; Number of workers is "
            << num_workers << "; My ID is " << rank << std::endl;  // client.cc:364
  printf("Connected.\n");
  if (o.messages) rc = run_msg_worker(d, o, gpu, num_workers, o.colocated ? num_workers : naggs);
  else rc = run_worker(d, o, gpu, rank == 0, num_workers);
  omr_dist_destroy(d);
  omrnet::Done done{omrnet::kMagic2, rank, rc};
  for (int fd : fds) {
    omrnet::send_all(fd, &done, sizeof(done));
    ::close(fd);
  }
  fprintf(stdout, "\ntest result is %d\n", rc);
  return rc;
}
