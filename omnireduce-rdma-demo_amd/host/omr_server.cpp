// omr_server.cpp — ./omr_server: the aggregator with the reference CLI (server.cc:222-356).
//
//   ./omr_server [-p port] [-d ib-dev] [-i ib-port] [-g gid-idx] [-s service-level] [-G gpu] worker_ip[,worker_ip...]
//
// It accepts the m workers of its list (server.cc:297-312 / sock_connect), gives each its ID by the position of its
// IP in the list (common.cc:123-133; workers sharing one IP ordered by the local id and GPU they announce), and
// learns from them its own index j among the n aggregators and n itself (the cm_con_data_t exchange,
// common.cc:1189-1232).  It then joins the workers' transport (RCCL over xGMI, or HIP IPC for processes sharing a
// GPU) as aggregator rank m + j and takes part in every round the workers run:
//   bulk rounds (omr_ar_plan_create_roles): it receives its shard's non-zero blocks from every worker, sums them in
//   rank order (server.cc:97-98) and returns the sums to every worker (server.cc:162);
//   -M on the workers (omr_msgd_*): the reference's wire messages of the global slots gs % n == j
//   (common.cc:381-383), replied to slot by slot as server.cc:56-199 does.
// With -C on the workers (co-located aggregation) it only introduces them and relays the transport id.
// -d/-i/-g/-s are accepted for drop-in compatibility and only printed (there is no verbs device here).
#include <getopt.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <string>
#include <vector>

#include "omr.h"
#include "omr_dist.h"
#include "omr_net.hpp"

static void usage(const char* argv0) {  // common.cc:1441-1457, with the default port fixed to the real one
  fprintf(stdout, "Usage:\n %s start a server and wait for connection\n\n", argv0);
  fprintf(stdout, "Options:\n");
  fprintf(stdout, " -p, --port <port> listen on/connect to port <port> (default 19875)\n");
  fprintf(stdout, " -d, --ib-dev <dev> accepted for compatibility (no verbs device is used)\n");
  fprintf(stdout, " -i, --ib-port <port> accepted for compatibility\n");
  fprintf(stdout, " -g, --gid_idx <git index> accepted for compatibility\n");
  fprintf(stdout, " -s, --service-level <sl> accepted for compatibility\n");
  fprintf(stdout, " -G <gpu> the GPU this aggregator uses (default $LOCAL_RANK or 0)\n");
  fprintf(stdout, " -h, --help show this help message\n");
}

namespace {

int result(int rc) {
  fprintf(stdout, "\ntest result is %d\n", rc);
  return rc;
}

// the aggregator's part of every round the workers run (they announced the count and the mode)
int aggregate(omr_dist* d, const omrnet::Hello2& h, int num_workers) {
  const uint32_t lanes = omr_num_lanes(h.block);
  const int total = h.warmups + h.rounds;
  hipStream_t st;
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return 1;
  int rc = 0;
  if (h.messages) {
    omr_msgd_plan* plan = nullptr;
    if (omr_msgd_plan_create(d, static_cast<uint32_t>(num_workers), h.n, h.block, lanes, OMR_NUM_THREADS, &plan)) {
      fprintf(stderr, "omr_msgd_plan_create: %s\n", omr_dist_last_error());
      return 1;
    }
    uint32_t maxr = 0;
    for (int r = 0; r < total && rc == 0; ++r) {
      if (omr_msgd_round_f32(plan, nullptr, nullptr, &maxr, st) || hipStreamSynchronize(st) != hipSuccess) {
        fprintf(stderr, "failed to run the round: %s\n", omr_dist_last_error());
        rc = 1;
      }
    }
    if (rc == 0) std::cout << "protocol rounds (largest slot): " << maxr << std::endl;
    omr_msgd_plan_destroy(plan);
  } else {
    omr_ar_plan* plan = nullptr;
    if (omr_ar_plan_create_roles(d, static_cast<uint32_t>(num_workers), h.n, h.block, lanes, OMR_NUM_THREADS, &plan)) {
      fprintf(stderr, "omr_ar_plan_create_roles: %s\n", omr_dist_last_error());
      return 1;
    }
    uint64_t uni = 0;
    for (int r = 0; r < total && rc == 0; ++r) {
      if (omr_sparse_round_f32(plan, nullptr, nullptr, nullptr, nullptr, nullptr, OMR_ROUND_ALLREDUCE, nullptr, &uni,
                               st) ||
          hipStreamSynchronize(st) != hipSuccess) {
        fprintf(stderr, "failed to run the round: %s\n", omr_dist_last_error());
        rc = 1;
      }
    }
    if (rc == 0) std::cout << "blocks aggregated per round: " << uni << std::endl;
    omr_ar_plan_destroy(plan);
  }
  (void)hipStreamDestroy(st);
  return rc;
}

}  // namespace

int main(int argc, char* argv[]) {
  int port = 19875, ib_port = 1, gid = -1, sl = 0, gpu = -1;  // server.cc:3-12
  const char* dev = nullptr;
  static option longopts[] = {{"port", 1, nullptr, 'p'},        {"ib-dev", 1, nullptr, 'd'},
                              {"ib-port", 1, nullptr, 'i'},     {"gid-idx", 1, nullptr, 'g'},
                              {"service-level", 1, nullptr, 's'}, {"help", 0, nullptr, 'h'},
                              {nullptr, 0, nullptr, 0}};
  while (true) {
    int c = getopt_long(argc, argv, "p:d:i:g:s:G:h", longopts, nullptr);
    if (c == -1) break;
    switch (c) {
      case 'p': port = static_cast<int>(strtoul(optarg, nullptr, 0)); break;
      case 'd': dev = optarg; break;
      case 'i': ib_port = static_cast<int>(strtoul(optarg, nullptr, 0)); break;
      case 'g': gid = static_cast<int>(strtoul(optarg, nullptr, 0)); break;
      case 's': sl = static_cast<int>(strtoul(optarg, nullptr, 0)); break;
      case 'G': gpu = atoi(optarg); break;
      default: usage(argv[0]); return 1;
    }
  }
  std::vector<std::string> workers = omrnet::split_list(optind == argc - 1 ? argv[optind] : nullptr);
  if (workers.empty()) {
    usage(argv[0]);
    return 1;
  }
  omrnet::print_config(true, workers, port, dev, ib_port, gid, sl);
  const int m = static_cast<int>(workers.size());
  int lfd = omrnet::listen_on(port);
  if (lfd < 0) {
    fprintf(stderr, "failed to listen on port %d\n", port);
    return result(1);
  }
  struct Conn {
    int fd;
    std::string ip;
    omrnet::Hello2 h;
    int rank;
  };
  std::vector<Conn> conns;
  while (static_cast<int>(conns.size()) < m) {
    int fd = ::accept(lfd, nullptr, nullptr);
    if (fd < 0) continue;
    omrnet::Hello2 h{};
    if (!omrnet::recv_all(fd, &h, sizeof(h)) || h.magic != omrnet::kMagic2) {
      ::close(fd);
      continue;
    }
    conns.push_back({fd, omrnet::peer_ip(fd), h, -1});
  }
  ::close(lfd);
  // every worker must agree on this aggregator's index, the aggregator count and the round they will run
  const omrnet::Hello2 h0 = conns[0].h;
  for (const auto& c : conns)
    if (c.h.agg != h0.agg || c.h.num_aggs != h0.num_aggs || c.h.transport != h0.transport ||
        c.h.messages != h0.messages || c.h.colocated != h0.colocated || c.h.n != h0.n || c.h.block != h0.block ||
        c.h.warmups != h0.warmups || c.h.rounds != h0.rounds) {
      fprintf(stderr, "machine ID or number error\n");  // common.cc:1225-1230
      return result(1);
    }
  const int j = h0.agg, n = h0.num_aggs;
  // IDs: list position of the peer IP (common.cc:123-133); workers on one IP ordered by (local id, GPU)
  std::stable_sort(conns.begin(), conns.end(), [](const Conn& a, const Conn& b) {
    return a.h.local != b.h.local ? a.h.local < b.h.local : a.h.gpu < b.h.gpu;
  });
  std::vector<bool> taken(m, false);
  for (int i = 0; i < m; ++i)
    for (auto& c : conns)
      if (c.rank < 0 && c.ip == workers[i]) {
        c.rank = i;
        taken[i] = true;
        break;
      }
  for (auto& c : conns) {  // peers whose address is not in the list (e.g. a hostname was given) fill the gaps
    if (c.rank >= 0) continue;
    for (int i = 0; i < m; ++i)
      if (!taken[i]) {
        c.rank = i;
        taken[i] = true;
        break;
      }
  }
  int rc = 0;
  for (auto& c : conns) {
    omrnet::Assign2 a{omrnet::kMagic2, c.rank, m, j};
    if (!omrnet::send_all(c.fd, &a, sizeof(a))) rc = 1;
  }
  // the transport id comes from worker 0; aggregator 0 relays it to the other workers
  char uid[omrnet::kIdBytes];
  auto root = std::find_if(conns.begin(), conns.end(), [](const Conn& c) { return c.rank == 0; });
  if (rc != 0 || !omrnet::recv_all(root->fd, uid, sizeof(uid))) {
    fprintf(stderr, "failed to receive the transport id from worker 0\n");
    return result(1);
  }
  if (j == 0)
    for (auto& c : conns)
      if (c.rank != 0 && !omrnet::send_all(c.fd, uid, sizeof(uid))) rc = 1;
  std::cout << "Number of aggregators: " << (h0.colocated ? m : n) << "; Number of workers is " << m
            << "; My ID is " << j << std::endl;  // server.cc:325
  printf("Connected.\n");
  if (!h0.colocated && rc == 0) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
      fprintf(stderr, "no HIP device\n");
      return result(1);
    }
    const char* lr = getenv("LOCAL_RANK");
    const int g = (gpu >= 0 ? gpu : (lr ? atoi(lr) : 0)) % ndev;
    omr_dist* d = nullptr;
    const int rank = m + j, world = m + n;
    int crc = hipSetDevice(g) != hipSuccess ? 1 : 0;
    if (crc == 0)
      crc = h0.transport == omrnet::kIpc ? omr_dist_create_ipc(uid, rank, world, &d)
                                         : omr_dist_create_rccl(uid, rank, world, &d);
    if (crc) {
      fprintf(stderr, "failed to connect: %s\n", omr_dist_last_error());
      rc = 1;
    } else {
      rc = aggregate(d, h0, m);
      omr_dist_destroy(d);
    }
  }
  for (auto& c : conns) {
    omrnet::Done dn{};
    if (!omrnet::recv_all(c.fd, &dn, sizeof(dn)) || dn.status != 0) rc = 1;
    ::close(c.fd);
  }
  return result(rc);
}
