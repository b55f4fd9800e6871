// omr_server.cpp — ./omr_server: the aggregator-side entry point with the reference CLI (server.cc:222-356).
//
//   ./omr_server [-p port] [-d ib-dev] [-i ib-port] [-g gid-idx] [-s service-level] worker_ip[,worker_ip...]
//
// In the MI355X build the aggregation itself is sharded over the workers' GPUs (each GPU sums one shard of the
// block space over xGMI, omr_dist.h), so this process is the rendezvous the reference's server is for its
// workers: it accepts the m workers (server.cc:297-312 / sock_connect), gives each its ID by the position of
// its IP in the worker list (common.cc:123-133, :1191-1224), relays worker 0's RCCL unique id to everyone (the
// cm_con_data_t exchange, common.cc:1160-1324), and reports when every worker has finished its rounds.
// -d/-i/-g/-s are accepted for drop-in compatibility and only printed (there is no verbs device here).
#include <getopt.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <string>
#include <vector>

#include "omr_net.hpp"

static void usage(const char* argv0) {  // common.cc:1441-1457, with the default port fixed to the real one
  fprintf(stdout, "Usage:\n %s start a server and wait for connection\n\n", argv0);
  fprintf(stdout, "Options:\n");
  fprintf(stdout, " -p, --port <port> listen on/connect to port <port> (default 19875)\n");
  fprintf(stdout, " -d, --ib-dev <dev> accepted for compatibility (no verbs device is used)\n");
  fprintf(stdout, " -i, --ib-port <port> accepted for compatibility\n");
  fprintf(stdout, " -g, --gid_idx <git index> accepted for compatibility\n");
  fprintf(stdout, " -s, --service-level <sl> accepted for compatibility\n");
  fprintf(stdout, " -h, --help show this help message\n");
}

int main(int argc, char* argv[]) {
  int port = 19875, ib_port = 1, gid = -1, sl = 0;  // server.cc:3-12
  const char* dev = nullptr;
  static option longopts[] = {{"port", 1, nullptr, 'p'},        {"ib-dev", 1, nullptr, 'd'},
                              {"ib-port", 1, nullptr, 'i'},     {"gid-idx", 1, nullptr, 'g'},
                              {"service-level", 1, nullptr, 's'}, {"help", 0, nullptr, 'h'},
                              {nullptr, 0, nullptr, 0}};
  while (true) {
    int c = getopt_long(argc, argv, "p:d:i:g:s:h", longopts, nullptr);
    if (c == -1) break;
    switch (c) {
      case 'p': port = static_cast<int>(strtoul(optarg, nullptr, 0)); break;
      case 'd': dev = optarg; break;
      case 'i': ib_port = static_cast<int>(strtoul(optarg, nullptr, 0)); break;
      case 'g': gid = static_cast<int>(strtoul(optarg, nullptr, 0)); break;
      case 's': sl = static_cast<int>(strtoul(optarg, nullptr, 0)); break;
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
    fprintf(stdout, "\ntest result is 1\n");
    return 1;
  }
  struct Conn {
    int fd;
    std::string ip;
    int gpu;
    int rank;
  };
  std::vector<Conn> conns;
  while (static_cast<int>(conns.size()) < m) {
    int fd = ::accept(lfd, nullptr, nullptr);
    if (fd < 0) continue;
    omrnet::Hello h{};
    if (!omrnet::recv_all(fd, &h, sizeof(h)) || h.magic != omrnet::kMagic) {
      ::close(fd);
      continue;
    }
    conns.push_back({fd, omrnet::peer_ip(fd), h.gpu, -1});
  }
  // IDs: list position of the peer IP (common.cc:123-133); workers on one IP ordered by their GPU index
  std::stable_sort(conns.begin(), conns.end(), [](const Conn& a, const Conn& b) { return a.gpu < b.gpu; });
  std::vector<bool> taken(m, false);
  for (int i = 0; i < m; ++i) {
    for (auto& c : conns)
      if (c.rank < 0 && c.ip == workers[i]) {
        c.rank = i;
        taken[i] = true;
        break;
      }
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
    omrnet::Assign a{omrnet::kMagic, c.rank, m};
    if (!omrnet::send_all(c.fd, &a, sizeof(a))) rc = 1;
  }
  char uid[omrnet::kIdBytes];
  auto root = std::find_if(conns.begin(), conns.end(), [](const Conn& c) { return c.rank == 0; });
  if (rc != 0 || !omrnet::recv_all(root->fd, uid, sizeof(uid))) {
    fprintf(stderr, "failed to receive the RCCL id from worker 0\n");
    fprintf(stdout, "\ntest result is 1\n");
    return 1;
  }
  for (auto& c : conns)
    if (c.rank != 0 && !omrnet::send_all(c.fd, uid, sizeof(uid))) rc = 1;
  std::cout << "Number of aggregators: " << 1 << "; Number of workers is " << m << "; My ID is " << 0 << std::endl;
  printf("Connected.\n");
  for (auto& c : conns) {
    omrnet::Done d{};
    if (!omrnet::recv_all(c.fd, &d, sizeof(d)) || d.magic != omrnet::kMagic || d.status != 0) rc = 1;
    ::close(c.fd);
  }
  ::close(lfd);
  fprintf(stdout, "\ntest result is %d\n", rc);
  return rc;
}
