// omr_net.hpp — the small TCP rendezvous between ./omr_server and ./omr_client.
//
// It stands in for the reference's TCP bootstrap (sock_connect / sock_sync_data, common.cc:50-197, and the
// cm_con_data_t exchange of connect_qp, common.cc:1160-1324): instead of QP numbers and rkeys, the peers
// exchange worker IDs and the RCCL unique id.  Worker IDs follow the reference rule: a worker's ID is the index
// of its IP in the server's worker list (common.cc:123-133, :1191-1224); workers sharing one IP (one node, one
// process per GPU) are ordered by the GPU index they announce.
#pragma once

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace omrnet {

constexpr uint32_t kMagic = 0x4f4d5230;  // "OMR0"
constexpr int kIdBytes = 128;

struct Hello {  // client -> server
  uint32_t magic;
  int32_t gpu;  // local GPU index: orders workers that share an IP
};
struct Assign {  // server -> client
  uint32_t magic;
  int32_t rank;
  int32_t world;
};
struct Done {  // client -> server
  uint32_t magic;
  int32_t rank;
  int32_t status;
};

// Protocol 2: the servers are aggregator ranks of the transport (m workers + n aggregators).  Each worker connects to
// every aggregator of its list in order and tells it its position and the list's length, as the reference's
// cm_con_data_t does (remoteId = i, num_machines = num_socks: common.cc:1189-1232); the aggregator answers with the
// worker's ID (its IP's position in the server's list, common.cc:123-133) and the number of workers.  Worker 0 then
// sends the transport id to every aggregator, and aggregator 0 relays it to the other workers.
constexpr uint32_t kMagic2 = 0x4f4d5232;  // "OMR2"
enum Transport : int32_t { kRccl = 0, kIpc = 1 };
struct Hello2 {  // worker -> aggregator j
  uint32_t magic;
  int32_t gpu, local;       // order workers sharing one IP
  int32_t agg, num_aggs;    // j, n
  int32_t transport;        // Transport
  int32_t messages;         // 1: the round as wire messages (-M)
  int32_t colocated;        // 1: the workers aggregate their own shards; the servers only meet them
  int32_t warmups, rounds;  // the number of rounds the aggregators must take part in
  uint32_t block;
  uint64_t n;
};
struct Assign2 {  // aggregator j -> worker
  uint32_t magic;
  int32_t rank, num_workers, agg;
};

// "host" or "host:port" (a port per aggregator lets several run on one host)
inline std::string host_of(const std::string& s) {
  const size_t c = s.rfind(':');
  return c == std::string::npos ? s : s.substr(0, c);
}
inline int port_of(const std::string& s, int dflt) {
  const size_t c = s.rfind(':');
  return c == std::string::npos ? dflt : atoi(s.c_str() + c + 1);
}

inline bool send_all(int fd, const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n) {
    ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
    if (k <= 0) {
      if (k < 0 && errno == EINTR) continue;
      return false;
    }
    c += k;
    n -= static_cast<size_t>(k);
  }
  return true;
}

inline bool recv_all(int fd, void* p, size_t n) {
  char* c = static_cast<char*>(p);
  while (n) {
    ssize_t k = ::recv(fd, c, n, 0);
    if (k <= 0) {
      if (k < 0 && errno == EINTR) continue;
      return false;
    }
    c += k;
    n -= static_cast<size_t>(k);
  }
  return true;
}

inline int listen_on(int port) {
  int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  if (fd < 0) return -1;
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_ANY);
  a.sin_port = htons(static_cast<uint16_t>(port));
  if (::bind(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) < 0 || ::listen(fd, 64) < 0) {
    ::close(fd);
    return -1;
  }
  return fd;
}

// connect with retries (the server may start after the clients, as the reference's sock_connect loops do)
inline int connect_to(const char* host, int port, int tries = 600) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  char ps[16];
  snprintf(ps, sizeof(ps), "%d", port);
  if (getaddrinfo(host, ps, &hints, &res) != 0 || res == nullptr) return -1;
  int fd = -1;
  for (int t = 0; t < tries; ++t) {
    fd = ::socket(res->ai_family, res->ai_socktype, res->ai_protocol);
    if (fd >= 0 && ::connect(fd, res->ai_addr, res->ai_addrlen) == 0) break;
    if (fd >= 0) ::close(fd);
    fd = -1;
    usleep(100000);
  }
  freeaddrinfo(res);
  if (fd >= 0) {
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  }
  return fd;
}

inline std::string peer_ip(int fd) {
  sockaddr_in a{};
  socklen_t len = sizeof(a);
  if (getpeername(fd, reinterpret_cast<sockaddr*>(&a), &len) != 0) return "";
  char buf[INET_ADDRSTRLEN];
  inet_ntop(AF_INET, &a.sin_addr, buf, sizeof(buf));
  return buf;
}

inline std::vector<std::string> split_list(const char* s) {  // "a,b,c" as client.cc:321-329
  std::vector<std::string> out;
  if (s == nullptr) return out;
  std::string cur;
  for (const char* c = s; *c; ++c) {
    if (*c == ',') {
      if (!cur.empty()) out.push_back(cur);
      cur.clear();
    } else {
      cur.push_back(*c);
    }
  }
  if (!cur.empty()) out.push_back(cur);
  return out;
}

// print_config (common.cc:1405-1427), same lines
inline void print_config(bool server, const std::vector<std::string>& peers, int port, const char* dev, int ib_port,
                         int gid, int sl) {
  fprintf(stdout, " ------------------------------------------------\n");
  for (size_t i = 0; i < peers.size(); ++i)
    fprintf(stdout, " %s %zu : %s\n", server ? "Client" : "Server", i, peers[i].c_str());
  fprintf(stdout, " TCP port : %u\n", port);
  fprintf(stdout, " Device name : \"%s\"\n", dev ? dev : "(null)");
  fprintf(stdout, " IB port : %u\n", ib_port);
  if (gid >= 0) fprintf(stdout, " GID index : %u\n", gid);
  fprintf(stdout, " Service level : %u\n", sl);
  fprintf(stdout, " ------------------------------------------------\n\n");
}

}  // namespace omrnet
